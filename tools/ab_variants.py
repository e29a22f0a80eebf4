#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in ONE process (cdna_hip_programming.md rule 24).

    python tools/ab_variants.py [--workload fedavg|iterative|weighted|secagg] [--clients N]
                                [--params P] [--rounds R] [--variants 0,1,2,3,4,5]

Prints per-variant median / min kernel ms and GB/s of algorithmic bytes.
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fedavg")
    ap.add_argument("--clients", type=int, default=1000)
    ap.add_argument("--params", type=int, default=11_689_512)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7,8,9,10,11,12,13,14")
    a = ap.parse_args()
    import torch

    from pygrid_amd import Engine

    mode = {"fedavg": 0, "iterative": 1, "weighted": 2, "secagg": None}[a.workload]
    P, N = a.params, a.clients
    eng = Engine(0)
    eng.set_layout([P])
    if mode is None:
        eng.reserve(N, 1, 2)
        alg = 16 * N * P + 12 * P
    else:
        eng.reserve(N)
        alg = 4 * N * P + 8 * P
    eng.synth_fill(1, N)
    sp = torch.cuda.current_stream().cuda_stream
    ck = torch.empty(P, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    s_out = torch.empty(P, dtype=torch.int64, device="cuda")
    eng.synth_ckpt_device(1, ck.data_ptr(), sp)
    if mode == 2:
        eng.set_weights([1.0 + (c % 3) for c in range(N)])
    variants = [int(v) for v in a.variants.split(",")]
    times = {v: [] for v in variants}

    def run():
        if mode is None:
            eng.secagg_device(s_out.data_ptr(), out.data_ptr(), 10, 3, sp)
        else:
            eng.fedavg_device(mode, ck.data_ptr(), out.data_ptr(), sp)

    for v in variants:  # warm every variant once
        eng.set_variant(v)
        run()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for v in variants:
            eng.set_variant(v)
            eng.reset_stats()
            for _ in range(a.reps):
                run()
            st = eng.stats()
            times[v].append(st["kernel_ms_total"] / st["kernel_launches"])
    res = {}
    for v in variants:
        med, mn = statistics.median(times[v]), min(times[v])
        res[v] = {"median_ms": round(med, 4), "min_ms": round(mn, 4), "GBps_median": round(alg / med / 1e6, 1)}
    print(json.dumps({"workload": a.workload, "P": P, "N": N, "alg_bytes": alg, "variants": res}))


if __name__ == "__main__":
    main()
