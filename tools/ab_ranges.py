#!/usr/bin/env python3
"""Cost of folding the shard in param ranges (the N > 1 bench path: range i is all-gathered beside
the fold of range i + 1) against one whole-shard fold, on one GPU, interleaved rounds.

    python tools/ab_ranges.py [--chunks 1,2,4,8,16,8t3]      (8t3: 8 ranges, last one halved 3 times)
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1000)
    ap.add_argument("--params", type=int, default=11_689_512)
    ap.add_argument("--chunks", default="1,2,4,8,16")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--streams", type=int, default=1, help="alternate range folds over this many streams")
    a = ap.parse_args()
    import torch

    from pygrid_amd import Engine
    from pygrid_amd.sharding import ALIGN, plan_ranges

    P, N = a.params, a.clients
    eng = Engine(0)
    eng.set_layout([P])
    eng.reserve(N)
    eng.synth_fill(1, N)
    eng.set_variant(a.variant)
    sp = torch.cuda.current_stream().cuda_stream
    ck = torch.empty(P, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    eng.synth_ckpt_device(1, ck.data_ptr(), sp)
    res = {}
    plans = {}
    for k in a.chunks.split(","):
        n, _, t = k.partition("t")
        plans[k] = [(o, b - o) for o, b in plan_ranges(P, int(n), ALIGN, int(t or 0))]
        res[k] = []

    main = torch.cuda.current_stream()
    side = [main] + [torch.cuda.Stream() for _ in range(a.streams - 1)]

    def step(k):
        if k == "1":
            eng.fedavg_device(0, ck.data_ptr(), out.data_ptr(), sp)
        else:
            for s in side[1:]:
                s.wait_stream(main)  # step boundary: every range after the previous step
            for i, (o, n) in enumerate(plans[k]):
                eng.fedavg_device_range(0, o, n, ck.data_ptr(), out.data_ptr(), side[i % len(side)].cuda_stream)
            for s in side[1:]:
                main.wait_stream(s)

    for k in plans:
        step(k)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k in plans:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                step(k)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / 3 * 1e3)
    alg = 4 * N * P + 8 * P
    print(json.dumps({"P": P, "N": N, "variant": a.variant, "streams": a.streams,
                      "chunks": {k: {"ms_median": round(statistics.median(v), 4),
                                     "GBps": round(alg / statistics.median(v) / 1e6, 1)} for k, v in res.items()}}))


if __name__ == "__main__":
    main()
