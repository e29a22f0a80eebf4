#!/usr/bin/env python3
"""Benchmark of the PyGrid cycle-close aggregation hot path on MI355X.

Metric (BASELINE.json): client-diff GB/s aggregated (% of HBM peak) at 1/2/4/8 MI355X; cycle
close ms.  Workload at N = 1: BASELINE configs[1], ResNet-18 (11,689,512 params) fp32 FedAvg
over 1,000 synthetic client diffs resident on one MI355X (46.8 GB).  A "step" is one cycle
close of that workload: the fused mean + apply kernel over all [1000][P] diffs, producing the
new checkpoint (for N > 1 also the RCCL all-gather that assembles it).

Scaling: weak.  Rank r owns a 11,689,512-param shard of a (N x 11.69M)-param model (the
parameter-axis sharding of SURVEY.md 8(e)), all 1,000 clients, so per-GPU work is fixed.

    python bench.py [--gpus N --steps K --warmup W] [--workload resnet18-fedavg|resnet18-iterative|
                     resnet18-weighted|resnet18-secagg] [--variant V] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md "HBM3E peak BW 8.0 TB/s spec"
RESNET18_P = 11_689_512
WORKLOADS = {
    # name: (mode, dtype, default clients, parties)
    "resnet18-fedavg": (0, 0, 1000, 1),
    "resnet18-iterative": (1, 0, 1000, 1),
    "resnet18-weighted": (2, 0, 1000, 1),
    "resnet18-secagg": (None, 1, 1000, 2),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="resnet18-fedavg", choices=sorted(WORKLOADS))
    ap.add_argument("--clients", type=int, default=None)
    ap.add_argument("--params", type=int, default=RESNET18_P, help="params per GPU shard")
    ap.add_argument("--variant", type=int, default=int(os.environ.get("PGH_VARIANT", "0")))
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    return ap.parse_args()


def cpu_baseline(P: int, seed: int, budget_s: float):
    """The oracle's restatement of cycle_manager.py:276-296 (allocating float32 adds, one thread,
    like the reference node's th.set_num_threads(1), main/__init__.py:8) on a bounded sample:
    the same P-param shard, 32 synthetic clients, repeated until `budget_s` of CPU work."""
    import numpy as np

    from oracle import coracle
    from oracle import oracle as O

    n = 32
    diffs = [[coracle.synth_f32(seed, O.STREAM_DIFF, c, 0, P, float(O.DIFF_SCALE))] for c in range(n)]
    ckpt = [coracle.synth_f32(seed, O.STREAM_CKPT, 0, 0, P, float(O.CKPT_SCALE))]
    reps, t0 = 0, time.perf_counter()
    while True:
        O.fedavg_mean(ckpt, diffs)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    gbs = reps * n * P * 4 / el / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"oracle numpy restatement of cycle_manager.py:276-296, P={P}, {n} clients, "
                      f"{reps} passes in {el:.1f}s, 1 thread",
            "cycle_close_ms_extrapolated_1000_clients": round(el / reps / n * 1000 * 1000, 1)}


def load_traffic(workload: str, variant: int, per_launch_bytes: float):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (profiles/), if present."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, None
    try:
        d = json.loads(f.read_text())
        e = d.get(workload, {}).get(str(variant))
        if e is None:
            return None, None
        return float(e["hbm_bytes_per_launch"]), e.get("source")
    except Exception:
        return None, None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from pygrid_amd import Engine
    from pygrid_amd.sharding import gather_flat, shard_bounds

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    mode, dtype, n_default, parties = WORKLOADS[args.workload]
    N = args.clients or n_default
    Pg = args.params
    P = Pg * world
    lo, hi = shard_bounds(P, world, rank)
    pg = hi - lo

    eng = Engine(local)
    eng.set_layout([P])
    eng.set_shard(lo, hi)
    eng.reserve(N, dtype, parties)
    eng.set_variant(args.variant)
    eng.synth_fill(args.seed, N)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    if dtype == 0:
        ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
        out = torch.empty_like(ckpt)
        eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
        if mode == 2:
            eng.set_weights([(c % 7 + 1) * 0.5 for c in range(N)])

        def step():
            eng.fedavg_device(mode, ckpt.data_ptr(), out.data_ptr(), sp)
            if world > 1:
                gather_flat(out, P, world, rank)
        diff_bytes = 4 * N * pg
        alg_bytes = 4 * N * pg + 8 * pg
        dt = "f32"
    else:
        s_out = torch.empty(pg, dtype=torch.int64, device="cuda")
        d_out = torch.empty(pg, dtype=torch.float32, device="cuda")

        def step():
            eng.secagg_device(s_out.data_ptr(), d_out.data_ptr(), 10, 3, sp)
            if world > 1:
                gather_flat(d_out, P, world, rank)
        diff_bytes = 8 * parties * N * pg
        alg_bytes = diff_bytes + 8 * pg + 4 * pg
        dt = "int64"
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    st = eng.stats()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kernel_ms = st["kernel_ms_total"] / max(st["kernel_launches"], 1)

    total_diff_bytes = diff_bytes * world * args.steps  # every rank processed the same shard size
    value = total_diff_bytes / el / 1e9
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
    traffic, traffic_src = load_traffic(args.workload, args.variant, alg_bytes)

    if rank == 0:
        rec = {
            "metric": "client-diff GB/s aggregated (% of HBM peak) at 1/2/4/8 MI355X; cycle close ms",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dt,
            "data": "synthetic (on-device counter-based generator, SURVEY.md 8(d); restated in oracle/oracle.py)",
            "config": {
                "workload": f"{args.workload}: P_shard={pg} params/GPU x {N} clients"
                            + (f" x {parties} parties int64" if dtype == 1 else " fp32") + ", resident in HBM",
                "clients": N, "params_per_gpu": pg, "params_total": P,
                "parallelism": f"param-shard{world}" + (" + RCCL all-gather" if world > 1 else ""),
                "kernel_variant": args.variant,
            },
            "pct_hbm_peak_per_gpu": round(100 * value / world / HBM_PEAK_GBS, 2),
            "cycle_close_ms": round(el / args.steps * 1e3, 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "k_fedavg" if dtype == 0 else "k_secagg",
                "kernel_ms_avg": round(kernel_ms, 4),
                "alg_bytes_per_launch": alg_bytes,
                "traffic_source": traffic_src,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline and dtype == 0:
            try:
                rec["cpu_baseline"] = cpu_baseline(pg, args.seed, args.cpu_seconds)
            except Exception as e:  # noqa: BLE001
                rec["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(rec), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
