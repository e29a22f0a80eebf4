"""A rank's world (torch.distributed over RCCL, or gloo for rehearsals and dry runs), the timed
loop, the JSON record, and the --check legs that hold sampled params of a full-size run against
the oracle (checker legs outside the timed region)."""
from __future__ import annotations

import os
import time

from benchlib.common import (DATA_DEVICE, DATA_HOST, HBM_PEAK_GBS, HOST_DATA_WORKLOADS, HW_QUEUES, METRIC,
                             PROCESS_TUNING)


class Ctx:
    """Per-rank setup shared by the workloads."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.group = args.group
        self.n_gpus = args.gpus if args.group else self.world  # GPUs measured (whole job)
        if self.group and self.world != 1:
            raise SystemExit("bench.py --group drives every GPU from one process: launch it once")
        if not self.group and self.world != args.gpus:
            # main() spawns the ranks itself when no launcher did; a launcher with another world
            # size would measure a different configuration than the one named
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher formed WORLD_SIZE {self.world}")
        # PGH_BENCH_DEVICE / PGH_DIST_BACKEND only exist to rehearse the N > 1 path with several
        # ranks on one GPU over gloo; the driver's runs use one GPU per rank and RCCL ("nccl").
        self.dry = args.dry_run
        self.device = int(os.environ.get("PGH_BENCH_DEVICE", self.local))
        self.backend = "gloo" if self.dry else os.environ.get("PGH_DIST_BACKEND", "nccl")
        self.tdev = "cpu" if self.dry else "cuda"
        if not self.dry:
            torch.cuda.set_device(self.device)
        if self.world > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.device))
            else:
                dist.init_process_group(self.backend)
            formed = int(self.sum_over_ranks(1.0))
            if formed != args.gpus:
                raise SystemExit(f"bench.py: formed a world of {formed} ranks, --gpus {args.gpus}")
        # what the exchange really ran over: torch's "nccl" backend IS RCCL on ROCm
        self.dist_backend = str(dist.get_backend()) if self.world > 1 else None
        self.rccl_ranks = self.world if self.dist_backend == "nccl" else 0
        self.coll = {"nccl": "RCCL", "gloo": "gloo (host)"}.get(self.dist_backend, self.dist_backend)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.tdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: float) -> float:
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.tdev)
        self.dist.all_reduce(t)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed(ctx, step, steps, warmup, eng):
    torch = ctx.torch
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    el = time.perf_counter() - t0
    return ctx.max_over_ranks(el), eng.stats()


def record(ctx, args, name, value, el, dt, config, roofline, extra=None, step_is="kernel"):
    """One JSON line.  `step_is` names what one timed step is: "kernel" (the resident lines: the
    fold of HBM-resident diffs, plus the collective at N > 1) -> `kernel_ms`; "close" (bytes in ->
    bytes out: the whole _average_plan_diffs slice) -> `cycle_close_ms`."""
    rec = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": ctx.n_gpus,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dt,
        "data": DATA_HOST if name in HOST_DATA_WORKLOADS else DATA_DEVICE,
        "config": config,
        "pct_hbm_peak_per_gpu": round(100 * value / ctx.n_gpus / HBM_PEAK_GBS, 2),
        ("kernel_ms" if step_is == "kernel" else "cycle_close_ms"): round(el / args.steps * 1e3, 4),
        "roofline": roofline, "cpu_baseline": None,
        "hip_hw_queues": HW_QUEUES, "process_tuning": dict(PROCESS_TUNING),
        "dist_backend": getattr(ctx, "dist_backend", None), "rccl_ranks": getattr(ctx, "rccl_ranks", 0),
    }
    if extra:
        rec.update(extra)
    return rec


def check_sampled(ctx, args, full, lo: int, hi: int, expected, against: str = None) -> dict:
    """``--check``: a checker leg outside the timed region (like cpu_baseline, the only other place
    this script runs the oracle).  Every rank takes its share of a strided 4,096-param sample of
    its own shard [lo, hi) (both edges included) and computes the oracle's values for them from its own
    inputs (``expected(idx)``); rank 0 gathers them and compares ``full`` -- the all-gathered new
    checkpoint, or the one shard at N = 1 -- at every rank's indices, bit for bit."""
    import numpy as np

    torch = ctx.torch
    # a strided sample of 4,096 params over the whole model (config 4's golden check),
    # this rank's share of it, plus its shard's edges
    k = max(1, -(-4096 // ctx.world))
    idx = np.unique(np.concatenate([[lo, hi - 1], lo + (np.arange(k, dtype=np.int64) * (hi - lo)) // k]))
    idx = idx[(idx >= lo) & (idx < hi)].astype(np.int64)
    want = np.ascontiguousarray(expected(idx), np.float32)
    mine = (idx.tolist(), want.view(np.uint32).tolist())
    if ctx.world > 1:
        got = [None] * ctx.world
        ctx.dist.all_gather_object(got, mine)
    else:
        got = [mine]
    if ctx.rank != 0:
        return None
    all_idx = np.array([i for g in got for i in g[0]], np.int64)
    all_want = np.array([w for g in got for w in g[1]], np.uint32)
    have = full[torch.from_numpy(all_idx).to(full.device)].float().cpu().numpy().view(np.uint32)
    bad = int((have != all_want).sum())
    return {"bit_exact": bad == 0, "mismatches": bad, "params_checked": int(all_idx.size), "ranks": ctx.world,
            "against": against or "oracle (coracle.fedavg over the sampled params of every client, from each rank's "
                                  "own inputs)",
            "after": "all-gather of the sharded new checkpoint" if ctx.world > 1 else "one GPU (no exchange)"}


def check_resident(ctx, args, full, mode, dtype, N, S, lo, hi, local_sums=None) -> dict:
    """``--check`` of the resident configs 2 and 3 (a checker leg outside the timed region): the
    oracle regenerates every client's diff (or S shares) at a strided 4,096-param sample on the CPU
    (oracle.synth_diff / synth_shares: the restatement of the on-device generator) and computes
    the expected values with the C oracle (coracle.fedavg / coracle.secagg); rank 0 compares the
    new checkpoint (config 3: the decoded sum) after the all-gather bit for bit, and every rank
    compares its own int64 Z_2^64 sums."""
    import numpy as np

    from oracle import coracle
    from oracle import oracle as O

    torch = ctx.torch
    if dtype == 0:
        w = np.array([(c % 7 + 1) * 0.5 for c in range(N)], np.float32) if mode == 2 else None

        def expected(idx):
            u = idx.astype(np.uint64)
            return coracle.fedavg(mode, np.stack([O.synth_diff(args.seed, c, u) for c in range(N)]),
                                  O.synth_ckpt(args.seed, u), w)
        return check_sampled(ctx, args, full, lo, hi, expected,
                             against=f"oracle (coracle.fedavg mode {mode} over the sampled params of all {N} clients, "
                                     "regenerated on the CPU)")
    bad_sums = [0]

    def expected_dec(idx):
        u = idx.astype(np.uint64)
        want_s, want_d = coracle.secagg(np.stack([O.synth_shares(args.seed, c, S, u) for c in range(N)]), idx.size)
        got = local_sums[torch.from_numpy(idx - lo).to(local_sums.device)].cpu().numpy()
        bad_sums[0] = int((got != want_s).sum())
        return want_d
    rec = check_sampled(ctx, args, full, lo, hi, expected_dec,
                        against=f"oracle (coracle.secagg over the sampled params of all {N} clients x {S} parties, "
                                "regenerated on the CPU): decoded float32 after the all-gather and every rank's "
                                "int64 sums")
    bad = int(ctx.sum_over_ranks(float(bad_sums[0])))
    if rec is not None:
        rec["sum_mismatches"] = bad
        rec["bit_exact"] = bool(rec["bit_exact"] and bad == 0)
    return rec
