"""cpu_baseline: the reference's CPU torch path timed on the box's own host cores (north_star: "next
to the reference CPU torch path timed on the box's own host cores in the same run, with the core
count stated").  Every figure runs in a child process that never touches the GPU, with glibc's
default allocator (the reference node's)."""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

from benchlib.common import WATCHDOG_MARGIN_S, run_child


def usable_cores() -> tuple:
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2/v1 CPU quota (a GPU
    lease's share of a bigger machine shows in the quota, not in os.cpu_count()).  Returns (cores,
    how they were determined)."""
    n = len(os.sched_getaffinity(0))
    how = "sched_getaffinity"
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
            per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None and int(quota) < n:
        n, how = max(1, int(quota)), "cgroup cpu quota"
    return n, how


def cpu_baseline(kind: str, P: int, seed: int, budget_s: float, n: int = 32, all_cores: int = 0, clients: int = 0):
    """The reference's path as the node runs it, in torch on CPU tensors at th.set_num_threads(1)
    (the node's setting, main/__init__.py:8), on a bounded sample: the same P-param shard, `n`
    synthetic clients, repeated until `budget_s` of CPU work.
      mean       cycle_manager.py:276-296                (oracle.fedavg_mean_torch)
      iterative  cycle_manager.py:266-269 + the plan     (oracle.fedavg_iterative_torch)
      secagg     syft share adds + fix-prec decode       (oracle.secagg_sum_torch), 2 parties
      weighted   no reference counterpart: the numpy oracle (oracle.fedavg_weighted)
    Also reported: the same at `all_cores` threads (default: usable_cores(), the GPU box's CPU
    share) and the numpy restatement at 1 thread.  `clients`: the workload's client count; when the
    sample holds fewer, the close figures are its per-byte rate extrapolated (labelled so)."""
    import numpy as np
    import torch

    cores_how = "given"
    if all_cores <= 0:
        all_cores, cores_how = usable_cores()

    from oracle import coracle
    from oracle import oracle as O

    if kind == "secagg":
        n = max(1, n // 4)
        rng = np.random.default_rng(seed)
        sh = [[rng.integers(-2**63, 2**63 - 1, P, dtype=np.int64, endpoint=True) for _ in range(2)] for _ in range(n)]
        tsh = [[torch.from_numpy(x) for x in c] for c in sh]
        sh_np = np.stack([np.stack(c) for c in sh])
        unit_bytes = 8 * 2 * P
        ref = lambda: O.secagg_sum_torch(tsh)  # noqa: E731
        port = lambda: O.fix_prec_decode(O.secagg_sum(sh_np))  # noqa: E731
        what = "syft share adds (torch int64 add, wrapping) + .float() / 10**3 decode (oracle.secagg_sum_torch)"
    else:
        diffs = [[coracle.synth_f32(seed, O.STREAM_DIFF, c, 0, P, float(O.DIFF_SCALE))] for c in range(n)]
        ckpt = [coracle.synth_f32(seed, O.STREAM_CKPT, 0, 0, P, float(O.CKPT_SCALE))]
        tdiffs = [[torch.from_numpy(t) for t in d] for d in diffs]
        tckpt = [torch.from_numpy(t) for t in ckpt]
        unit_bytes = 4 * P
        w = np.linspace(0.5, 2.0, n).astype(np.float32)
        if kind == "iterative":
            ref = lambda: O.fedavg_iterative_torch(tckpt, tdiffs)  # noqa: E731
            port = lambda: O.fedavg_iterative(ckpt, diffs)  # noqa: E731
            what = "cycle_manager.py:266-269 + 01-Create-plan.ipynb:450-454 (oracle.fedavg_iterative_torch)"
        elif kind == "weighted":
            ref = None
            port = lambda: O.fedavg_weighted(ckpt, diffs, w)  # noqa: E731
            what = "no reference counterpart: numpy oracle (oracle.fedavg_weighted)"
        else:
            ref = lambda: O.fedavg_mean_torch(tckpt, tdiffs)  # noqa: E731
            port = lambda: O.fedavg_mean(ckpt, diffs)  # noqa: E731
            what = "cycle_manager.py:276-296 (oracle.fedavg_mean_torch)"

    def rate(fn, budget):
        fn()  # warm: allocator, thread pool after set_num_threads
        reps, t0 = 0, time.perf_counter()
        while True:
            fn()
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return reps * n * unit_bytes / el / 1e9, reps, el

    threads = torch.get_num_threads()
    try:
        torch.set_num_threads(1)
        gbs, reps, el = rate(ref or port, budget_s * 0.5)
        torch.set_num_threads(all_cores)
        gbs_all, _, _ = rate(ref, budget_s * 0.25) if ref else (None, 0, 0)
    finally:
        torch.set_num_threads(threads)
    gbs_np, _, _ = rate(port, budget_s * 0.25) if ref else (gbs, 0, 0)
    close_1000 = lambda g: round(unit_bytes * 1000 / (g * 1e9) * 1e3, 1)  # noqa: E731
    clients = clients or n
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{what}, {f'torch {torch.__version__} CPU tensors' if ref else 'numpy'}, P={P}, {n} clients, "
                      f"{reps} passes in {el:.1f}s, 1 thread (the node's th.set_num_threads(1))",
            "sample_clients": n, "workload_clients": clients,
            # the close figures: the sample's per-byte rate applied to 1,000 / the workload's clients
            "extrapolated": clients != n or n != 1000,
            "cycle_close_ms_per_1000_clients": close_1000(gbs),
            "cycle_close_ms_workload": round(unit_bytes * clients / (gbs * 1e9) * 1e3, 1),
            "all_cores": ({"value": round(gbs_all, 3), "cores": all_cores, "cores_from": cores_how,
                           "cycle_close_ms_per_1000_clients": close_1000(gbs_all)} if gbs_all else None),
            "numpy_restatement_1_thread": round(gbs_np, 3), "cpu_model": cpu_model()}


def in_reference_allocator(fn: str, kwargs: dict, blobs=None, reserve=None):
    """Run ``bench.<fn>(**kwargs)`` in a child process with glibc's default allocator
    (PGH_MALLOC_TUNE=0): importing pygrid_amd raises glibc's mmap threshold (pygrid_amd.hostmem),
    which would also spare the reference's torch code its per-add page faults -- the node it
    stands for runs without that.  ``blobs`` (name -> bytes) reach the child as files.  The child
    never touches the GPU.  ``reserve``: seconds of the run's budget it must leave (default: up to
    the watchdog's margin, for a child that is part of the headline itself)."""
    import shutil
    import subprocess
    import tempfile

    tmp = Path(tempfile.mkdtemp(prefix="pgh_cpu_"))
    try:
        files = {}
        for name, data in (blobs or {}).items():
            paths = []
            for i, b in enumerate(data if isinstance(data, (list, tuple)) else [data]):
                f = tmp / f"{name}_{i}.bin"
                f.write_bytes(b)
                paths.append(str(f))
            files[name] = paths if isinstance(data, (list, tuple)) else paths[0]
        code = ("import json, sys; from pathlib import Path; sys.argv = ['bench.py']; from benchlib import baseline as bench\n"
                "spec = json.loads(sys.stdin.read())\n"
                "kw = dict(spec['kwargs'])\n"
                "for k, v in spec['files'].items():\n"
                "    kw[k] = [Path(p).read_bytes() for p in v] if isinstance(v, list) else Path(v).read_bytes()\n"
                "print(json.dumps(getattr(bench, spec['fn'])(**kw)))")
        r, err = run_child(None, "cpu_baseline", [sys.executable, "-c", code], 600,
                           reserve=WATCHDOG_MARGIN_S + 5 if reserve is None else reserve, capture_output=True,
                           input=json.dumps({"fn": fn, "kwargs": kwargs, "files": files}),
                           env=dict(os.environ, PGH_MALLOC_TUNE="0"))
        if err:
            raise RuntimeError(f"CPU baseline child: {err['error']}")
        if r.returncode != 0:
            raise RuntimeError(f"CPU baseline child failed: {r.stderr.strip().splitlines()[-1:]}")
        out = json.loads(r.stdout.strip().splitlines()[-1])
        out["allocator"] = "glibc defaults (the reference node's): measured in a child without pygrid_amd's heap thresholds"
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cpu_baseline_state(ck_pb: bytes, d_pbs, P: int, n_target: int, budget_s: float):
    """The node's whole bytes -> bytes cycle close on the host (oracle.cycle_close_state_torch:
    State parse + per-tensor torch.tensor conversion, mean, apply, serialize; cycle_manager.py:
    240-303, model_manager.py:79-103) at th.set_num_threads(1).  With all n_target diffs given it
    is timed as is (repeated for budget_s); otherwise closes of 1 and len(d_pbs) diffs are timed
    and the close of n_target diffs extrapolated linearly (fixed + per-diff cost)."""
    import torch

    from oracle import oracle as O

    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        def close_s(pbs, min_s):
            reps, t0 = 0, time.perf_counter()
            while True:
                O.cycle_close_state_torch(ck_pb, pbs)
                reps += 1
                el = time.perf_counter() - t0
                if el >= min_s:
                    return el / reps, reps
        if len(d_pbs) == n_target:
            O.cycle_close_state_torch(ck_pb, d_pbs)  # warm
            t, reps = close_s(d_pbs, budget_s)
            how = f"{reps} closes of {n_target} diffs timed"
            extrap = False
        else:
            t1, _ = close_s(d_pbs[:1], 0.0)
            tn, _ = close_s(d_pbs, 0.0)
            per = (tn - t1) / (len(d_pbs) - 1)
            t = t1 + (n_target - 1) * per
            how = (f"extrapolated: closes of 1 and {len(d_pbs)} diffs timed ({t1 * 1e3:.0f} / {tn * 1e3:.0f} ms, "
                   f"{per * 1e3:.0f} ms per diff), close of {n_target} = fixed + {n_target} x per-diff")
            extrap = True
    finally:
        torch.set_num_threads(threads)
    return {"value": round(4 * n_target * P / t / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle.cycle_close_state_torch: State bytes -> new checkpoint bytes (protobuf ParseFromString "
                      "over the restated schema, torch.tensor(contents_float32) per tensor, reduce(th.add) / th.div / "
                      f"subtract, contents_float32.extend(tolist()) + SerializeToString), torch {torch.__version__}, "
                      f"P={P}, 1 thread; {how}",
            "cycle_close_ms": round(t * 1e3, 2), "extrapolated": extrap, "cpu_model": cpu_model()}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# workload -> (kind, sample clients, note): the reference's arithmetic each resident / streamed
# workload replaces (the bytes -> bytes workloads time the node's whole close themselves)
BASELINE_OF = {
    "resnet18-fedavg": ("mean", 32, None), "resnet18-iterative": ("iterative", 32, None),
    "resnet18-weighted": ("weighted", 32, None), "resnet18-secagg": ("secagg", 32, None),
    "secagg-clients": ("secagg", 32, None),
    "c4-stream": ("mean", 8, "extrapolated: per-byte rate of an 8-client sample of the {N}-client shard"),
    "c5-ingest": ("iterative", 4, "extrapolated: per-byte rate of a 4-client sample of the {N}-client shard, diffs "
                                  "already in host memory (no ingest)"),
}


def wants_cpu_baseline(args) -> bool:
    return not args.no_cpu_baseline and not args.group and args.workload in BASELINE_OF


def pre_world_cpu_baseline(args, reserve: float) -> dict:
    """The reference's arithmetic for this workload timed on the host (cpu_baseline above) on a
    bounded sample of one GPU's shard -- at EVERY N, by rank 0 (or the
    parent that spawns the ranks) before any rank touches a GPU, so no rank's GPU work shares the
    host cores with it.  Weak scaling: the shard, and so the sample, is the same at every N."""
    from benchlib.common import WORKLOADS

    kind, n, note = BASELINE_OF[args.workload]
    _, _, n_default, _, pg_default = WORKLOADS[args.workload]
    P, N = args.params or pg_default, args.clients or n_default
    try:
        out = in_reference_allocator("cpu_baseline", {"kind": kind, "P": P, "seed": args.seed,
                                                      "budget_s": args.cpu_seconds, "n": n, "clients": N},
                                     reserve=reserve)
        if note and "sample" in out:
            out["sample"] += "; " + note.format(N=N)
        out["measured"] = (f"before the {args.gpus}-GPU world formed, on the host cores of the run's rank 0"
                           if args.gpus > 1 else "before the timed run, no GPU work beside it")
        return out
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}
