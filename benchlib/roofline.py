"""The dominant kernel against the HBM roofline: achieved bytes from HIP-event launch times, and
HBM traffic from rocprofv3 --pmc passes run by bench.py itself (or the committed summary)."""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

from benchlib.common import HBM_PEAK_GBS, ROOT, child_env, run_child


def kernels_sha256() -> str:
    import hashlib

    h = hashlib.sha256()
    for f in ("pygrid_amd/csrc/pgh_kernels.hip", "pygrid_amd/csrc/pgh_kernels.h"):
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()


def load_traffic(workload: str, variant: int, alg_bytes: float):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (profiles/pmc_traffic.json).
    When this launch's algorithmic bytes differ from the profiled launch's (e.g. a range-split
    fold at N > 1), the measured traffic/algorithmic ratio is applied and the source says so.  A
    summary measured on other kernel sources (kernels_sha256 differs) is not quoted: traffic is
    then null and the source says it is stale."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, None
    try:
        e = json.loads(f.read_text()).get(workload, {}).get(str(variant))
        if e is None:
            return None, None
        if e.get("kernels_sha256") != kernels_sha256():
            return None, f"stale: {e.get('source')} was measured on other kernel sources (re-run tools/profile_round.sh)"
        if abs(float(e.get("alg_bytes_per_launch", alg_bytes)) - alg_bytes) <= 1e-6 * alg_bytes:
            return float(e["hbm_bytes_per_launch"]), e.get("source")
        return float(e["ratio"]) * alg_bytes, f"{e.get('source')}; ratio {e['ratio']:.6f} applied to this launch"
    except Exception:
        return None, None


PMC_KERNEL = {"resnet18-fedavg": "k_fedavg", "resnet18-iterative": "k_fedavg", "resnet18-weighted": "k_fedavg",
              "resnet18-secagg": "k_secagg"}


def under_profiler() -> bool:
    return any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def measure_live_traffic(args, timeout_s=(240, 120)):
    """roofline.traffic measured in THIS run: before the parent touches the GPU, the same workload
    runs twice as a child under ``rocprofv3 --pmc`` (FETCH_SIZE, then WRITE_SIZE: one counter
    block per pass, as MI355X_MICROARCH.md's HBM section prescribes), 2 steps each; HBM bytes per
    launch of the dominant kernel = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950's FETCH_SIZE
    counts half the bytes of wide streaming reads).  Returns (bytes per launch, the child's
    algorithmic bytes per launch, note) or None (no profiler, a failed or timed-out pass: the
    committed summary is quoted instead)."""
    import shutil
    import subprocess
    import tempfile

    kernel = PMC_KERNEL.get(args.workload)
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if kernel is None or not Path(prof).exists():
        return None
    sys.path.insert(0, str(ROOT / "tools"))
    from pmc_summarize import per_launch

    tmp = Path(tempfile.mkdtemp(prefix="pgh_pmc_"))
    child = [sys.executable, str(ROOT / "bench.py"), "--workload", args.workload, "--steps", "2", "--warmup", "1",
             "--no-cpu-baseline", "--no-e2e", "--no-live-traffic", "--no-config-lines", "--seed", str(args.seed)]
    if args.variant is not None:
        child += ["--variant", str(args.variant)]
    for flag, v in (("--clients", args.clients), ("--params", args.params)):
        if v:
            child += [flag, str(v)]
    got, alg = {}, None
    try:
        # the first pass may pay a fresh box's first `import torch` (1-2 minutes): a longer limit
        for counter, limit in zip(("FETCH_SIZE", "WRITE_SIZE"), timeout_s):
            r, err = run_child(args, f"pmc_{counter}", [prof, "--pmc", counter, "-d", str(tmp / counter), "-o", "run",
                                                        "--output-format", "csv", "--"] + child,
                               limit, kill="KILL", capture_output=True, env=child_env())
            if err:
                print(f"bench.py: live PMC pass {counter}: {err['error']}; quoting the committed traffic",
                      file=sys.stderr)
                return None
            if r.returncode != 0:
                print(f"bench.py: live PMC pass {counter} failed (rc {r.returncode}); quoting the committed "
                      f"traffic", file=sys.stderr)
                return None
            got[counter] = per_launch(tmp / counter, counter, kernel)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            alg = json.loads(lines[-1])["roofline"]["alg_bytes_per_launch"] if lines else alg
    except (Exception, SystemExit) as e:  # noqa: BLE001 -- evidence only: never fails the bench
        print(f"bench.py: live PMC passes unusable ({e}); quoting the committed traffic", file=sys.stderr)
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch, n, _ = got["FETCH_SIZE"]
    write, _, _ = got["WRITE_SIZE"]
    where = "on GPU 0 before any rank of this world touched a GPU" if args.gpus > 1 else "before its timed run"
    note = (f"live: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of this workload (2 steps each, "
            f"{n} {kernel} launches per pass, one GPU) run by bench.py {where}; (2*FETCH_SIZE + WRITE_SIZE)*1024")
    return (2 * fetch + write) * 1024, alg, note


def wants_live_traffic(args) -> bool:
    """Every N: the passes run before the world forms, on rank 0 (or the
    parent that spawns the ranks), on GPU 0 alone."""
    return (not args.group and not args.dry_run and not args.no_live_traffic and args.workload in PMC_KERNEL
            and not under_profiler())


# (hbm bytes per launch, algorithmic bytes per launch, note) from measure_live_traffic: set in the
# process that measured it, or handed to the ranks it spawns in PGH_BENCH_LIVE_TRAFFIC
LIVE_TRAFFIC = None
LIVE_TRAFFIC_ENV = "PGH_BENCH_LIVE_TRAFFIC"


def live_traffic():
    if LIVE_TRAFFIC is not None:
        return LIVE_TRAFFIC
    env = os.environ.get(LIVE_TRAFFIC_ENV)
    return tuple(json.loads(env)) if env else None


def roofline_of(st, workload, variant, kernel, n_gpus=1):
    """Dominant kernel against one GPU's HBM peak.  A group's stats sum the bytes of its GPUs and
    take the slowest GPU's times (they run concurrently): bytes are divided by n_gpus here.
    ``traffic`` is this run's own PMC measurement when bench.py made one (LIVE_TRAFFIC), else the
    committed summary (profiles/pmc_traffic.json), quoted only for the current kernel sources."""
    n = max(st["kernel_launches"], 1)
    ms = st["kernel_ms_total"] / n
    alg = st["kernel_bytes_total"] / n / n_gpus
    # Launches on two streams (param ranges at N > 1) overlap; each one's event span then includes
    # time shared with its neighbour, so the duration per launch is the busy time (the union of
    # the launch intervals) divided by the launches.  Without overlap the two are equal.
    busy = st.get("kernel_busy_ms_total") or st["kernel_ms_total"]
    overlapped = busy < 0.99 * st["kernel_ms_total"]
    dur = busy / n if overlapped else ms
    achieved = alg / (dur / 1e3) / 1e9
    traffic, src = load_traffic(workload, variant, alg)
    committed = traffic
    lt = live_traffic()
    if lt is not None and kernel == PMC_KERNEL.get(workload):
        live, live_alg, note = lt
        if live_alg and abs(live_alg - alg) <= 1e-6 * alg:
            traffic, src = live, note
        elif live_alg:
            traffic, src = live / live_alg * alg, note + f"; ratio {live / live_alg:.6f} applied to this launch"
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
         "kernel_ms_avg": round(dur, 4), "alg_bytes_per_launch": int(alg), "launches": st["kernel_launches"],
         "traffic_source": src}
    if traffic is not None and committed is not None and traffic is not committed:
        r["traffic_committed"] = committed  # the last evidence pass's figure, for comparison
    if overlapped:
        r["launch_overlap"] = {"event_span_ms_avg": round(ms, 4), "busy_ms_total": round(busy, 3),
                               "note": "launches overlap on two streams: duration = busy time / launches"}
    return r
