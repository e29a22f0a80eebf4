"""bench.py's shared pieces: the workload table, the JSON line's constants, and the run's one
deadline -- child runs under ``timeout`` within what is left of it, the
watchdog that prints the headline line before it, stage durations for the line's ``budget``."""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BENCH = ROOT / "bench.py"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


from pygrid_amd import hipenv  # noqa: E402

# Before anything touches HIP (the ranks this script spawns inherit it), this harness ASKS for 16
# hardware queues (PGH_HW_QUEUES: explicit, so hipenv applies it; an operator's own PGH_HW_QUEUES
# wins), so the N > 1 step's RCCL all-gather does not share a queue with the next range's fold.
# Importing pygrid_amd changes nothing by itself; the glibc thresholds are applied in main()
# (pygrid_amd.tune_process), never in the CPU-baseline children.
os.environ.setdefault("PGH_HW_QUEUES", str(hipenv.DEFAULT_HW_QUEUES))
HW_QUEUES = hipenv.prepare()
PROCESS_TUNING = {"hw_queues": HW_QUEUES, "malloc": False}

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md "HBM3E peak BW 8.0 TB/s spec"
METRIC = "client-diff GB/s aggregated (% of HBM peak) at 1/2/4/8 MI355X; cycle close ms"
RESNET18_P = 11_689_512
# name: (mode, dtype, clients, parties, params per GPU)
WORKLOADS = {
    "resnet18-fedavg": (0, 0, 1000, 1, RESNET18_P),
    "resnet18-iterative": (1, 0, 1000, 1, RESNET18_P),
    "resnet18-weighted": (2, 0, 1000, 1, RESNET18_P),
    "resnet18-secagg": (None, 1, 1000, 2, RESNET18_P),
    "secagg-clients": (None, 1, 1000, 2, RESNET18_P),  # clients per GPU; P is the whole model on every rank
    "c4-stream": (0, 0, 10_000, 1, 12_500_000),
    "c5-ingest": (1, 0, 64, 1, 125_000_000),
    "mnist-state": (0, 0, 3, 1, 311_650),
    "resnet18-state": (0, 0, 100, 1, RESNET18_P),
    "resnet18-report": (0, 0, 100, 1, RESNET18_P),
    "resnet18-secagg-state": (None, 1, 16, 2, RESNET18_P),
}


DATA_DEVICE = "synthetic (on-device counter-based generator, SURVEY.md 8(d); restated in oracle/oracle.py)"
DATA_HOST = ("synthetic (seeded numpy arrays in host memory, as State protobuf bytes where the workload "
             "takes bytes: pygrid_amd.state_schema)")
HOST_DATA_WORKLOADS = {"c5-ingest", "mnist-state", "resnet18-state", "resnet18-report", "resnet18-secagg-state"}


# ---- the run's deadline ------------------------------------------------------
# One absolute deadline (wall clock) for this process and everything it starts: child runs get a
# deadline of their own (PGH_BENCH_DEADLINE, inside their `timeout` limit), ranks spawned here share
# this one.  Stage durations go on the line under `budget`.
DEFAULT_BUDGET_S = 540.0
MIN_CHILD_S = 20.0        # a child that would get less is not started (its slot says why)
WATCHDOG_MARGIN_S = 10.0  # the watchdog prints the headline line this long before the deadline
RUN = {"t0": time.time(), "deadline": None, "budget_s": None, "stage": "start", "stages": {}, "printed": False}
_EMIT = threading.Lock()


def set_deadline(args):
    budget = args.budget_s if args.budget_s is not None else float(os.environ.get("PGH_BENCH_BUDGET_S",
                                                                                  DEFAULT_BUDGET_S))
    deadline = RUN["t0"] + budget
    inherited = os.environ.get("PGH_BENCH_DEADLINE")
    if inherited:  # a child run (its parent's limit) or a spawned rank (its parent's deadline)
        deadline = min(deadline, float(inherited))
    RUN["deadline"], RUN["budget_s"] = deadline, round(deadline - RUN["t0"], 1)
    os.environ["PGH_BENCH_DEADLINE"] = repr(deadline)


def remaining() -> float:
    return float("inf") if RUN["deadline"] is None else RUN["deadline"] - time.time()


def headline_reserve(args) -> float:
    if args.headline_reserve_s is not None:
        return float(args.headline_reserve_s)
    return 150.0 if args.gpus == 1 else 120.0


def stub_sleep(stage: str):
    """Test hook (tests/test_bench_launch.py): PGH_BENCH_STUB="config4=1000,group=0" replaces the
    named child runs by a stand-in that sleeps that long and prints a dry-run line."""
    for item in os.environ.get("PGH_BENCH_STUB", "").split(","):
        name, _, secs = item.partition("=")
        if name.strip() == stage:
            return float(secs or 0)
    return None


def run_child(args, stage: str, cmd, want_s: float, reserve=None, kill="TERM", **kw):
    """Run one child line under ``timeout -k 10 <limit>`` with limit = min(want_s, what is left of
    the run's budget minus ``reserve`` (default: the headline's)).  Returns (CompletedProcess or
    None, error dict or None): a child given less than MIN_CHILD_S is not started, one that hits
    its limit is reported as a timeout; either way the caller puts the error in the child's slot
    and the run goes on."""
    import subprocess

    keep = reserve if reserve is not None else headline_reserve(args)
    limit = int(min(want_s, remaining() - keep))
    if limit < MIN_CHILD_S:
        RUN["stages"][stage] = "skipped"
        return None, {"error": f"skipped: {max(remaining(), 0):.0f} s of the run's {RUN['budget_s']} s budget left, "
                               f"{keep:.0f} s kept for the headline", "stage": stage}
    secs = stub_sleep(stage)
    if secs is not None:
        cmd = [sys.executable, "-c", "import json, sys, time; time.sleep(float(sys.argv[1])); "
               "print(json.dumps({'dry_run': True, 'stub': sys.argv[2]}))", str(secs), stage]
    env = kw.pop("env", None) or child_env()
    env["PGH_BENCH_DEADLINE"] = repr(time.time() + limit - 5)  # the child's own watchdog fires first
    print(f"bench.py: {stage}: {limit} s limit ({remaining():.0f} s of the budget left)", file=sys.stderr, flush=True)
    RUN["stage"] = stage
    t = time.time()
    try:
        r = subprocess.run(["timeout", "-s", kill, "-k", "10", str(limit)] + list(cmd), cwd=str(ROOT), env=env,
                           text=True, **kw)
    except OSError as e:
        return None, {"error": f"{stage} child did not start: {e}", "stage": stage}
    finally:
        RUN["stages"][stage] = round(time.time() - t, 1)
    if r.returncode in (124, 137) and time.time() - t >= limit - 1:
        return r, {"error": f"timeout after {limit} s", "stage": stage, "command": " ".join(map(str, cmd[1:]))}
    return r, None


def json_lines(text) -> list:
    return [ln for ln in (text or "").splitlines() if ln.startswith("{")]


def headline_error_line(args, why: str, n_gpus=None) -> dict:
    """The headline line when the headline could not finish: the contract's keys, value null."""
    return {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": n_gpus or args.gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32" if args.workload != "resnet18-secagg" else "int64",
            "data": DATA_DEVICE, "config": {"workload": args.workload}, "roofline": None, "cpu_baseline": None,
            "error": why, "stage": RUN["stage"]}


def emit(rec: dict) -> bool:
    """Print THE result line (once per process: the watchdog and the normal path race for it)."""
    with _EMIT:
        if RUN["printed"]:
            return False
        RUN["printed"] = True
        rec["budget"] = {"budget_s": RUN["budget_s"], "elapsed_s": round(time.time() - RUN["t0"], 1),
                         "stages_s": dict(RUN["stages"])}
        print(json.dumps(rec), flush=True)
        return True


def start_watchdog(args, pre: dict):
    """Print the headline line anyway shortly before the deadline (rank 0; the other ranks just
    exit a little later), then end the process: a hung collective or a slow stage costs the
    headline's value, never the whole line."""
    if RUN["deadline"] is None:
        return
    rank = int(os.environ.get("RANK", "0"))
    margin = WATCHDOG_MARGIN_S if rank == 0 else WATCHDOG_MARGIN_S / 2

    def fire():
        while remaining() > margin:
            time.sleep(min(remaining() - margin, 2.0))
        why = f"stage '{RUN['stage']}' did not finish within the run's {RUN['budget_s']} s budget"
        done = RUN["printed"]  # the result is out: only the teardown is late
        if rank == 0 and not done:
            rec = headline_error_line(args, why)
            rec.update(pre)
            emit(rec)
        print(f"bench.py: {why}; exiting", file=sys.stderr, flush=True)
        os._exit(0 if done else 3)

    threading.Thread(target=fire, name="pgh-bench-deadline", daemon=True).start()


LAUNCHER_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK",
                "ROLE_RANK", "GROUP_WORLD_SIZE", "ROLE_WORLD_SIZE", "ROLE_NAME", "PGH_BENCH_SPAWNED")


def child_env() -> dict:
    """This environment without the launcher's rank variables (torch.distributed.run's, including
    every TORCHELASTIC_* one: a child world that inherited TORCHELASTIC_USE_AGENT_STORE would wait
    on the launcher's store), so a child forms its own world or none."""
    return {k: v for k, v in os.environ.items()
            if k not in LAUNCHER_ENV and not k.startswith("TORCHELASTIC_") and k != "PGH_BENCH_LIVE_TRAFFIC"}


def time_for(stage: str, need_s: float) -> bool:
    """Whether an optional part of the headline (need_s: its usual duration) still fits before the
    watchdog; if not it is skipped and the line says so."""
    if remaining() - WATCHDOG_MARGIN_S >= need_s:
        return True
    RUN["stages"][stage] = "skipped"
    return False


def skipped(stage: str) -> dict:
    return {"skipped": f"{max(remaining(), 0):.0f} s of the run's {RUN['budget_s']} s budget left", "stage": stage}
