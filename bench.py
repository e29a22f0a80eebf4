#!/usr/bin/env python3
"""Benchmark of the PyGrid cycle-close aggregation hot path on MI355X.

Metric (BASELINE.json): client-diff GB/s aggregated (% of HBM peak) at 1/2/4/8 MI355X; cycle
close ms.  Default workload (N = 1: BASELINE configs[1]): ResNet-18 (11,689,512 params) fp32
FedAvg over 1,000 synthetic client diffs resident on one MI355X (46.8 GB).  A "step" is one cycle
close of that workload: the fused mean + apply kernel over all [1000][P] diffs producing the new
checkpoint (for N > 1 also the RCCL all-gather that assembles it).

Scaling: weak.  Rank r owns a P_g-param shard of a (N x P_g)-param model (the parameter-axis
sharding of SURVEY.md 8(e)) and all clients, so per-GPU work is fixed as N grows.

Other BASELINE configs (--workload), each printed as its own JSON line of the same shape:
  resnet18-iterative / resnet18-weighted   config 2 with the iterative plan / weighted FedAvg
  resnet18-secagg        config 3: 1,000 clients x 2-party int64 shares (187 GB) resident
  secagg-clients         config 3 with the CLIENTS sharded: every rank sums the shares of its own
                         1,000 clients over the whole ResNet-18 vector, int64 reduce-scatter +
                         decode + all-gather over RCCL, range by range beside the share sum
                         (weak scaling in clients: 1,000 x N clients in total)
  c4-stream              config 4 per-GPU shard: 12.5M params x 10,000 clients (500 GB) streamed
                         through a 1,000-slot HBM ring, chunks generated on the GPU
  c5-ingest              config 5 per-GPU shard: 125M params x 64 clients iterative, diffs streamed
                         host (pinned) -> HBM over PCIe, folded while the next ones copy
  mnist-state            config 1: 3 clients' State protobuf bytes -> new checkpoint bytes
  resnet18-state         ResNet-18 (62 tensors) x 100 clients, State bytes on the host -> new
                         checkpoint bytes: the whole cycle close a node runs (PCIe-inclusive)
  resnet18-secagg-state  config 3 from the wire: ResNet-18 x N clients x 2 parties of int64 shares as
                         State bytes (packed varints, ~9.5 B per value) in host memory -> HBM as
                         received -> decoded on the GPU -> Z_2^64 sum + decode (PCIe-inclusive)
  resnet18-report        the same cycle with report-time aggregation: each
                         State diff is folded into HBM as it is reported, the checkpoint uploaded
                         at cycle start; reports the cycle close latency after the last report

The default run (resnet18-fedavg) also carries configs 1, 3, 4 and 5 as sub-lines (`config1` ...
`config5`), each a fresh child run with a bit-exact check, and -- at N > 1 -- the one-process group
over the same GPUs (`group`).  The whole run keeps to one deadline (--budget-s, under the driver's
600 s): every child gets at most what is left after the headline's reserve, a child that runs out
leaves {"error": "timeout after ... s", "stage": ...} in its slot, and the headline line is printed
whatever happens (a watchdog prints it with an error when the headline itself cannot finish).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="resnet18-fedavg", choices=sorted(WORKLOADS))
    ap.add_argument("--clients", type=int, default=None)
    ap.add_argument("--params", type=int, default=None, help="params per GPU shard")
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--ring", type=int, default=None, help="stream workloads: HBM ring slots")
    ap.add_argument("--gather-chunks", type=int, default=8, help="N > 1: fold ranges overlapped with all-gather")
    ap.add_argument("--gather-tail", type=int, default=3,
                    help="N > 1: halve the last range this many times (shorter exposed collective)")
    ap.add_argument("--synth", choices=["fast", "irwin-hall"], default="fast",
                    help="c4-stream: on-device generator of the arriving diffs (fast: one hash per 4 params)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-e2e", action="store_true",
                    help="resident config-2 lines: skip the bytes -> bytes end-to-end close measured beside them")
    ap.add_argument("--group", action="store_true",
                    help="one process drives all --gpus GPUs through one library context (pgh_create_group: "
                         "how the node's single process uses the node's GPUs) instead of one rank per GPU")
    ap.add_argument("--e2e-distinct", type=int, default=64,
                    help="end-to-end close: distinct client State messages in host memory (re-sent as the others)")
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="N = 1 resident lines: skip the two rocprofv3 --pmc passes that measure roofline.traffic "
                         "in this run (the committed profiles/pmc_traffic.json is quoted instead)")
    ap.add_argument("--report-gap-ms", type=float, default=0.0,
                    help="resnet18-report: pause between reports (0: back to back; a node decodes each report's "
                         "base64 for ~4-7 ms anyway, tools/node_sim.py)")
    ap.add_argument("--close-gap-ms", type=float, default=0.0,
                    help="resnet18-report: pause between the last report and the close (the cycle's end "
                         "comes later than its last report; 0: at once)")
    ap.add_argument("--sync-before-close", action="store_true",
                    help="resnet18-report: wait for the GPU before the close and time that wait apart")
    ap.add_argument("--no-group-line", action="store_true",
                    help="N > 1 per-rank runs: skip the one-process group over the same GPUs measured after the "
                         "ranks exit (the JSON line's `group` record)")
    ap.add_argument("--no-tune", action="store_true",
                    help="leave glibc's allocator thresholds alone (pygrid_amd.tune_process(malloc=...))")
    ap.add_argument("--dry-run", action="store_true",
                    help="form the world (gloo, no GPU), print the world size on rank 0 and exit")
    ap.add_argument("--check", action="store_true",
                    help="c4-stream / c5-ingest: after the timed steps, every rank samples params of its shard, "
                         "the oracle computes them from that rank's inputs, rank 0 compares the all-gathered "
                         "new checkpoint bit for bit (a checker leg outside the timed region)")
    ap.add_argument("--no-config-lines", action="store_true",
                    help="default workload: skip the config lines (mnist-state --check on one GPU; resnet18-secagg, "
                         "c4-stream, c5-ingest --check over the same --gpus; each in a fresh child run) attached "
                         "under `config1` / `config3` / `config4` / `config5`")
    ap.add_argument("--config-clients", type=int, default=None,
                    help="rehearsal on one GPU only (tools/rehearse_multi.sh): clients of the config-3/4/5 child "
                         "lines (default: each config's own count)")
    ap.add_argument("--budget-s", type=float, default=None,
                    help=f"deadline of the whole run, seconds (default: PGH_BENCH_BUDGET_S or {DEFAULT_BUDGET_S:.0f}, "
                         "under the driver's 600 s).  Every child line gets min(its own limit, what is left minus "
                         "--headline-reserve-s); the headline line is printed whatever happens")
    ap.add_argument("--headline-reserve-s", type=float, default=None,
                    help="seconds of the budget kept for the headline world (default 150 at N = 1: its "
                         "end-to-end and report-time closes and cpu_baseline; 120 at N > 1)")
    return ap.parse_args()


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


def spawn_ranks(args) -> int:
    """``--gpus N`` (N > 1) started without a launcher: run the child lines first (this parent
    imports neither torch nor the engine, so it never touches a GPU), then start N rank processes
    of this script with the environment torch.distributed.run would give them (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT) and the run's deadline, and return the
    worst exit status.  If one rank fails the others are stopped (their own PIDs) instead of
    waiting in a collective forever, and at the deadline every rank is.  Rank 0's result line
    (or, failing that, an error line) gets the child lines and is printed here."""
    import socket
    import subprocess

    pre = pre_world_lines(args)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    RUN["stage"] = "headline"
    t = time.time()
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PGH_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, text=True))
    rc = 0
    live = list(procs)
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()  # rank 0's pipe is drained as it writes
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0:
                rc = rc or r
                for q in live:
                    q.terminate()
        if live and remaining() < 0:  # the ranks' own watchdogs should have ended them by now
            rc = rc or 124
            for q in live:
                q.kill()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    reader.join(10)
    RUN["stages"]["headline"] = round(time.time() - t, 1)
    text = out[0] if out else ""
    for ln in text.splitlines():
        if not ln.startswith("{"):
            print(ln, flush=True)
    lines = json_lines(text)
    if lines:
        rec = json.loads(lines[-1])
        rec.pop("budget", None)
    else:
        rec = headline_error_line(args, f"the {args.gpus} ranks exited {rc} without a result line")
    rec.update(pre)
    emit(rec)
    return rc or (1 if rec.get("error") else 0)


GROUP_WORKLOADS = {"resnet18-fedavg", "resnet18-iterative", "resnet18-weighted", "resnet18-secagg", "secagg-clients"}


LAUNCHER_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK",
                "ROLE_RANK", "GROUP_WORLD_SIZE", "ROLE_WORLD_SIZE", "ROLE_NAME", "PGH_BENCH_SPAWNED")


def child_env() -> dict:
    """This environment without the launcher's rank variables (torch.distributed.run's, including
    every TORCHELASTIC_* one: a child world that inherited TORCHELASTIC_USE_AGENT_STORE would wait
    on the launcher's store), so a child forms its own world or none."""
    return {k: v for k, v in os.environ.items() if k not in LAUNCHER_ENV and not k.startswith("TORCHELASTIC_")}


def wants_group_line(args) -> bool:
    return args.gpus > 1 and not args.group and not args.no_group_line and args.workload in GROUP_WORKLOADS


def group_line(args, limit_s: int = 240) -> dict:
    """The path the node deploys at N > 1 (its single process drives every GPU through one library
    context, ``pgh_create_group``), measured on the same GPUs before the
    per-rank world forms: ``bench.py --group --gpus N`` in a FRESH child (no process that touched a
    GPU re-execs), summarised for the per-rank line.  ``rccl`` says whether the group's exchange ran
    over RCCL (distinct devices) or peer copies."""
    import subprocess

    cmd = [sys.executable, str(Path(__file__).resolve()), "--group", "--gpus", str(args.gpus), "--workload",
           args.workload, "--steps", str(args.steps), "--warmup", str(args.warmup), "--seed", str(args.seed),
           "--no-cpu-baseline", "--no-live-traffic"]
    if args.dry_run:
        cmd.append("--dry-run")
    if args.clients:
        cmd += ["--clients", str(args.clients)]
    if args.params:
        cmd += ["--params", str(args.params)]
    # stderr passes through: the child's progress stays visible
    r, err = run_child(args, "group", cmd, limit_s, stdout=subprocess.PIPE)
    if err:
        return err
    lines = json_lines(r.stdout)
    if r.returncode != 0 or not lines:
        return {"error": f"group child exited {r.returncode} (its stderr is above)", "stage": "group",
                "command": " ".join(cmd[1:])}
    g = json.loads(lines[-1])
    if g.get("dry_run"):
        return g
    if g.get("error"):
        return {"error": g["error"], "stage": "group", "command": " ".join(cmd[1:])}
    cfg = g.get("config", {})
    out = {"value": g.get("value"), "unit": g.get("unit"), "n_gpus": g.get("n_gpus"),
           "ms_per_step": g.get("ms_per_step"), "kernel_ms": g.get("kernel_ms"),
           "pct_hbm_peak_per_gpu": g.get("pct_hbm_peak_per_gpu"),
           "frac": (g.get("roofline") or {}).get("frac"), "rccl": cfg.get("rccl"),
           "exchange": cfg.get("exchange"), "parallelism": cfg.get("parallelism"),
           "devices": cfg.get("devices"), "command": " ".join(cmd[1:])}
    for k in ("cycle_close_e2e", "cycle_close_report_time"):
        if k in g:
            out[k] = g[k]
    return out


# key: (workload, GPUs (None: this run's --gpus), steps cap, with its cpu_baseline, time limit s).
# In run order: the cheap config-1 close first, then the configs only a multi-GPU run exercises in
# their stated form (4, 5), then config 3 (187.7 GB resident per GPU).  Each limit is ~10x what the
# child took at N = 1 (profiles/r05b: 9 / 4 / 9 / 18 s), so one hung child cannot starve the others.
CONFIG_LINES = {"config1": ("mnist-state", 1, None, True, 120), "config4": ("c4-stream", None, 5, False, 180),
                "config5": ("c5-ingest", None, 5, False, 180), "config3": ("resnet18-secagg", None, 10, True, 240)}
FOLD_BYTES_NOTE = {
    "c5-ingest": "fold batch 2: each fold launch also reads and writes the running state (4 B + 4 B per param "
                 "per 2 clients), so the fold kernel moves 2x its diff bytes; fold_frac counts those bytes, "
                 "e2e_frac only the diff bytes (the step is PCIe-bound)",
    "c4-stream": "value and e2e_frac include the on-device generation of every chunk (4 B written per param per "
                 "client, alternating with the fold); fold_frac is the fold kernel alone",
    "resnet18-secagg": "fold_frac: 8*S*N*P + 12*P bytes (shares in; int64 sum and float32 decode out) over the "
                       "k_secagg launch time; e2e_frac: the share bytes 8*S*N*P over the whole step",
    "mnist-state": "latency line (bytes in -> bytes out, 3 clients): cycle_close_ms is the figure; fold_frac is "
                   "the 0.3M-param fold kernel alone",
}


def wants_config_lines(args) -> bool:
    return args.workload == "resnet18-fedavg" and not args.group and not args.no_config_lines and not under_profiler()


def config_line(args, key: str) -> dict:
    """One BASELINE config as a fresh child run (``bench.py --gpus N --workload <w> --check``: it
    forms its own N ranks; no process that touched a GPU re-execs), summarised for this line: what
    ran (ranks, backend), its value with ``e2e_frac`` = value / (GPUs x HBM peak), the dominant
    kernel's own roofline fraction ``fold_frac`` (the two differ: FOLD_BYTES_NOTE says how), the
    bit-exact check and, where the config has one, its cpu_baseline."""
    import subprocess

    workload, gpus, steps_cap, cpu, limit_s = CONFIG_LINES[key]
    gpus = gpus or args.gpus
    steps = min(args.steps, steps_cap) if steps_cap else args.steps
    cmd = [sys.executable, str(Path(__file__).resolve()), "--gpus", str(gpus), "--workload", workload,
           "--steps", str(steps), "--warmup", str(1 if steps_cap else args.warmup), "--seed", str(args.seed),
           "--no-live-traffic", "--no-group-line", "--no-config-lines", "--check",
           "--cpu-seconds", str(args.cpu_seconds)]
    if not cpu or args.no_cpu_baseline:
        cmd.append("--no-cpu-baseline")
    if args.config_clients and workload != "mnist-state":
        cmd += ["--clients", str(args.config_clients)]
    if args.dry_run:
        cmd.append("--dry-run")
    r, err = run_child(args, key, cmd, limit_s, stdout=subprocess.PIPE)
    if err:
        return err
    lines = json_lines(r.stdout)
    g = json.loads(lines[-1]) if lines else {}
    if r.returncode != 0 or not lines:  # the child's own watchdog line says where it stopped
        return {"error": g.get("error") or f"{workload} child exited {r.returncode} (its stderr is above)",
                "stage": key, "child_stage": g.get("stage"), "command": " ".join(cmd[1:])}
    if g.get("dry_run"):
        return g
    if g.get("error"):
        return {"error": g["error"], "stage": key, "command": " ".join(cmd[1:])}
    keep = ("value", "unit", "n_gpus", "steps", "ms_per_step", "kernel_ms", "cycle_close_ms", "dtype",
            "pct_hbm_peak_per_gpu", "dist_backend", "rccl_ranks", "check", "fold_kernel_client_diff_GBps_aggregated",
            "fold_kernel_client_diff_GBps_per_gpu", "ingest_GBps_per_gpu", "bound_by", "cpu_baseline")
    out = {k: g[k] for k in keep if k in g}
    cfg, roof = g.get("config") or {}, g.get("roofline") or {}
    out["workload"] = cfg.get("workload")
    out["parallelism"] = cfg.get("parallelism")
    if g.get("value") is not None:
        out["e2e_frac"] = round(g["value"] / (g.get("n_gpus") or gpus) / HBM_PEAK_GBS, 4)
    out["fold_frac"] = roof.get("frac")
    out["fold_kernel"] = {k: roof.get(k) for k in ("kernel", "kernel_ms_avg", "alg_bytes_per_launch", "achieved",
                                                   "launches")}
    out["fold_bytes_note"] = FOLD_BYTES_NOTE.get(workload)
    out["command"] = " ".join(cmd[1:])
    return out


def attach_config_lines(args, rec: dict):
    if wants_config_lines(args):
        for key in CONFIG_LINES:
            rec[key] = config_line(args, key)


def pre_world_lines(args, out=None) -> dict:
    """The child lines of this run -- configs 1, 3, 4, 5 and the one-process group over the same
    GPUs -- run BEFORE this process, or any rank of its world, touches a GPU: a parent holding a
    HIP context while its child runs slowed the child's config-4 step by 13 % (176 vs 154 ms,
    profiles/r04g/).  Under torch.distributed.run rank 0 runs them while the other ranks wait on
    the launcher's store (no GPU touched; the wait ends by the run's deadline); at N = 1, and in
    the parent that spawns ranks itself, this process runs them first.  Each is limited by the
    run's budget (run_child).  Fills and returns ``out``."""
    out = {} if out is None else out
    spawned = os.environ.get("PGH_BENCH_SPAWNED") == "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if spawned or args.group or not (wants_group_line(args) or wants_config_lines(args)):
        return out
    rank = int(os.environ.get("RANK", "0"))

    def run():
        attach_config_lines(args, out)
        if wants_group_line(args):
            out["group"] = group_line(args)

    if world == 1:
        run()
        return out
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() != "true":
        # another launcher: no store to wait on before the process group forms; rank 0 runs them
        # first and the others wait in init_process_group (their GPUs touched: no deadlock risk)
        if rank == 0:
            run()
        return out
    # torch.distributed.run: a barrier on the launcher's own store, before any process group exists
    from datetime import timedelta

    import torch.distributed as dist

    # the other ranks wait no longer than the run's deadline (their watchdog ends them after it)
    wait_s = max(30.0, remaining())
    store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), is_master=False,
                          timeout=timedelta(seconds=wait_s))
    key = f"pgh_bench_pre_world_{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}"
    if rank == 0:
        try:
            run()
        finally:
            store.set(key, "done")
    else:
        try:
            store.wait([key], timedelta(seconds=wait_s))
        except Exception as e:  # noqa: BLE001 -- go on: rank 0's watchdog still prints the line
            print(f"bench.py: rank {rank}: no word from rank 0's child lines ({e})", file=sys.stderr, flush=True)
    return out


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


def cpu_baseline(kind: str, P: int, seed: int, budget_s: float, n: int = 32, all_cores: int = 0):
    """The reference's path as the node runs it, in torch on CPU tensors at th.set_num_threads(1)
    (the node's setting, main/__init__.py:8), on a bounded sample: the same P-param shard, `n`
    synthetic clients, repeated until `budget_s` of CPU work.
      mean       cycle_manager.py:276-296                (oracle.fedavg_mean_torch)
      iterative  cycle_manager.py:266-269 + the plan     (oracle.fedavg_iterative_torch)
      secagg     syft share adds + fix-prec decode       (oracle.secagg_sum_torch), 2 parties
      weighted   no reference counterpart: the numpy oracle (oracle.fedavg_weighted)
    Also reported: the same at `all_cores` threads (default: usable_cores(), the GPU box's CPU
    share) and the numpy restatement at 1 thread."""
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
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{what}, {f'torch {torch.__version__} CPU tensors' if ref else 'numpy'}, P={P}, {n} clients, "
                      f"{reps} passes in {el:.1f}s, 1 thread (the node's th.set_num_threads(1))",
            "cycle_close_ms_per_1000_clients": close_1000(gbs),
            "all_cores": ({"value": round(gbs_all, 3), "cores": all_cores, "cores_from": cores_how,
                           "cycle_close_ms_per_1000_clients": close_1000(gbs_all)} if gbs_all else None),
            "numpy_restatement_1_thread": round(gbs_np, 3), "cpu_model": cpu_model()}


def in_reference_allocator(fn: str, kwargs: dict, blobs=None):
    """Run ``bench.<fn>(**kwargs)`` in a child process with glibc's default allocator
    (PGH_MALLOC_TUNE=0): importing pygrid_amd raises glibc's mmap threshold (pygrid_amd.hostmem),
    which would also spare the reference's torch code its per-add page faults -- the node it
    stands for runs without that.  ``blobs`` (name -> bytes) reach the child as files.  The child
    never touches the GPU."""
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
        code = ("import json, sys; from pathlib import Path; sys.argv = ['bench.py']; import bench\n"
                "spec = json.loads(sys.stdin.read())\n"
                "kw = dict(spec['kwargs'])\n"
                "for k, v in spec['files'].items():\n"
                "    kw[k] = [Path(p).read_bytes() for p in v] if isinstance(v, list) else Path(v).read_bytes()\n"
                "print(json.dumps(getattr(bench, spec['fn'])(**kw)))")
        # part of the headline: it may use the budget up to the watchdog's margin
        r, err = run_child(None, "cpu_baseline", [sys.executable, "-c", code], 600,
                           reserve=WATCHDOG_MARGIN_S + 5, capture_output=True,
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
    got, alg = {}, None
    try:
        # the first pass may pay a fresh box's first `import torch` (1-2 minutes): a longer limit
        for counter, limit in zip(("FETCH_SIZE", "WRITE_SIZE"), timeout_s):
            r, err = run_child(args, f"pmc_{counter}", [prof, "--pmc", counter, "-d", str(tmp / counter), "-o", "run",
                                                        "--output-format", "csv", "--"] + child,
                               limit, kill="KILL", capture_output=True, env=dict(os.environ))
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
    note = (f"live: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of this workload (2 steps each, "
            f"{n} {kernel} launches per pass) run by bench.py before its timed run; (2*FETCH_SIZE + WRITE_SIZE)*1024")
    return (2 * fetch + write) * 1024, alg, note


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


LIVE_TRAFFIC = None  # (hbm bytes per launch, algorithmic bytes per launch, note): measure_live_traffic


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
    if LIVE_TRAFFIC is not None and kernel == PMC_KERNEL.get(workload):
        live, live_alg, note = LIVE_TRAFFIC
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


def run_resident(ctx, args, eng, mode, dtype, N, parties, pg, P, lo, hi):
    torch = ctx.torch

    eng.reserve(N, dtype, parties)
    eng.synth_fill(args.seed, N)
    sp = torch.cuda.current_stream().cuda_stream
    if dtype == 0:
        ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
        out = torch.empty_like(ckpt)
        eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
        if mode == 2:
            eng.set_weights([(c % 7 + 1) * 0.5 for c in range(N)])
        if ctx.world > 1:
            # fold the shard in 8 param ranges; RCCL all-gathers range i beside the fold of i + 1
            from pygrid_amd.sharding import OverlappedGather
            og = OverlappedGather(P, ctx.world, ctx.rank, chunks=args.gather_chunks, tail=args.gather_tail)
            lp = og.local.data_ptr()

            def step():
                og.run(lambda off, n, st: eng.fedavg_device_range(mode, off, n, ckpt.data_ptr(), lp, st))
                og.assemble()
        else:
            def step():
                eng.fedavg_device(mode, ckpt.data_ptr(), out.data_ptr(), sp)
        diff_bytes, dt, kernel = 4 * N * pg, "f32", "k_fedavg"
    else:
        s_out = torch.empty(pg, dtype=torch.int64, device="cuda")
        d_out = torch.empty(pg, dtype=torch.float32, device="cuda")
        if ctx.world > 1:
            # decoded shard gathered range by range beside the share sum of the next range
            from pygrid_amd.sharding import OverlappedGather
            og = OverlappedGather(P, ctx.world, ctx.rank, chunks=args.gather_chunks, tail=args.gather_tail)
            lp = og.local.data_ptr()

            def step():
                og.run(lambda off, n, st: eng.secagg_device_range(off, n, s_out.data_ptr(), lp, 10, 3, st))
                og.assemble()
        else:
            def step():
                eng.secagg_device(s_out.data_ptr(), d_out.data_ptr(), 10, 3, sp)
        diff_bytes, dt, kernel = 8 * parties * N * pg, "int64", "k_secagg"
    torch.cuda.synchronize()
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    checked = None
    if args.check:
        full = og.assemble() if ctx.world > 1 else (out if dtype == 0 else d_out)
        checked = check_resident(ctx, args, full, mode, dtype, N, parties, lo, hi, s_out if dtype == 1 else None)
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    cfg = {"workload": f"{args.workload}: P_shard={pg} params/GPU x {N} clients"
                       + (f" x {parties} parties int64" if dtype == 1 else " fp32") + ", resident in HBM",
           "clients": N, "params_per_gpu": pg, "params_total": P,
           "parallelism": f"param-shard{ctx.world}" + (
               f" + {ctx.coll} all-gather ({args.gather_chunks} ranges, last halved {args.gather_tail}x, overlapped with the fold)" if ctx.world > 1 else ""),
           "kernel_variant": eng.effective_variant(mode if dtype == 0 else 16)}
    rec = record(ctx, args, args.workload, value, el, dt, cfg,
                 roofline_of(st, args.workload, cfg["kernel_variant"], kernel),
                 {"check": checked} if args.check else None)
    kind = "secagg" if dtype == 1 else {0: "mean", 1: "iterative", 2: "weighted"}[mode]
    return attach_cpu_baseline(ctx, args, rec, kind, pg)


def attach_cpu_baseline(ctx, args, rec, kind, P, n=32, note=None):
    """rank 0 at N = 1 only: the reference's arithmetic for this workload timed on the host
    (cpu_baseline above), on a bounded sample of the same P-param shard."""
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        try:
            rec["cpu_baseline"] = in_reference_allocator(
                "cpu_baseline", {"kind": kind, "P": P, "seed": args.seed, "budget_s": args.cpu_seconds, "n": n})
            if note:
                rec["cpu_baseline"]["sample"] += "; " + note
        except Exception as e:  # noqa: BLE001
            rec["cpu_baseline"] = {"error": str(e)}
    return rec


def run_secagg_clients(ctx, args, eng, N, S, P):
    """Config 3 with client sharding (north_star: reduce-scatter when clients are sharded): rank r
    holds the 2-party int64 shares of its own N clients for all P params (a different client set
    per rank: seed + rank), sums them range by range, and OverlappedReduceScatter reduce-scatters
    the Z_2^64 sums, decodes each rank's slice and all-gathers the decoded vector."""
    torch = ctx.torch
    from pygrid_amd.sharding import OverlappedReduceScatter

    eng.reserve(N, 1, S)
    eng.synth_fill(args.seed + ctx.rank, N)
    og = OverlappedReduceScatter(P, ctx.world, ctx.rank, chunks=args.gather_chunks, tail=args.gather_tail)
    sp = og.sums.data_ptr()

    def step():
        og.run(lambda a, n, st: eng.secagg_device_range(a, n, sp, 0, 10, 3, st),
               lambda t, d, st: eng.secagg_decode_device(t.data_ptr(), t.numel(), d.data_ptr(), 10, 3, st))
        og.assemble()
    torch.cuda.synchronize()
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    diff_bytes = 8 * S * N * P
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    cfg = {"workload": f"secagg-clients: {N} clients/GPU x {S} parties int64 x P={P} (ResNet-18) on every rank, "
                       "clients sharded, resident in HBM",
           "clients": N * ctx.world, "clients_per_gpu": N, "params_per_gpu": P, "params_total": P,
           "parallelism": f"client-shard{ctx.world} + {ctx.coll or 'no'} int64 reduce-scatter / decode / all-gather "
                          f"({args.gather_chunks} ranges, last halved {args.gather_tail}x, overlapped with the share sum)",
           "kernel_variant": eng.effective_variant(16)}
    # roofline: the share-sum launches (k_secagg); the decode kernel (12 B/param) is not in the stats
    rec = record(ctx, args, "secagg-clients", value, el, "int64", cfg,
                 roofline_of(st, "secagg-clients", cfg["kernel_variant"], "k_secagg"))
    return attach_cpu_baseline(ctx, args, rec, "secagg", P)


def run_c4(ctx, args, eng, N, pg, P):
    """Config 4 shard: N clients streamed through an R-slot ring; each chunk generated on the GPU
    (stand-in for arriving data) and folded in client order, generator and fold alternating on one
    stream (r02p: 12-14 % faster than beside it)."""
    torch = ctx.torch
    from pygrid_amd.sharding import gather_flat

    R = args.ring or 1000
    chunk = R // 2
    eng.reserve(R)
    eng.set_synth_kind(1 if args.synth == "fast" else 0)
    ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ckpt)
    sp = torch.cuda.current_stream().cuda_stream
    eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
    torch.cuda.synchronize()

    full = [out]

    def step():
        eng.stream_begin(0, chunk)
        for c0 in range(0, N, chunk):
            eng.synth_ingest(args.seed, c0, min(chunk, N - c0))
        eng.stream_finish_device(ckpt.data_ptr(), out.data_ptr(), sp)
        if ctx.world > 1:
            full[0] = gather_flat(out, P, ctx.world, ctx.rank)
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    checked = None
    if args.check:
        def expected(idx):
            import numpy as np

            from oracle import coracle
            from oracle import oracle as O

            u = idx.astype(np.uint64)
            gen = O.synth_diff_fast if args.synth == "fast" else O.synth_diff
            return coracle.fedavg(0, np.stack([gen(args.seed, k, u) for k in range(N)]), O.synth_ckpt(args.seed, u))
        checked = check_sampled(ctx, args, full[0], eng.lo, eng.hi, expected)
    diff_bytes = 4 * N * pg
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    kern_gbs = ctx.sum_over_ranks(4 * N * pg * args.steps / (st["kernel_ms_total"] / 1e3) / 1e9)
    cfg = {"workload": f"c4-stream: P_shard={pg} params/GPU x {N} clients fp32 (SURVEY 8(d) config 4 shard), "
                       f"{R}-slot HBM ring, {chunk}-client chunks generated on-device ({args.synth} generator)",
           "clients": N, "params_per_gpu": pg, "params_total": P, "ring_slots": R, "generator": args.synth,
           "parallelism": f"param-shard{ctx.world}" + (f" + {ctx.coll} all-gather" if ctx.world > 1 else ""),
           "kernel_variant": eng.effective_variant()}
    extra = {"fold_kernel_client_diff_GBps_aggregated": round(kern_gbs, 1),
             "note": "value includes on-device generation of every chunk (writes 4 B/param/client, "
                     "alternating with the fold); the fold kernels alone are fold_kernel_*"}
    if args.check:
        extra["check"] = checked
    rec = record(ctx, args, "c4-stream", value, el, "f32", cfg,
                 roofline_of(st, "c4-stream", cfg["kernel_variant"], "k_fedavg"), extra)
    return attach_cpu_baseline(ctx, args, rec, "mean", pg, n=8,
                               note=f"extrapolated: per-byte rate of an 8-client sample of the {N}-client shard")


def run_c5(ctx, args, eng, N, pg, P):
    """Config 5 shard: iterative plan over N clients whose diffs arrive from page-locked host
    memory; every H2D copy overlaps the fold of the previously copied clients."""
    torch = ctx.torch
    import numpy as np

    from pygrid_amd import PinnedBuffer
    from pygrid_amd.sharding import gather_flat

    R = args.ring or 8
    n_host = 4  # distinct host buffers, re-sent as different clients
    bufs = [PinnedBuffer((pg,)) for _ in range(n_host)]  # shard-sized host diffs
    rng = np.random.default_rng(args.seed + ctx.rank)
    for b in bufs:
        b.array[:] = rng.standard_normal(pg, dtype=np.float32) * np.float32(1e-2)
    eng.reserve(R)
    ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ckpt)
    sp = torch.cuda.current_stream().cuda_stream
    eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
    torch.cuda.synchronize()

    full = [out]

    def step():
        eng.stream_begin(1, 2)
        for k in range(N):
            eng.ingest(k, bufs[k % n_host].array)
        eng.stream_finish_device(ckpt.data_ptr(), out.data_ptr(), sp)
        if ctx.world > 1:
            full[0] = gather_flat(out, P, ctx.world, ctx.rank)
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    checked = None
    if args.check:
        lo = eng.lo

        def expected(idx):
            from oracle import coracle
            from oracle import oracle as O

            d = np.stack([bufs[k % n_host].array[idx - lo] for k in range(N)])
            return coracle.fedavg(1, d, O.synth_ckpt(args.seed, idx.astype(np.uint64)))
        checked = check_sampled(ctx, args, full[0], eng.lo, eng.hi, expected)
    diff_bytes = 4 * N * pg
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    kern_gbs = 4 * N * pg * args.steps / (st["kernel_ms_total"] / 1e3) / 1e9
    ingest_gbs = st["h2d_bytes_total"] / (st["h2d_ms_total"] / 1e3) / 1e9 if st["h2d_ms_total"] else None
    cfg = {"workload": f"c5-ingest: P_shard={pg} params/GPU x {N} clients fp32 iterative plan (SURVEY 8(d) "
                       f"config 5 shard), pinned host -> HBM over PCIe, {R}-slot ring, fold batch 2",
           "clients": N, "params_per_gpu": pg, "params_total": P, "ring_slots": R,
           "parallelism": f"param-shard{ctx.world}" + (f" + {ctx.coll} all-gather" if ctx.world > 1 else ""),
           "kernel_variant": eng.effective_variant(1)}
    extra = {"bound_by": "PCIe host->device (Gen5 x16, 63 GB/s spec per GPU)",
             "ingest_GBps_per_gpu": round(ingest_gbs, 2) if ingest_gbs else None,
             "fold_kernel_client_diff_GBps_per_gpu": round(kern_gbs, 1)}
    if args.check:
        extra["check"] = checked
    rec = record(ctx, args, "c5-ingest", value, el, "f32", cfg,
                 roofline_of(st, "c5-ingest", cfg["kernel_variant"], "k_fedavg"), extra)
    attach_cpu_baseline(ctx, args, rec, "iterative", pg, n=4,
                        note=f"extrapolated: per-byte rate of a 4-client sample of the {N}-client shard, diffs "
                             "already in host memory (no ingest)")
    for b in bufs:
        b.free()
    return rec


def run_mnist_state(ctx, args, eng):
    """Config 1: bytes in, bytes out (State protobuf diffs -> new checkpoint bytes), 3 clients."""
    import numpy as np

    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import MNIST_SHAPES

    golden = None
    if args.check:
        # checker leg: the golden fixture's inputs (tests/golden/mnist_synth.json: the oracle's
        # counter-based generator, seed 1234), so the new checkpoint can be held against its SHA-256
        import hashlib

        from oracle.gen_golden import mnist_inputs, split

        golden = json.loads((ROOT / "tests" / "golden" / "mnist_synth.json").read_text())
        flat_d, flat_c = mnist_inputs(golden["seed"], golden["n_clients"])
        sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
        if sha(flat_d) != golden["sha256_diffs"] or sha(flat_c) != golden["sha256_ckpt"]:
            raise SystemExit("bench.py mnist-state --check: the regenerated inputs are not the golden fixture's")
        ck = split(flat_c, MNIST_SHAPES)
        ds = [split(d, MNIST_SHAPES) for d in flat_d]
    else:
        rng = np.random.default_rng(args.seed)
        ck = [rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in MNIST_SHAPES]
        ds = [[rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2) for s in MNIST_SHAPES] for _ in range(3)]
    ck_pb = build_state_fast(ck)
    d_pb = [build_state_fast(d) for d in ds]
    # config 1 hosts a non-iterative plan: the operator's opt-in lets the engine run it as MEAN
    # once it probes bit-identical (pygrid_amd.cycle.mean_plan_policy; the default declines it)
    agg = CycleAggregator(eng, mean_plans="probe")

    def avg_plan(diffs):  # config 1's hosted non-iterative avg plan: the plain mean (cycle_manager.py:270-271)
        import torch as th
        from functools import reduce
        return [th.div(reduce(th.add, [d[j] for d in diffs]), len(diffs)) for j in range(len(diffs[0]))]

    plan_key = b"config-1 avg_plan: stands in for the hosted Plan's serialized bytes (avg_plan_rec.value)"
    t0 = time.perf_counter()
    agg.average_plan_diffs({}, ck_pb, d_pb, avg_plan, plan_key=plan_key)  # the plan is probed once, here
    first_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(args.warmup):
        agg.average_plan_diffs({}, ck_pb, d_pb, avg_plan, plan_key=plan_key)
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        new = agg.average_plan_diffs({}, ck_pb, d_pb, avg_plan, plan_key=plan_key)
    el = time.perf_counter() - t0
    st = eng.stats()
    P = sum(int(np.prod(s)) for s in MNIST_SHAPES)
    value = 4 * 3 * P * args.steps / el / 1e9
    cfg = {"workload": "mnist-state: MNIST 784-392-10 (P=311,650), 3 clients, non-iterative hosted avg_plan (the "
                       "plain mean: probed bit-identical to reduce(th.add)/N once per plan, verdict cached by the "
                       "plan's bytes), State bytes -> checkpoint bytes (scan + H2D + fused mean/apply + D2H + "
                       "fresh framing)", "clients": 3, "params_per_gpu": P,
           "params_total": P, "parallelism": "single GPU", "kernel_variant": eng.effective_variant()}
    extra = {"new_checkpoint_bytes": len(new), "first_close_ms_with_plan_probe": round(first_ms, 3),
             "note": "latency-bound: host protobuf scan, 3 H2D copies and a 0.3M-param kernel"}
    if golden is not None:
        from pygrid_amd.state_schema import parse_state

        flat = np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in parse_state(new)])
        got = hashlib.sha256(flat.tobytes()).hexdigest()
        extra["check"] = {"bit_exact": got == golden["sha256_mean"], "sha256_new_checkpoint_params": got,
                          "params_checked": int(flat.size),
                          "against": "tests/golden/mnist_synth.json sha256_mean (the oracle's mean of the golden "
                                     "inputs, pinned by the reference's avg_plan KAT; DESIGN.md section 4)"}
    rec = record(ctx, args, "mnist-state", value, el, "f32", cfg,
                 roofline_of(st, "mnist-state", eng.effective_variant(), "k_fedavg"), extra, step_is="close")
    if not args.no_cpu_baseline:
        try:
            rec["cpu_baseline"] = in_reference_allocator("cpu_baseline_state",
                                                         {"P": P, "n_target": 3, "budget_s": 4.0},
                                                         {"ck_pb": ck_pb, "d_pbs": list(d_pb)})
        except Exception as e:  # noqa: BLE001
            rec["cpu_baseline"] = {"error": str(e)}
    return rec


def run_resnet18_state(ctx, args, eng, N):
    """Bytes in, bytes out at ResNet-18 size: N clients' State protobuf diffs (host memory) ->
    new checkpoint bytes.  Includes payload location, host->HBM over PCIe, fused mean/apply,
    HBM->host and the checkpoint patch: what `_average_plan_diffs` costs the node."""
    import numpy as np

    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    rng = np.random.default_rng(args.seed)
    ck_pb = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                  for s in RESNET18_SHAPES]) for _ in range(4)]
    d_pb = [distinct[k % 4] for k in range(N)]  # 4 distinct messages re-sent (host memory)
    agg = CycleAggregator(eng)
    for _ in range(args.warmup):
        agg.average_plan_diffs({}, ck_pb, d_pb)
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        new = agg.average_plan_diffs({}, ck_pb, d_pb)
    el = time.perf_counter() - t0
    st = eng.stats()
    P = RESNET18_P
    value = 4 * N * P * args.steps / el / 1e9
    cfg = {"workload": f"resnet18-state: ResNet-18 (62 tensors, P={P}) x {N} clients, State protobuf bytes in host "
                       "memory -> new checkpoint bytes (scan + host->HBM + fused mean/apply + HBM->host + patch)",
           "clients": N, "params_per_gpu": P, "params_total": P, "parallelism": "single GPU", "kernel_variant": eng.effective_variant()}
    extra = {"h2d_GBps": round(st["h2d_bytes_total"] / (st["h2d_ms_total"] / 1e3) / 1e9, 2) if st["h2d_ms_total"] else None,
             "h2d_ms_per_close": round(st["h2d_ms_total"] / args.steps, 2),
             "new_checkpoint_bytes": len(new),
             "note": "PCIe-inclusive cycle close from host bytes (never `value` for the resident configs)"}
    rec = record(ctx, args, "resnet18-state", value, el, "f32", cfg,
                 roofline_of(st, "resnet18-state", eng.effective_variant(), "k_fedavg"), extra, step_is="close")
    if not args.no_cpu_baseline:
        rec["cpu_baseline"] = in_reference_allocator("cpu_baseline_state", {"P": P, "n_target": N, "budget_s": 0.0},
                                                     {"ck_pb": ck_pb, "d_pbs": list(distinct[:3])})
    return rec


def run_resnet18_secagg_state(ctx, args, eng, N, S):
    """Secure aggregation from share State bytes: per step, N clients x S parties of int64 shares
    (State messages with packed-varint payloads, 2 distinct clients re-sent from host memory) go
    to HBM as they are, are decoded there (k_varint_decode) and summed + decoded (k_secagg)."""
    import numpy as np

    from pygrid_amd.state_schema import build_state_i64_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    P = sum(numel)
    rng = np.random.default_rng(args.seed)
    msgs = []
    for _ in range(2):
        sh = rng.integers(-2**63, 2**63 - 1, (S, P), dtype=np.int64, endpoint=True)
        parts = [np.split(sh[s], np.cumsum(numel)[:-1]) for s in range(S)]
        msgs.append([build_state_i64_fast(p) for p in parts])
    wire = sum(len(m) for m in msgs[0])  # bytes per client (S messages)
    eng.set_layout(numel)
    eng.reserve(N, 1, S)

    def step():
        eng.reset()
        for c in range(N):
            eng.ingest_state_shares(c, msgs[c % 2])
        return eng.secagg(10, 3)

    for _ in range(args.warmup):
        step()
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t0
    st = eng.stats()
    value = 8 * S * N * P * args.steps / el / 1e9
    cfg = {"workload": f"resnet18-secagg-state: ResNet-18 (62 tensors, P={P}) x {N} clients x {S} parties of int64 "
                       "shares as State bytes (packed varint) in host memory -> HBM -> GPU varint decode -> Z_2^64 "
                       "sum + fixed-point decode -> host", "clients": N, "parties": S, "params_per_gpu": P,
           "params_total": P, "parallelism": "single GPU", "kernel_variant": eng.effective_variant(16)}
    extra = {"wire_bytes_per_client": wire, "wire_GBps": round(wire * N * args.steps / el / 1e9, 2),
             "h2d_GBps": round(st["h2d_bytes_total"] / (st["h2d_ms_total"] / 1e3) / 1e9, 2) if st["h2d_ms_total"] else None,
             "note": "PCIe-inclusive: value counts the decoded int64 share bytes (8 B per value) per second; "
                     "wire_GBps the varint bytes received"}
    rec = record(ctx, args, "resnet18-secagg-state", value, el, "int64", cfg,
                 roofline_of(st, "resnet18-secagg-state", cfg["kernel_variant"], "k_secagg"), extra, step_is="close")
    if not args.no_cpu_baseline:
        from oracle import oracle as O  # cpu_baseline leg only
        import torch
        threads = torch.get_num_threads()
        torch.set_num_threads(1)
        try:
            t0 = time.perf_counter()
            O.secagg_close_state_torch([msgs[0]])
            one = time.perf_counter() - t0
        finally:
            torch.set_num_threads(threads)
        rec["cpu_baseline"] = {
            "value": round(8 * S * P / one / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle.secagg_close_state_torch on 1 client x 2 parties (protobuf ParseFromString over the "
                      "restated schema, torch.tensor(contents_int64) per tensor, torch int64 share adds, "
                      ".float() / 10**3), 1 thread; per-client rate, extrapolated",
            "cycle_close_ms_per_client": round(one * 1e3, 1), "cpu_model": cpu_model()}
    return rec


def run_resnet18_report(ctx, args, eng, N):
    """Report-time aggregation (pygrid_amd.incremental.IncrementalCycle): per step one cycle of N
    assigned workers of which ~20 % never report (the reference's expected failure rate,
    routes.py:314; worker 0 among them, so nothing can fold before close) and the rest report in a
    shuffled order.  Each State diff goes to its HBM slot as it is reported; close drops the
    non-reporters and folds the reporters' slots in assignment order (row table), then patches the
    new checkpoint bytes.  `value` is PCIe-inclusive like resnet18-state; `close_ms_after_last_
    report` is what the node waits for once the last diff is in (cycle_manager.py:180-217)."""
    import numpy as np

    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    rng = np.random.default_rng(args.seed)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ck_pb = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                  for s in RESNET18_SHAPES]) for _ in range(4)]
    reporters = [w for w in range(N) if w != 0 and rng.random() >= 0.2]
    arrival = [int(w) for w in rng.permutation(reporters)]
    slots, batch = args.ring or N, 8
    closes, early, at_close, pending = [], [], [], []

    def cycle():
        inc = IncrementalCycle(eng, numel, slots=slots, fold_batch=batch, checkpoint=ck_pb)
        for w in range(N):
            inc.assigned(w)
        for w in arrival:
            inc.reported(w, distinct[w % 4])
            if args.report_gap_ms:
                time.sleep(args.report_gap_ms / 1e3)
        if args.close_gap_ms:
            time.sleep(args.close_gap_ms / 1e3)
        early.append(inc.n_folded)
        t0 = time.perf_counter()
        if args.sync_before_close:  # the GPU work the reports left queued, timed apart from the close call
            eng.sync()
            pending.append((time.perf_counter() - t0) * 1e3)
            t0 = time.perf_counter()
        new = inc.close(ck_pb)
        closes.append((time.perf_counter() - t0) * 1e3)
        at_close.append(inc.last_close["n"] - inc.last_close["early"])
        return new

    for _ in range(args.warmup):
        cycle()
    for x in (closes, early, at_close, pending):
        x.clear()
    eng.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        new = cycle()
    el = time.perf_counter() - t0
    st = eng.stats()
    P = RESNET18_P
    nrep = len(reporters)
    value = 4 * nrep * P * args.steps / el / 1e9
    cfg = {"workload": f"resnet18-report: ResNet-18 (62 tensors, P={P}), {N} workers assigned, {nrep} report "
                       f"(worker 0 and ~20 % others never do, routes.py:314) in shuffled order; each State diff "
                       f"goes to its HBM slot when reported ({slots} slots), checkpoint uploaded at cycle start, "
                       "close = fold of the reporters' slots in assignment order + new checkpoint bytes from HBM",
           "clients": nrep, "assigned": N, "params_per_gpu": P, "params_total": P, "parallelism": "single GPU",
           "kernel_variant": eng.effective_variant()}
    extra = {"close_ms_after_last_report": round(float(np.median(closes)), 3),
             "close_ms_after_last_report_all": [round(c, 3) for c in closes],
             "folded_before_close": int(np.median(early)) if early else 0,
             "rows_folded_at_close": int(np.median(at_close)) if at_close else 0,
             "report_gap_ms": args.report_gap_ms,
             "close_gap_ms": args.close_gap_ms,
             "pending_gpu_ms_at_close": [round(x, 3) for x in pending] if pending else None,
             "h2d_GBps": round(st["h2d_bytes_total"] / (st["h2d_ms_total"] / 1e3) / 1e9, 2) if st["h2d_ms_total"] else None,
             "new_checkpoint_bytes": len(new),
             "note": "PCIe-inclusive whole cycle (reports + close); compare close_ms_after_last_report with "
                     "resnet18-state's cycle_close_ms (all diffs ingested and folded at close)"}
    rec = record(ctx, args, "resnet18-report", value, el, "f32", cfg,
                 roofline_of(st, "resnet18-report", eng.effective_variant(), "k_fedavg_rows"), extra, step_is="close")
    if not args.no_cpu_baseline:  # the reference decodes and folds every diff at close
        rec["cpu_baseline"] = in_reference_allocator("cpu_baseline_state", {"P": P, "n_target": nrep, "budget_s": 0.0},
                                                     {"ck_pb": ck_pb, "d_pbs": list(distinct[:3])})
    return rec


def state_messages(shapes, n_distinct: int, seed: int):
    """Checkpoint + n_distinct client diffs as State bytes (distinct payloads, so a close of many
    clients streams from host DRAM rather than from cache): one seeded base vector, the diffs
    are rolled copies of it written into the template's payload spans by the C++ patcher."""
    import numpy as np

    from pygrid_amd.state import serialize_model_params
    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng(seed)
    P = sum(int(np.prod(s)) for s in shapes)
    ck_pb = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in shapes])
    base = rng.standard_normal(P, dtype=np.float32) * np.float32(1e-2)
    diffs = [serialize_model_params(ck_pb, np.roll(base, 9973 * k)) for k in range(n_distinct)]
    return ck_pb, diffs


def e2e_close(ctx, args, eng, n_clients: int, steps: int = 2):
    """BASELINE.md's cycle close, end to end: n_clients ResNet-18 diffs as State bytes in host
    memory -> new checkpoint bytes through CycleAggregator.average_plan_diffs (the slice
    cycle_manager.py:240-303: checkpoint upload, every diff's payload -> HBM over PCIe, fused
    mean/apply, HBM -> host, State patch).  Wall time per close, 1 warm-up close first."""
    import numpy as np

    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.workloads import RESNET18_SHAPES

    ck_pb, distinct = state_messages(RESNET18_SHAPES, min(args.e2e_distinct, n_clients), args.seed)
    diffs = [distinct[k % len(distinct)] for k in range(n_clients)]
    agg = CycleAggregator(eng)
    agg.average_plan_diffs({}, ck_pb, diffs)
    eng.reset_stats()
    t = []
    for _ in range(steps):
        t0 = time.perf_counter()
        new = agg.average_plan_diffs({}, ck_pb, diffs)
        t.append(time.perf_counter() - t0)
    st = eng.stats()
    ms = float(np.median(t)) * 1e3
    return {"cycle_close_ms": round(ms, 2), "closes_ms": [round(x * 1e3, 2) for x in t], "clients": n_clients,
            "client_diff_GBps": round(4 * RESNET18_P * n_clients / (ms / 1e3) / 1e9, 2),
            "h2d_GBps_per_gpu": round(st["h2d_bytes_total"] / max(ctx.n_gpus, 1) / (st["h2d_ms_total"] / 1e3) / 1e9, 2)
            if st["h2d_ms_total"] else None,
            "fold_kernel_ms": round(st["kernel_ms_total"] / max(st["kernel_launches"], 1), 3),
            "new_checkpoint_bytes": len(new), "distinct_messages_in_host_memory": len(distinct),
            "gpus": ctx.n_gpus,
            "definition": "wall time of CycleAggregator.average_plan_diffs: ResNet-18 checkpoint + client diffs as "
                          "State bytes in host memory -> new checkpoint bytes (BASELINE.md cycle close; PCIe-inclusive)"}


def report_close(ctx, args, eng, cycles: int = 8, assigned: int = 100):
    """The close as a node running report-time aggregation sees it, triggered
    the way the reference triggers it: the report that completes the cycle requests the close
    (``submit_worker_diff`` -> ``run_task_once("complete_cycle", ...)``, cycle_manager.py:176-178)
    and Flask-Executor runs it on its own thread (tasks/cycle.py:9-25).  Per cycle `assigned`
    ResNet-18 workers, ~20 % never report (worker 0 among them, routes.py:314), the rest in shuffled
    order, each State diff to HBM (and folded) when reported.  Timed: from the last report's
    ``reported`` returning to the new checkpoint bytes ready on the executor thread -- nothing
    waits between the two, nothing syncs the GPU before the clock starts.  Two arrival patterns:
    reports `paced` 5 ms apart (a node handles each report for tens of ms anyway, its DB write
    included, tools/node_sim.py; the headline) and `back_to_back`.  1 warm-up cycle each."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    rng = np.random.default_rng(args.seed + 17)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ck_pb = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                  for s in RESNET18_SHAPES]) for _ in range(4)]
    reporters = [w for w in range(assigned) if w != 0 and rng.random() >= 0.2]
    arms = {}
    with ThreadPoolExecutor(1, thread_name_prefix="executor") as executor:
        for arrival, gap_ms in (("paced", 5.0), ("back_to_back", 0.0)):
            for kind in ("default",):
                closes, left = [], []
                for cyc in range(cycles + 1):
                    inc = IncrementalCycle(eng, numel, slots=assigned, checkpoint=ck_pb)
                    for w in range(assigned):
                        inc.assigned(w)
                    for i, w in enumerate(rng.permutation(reporters)):
                        if i and gap_ms:
                            time.sleep(gap_ms / 1e3)  # between reports; none after the last one
                        inc.reported(int(w), distinct[int(w) % 4])
                    t0 = time.perf_counter()
                    ck_pb = executor.submit(inc.close, ck_pb).result()
                    if cyc:
                        closes.append((time.perf_counter() - t0) * 1e3)
                        left.append(inc.last_close["n"] - inc.last_close["early"])
                arms[f"{arrival}_{kind}"] = {"close_ms": round(float(np.median(closes)), 3),
                                            "closes_ms": [round(c, 3) for c in closes],
                                            "rows_left_to_fold_at_close": int(np.median(left))}
    head = arms["paced_default"]
    return {"close_ms_after_last_report": head["close_ms"], "arms": arms,
            "folds": "certain-only (the speculative folds of ABI 6-7 were retired in r05)",
            "assigned": assigned, "reporters": len(reporters), "gpus": ctx.n_gpus,
            "definition": "the reference's trigger: the last report's handler returns, the close runs at once on "
                          "an executor thread (run_task_once, cycle_manager.py:176-178); timed from that return "
                          "to the new checkpoint bytes (fold what the DB order still changes + FINAL pass + "
                          "PCIe D2H + State framing), no pause and no GPU sync in between; headline = product "
                          "default, reports paced 5 ms apart; cycles chained through the resident checkpoint"}


def group_exchange(eng) -> str:
    """How a group's collective ran: RCCL (distinct devices) or the library's peer copies (repeated
    devices, PGH_RCCL=0, or a group of one before its first collective)."""
    return {1: "RCCL (ncclAllGather / ncclReduceScatter)", 0: "peer-copy"}.get(eng.group_backend(), "no collective")


def run_group_resident(ctx, args, eng, mode, dtype, N, parties, Pg):
    """The resident configs on a one-process group: GPU g folds its Pg-param shard of a
    (G x Pg)-param model over all N clients (weak scaling like the per-rank runs), then the new
    checkpoint is all-gathered into a full copy on every GPU (ncclAllGather); secagg writes the
    decoded sum into a page-locked host array slice by slice."""
    import numpy as np

    from pygrid_amd import PinnedBuffer

    G = ctx.n_gpus
    P = Pg * G
    eng.set_layout([P])
    eng.reserve(N, dtype, parties)
    eng.synth_fill(args.seed, N)
    bufs = []
    if dtype == 0:
        eng.ckpt_upload(np.full(P, 0.01, np.float32))
        if mode == 2:
            eng.set_weights([(c % 7 + 1) * 0.5 for c in range(N)])

        def step():
            eng.fedavg_resident(mode)
            eng.allgather_resident()
        diff_bytes, dt, kernel = 4 * N * P, "f32", "k_fedavg"
    else:
        bufs = [PinnedBuffer((P,), np.int64), PinnedBuffer((P,), np.float32)]

        def step():
            eng.secagg(10, 3, out_sum=bufs[0].array, out_dec=bufs[1].array)
        diff_bytes, dt, kernel = 8 * parties * N * P, "int64", "k_secagg"
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    value = diff_bytes * args.steps / el / 1e9
    cfg = {"workload": f"{args.workload}: P_shard={Pg} params/GPU x {N} clients"
                       + (f" x {parties} parties int64" if dtype == 1 else " fp32") + ", resident in HBM",
           "clients": N, "params_per_gpu": Pg, "params_total": P,
           "parallelism": f"param-shard{G} in one process (pgh_create_group, one host thread per GPU)" + (
               f" + {group_exchange(eng)} all-gather of the new checkpoint" if dtype == 0 else " + host slices"),
           "rccl": eng.group_backend() == 1, "exchange": group_exchange(eng), "devices": ctx.devices,
           "kernel_variant": eng.effective_variant(mode if dtype == 0 else 16)}
    rec = record(ctx, args, args.workload, value, el, dt, cfg,
                 roofline_of(st, args.workload, cfg["kernel_variant"], kernel, G))
    for b in bufs:
        b.free()
    return rec


def run_group_secagg_clients(ctx, args, eng, N, S, P):
    """Config 3 client-sharded on a one-process group: GPU g holds its own N clients x S parties
    over the whole model, the Z_2^64 sums are reduce-scattered (ncclReduceScatter, uint64 SUM), GPU
    g decodes its slice and writes it into the page-locked host outputs."""
    import numpy as np

    from pygrid_amd import PinnedBuffer

    G = ctx.n_gpus
    eng.set_layout([P])
    eng.set_client_sharding(True)
    eng.reserve(N * G, 1, S)
    eng.synth_fill(args.seed, N * G)
    bufs = [PinnedBuffer((P,), np.int64), PinnedBuffer((P,), np.float32)]

    def step():
        eng.secagg(10, 3, out_sum=bufs[0].array, out_dec=bufs[1].array)
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    value = 8 * S * N * G * P * args.steps / el / 1e9
    cfg = {"workload": f"secagg-clients: {N} clients/GPU x {S} parties int64 x P={P} (ResNet-18), clients sharded "
                       "over the GPUs of one process, resident in HBM",
           "clients": N * G, "clients_per_gpu": N, "params_per_gpu": P, "params_total": P,
           "parallelism": f"client-shard{G} in one process (pgh_create_group) + {group_exchange(eng)} reduce-scatter of "
                          "the Z_2^64 sums + per-GPU decode + host slices",
           "rccl": eng.group_backend() == 1, "exchange": group_exchange(eng), "devices": ctx.devices,
           "kernel_variant": eng.effective_variant(16)}
    rec = record(ctx, args, "secagg-clients", value, el, "int64", cfg,
                 roofline_of(st, "secagg-clients", cfg["kernel_variant"], "k_secagg", G))
    for b in bufs:
        b.free()
    return rec


def main_group(ctx, args):
    from pygrid_amd import Engine

    mode, dtype, n_default, parties, pg_default = WORKLOADS[args.workload]
    N = args.clients or n_default
    Pg = args.params or pg_default
    # PGH_BENCH_DEVICES (e.g. "0,0") only exists to rehearse a group on a one-GPU box
    devs = os.environ.get("PGH_BENCH_DEVICES")
    devices = [int(x) for x in devs.split(",")] if devs else list(range(args.gpus))
    if len(devices) != args.gpus:
        raise SystemExit(f"PGH_BENCH_DEVICES names {len(devices)} devices, --gpus {args.gpus}")
    ctx.devices = devices
    eng = Engine(devices=devices)
    if args.variant is not None:
        eng.set_variant(args.variant)
    if args.workload == "secagg-clients":
        rec = run_group_secagg_clients(ctx, args, eng, N, parties, Pg)
    elif args.workload in ("resnet18-state", "mnist-state", "resnet18-report"):
        rec = {"resnet18-state": run_resnet18_state, "mnist-state": lambda c, a, e, n: run_mnist_state(c, a, e),
               "resnet18-report": run_resnet18_report}[args.workload](ctx, args, eng, N)
        rec["config"]["parallelism"] = f"param-shard{ctx.n_gpus} in one process (pgh_create_group)"
    elif args.workload in ("c4-stream", "c5-ingest"):
        raise SystemExit(f"--group: {args.workload} runs per rank (torch.distributed.run)")
    else:
        rec = run_group_resident(ctx, args, eng, mode, dtype, N, parties, Pg)
        if args.workload == "resnet18-fedavg" and not args.no_e2e:
            RUN["stage"] = "cycle_close_e2e"
            rec["cycle_close_e2e"] = e2e_close(ctx, args, eng, N) if time_for("cycle_close_e2e", 40) \
                else skipped("cycle_close_e2e")
            RUN["stage"] = "cycle_close_report_time"
            rec["cycle_close_report_time"] = report_close(ctx, args, eng) \
                if time_for("cycle_close_report_time", 45) else skipped("cycle_close_report_time")
    emit(rec)
    RUN["stage"] = "teardown"
    eng.close()


def time_for(stage: str, need_s: float) -> bool:
    """Whether an optional part of the headline (need_s: its usual duration) still fits before the
    watchdog; if not it is skipped and the line says so."""
    if remaining() - WATCHDOG_MARGIN_S >= need_s:
        return True
    RUN["stages"][stage] = "skipped"
    return False


def skipped(stage: str) -> dict:
    return {"skipped": f"{max(remaining(), 0):.0f} s of the run's {RUN['budget_s']} s budget left", "stage": stage}


def main():
    args = parse()
    set_deadline(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.group:
        sys.exit(spawn_ranks(args))  # no launcher: form the N-rank world here (no GPU touched yet)
    pre = {}
    start_watchdog(args, pre)
    if not args.no_tune:
        import pygrid_amd

        # the harness opts in to the allocator thresholds a tuned node would use (the hardware
        # queues were requested at import); cpu_baseline children run with glibc's defaults
        PROCESS_TUNING.update(pygrid_amd.tune_process(hw_queues=False))
        PROCESS_TUNING["hw_queues"] = HW_QUEUES
    pre_world_lines(args, pre)  # child lines first: nothing of this world holds a GPU yet
    global LIVE_TRAFFIC
    if (args.gpus == 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.group and not args.dry_run
            and not args.no_live_traffic and args.workload in PMC_KERNEL and not under_profiler()):
        LIVE_TRAFFIC = measure_live_traffic(args)  # child processes; this one has not touched the GPU yet
    RUN["stage"] = "headline"
    t_head = time.time()
    if stub_sleep("headline"):  # test hook: a headline that cannot finish in time
        time.sleep(stub_sleep("headline"))
    ctx = Ctx(args)
    if args.dry_run:
        rec = {"dry_run": True, "n_gpus": ctx.n_gpus, "backend": ctx.backend, "group": ctx.group,
               "workload": args.workload, "dist_backend": ctx.dist_backend, "rccl_ranks": ctx.rccl_ranks,
               "check": args.check}
        ctx.close()
        if ctx.rank == 0:
            rec.update(pre)
            emit(rec)
        return
    if ctx.group:
        main_group(ctx, args)
        return
    from pygrid_amd import Engine
    from pygrid_amd.sharding import shard_bounds

    mode, dtype, n_default, parties, pg_default = WORKLOADS[args.workload]
    N = args.clients or n_default
    Pg = args.params or pg_default
    P = Pg if args.workload == "secagg-clients" else Pg * ctx.world
    lo, hi = (0, P) if args.workload == "secagg-clients" else shard_bounds(P, ctx.world, ctx.rank)
    eng = Engine(ctx.device)
    eng.set_layout([P])
    eng.set_shard(lo, hi)
    if args.variant is not None:
        eng.set_variant(args.variant)
    if args.workload == "c4-stream":
        rec = run_c4(ctx, args, eng, N, hi - lo, P)
    elif args.workload == "c5-ingest":
        rec = run_c5(ctx, args, eng, N, hi - lo, P)
    elif args.workload == "secagg-clients":
        rec = run_secagg_clients(ctx, args, eng, N, parties, P)
    elif args.workload == "mnist-state":
        rec = run_mnist_state(ctx, args, eng)
    elif args.workload == "resnet18-state":
        rec = run_resnet18_state(ctx, args, eng, N)
    elif args.workload == "resnet18-report":
        rec = run_resnet18_report(ctx, args, eng, N)
    elif args.workload == "resnet18-secagg-state":
        rec = run_resnet18_secagg_state(ctx, args, eng, N, parties)
    else:
        rec = run_resident(ctx, args, eng, mode, dtype, N, parties, hi - lo, P, lo, hi)
        if args.workload == "resnet18-fedavg" and ctx.world == 1 and not args.no_e2e:
            # the bytes -> bytes close of the same config (BASELINE.md cycle close), beside the kernel line
            RUN["stage"] = "cycle_close_e2e"
            rec["cycle_close_e2e"] = e2e_close(ctx, args, eng, N) if time_for("cycle_close_e2e", 40) \
                else skipped("cycle_close_e2e")
            RUN["stage"] = "cycle_close_report_time"
            rec["cycle_close_report_time"] = report_close(ctx, args, eng) \
                if time_for("cycle_close_report_time", 45) else skipped("cycle_close_report_time")
    RUN["stage"] = "teardown"
    eng.close()
    del eng
    if ctx.world > 1:
        ctx.torch.cuda.synchronize()
        ctx.torch.cuda.empty_cache()
        ctx.barrier()
    ctx.close()
    RUN["stages"]["headline"] = round(time.time() - t_head, 1)
    if ctx.rank == 0:
        rec.update(pre)  # measured before this world touched a GPU (pre_world_lines)
        emit(rec)


if __name__ == "__main__":
    main()
