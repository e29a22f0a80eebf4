"""How bench.py forms its worlds: N rank processes without a launcher (spawn_ranks), and the child
lines -- configs 1, 3, 4, 5, the one-process group, the CPU baseline and the live PMC passes --
run before this process or any rank of its world touches a GPU (pre_world_lines)."""
from __future__ import annotations

import json
import os
import sys
import threading
import time

from benchlib.common import (BENCH, HBM_PEAK_GBS, RUN, child_env, emit, headline_error_line, json_lines, remaining,
                             run_child)
from benchlib.roofline import under_profiler


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
        procs.append(subprocess.Popen([sys.executable, str(BENCH), *sys.argv[1:]], env=env,
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


def wants_group_line(args) -> bool:
    return args.gpus > 1 and not args.group and not args.no_group_line and args.workload in GROUP_WORKLOADS


def group_line(args, limit_s: int = 240) -> dict:
    """The path the node deploys at N > 1 (its single process drives every GPU through one library
    context, ``pgh_create_group``), measured on the same GPUs before the
    per-rank world forms: ``bench.py --group --gpus N`` in a FRESH child (no process that touched a
    GPU re-execs), summarised for the per-rank line.  ``rccl`` says whether the group's exchange ran
    over RCCL (distinct devices) or peer copies."""
    import subprocess

    cmd = [sys.executable, str(BENCH), "--group", "--gpus", str(args.gpus), "--workload",
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
    "c5-ingest": "fold batch 4 (half the 8-slot ring): each fold launch also reads and writes the running state "
                 "(4 B + 4 B per param per 4 clients), so the fold kernel moves 1.5x its diff bytes; fold_frac counts "
                 "those bytes, e2e_frac only the diff bytes (the step is PCIe-bound)",
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
    cmd = [sys.executable, str(BENCH), "--gpus", str(gpus), "--workload", workload,
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
    """Everything of this run that must not share the GPU (or the host cores) with a rank's timed
    work -- the child lines (configs 1, 3, 4, 5 and the one-process group over the same GPUs), the
    live PMC passes behind ``roofline.traffic`` and the ``cpu_baseline`` child -- runs BEFORE this
    process, or any rank of its world, touches a GPU: a parent holding a HIP context while its
    child runs slowed the child's config-4 step by 13 % (176 vs 154 ms, profiles/r04g/).  Under
    torch.distributed.run rank 0 runs them while the other ranks wait on the launcher's store (no
    GPU touched; the wait ends by the run's deadline); at N = 1, and in the parent that spawns
    ranks itself, this process runs them first.  Each is limited by the run's budget (run_child).
    The PMC figure reaches the ranks a parent spawns in PGH_BENCH_LIVE_TRAFFIC; the rest merges
    into the headline line.  Fills and returns ``out``."""
    from benchlib import roofline
    from benchlib.baseline import pre_world_cpu_baseline, wants_cpu_baseline
    from benchlib.common import headline_reserve

    out = {} if out is None else out
    spawned = os.environ.get("PGH_BENCH_SPAWNED") == "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    jobs = (wants_config_lines(args), wants_group_line(args), roofline.wants_live_traffic(args),
            wants_cpu_baseline(args))
    if spawned or args.group or not any(jobs):
        return out
    rank = int(os.environ.get("RANK", "0"))

    def run():
        configs, group, live, cpu = jobs
        if configs:
            attach_config_lines(args, out)
        if group:
            out["group"] = group_line(args)
        if live:
            RUN["stage"] = "live_traffic"
            roofline.LIVE_TRAFFIC = roofline.measure_live_traffic(args)
            if roofline.LIVE_TRAFFIC is not None:
                os.environ[roofline.LIVE_TRAFFIC_ENV] = json.dumps(list(roofline.LIVE_TRAFFIC))
        if cpu:
            RUN["stage"] = "cpu_baseline"
            out["cpu_baseline"] = pre_world_cpu_baseline(args, reserve=headline_reserve(args))

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
