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
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

# benchlib.common asks for the hardware queues before anything touches HIP (first import)
from benchlib.common import (DEFAULT_BUDGET_S, HW_QUEUES, PROCESS_TUNING, RUN, WORKLOADS, emit,  # noqa: E402
                             set_deadline, skipped, start_watchdog, stub_sleep, time_for)
from benchlib.closes import (e2e_close, report_close, run_mnist_state, run_resnet18_report,  # noqa: E402
                             run_resnet18_secagg_state, run_resnet18_state)
from benchlib.launch import pre_world_lines, spawn_ranks  # noqa: E402
from benchlib.resident import (run_c4, run_c5, run_group_resident, run_group_secagg_clients,  # noqa: E402
                               run_resident, run_secagg_clients)
from benchlib.world import Ctx, check_sampled  # noqa: E402,F401 -- check_sampled: tests/test_bench_launch.py
from benchlib.baseline import usable_cores  # noqa: E402,F401 -- tests/test_bench_launch.py
from benchlib.roofline import roofline_of, under_profiler  # noqa: E402,F401 -- tests/test_bench_launch.py


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
    # child lines, live PMC passes and the CPU baseline first: nothing of this world holds a GPU yet
    pre_world_lines(args, pre)
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
