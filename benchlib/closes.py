"""The bytes -> bytes workloads: a cycle close from State protobuf bytes in host memory to the new
checkpoint's bytes (config 1, ResNet-18 closes, shares from the wire) and the report-time close
under the reference's trigger."""
from __future__ import annotations

import json
import time

from benchlib.baseline import cpu_model, in_reference_allocator
from benchlib.common import RESNET18_P, ROOT
from benchlib.roofline import roofline_of
from benchlib.world import record


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
