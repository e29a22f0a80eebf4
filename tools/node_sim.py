#!/usr/bin/env python3
"""What a PyGrid node sees per cycle with the engine wired in: the
report handler's work for each client (fl_events.py:257-261: the JSON's base64 diff text ->
bytes -> submit), here `report.b64decode` + `IncrementalCycle.reported` (the diff straight into
an HBM slot), and the close when the cycle ends (cycle_manager.py:217).  ResNet-18, 100 workers
assigned per cycle, ~20 % never report (routes.py:314), shuffled arrival, several cycles chained
through the resident checkpoint.

    python tools/node_sim.py [cycles] [--pinned] [--tune] [--phases] [--no-speculate] [--close-gap-ms=50]

Prints one JSON line: per-report handler latency (decode, ingest, total: p50 / p99 / max), the host
bytes copied into the library's staging ring per report, and the close latency per cycle.
``--pinned``: the report is decoded into a page-locked block (``report.PinnedPool``) and DMA'd as
it lies.  ``--tune``: ``pygrid_amd.tune_process()`` first (glibc thresholds;
the engine's own share of the close is the untuned run).  ``--no-speculate``: fold only certain
positions early.  ``--close-gap-ms``: pause between the last report and the close (0: at once, as
when the report that reaches ``max_diffs`` triggers ``complete_cycle``; 50 by default, a
``cycle.end`` close).
"""
import base64
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine  # noqa: E402
from pygrid_amd.incremental import IncrementalCycle  # noqa: E402
from pygrid_amd.report import b64decode  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import RESNET18_SHAPES  # noqa: E402


def pct(xs, q):
    return round(float(np.percentile(xs, q)), 3)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cycles = int(args[0]) if args else 4
    speculate = False if "--no-speculate" in sys.argv else None
    gap_ms = next((float(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--close-gap-ms=")), 50.0)
    tuned = None
    if "--tune" in sys.argv:
        import pygrid_amd

        tuned = pygrid_amd.tune_process(hw_queues=False)
    pool = None
    if "--pinned" in sys.argv:
        from pygrid_amd.report import PinnedPool

        pool = PinnedPool(max_blocks=8)
    rng = np.random.default_rng(2024)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ckpt = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    # the report payload as the JSON carries it: base64 text of the State diff (4 distinct diffs, re-sent)
    texts = [base64.b64encode(build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                                for s in RESNET18_SHAPES])).decode("ascii") for _ in range(4)]
    eng = Engine(0)
    phases = {}
    if "--phases" in sys.argv:  # time the engine calls inside close (as tools/time_report_close.py)
        import functools

        from pygrid_amd import state as st

        def wrap(obj, name):
            f = getattr(obj, name)

            @functools.wraps(f)
            def g(*a, **k):
                t0 = time.perf_counter()
                r = f(*a, **k)
                phases[name] = round(phases.get(name, 0) + (time.perf_counter() - t0) * 1e3, 3)
                return r
            setattr(obj, name, g)
        for nm in ("fold_slots_finish_resident", "ckpt_patch_into", "fold_slots"):
            wrap(eng, nm)
        wrap(st, "fresh_frame_bytes")
    dec, ing, tot, closes, close_phases, staged = [], [], [], [], [], []
    for cyc in range(cycles + 1):  # cycle 0 warms up
        n = 100
        reporters = [w for w in range(n) if rng.random() >= 0.2]
        inc = IncrementalCycle(eng, numel, slots=n, fold_batch=8, checkpoint=ckpt, speculate=speculate)
        for w in range(n):
            inc.assigned(w)
        for w in rng.permutation(reporters):
            s0 = eng.stats()["h2d_staged_bytes_total"]
            t0 = time.perf_counter()
            diff = b64decode(texts[int(w) % 4], into=pool)  # fl_events.py:257
            t1 = time.perf_counter()
            inc.reported(int(w), diff)           # submit_worker_diff, cycle_manager.py:151-178
            t2 = time.perf_counter()
            del diff                             # the handler returns (its pinned block goes back)
            if cyc:
                dec.append((t1 - t0) * 1e3)
                ing.append((t2 - t1) * 1e3)
                tot.append((t2 - t0) * 1e3)
                staged.append(eng.stats()["h2d_staged_bytes_total"] - s0)
        if gap_ms:
            time.sleep(gap_ms / 1e3)  # the cycle ends some time after the last report (cycle.end timer)
        phases.clear()
        t0 = time.perf_counter()
        new = inc.close(ckpt)
        t1 = time.perf_counter()
        ckpt = new  # the previous checkpoint's bytes are freed here (the node drops them after the save)
        t2 = time.perf_counter()
        if cyc:
            closes.append((t2 - t0) * 1e3)
            close_phases.append(dict(phases, close_call=round((t1 - t0) * 1e3, 3), free_old=round((t2 - t1) * 1e3, 3),
                                     folded_before_close=inc.folded_early))
    eng.close()
    if pool is not None:
        pool.close()
    print(json.dumps({
        "pinned_reports": pool is not None, "process_tuning": tuned, "speculative_folds": inc.speculate,
        "close_gap_ms": gap_ms,
        "pinned_pool": {"hits": pool.hits, "misses": pool.misses} if pool is not None else None,
        "host_staging_bytes_per_report": {"mean": round(float(np.mean(staged)), 1), "max": int(max(staged))},
        "workload": "ResNet-18 (62 tensors), 100 assigned per cycle, ~20 % never report, shuffled arrival, "
                    "base64 text -> report.b64decode -> IncrementalCycle.reported; close close_gap_ms after the last report",
        "cycles": cycles, "reports": len(tot),
        "report_b64decode_ms": {"p50": pct(dec, 50), "p99": pct(dec, 99), "max": round(max(dec), 3)},
        "report_ingest_ms": {"p50": pct(ing, 50), "p99": pct(ing, 99), "max": round(max(ing), 3)},
        "report_handler_ms": {"p50": pct(tot, 50), "p99": pct(tot, 99), "max": round(max(tot), 3)},
        "close_ms": [round(c, 3) for c in closes], "close_phases_ms": close_phases}))


if __name__ == "__main__":
    main()
