#!/usr/bin/env python3
"""Where the report-time close's time goes, measured the way bench.py's cycle_close_report_time
triggers it (ResNet-18, 100 assigned, ~72 report in shuffled order 5 ms apart, worker 0 never, the
close submitted to an executor thread the moment the last report returned): per cycle, the
executor hand-off, ``seal``, the host time of every engine call inside ``finish``
(``fold_slots_finish_resident``: the launches; ``ckpt_patch_into``: the FINAL pass's D2H pieces
waited for and copied out into the new checkpoint bytes), the prepared frame's join, and the total.

    python tools/close_phases.py [cycles] [--gap-ms 5]

One JSON line per cycle, then the medians.  Run it under ``rocprofv3 --kernel-trace
--memory-copy-trace`` for the device timeline of the same closes (the copies HIP runs as
``__amd_rocclr_copyBuffer`` kernels are in the kernel trace only: DESIGN.md section 5).
"""
from __future__ import annotations

import argparse
import functools
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cycles", nargs="?", type=int, default=8)
    ap.add_argument("--gap-ms", type=float, default=5.0)
    args = ap.parse_args()

    import numpy as np

    import pygrid_amd
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    pygrid_amd.tune_process(hw_queues=False)  # bench.py's process tuning (allocator thresholds)
    rng = np.random.default_rng(1234 + 17)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                  for s in RESNET18_SHAPES]) for _ in range(4)]
    assigned = 100
    reporters = [w for w in range(assigned) if w != 0 and rng.random() >= 0.2]
    T = {}

    def timed(obj, name, key=None):
        f = getattr(obj, name)

        @functools.wraps(f)
        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                T[key or name] = T.get(key or name, 0.0) + (time.perf_counter() - t0) * 1e3
        setattr(obj, name, g)

    eng = Engine(0)
    for n in ("fold_slots_finish_resident", "ckpt_patch_into", "fold_slots", "ckpt_upload_state"):
        timed(eng, n)
    for n in ("seal", "finish"):
        timed(IncrementalCycle, n)
    rows = []
    with ThreadPoolExecutor(1, thread_name_prefix="executor") as ex:
        for cyc in range(args.cycles + 1):
            inc = IncrementalCycle(eng, numel, slots=assigned, checkpoint=ck)
            for w in range(assigned):
                inc.assigned(w)
            for i, w in enumerate(rng.permutation(reporters)):
                if i and args.gap_ms:
                    time.sleep(args.gap_ms / 1e3)
                inc.reported(int(w), distinct[int(w) % 4])
            T.clear()
            started = []

            def close(ck_pb):
                started.append(time.perf_counter())
                return inc.close(ck_pb)
            t0 = time.perf_counter()
            ck = ex.submit(close, ck).result()
            total = (time.perf_counter() - t0) * 1e3
            if cyc == 0:
                continue  # warm-up
            r = {"total_ms": round(total, 3), "handoff_ms": round((started[0] - t0) * 1e3, 3),
                 **{k: round(v, 3) for k, v in T.items()},
                 "rows_at_close": inc.last_close["n"] - inc.last_close["early"]}
            r["finish_other_ms"] = round(r.get("finish", 0) - r.get("fold_slots_finish_resident", 0)
                                         - r.get("ckpt_patch_into", 0), 3)
            rows.append(r)
            print(json.dumps(r), flush=True)
    med = {k: round(float(np.median([r[k] for r in rows if k in r])), 3) for k in rows[0]}
    print(json.dumps({"median": med, "cycles": len(rows), "gap_ms": args.gap_ms}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
