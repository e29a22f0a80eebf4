"""Copy accounting under ``rocprofv3 --memory-copy-trace``: how many host <->
HBM copies the library issues in a few report-time cycles and end-to-end closes, against what the
profiler records, and whether any are still queued when the process ends.

    rocprofv3 --memory-copy-trace --kernel-trace -d OUT -o run --output-format csv -- \\
        python3 tools/probe_copies.py [--settle-s S] [--pageable]

Per cycle: 12 ResNet-18-sized State diffs (47 MB each) reported into HBM slots (page-locked
blocks unless --pageable), certain-only folds, the close's FINAL pass and its D2H pieces.  Prints
one JSON line with the copies issued (ingests, D2H pieces by size) so the trace's rows can be
matched; ``--settle-s`` waits that long after ``Engine.close()`` (every stream synchronised) before
the interpreter exits, to tell copies still in flight at teardown from completions the profiler
never receives.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=3)
    ap.add_argument("--reports", type=int, default=12)
    ap.add_argument("--settle-s", type=float, default=0.0)
    ap.add_argument("--pageable", action="store_true")
    args = ap.parse_args()

    import numpy as np

    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.report import PinnedPool
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    rng = np.random.default_rng(3)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    diffs = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2) for s in RESNET18_SHAPES])
             for _ in range(2)]
    pool = None if args.pageable else PinnedPool(max_blocks=4)
    if pool is not None:  # the report handler's decode lands in page-locked blocks (node.install)
        import ctypes

        blocks = []
        for d in diffs:
            arr, addr = pool.acquire(len(d))
            ctypes.memmove(addr, d, len(d))
            blocks.append(arr)
        diffs = blocks
    n_ingest = 0
    t0 = time.perf_counter()
    eng = Engine(0)
    for _ in range(args.cycles):
        inc = IncrementalCycle(eng, numel, slots=args.reports + 2, checkpoint=ck, fold_batch=4)
        for w in range(args.reports + 1):
            inc.assigned(w)
        for w in range(1, args.reports + 1):  # worker 0 never reports: everything folds at close
            inc.reported(w, diffs[w % 2])
            n_ingest += 1
        ck = inc.close(ck)
    eng.close()
    closed_at = time.perf_counter() - t0
    if args.settle_s:
        time.sleep(args.settle_s)
    p_bytes = 4 * sum(numel)
    piece = 8 << 20
    print(json.dumps({"cycles": args.cycles, "reports_ingested": n_ingest, "page_locked_reports": pool is not None,
                      "d2h_pieces_per_close": -(-p_bytes // piece), "checkpoint_bytes": p_bytes,
                      "engine_closed_after_s": round(closed_at, 3), "settle_s": args.settle_s}), flush=True)
    if pool is not None:
        del diffs, blocks
        pool.close()
    return 0


if __name__ == "__main__":
    main()
