#!/usr/bin/env python3
"""Where a speculative close started at once after the last report goes (bench.py's
cycle_close_report_time arms): every Engine call made by the last report's ``reported`` and by the
close, with its start / end relative to the moment the last ``reported`` returned.

    python tools/probe_spec_close.py [cycles] [--gap-ms=5] [--no-peek] [--certain]

Prints one JSON line per cycle (after a warm-up cycle): the call log of the last report and of the
close, the close's wall time and ``last_close``.
"""
import functools
import json
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine  # noqa: E402
from pygrid_amd import state as st  # noqa: E402
from pygrid_amd.incremental import IncrementalCycle  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import RESNET18_SHAPES  # noqa: E402

LOG = []
LOCK = threading.Lock()


def wrap(obj, name):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            with LOCK:
                LOG.append((name, threading.current_thread().name, t0, time.perf_counter()))
    setattr(obj, name, g)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cycles = int(args[0]) if args else 3
    gap = next((float(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--gap-ms=")), 5.0)
    opts = {"speculate": False} if "--certain" in sys.argv else {"speculate": True, "peek": "--no-peek" not in sys.argv}
    rng = np.random.default_rng(7)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                  for s in RESNET18_SHAPES]) for _ in range(4)]
    reporters = [w for w in range(100) if w != 0 and rng.random() >= 0.2]
    eng = Engine(0)
    for name in ("ingest_state", "fold_slots_keep", "fold_slots", "fold_mark", "fold_unmark", "fold_rewind",
                 "fold_peek", "peek_patch_into", "fold_slots_finish_resident", "ckpt_patch_into", "fold_busy",
                 "peek_valid", "ckpt_upload_state"):
        if hasattr(eng, name):
            wrap(eng, name)
    wrap(st, "fresh_checkpoint")
    with ThreadPoolExecutor(1, thread_name_prefix="executor") as ex:
        for cyc in range(cycles + 1):
            inc = IncrementalCycle(eng, numel, slots=100, checkpoint=ck, **opts)
            for w in range(100):
                inc.assigned(w)
            order = [int(w) for w in rng.permutation(reporters)]
            for i, w in enumerate(order):
                if i and gap:
                    time.sleep(gap / 1e3)
                if i == len(order) - 1:
                    with LOCK:
                        LOG.clear()
                    t_rep = time.perf_counter()
                inc.reported(w, distinct[w % 4])
            t0 = time.perf_counter()
            ck = ex.submit(inc.close, ck).result()
            t1 = time.perf_counter()
            time.sleep(0.05)  # let a late timer / peek thread log
            if cyc:
                with LOCK:
                    calls = [(n, th, round((a - t0) * 1e3, 3), round((b - t0) * 1e3, 3)) for n, th, a, b in LOG]
                print(json.dumps({"cycle": cyc, "opts": opts, "close_ms": round((t1 - t0) * 1e3, 3),
                                  "last_report_ms": round((t0 - t_rep) * 1e3, 3), "last_close": inc.last_close,
                                  "calls_ms_from_close_start": calls}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
