#!/usr/bin/env python3
"""Where the report-time close goes (bench.py --workload resnet18-report: ResNet-18, 100 assigned,
~83 report in shuffled order, worker 0 never): every Engine call and codec step inside
IncrementalCycle.close timed, per cycle.

    python tools/time_report_close.py [cycles] [--idle SECONDS] [--profile]
"""
import functools
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine, _lib  # noqa: E402
from pygrid_amd import state as st  # noqa: E402
from pygrid_amd.incremental import IncrementalCycle  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import RESNET18_SHAPES  # noqa: E402

rng = np.random.default_rng(1234)
numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2) for s in RESNET18_SHAPES])
            for _ in range(4)]
N = 100
reporters = [w for w in range(N) if w != 0 and rng.random() >= 0.2]
arrival = [int(w) for w in rng.permutation(reporters)]
eng = Engine(0)
T = {}


def wrap(obj, name, key=None):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T[key or name] = round(T.get(key or name, 0) + (time.perf_counter() - t0) * 1e3, 3)
        return r
    setattr(obj, name, g)


for n in ("fold_slots", "fold_slots_finish_resident", "ckpt_patch_into", "ckpt_upload_state", "set_weights"):
    wrap(eng, n)
wrap(IncrementalCycle, "_advance")
wrap(IncrementalCycle, "_fold_ready")
wrap(st, "fresh_frame_bytes")
wrap(_lib, "fresh_bytes")
new = None  # the previous close's bytes stay alive until the next close returns (as in a node)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    inc = IncrementalCycle(eng, numel, slots=N, fold_batch=8, checkpoint=ck)
    for w in range(N):
        inc.assigned(w)
    for w in arrival:
        inc.reported(w, distinct[w % 4])
    eng.sync()
    if "--idle" in sys.argv:  # the cycle ends some time after the last report (cycle.end timer)
        time.sleep(float(sys.argv[sys.argv.index("--idle") + 1]))
    T.clear()
    import gc
    gc0 = gc.get_count()
    if "--profile" in sys.argv and it == 3:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        out = inc.close(ck)
        pr.disable()
        el = time.perf_counter() - t0
        pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
    else:
        t0 = time.perf_counter()
        out = inc.close(ck)
        el = time.perf_counter() - t0
    new = out
    print(it, round(el * 1e3, 3), T, "gc", gc0, gc.get_count(), flush=True)
