#!/usr/bin/env python3
"""Where the one slow (~7 ms) close among the first few CycleAggregator.average_plan_diffs calls
goes (r01ap: all of it inside the second close's checkpoint patch): every Engine method, the State
scan and the fresh-checkpoint steps timed inside the real call.

    python tools/time_mnist_second.py [closes]
Environment knobs worth comparing: MALLOC_MMAP_THRESHOLD_ (fixes glibc's dynamic mmap threshold),
(PGH_PREFAULT=0 was the r01 arm; the pre-fault is now always on)."""
import functools
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine, _lib  # noqa: E402
from pygrid_amd import cycle as cyc  # noqa: E402
from pygrid_amd.cycle import CycleAggregator  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import MNIST_SHAPES  # noqa: E402

rng = np.random.default_rng(1)
ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) for s in MNIST_SHAPES])
ds = [build_state_fast([rng.standard_normal(s, dtype=np.float32) for s in MNIST_SHAPES]) for _ in range(3)]
eng = Engine(0)
agg = CycleAggregator(eng)
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


for n in ("reset", "ckpt_upload_state", "ingest_state", "fedavg_resident", "ckpt_patch_state", "ckpt_patch_into",
          "set_layout", "reserve"):
    wrap(eng, n)
wrap(cyc.state_codec, "tensor_numels")
wrap(_lib, "fresh_bytes")
from pygrid_amd import state_schema as SS  # noqa: E402

wrap(SS, "tensor_shapes")
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    T.clear()
    t0 = time.perf_counter()
    agg.average_plan_diffs({}, ck, ds)
    print(it, round((time.perf_counter() - t0) * 1e3, 3), T, flush=True)
