#!/usr/bin/env python3
"""Where the one slow (~7 ms) close among the first few CycleAggregator.average_plan_diffs calls
goes: every Engine method and the State scan timed inside the real call."""
import functools
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine  # noqa: E402
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


def wrap(obj, name):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T[name] = round(T.get(name, 0) + (time.perf_counter() - t0) * 1e3, 3)
        return r
    setattr(obj, name, g)


for n in ("reset", "ckpt_upload_state", "ingest_state", "fedavg_resident", "ckpt_patch_state", "set_layout", "reserve"):
    wrap(eng, n)
wrap(cyc.state_codec, "tensor_numels")
for it in range(6):
    T.clear()
    t0 = time.perf_counter()
    agg.average_plan_diffs({}, ck, ds)
    print(it, round((time.perf_counter() - t0) * 1e3, 3), T, flush=True)
