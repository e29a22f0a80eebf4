#!/usr/bin/env python3
"""MNIST State-bytes close (CycleAggregator.average_plan_diffs), wall time of every call from the
first on, back to back and then with idle gaps between closes (a node closes a cycle every few
minutes, not in a loop): is the fast close a warm-loop artefact?"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine  # noqa: E402
from pygrid_amd.cycle import CycleAggregator  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import MNIST_SHAPES  # noqa: E402

rng = np.random.default_rng(1)
ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) for s in MNIST_SHAPES])
ds = [build_state_fast([rng.standard_normal(s, dtype=np.float32) for s in MNIST_SHAPES]) for _ in range(3)]
t0 = time.perf_counter()
eng = Engine(0)
agg = CycleAggregator(eng)
print(f"engine create {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)


def close():
    t = time.perf_counter()
    agg.average_plan_diffs({}, ck, ds)
    return round(1e3 * (time.perf_counter() - t), 3)


print("back to back:", [close() for _ in range(12)], flush=True)
for gap in (0.1, 1.0, 3.0):
    out = []
    for _ in range(4):
        time.sleep(gap)
        out.append(close())
    print(f"after {gap} s idle:", out, flush=True)
