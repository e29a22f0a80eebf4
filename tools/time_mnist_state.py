#!/usr/bin/env python3
"""Per-call wall time of one MNIST State-bytes cycle close (CycleAggregator.average_plan_diffs):
where the ~0.3 ms go.  Run with PGH_BLOCK_BYTES=0 for the row-major slab."""
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
eng = Engine(0)
agg = CycleAggregator(eng)
for _ in range(5):
    agg.average_plan_diffs({}, ck, ds)
T = {}


def t(name, f, *a):
    t0 = time.perf_counter()
    r = f(*a)
    T.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
    return r


for _ in range(50):
    t0 = time.perf_counter()
    agg._prepare(agg._numel, 3)
    T.setdefault("prepare", []).append((time.perf_counter() - t0) * 1e3)
    t("ckpt_upload_state", eng.ckpt_upload_state, ck)
    for i, d in enumerate(ds):
        t(f"ingest_state{i}", eng.ingest_state, i, d)
    t("fedavg_resident", eng.fedavg_resident, 0)
    t("ckpt_patch_state", eng.ckpt_patch_state, ck)
    t0 = time.perf_counter()
    agg.average_plan_diffs({}, ck, ds)
    T.setdefault("whole", []).append((time.perf_counter() - t0) * 1e3)
print({k: round(float(np.median(v)), 4) for k, v in T.items()}, "stats ld", eng.stats()["ld"], "slab", eng.slab()[1:])
