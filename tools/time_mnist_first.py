#!/usr/bin/env python3
"""Phase times of the first MNIST State-bytes closes on a fresh Engine (what the 10.7 / 7.5 ms
first closes of tools/time_mnist_cold.py spend their time on)."""
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
numel = [int(np.prod(s)) for s in MNIST_SHAPES]
for it in range(4):
    T = {}

    def t(name, f, *a):
        t0 = time.perf_counter()
        r = f(*a)
        T[name] = round((time.perf_counter() - t0) * 1e3, 3)
        return r
    t("prepare", agg._prepare, numel, 3)
    t("upload", eng.ckpt_upload_state, ck)
    for i, d in enumerate(ds):
        t(f"ingest{i}", eng.ingest_state, i, d)
    t("fold", eng.fedavg_resident, 0)
    t("sync", eng.sync)
    t("patch", eng.ckpt_patch_state, ck)
    print(it, T, flush=True)
