#!/usr/bin/env python3
"""Phase times of one ResNet-18 x 100 clients State-bytes cycle close (CycleAggregator.
average_plan_diffs, the bench's resnet18-state line): where the time beyond the H2D goes."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd import Engine  # noqa: E402
from pygrid_amd.cycle import CycleAggregator  # noqa: E402
from pygrid_amd.state_schema import build_state_fast  # noqa: E402
from pygrid_amd.workloads import RESNET18_SHAPES  # noqa: E402

N = 100
rng = np.random.default_rng(1)
ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
distinct = [build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2) for s in RESNET18_SHAPES])
            for _ in range(4)]
ds = [distinct[k % 4] for k in range(N)]
eng = Engine(0)
agg = CycleAggregator(eng)
for _ in range(2):
    agg.average_plan_diffs({}, ck, ds)
T = {}


def t(name, f, *a):
    t0 = time.perf_counter()
    r = f(*a)
    T.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
    return r


for _ in range(5):
    t0 = time.perf_counter()
    agg._prepare(agg._numel, N)
    T.setdefault("prepare", []).append((time.perf_counter() - t0) * 1e3)
    t("ckpt_upload_state", eng.ckpt_upload_state, ck)
    t1 = time.perf_counter()
    for i, d in enumerate(ds):
        t("ingest_first" if i == 0 else ("ingest_last" if i == N - 1 else "ingest_mid"), eng.ingest_state, i, d)
    T.setdefault("ingest_all", []).append((time.perf_counter() - t1) * 1e3)
    t("fedavg_resident", eng.fedavg_resident, 0)
    t("ckpt_patch_state", eng.ckpt_patch_state, ck)
    eng.reset_stats()
    t0 = time.perf_counter()
    agg.average_plan_diffs({}, ck, ds)
    T.setdefault("whole", []).append((time.perf_counter() - t0) * 1e3)
    st = eng.stats()
    T.setdefault("stats_h2d_ms", []).append(st["h2d_ms_total"])
print({k: round(float(np.median(v)), 3) for k, v in T.items()})
