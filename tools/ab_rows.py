#!/usr/bin/env python3
"""Interleaved A/B of the report-time close fold K1r (``k_fedavg_rows``, pgh_fold_slots_finish_resident)
over a scattered row table, in ONE process (~80 rows at close).

    python tools/ab_rows.py [--params P] [--slots S] [--rows R] [--mode 0] [--rounds 10] [--variants 0,11]

Every round re-generates the slab on the GPU (untimed), then times one finish-fold per variant
(HIP events: pgh_stats kernel_ms_last) over the same R of S slots in shuffled order.  Prints one
JSON line: per-variant median / min ms and TB/s of algorithmic bytes (4 R P + 8 P).
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=11_689_512)
    ap.add_argument("--slots", type=int, default=100)
    ap.add_argument("--rows", type=int, default=83)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--variants", default="0,11")
    a = ap.parse_args()
    import numpy as np

    from pygrid_amd import Engine

    P, S, R = a.params, a.slots, a.rows
    rng = np.random.default_rng(5)
    rows = [int(x) for x in rng.permutation(S)[:R]]
    eng = Engine(0)
    eng.set_layout([P])
    eng.reserve(S)
    ck = np.full(P, 0.01, np.float32)
    if a.mode == 2:
        eng.set_weights([1.0 + (c % 3) for c in range(R)])
    variants = [int(v) for v in a.variants.split(",")]
    times = {v: [] for v in variants}
    alg = 4 * R * P + 8 * P
    for rnd in range(a.rounds + 1):
        order = variants if rnd % 2 == 0 else variants[::-1]
        for v in order:
            eng.reset()
            eng.synth_fill(1, S)          # untimed: the slab holds S clients again
            eng.ckpt_upload(ck)
            if a.mode == 2:
                eng.set_weights([1.0 + (c % 3) for c in range(R)])
            eng.set_variant(v)
            eng.sync()
            eng.reset_stats()
            eng.fold_slots_finish_resident(a.mode, rows)
            eng.sync()
            st = eng.stats()
            if rnd:  # round 0 warms every variant
                times[v].append(st["kernel_ms_total"] / max(st["kernel_launches"], 1))
    eng.close()
    out = {v: {"median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
               "TBps_median": round(alg / statistics.median(t) / 1e9, 3)} for v, t in times.items()}
    print(json.dumps({"params": P, "rows": R, "slots": S, "mode": a.mode, "rounds": a.rounds,
                      "alg_bytes": alg, "variants": out}))


if __name__ == "__main__":
    main()
