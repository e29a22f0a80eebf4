#!/usr/bin/env python3
"""Where the close's ``ckpt_patch_into`` time goes (r03k: 2.0-2.8 ms for 47 MB whether 0 or 83 rows
were left to fold).  ResNet-18 resident checkpoint, one FINAL fold, then the fresh-framed output
written from HBM, timed over --reps for: a fresh output (framed now), a prepared output (framed and
faulted in beforehand), and the D2H alone into a page-locked buffer (``ckpt_download``).

    python tools/patch_probe.py [--reps 10]      (r01 knobs PGH_PREFAULT / PGH_D2H_PIECE_MB: now fixed defaults)
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np

    from pygrid_amd import Engine, PinnedBuffer
    from pygrid_amd import state as st
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    rng = np.random.default_rng(3)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) for s in RESNET18_SHAPES])
    eng = Engine(0)
    eng.set_layout(numel)
    eng.reserve(2)
    eng.ckpt_upload_state(ck)
    eng.ingest_state(0, ck)
    eng.fedavg_resident(0)
    eng.sync()
    out = {}

    def run(name, fn, prep=None):
        ts = []
        for _ in range(a.reps + 1):
            p = prep() if prep else None
            eng.sync()
            t0 = time.perf_counter()
            r = fn(p)
            ts.append((time.perf_counter() - t0) * 1e3)
            del r, p
        out[name] = {"median_ms": round(statistics.median(ts[1:]), 3), "min_ms": round(min(ts[1:]), 3)}

    run("fresh_output", lambda p: st.fresh_checkpoint(eng, ck))
    run("prepared_output", lambda p: st.fresh_checkpoint(eng, ck, prepared=p), lambda: st.prepared_fresh_frame(ck))
    pb = PinnedBuffer((sum(numel),))
    run("d2h_pinned_only", lambda p: eng._lib.pgh_ckpt_download(eng._h, pb.array.ctypes.data))
    run("download_pageable", lambda p: eng.ckpt_download())
    run("frame_only", lambda p: st.fresh_frame_bytes(ck))
    run("prepare_only", lambda p: st.prepared_fresh_frame(ck))
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
