#!/usr/bin/env python3
"""The report-time close's D2H pieces against the oracle, close by close (profiles/r06s/: round
6's K6 k_copy_to_host, since removed, copied out FINAL ranges that had not run yet): a 20 M-param
shard (10 pieces of 8 MiB, 8 cells), three chained report-time closes, in REPS fresh contexts per
PGH_D2H_STREAM mode; on a mismatch, which cycle, which pieces (flat index * 4 // 8 MiB), how many
floats, whether the device-resident result is right, and what the wrong host floats equal: zeros,
the previous checkpoint, the old contents of the FINAL output buffer (the result two closes back),
another piece of the result.  Exit status 1 if any close was wrong.

    python tools/diag_d2h_race.py [reps] [modes, e.g. 1,0]
"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

PIECE = 8 << 20


def run(mode: str, reps: int):
    os.environ["PGH_D2H_STREAM"] = mode
    from oracle import oracle as O
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    F = np.float32
    shapes = [(4000, 5000), (7,)]
    numel = [int(np.prod(s)) for s in shapes]
    bad = 0
    for rep in range(reps):
        with Engine(0) as eng:  # a fresh context per repetition (K6's failures came early in a process)
            rng = np.random.default_rng(931 + rep)
            ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
            ck_pb = build_state_fast(ckpt)
            hist = [np.concatenate([a.reshape(-1) for a in ckpt])]
            for cyc in range(3):
                diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(3)]
                inc = IncrementalCycle(eng, numel, slots=4, checkpoint=ck_pb)
                for w in range(4):
                    inc.assigned(w)
                for w in (2, 1, 3):
                    inc.reported(w, build_state_fast(diffs[w - 1]))
                prev = np.concatenate([a.reshape(-1) for a in ckpt])
                prev2 = hist[-2] if len(hist) >= 2 else None
                ck_pb = inc.close(ck_pb)
                ckpt = O.fedavg_mean(ckpt, diffs)
                want = np.concatenate([a.reshape(-1) for a in ckpt]).view(np.uint32)
                got = np.concatenate([a.reshape(-1) for a in parse_state(ck_pb)]).astype(F).view(np.uint32)
                diff = np.flatnonzero(got != want)
                hist.append(want.view(F))
                if diff.size:
                    dev = eng.ckpt_download().astype(F).view(np.uint32)
                    dev_bad = int((dev != want).sum())
                    two_back = int((got[diff] == prev2.view(np.uint32)[diff]).sum()) if prev2 is not None else -1
                    print(f"  device-resident result: {dev_bad} floats wrong; wrong host floats equal to the "
                          f"result two closes back (d_out's old content): {two_back}", flush=True)
                    bad += 1
                    pieces = sorted(set((diff * 4 // PIECE).tolist()))
                    stale = int((got[diff] == prev.view(np.uint32)[diff]).sum())
                    other = 0
                    for d in diff[:2000]:
                        off = d % (PIECE // 4)
                        cands = want[off::PIECE // 4]
                        other += int(np.any(cands == got[d]))
                    print(f"mode {mode} rep {rep} cycle {cyc}: {diff.size} floats differ, pieces {pieces}, "
                          f"first {diff[0]} last {diff[-1]}; equal to the previous checkpoint: {stale}; "
                          f"equal to the same offset of another piece (first 2000): {other}; "
                          f"zeros: {int((got[diff] == 0).sum())}", flush=True)
                    ck_pb = build_state_fast(ckpt)  # continue from the right checkpoint
    print(f"mode {mode}: {bad} bad closes of {3 * reps}", flush=True)
    return bad


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    modes = (sys.argv[2] if len(sys.argv) > 2 else "1,0").split(",")
    # one mode per process: the library reads PGH_D2H_STREAM when a context is made
    if len(modes) > 1:
        import subprocess

        rc = 0
        for m in modes:
            rc |= subprocess.call([sys.executable, "-u", __file__, str(reps), m])
        sys.exit(rc)
    sys.exit(1 if run(modes[0], reps) else 0)
