#!/usr/bin/env python3
"""Where a report's base64 decode writes matters (r03 node_sim: decode into page-locked blocks took
5.1 ms p50 vs 4.1 ms into fresh bytes).  Times report.b64decode of a ResNet-18-sized diff (62 MB of
text) into: fresh bytes, a PinnedPool block (reused), and the same pool after the block was
first-touched by a plain memset -- medians over --reps, one JSON line.

    python tools/b64_into.py [--reps 20] [--threads 0]
"""
import argparse
import base64
import gc
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--mb", type=float, default=46.76)
    a = ap.parse_args()
    import numpy as np

    from pygrid_amd.report import PinnedPool, b64decode

    raw = np.random.default_rng(1).integers(0, 256, int(a.mb * 1e6), dtype=np.uint8).tobytes()
    text = base64.b64encode(raw).decode()
    out = {"decoded_bytes": len(raw), "threads": a.threads}

    def timeit(fn):
        ts = []
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            r = fn()
            ts.append((time.perf_counter() - t0) * 1e3)
            del r
            gc.collect()
        return round(statistics.median(ts[1:]), 3)

    out["fresh_bytes_ms"] = timeit(lambda: b64decode(text, threads=a.threads))
    pool = PinnedPool(max_blocks=2)
    out["pinned_block_ms"] = timeit(lambda: b64decode(text, threads=a.threads, into=pool))
    out["pinned_hits"] = pool.hits  # 0 without a GPU: the pool falls back to ordinary memory
    pool.close()
    buf = bytearray(len(raw) + 64)
    from pygrid_amd import _lib
    import ctypes as C

    lib = _lib.load()
    src = text.encode()
    addr = C.addressof((C.c_char * len(buf)).from_buffer(buf))
    n = C.c_size_t(0)

    def into_reused():
        rc = lib.pgh_b64_decode(src, len(src), C.c_void_p(addr), C.byref(n), a.threads)
        assert rc == 0
    out["reused_pageable_ms"] = timeit(into_reused)
    out["text_MB"] = round(len(text) / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
