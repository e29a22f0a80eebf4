#!/usr/bin/env python3
"""Host base64 decode of a ResNet-18-sized diff (fl_events.py:257): Python vs native, by threads.
(r02 A/B knobs, since removed from the library: PGH_B64_GENERAL=1 forced the general path, PGH_B64_POPULATE=0 skipped the
output pre-population.)"""
import base64
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from pygrid_amd.report import b64decode  # noqa: E402

d = np.random.default_rng(0).integers(0, 256, 47_000_000, dtype=np.uint8).tobytes()
e = base64.b64encode(d)
m = base64.encodebytes(d)
b64decode(b"QQ==")
for label, text in (("plain", e), ("mime76", m)):
    for th in (0, 1, 4, 16):
        ts = []
        for _ in range(4):
            t = time.perf_counter()
            out = b64decode(text, threads=th)
            ts.append((time.perf_counter() - t) * 1e3)
        assert out == d
        print(f"{label} native threads={th or 'auto'}: {sorted(ts)[1]:.1f} ms ({len(text) / sorted(ts)[1] / 1e6:.2f} GB/s of text)")
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        base64.b64decode(text)
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"{label} python: {sorted(ts)[1]:.1f} ms")
