"""Report path helper: the diff's base64 decode (``fl_events.report``,
``apps/node/src/app/main/events/model_centric/fl_events.py:257``) done natively.

``b64decode(s)`` is a drop-in for ``base64.b64decode(s)`` (same result, same
``binascii.Error`` on bad padding) that splits the work over host threads; the node's
``report`` handler can call it instead of the Python codec for multi-MB diffs.
"""
from __future__ import annotations

import binascii
import ctypes as C

from . import _lib


def b64decode(s, threads: int = 0) -> bytes:
    if isinstance(s, str):
        s = s.encode("ascii")
    elif not isinstance(s, bytes):
        s = bytes(s)
    lib = _lib.load()
    n = C.c_size_t(0)
    # one pass for a clean string: allocate the size its tail implies, decode (which checks the rest)
    if len(s) >= (1 << 16) and lib.pgh_b64_clean_size(s, len(s), C.byref(n)) == 0:
        out, dst = _lib.fresh_bytes(n.value)
        rc = lib.pgh_b64_decode_clean(s, len(s), dst, n.value, C.byref(n), int(threads))
        if rc == 0:
            return out
        if rc == -5:
            raise binascii.Error("Incorrect padding")
        # PGH_E_STATE: not clean (junk, line breaks): the general route
    if lib.pgh_b64_decode(s, len(s), None, C.byref(n), int(threads)) != 0:  # validate + exact size
        raise binascii.Error("Incorrect padding")
    out, dst = _lib.fresh_bytes(n.value)  # fresh, unshared bytes object: decoded into in place
    if n.value:
        if lib.pgh_b64_decode(s, len(s), dst, C.byref(n), int(threads)) != 0:
            raise binascii.Error("Incorrect padding")
    return out
