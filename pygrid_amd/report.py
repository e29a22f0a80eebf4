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


_utf8 = C.pythonapi.PyUnicode_AsUTF8AndSize
_utf8.restype = C.c_void_p
_utf8.argtypes = [C.py_object, C.POINTER(C.c_ssize_t)]


def _text(s):
    """(keep-alive object, address or bytes, length) of the base64 text.  A str -- what the
    report's JSON yields, 62 MB for a ResNet-18 diff -- is read in place: an ASCII str stores its
    characters as one byte each, and PyUnicode_AsUTF8AndSize returns that buffer without a copy
    (``s.encode()`` would copy all of it, then free it)."""
    if isinstance(s, str):
        if not s.isascii():  # as base64.b64decode: "string argument should contain only ASCII characters"
            raise ValueError("string argument should contain only ASCII characters")
        n = C.c_ssize_t(0)
        addr = _utf8(s, C.byref(n))
        return s, addr, n.value
    if not isinstance(s, bytes):
        s = bytes(s)
    return s, s, len(s)


def b64decode(s, threads: int = 0) -> bytes:
    keep, src, length = _text(s)  # `keep` holds the text's buffer alive for the calls below
    lib = _lib.load()
    n = C.c_size_t(0)
    # one pass for a clean string: allocate the size its tail implies, decode (which checks the rest)
    if length >= (1 << 16) and lib.pgh_b64_clean_size(src, length, C.byref(n)) == 0:
        out, dst = _lib.fresh_bytes(n.value)
        rc = lib.pgh_b64_decode_clean(src, length, dst, n.value, C.byref(n), int(threads))
        if rc == 0:
            return out
        if rc == -5:
            raise binascii.Error("Incorrect padding")
        # PGH_E_STATE: not clean (junk, line breaks): the general route
    if lib.pgh_b64_decode(src, length, None, C.byref(n), int(threads)) != 0:  # validate + exact size
        raise binascii.Error("Incorrect padding")
    out, dst = _lib.fresh_bytes(n.value)  # fresh, unshared bytes object: decoded into in place
    if n.value:
        if lib.pgh_b64_decode(src, length, dst, C.byref(n), int(threads)) != 0:
            raise binascii.Error("Incorrect padding")
    del keep
    return out
