"""Report path helper: the diff's base64 decode (``fl_events.report``,
``apps/node/src/app/main/events/model_centric/fl_events.py:257``) done natively.

``b64decode(s)`` is a drop-in for ``base64.b64decode(s)`` (same result, same
``binascii.Error`` on bad padding) that splits the work over host threads; the node's
``report`` handler can call it instead of the Python codec for multi-MB diffs.

``b64decode(s, into=pool)`` decodes into a page-locked block of a ``PinnedPool`` and returns a
read-only ``memoryview`` of the diff: ``pgh_ingest_state`` then DMAs its payload spans to HBM as
they lie, instead of host threads first copying them into the library's pinned staging ring (one
host-DRAM read and one write of the whole diff less per report, and the copy threads' time).  The
view is what the node stores in its DB (``WorkerCycle.diff``: SQLAlchemy's LargeBinary binds any
buffer) and what it hands the engine; the block goes back to the pool when the last reference to
the view is gone, so a diff the DB layer or a parked report still holds is never overwritten.
"""
from __future__ import annotations

import binascii
import ctypes as C
import threading
from typing import List, Optional, Tuple

from . import _lib


_utf8 = C.pythonapi.PyUnicode_AsUTF8AndSize
_utf8.restype = C.c_void_p
_utf8.argtypes = [C.py_object, C.POINTER(C.c_ssize_t)]

_BLOCK_ALIGN = 2 << 20


class _Return:
    """Attached to the ctypes array a decoded view exports: gives the block back when collected."""

    def __init__(self, pool: "PinnedPool", addr: int, cap: int):
        self.pool, self.addr, self.cap = pool, addr, cap

    def __del__(self):
        try:
            self.pool._give(self.addr, self.cap)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class PinnedPool:
    """Page-locked host blocks (``pgh_host_alloc``) for decoded report diffs.  At most
    ``max_blocks`` blocks (each rounded up to 2 MiB) are allocated; a report beyond that -- more
    reports in flight than blocks, or a diff larger than ``max_block_bytes`` -- is decoded into
    ordinary memory, as without a pool.  Counters: ``hits`` (decoded into a block), ``misses``.

    Blocks are marked async (``pgh_host_async``): an ingest of a diff lying in one returns with its
    DMA queued, and a block that comes back is handed out again only after ``pgh_host_wait`` --
    the report handler does not wait for PCIe, the next decode never overwrites bytes in flight."""

    def __init__(self, max_blocks: int = 16, max_block_bytes: int = 1 << 30):
        self.max_blocks = int(max_blocks)
        self.max_block_bytes = int(max_block_bytes)
        self._free: List[Tuple[int, int]] = []  # (cap, addr), returned blocks
        self._n = 0
        self._closed = False
        self._lock = threading.Lock()
        self.hits = self.misses = 0

    def acquire(self, n: int):
        """(ctypes array of ``n`` writable bytes over a pinned block, its address) or None."""
        if n <= 0 or n > self.max_block_bytes:
            self.misses += 1
            return None
        lib = _lib.load()
        evict = None
        with self._lock:
            if self._closed:
                return None
            fits = [b for b in self._free if b[0] >= n]
            if fits:
                cap, addr = min(fits)
                self._free.remove((cap, addr))
            else:
                if self._n >= self.max_blocks and self._free:  # every idle block too small: replace one
                    evict = min(self._free)
                    self._free.remove(evict)
                    self._n -= 1
                if self._n >= self.max_blocks:
                    self.misses += 1
                    return None
                self._n += 1  # reserved; allocated below, outside the lock
                cap, addr = (n + _BLOCK_ALIGN - 1) // _BLOCK_ALIGN * _BLOCK_ALIGN, None
        if evict is not None:
            lib.pgh_host_free(C.c_void_p(evict[1]))  # waits for a DMA still reading it
        if addr is None:
            p = C.c_void_p()
            if lib.pgh_host_alloc(cap, C.byref(p)) != 0:
                with self._lock:
                    self._n -= 1
                    self.misses += 1
                return None
            addr = p.value
            # an ingest from the block returns with its DMA queued, not done (pgh_host_async) ...
            lib.pgh_host_async(C.c_void_p(addr), cap, 1)
        else:
            # ... so a returned block is written again only after that DMA has read it
            lib.pgh_host_wait(C.c_void_p(addr), cap)
        with self._lock:
            self.hits += 1
        arr = (C.c_uint8 * n).from_address(addr)
        arr._pgh_block = _Return(self, addr, cap)  # lives as long as any view of arr
        return arr, addr

    def _give(self, addr: int, cap: int):
        with self._lock:
            if self._closed:
                _lib.load().pgh_host_free(C.c_void_p(addr))
                self._n -= 1
                return
            self._free.append((cap, addr))

    @property
    def blocks(self) -> int:
        return self._n

    def close(self):
        """Free the idle blocks now; blocks still referenced are freed when they come back."""
        with self._lock:
            self._closed = True
            free, self._free = self._free, []
            self._n -= len(free)
        for _, addr in free:
            _lib.load().pgh_host_free(C.c_void_p(addr))


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


def _out(n: int, into: Optional[PinnedPool]):
    """(object to return, its writable address) for n decoded bytes."""
    if into is not None and n:
        got = into.acquire(n)
        if got is not None:
            arr, addr = got
            return arr, addr
    return _lib.fresh_bytes(n)


def _result(out):
    return out if isinstance(out, bytes) else memoryview(out).cast("B").toreadonly()


def b64decode(s, threads: int = 0, into: Optional[PinnedPool] = None):
    """``base64.b64decode(s)``.  Returns ``bytes``, or -- with ``into`` -- a read-only memoryview
    over a page-locked block of that pool (``bytes`` when the pool has no block to give)."""
    keep, src, length = _text(s)  # `keep` holds the text's buffer alive for the calls below
    lib = _lib.load()
    n = C.c_size_t(0)
    # one pass for a clean string: allocate the size its tail implies, decode (which checks the rest)
    if length >= (1 << 16) and lib.pgh_b64_clean_size(src, length, C.byref(n)) == 0:
        out, dst = _out(n.value, into)
        rc = lib.pgh_b64_decode_clean(src, length, dst, n.value, C.byref(n), int(threads))
        if rc == 0:
            return _result(out)
        if rc == -5:
            raise binascii.Error("Incorrect padding")
        # PGH_E_STATE: not clean (junk, line breaks): the general route
        del out
    if lib.pgh_b64_decode(src, length, None, C.byref(n), int(threads)) != 0:  # validate + exact size
        raise binascii.Error("Incorrect padding")
    out, dst = _out(n.value, into)  # fresh, unshared: decoded into in place
    if n.value:
        if lib.pgh_b64_decode(src, length, dst, C.byref(n), int(threads)) != 0:
            raise binascii.Error("Incorrect padding")
    del keep
    return _result(out)
