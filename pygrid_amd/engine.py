"""Python handle on one libpygrid_hip context (one GPU, one parameter shard).

This is plumbing over the C ABI: every computation happens in the HIP kernels of
``pygrid_amd/csrc``.  There is deliberately no CPU implementation here -- an Engine cannot be
constructed without the library and a visible GPU (``EngineUnavailableError``).
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .exceptions import AggregationError, EngineUnavailableError, StateParseError

MEAN, ITERATIVE_MEAN, WEIGHTED_MEAN = 0, 1, 2
STREAM_SECAGG = 16
DEFAULT_VARIANT = -1  # PGH_DEFAULT_VARIANT: auto by shard size
F32, I64 = 0, 1
MODE_NAMES = {MEAN: "mean", ITERATIVE_MEAN: "iterative_mean", WEIGHTED_MEAN: "weighted_mean"}


def device_count() -> int:
    lib = _lib.load()
    n = C.c_int(0)
    if lib.pgh_device_count(C.byref(n)) != 0:
        return 0
    return n.value


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class PinnedBuffer:
    """Page-locked host memory (pgh_host_alloc) viewed as a numpy array; ingest DMAs it directly."""

    def __init__(self, shape, dtype=np.float32):
        self._lib = _lib.load()
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = C.c_void_p()
        if self._lib.pgh_host_alloc(n, C.byref(p)) != 0:
            raise AggregationError(self._lib.pgh_last_error(None).decode())
        self._p = p
        buf = (C.c_uint8 * n).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dtype).reshape(shape)

    def free(self):
        if getattr(self, "_p", None):
            self.array = None
            self._lib.pgh_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class _Serialized:
    """The library with every call made under one lock: a context is single-owner, and ctypes
    releases the GIL, so two Python threads sharing an Engine would otherwise enter it together.
    A failing call's message (``pgh_last_error``, one per context) is read under the same lock
    and kept per thread, so another thread's call cannot overwrite it before ``_check`` sees it."""

    def __init__(self, lib, lock):
        self._l, self._m = lib, lock
        self.errors = threading.local()

    def __getattr__(self, name):
        fn = getattr(self._l, name)

        def call(*args):
            with self._m:
                rc = fn(*args)
                if isinstance(rc, int) and rc < 0:
                    ctx = args[0] if args and isinstance(args[0], C.c_void_p) else None
                    self.errors.msg = self._l.pgh_last_error(ctx).decode(errors="replace")
                return rc
        return call


class Engine:
    """One libpygrid_hip context: one GPU (``device``), or several GPUs of this node driven from
    this process (``devices=[0, 1, ...]``: ``pgh_create_group``, parameter shards across the GPUs,
    bit-identical results, one host thread per GPU inside the library)."""

    def __init__(self, device: int = 0, pinned_bytes: int = 0, devices: Optional[Sequence[int]] = None,
                 _borrowed=None):
        self._lib = _Serialized(_lib.load(), threading.RLock()) if _borrowed is None else _borrowed[1]
        self._owned = _borrowed is None
        if _borrowed is not None:
            h = _borrowed[0]
            devs = [int(device)]
        elif devices is not None:
            devs = [int(d) for d in devices]
            if not devs:
                raise EngineUnavailableError("a group needs at least one device")
            h = C.c_void_p()
            arr = (C.c_int * len(devs))(*devs)
            rc = self._lib.pgh_create_group(len(devs), arr, int(pinned_bytes), C.byref(h))
            if rc != 0:
                msg = getattr(self._lib.errors, "msg", "")
                raise EngineUnavailableError(f"pgh_create_group(devices={devs}) failed: {msg}")
        else:
            devs = [int(device)]
            h = C.c_void_p()
            rc = self._lib.pgh_create(int(device), int(pinned_bytes), C.byref(h))
            if rc != 0:
                msg = getattr(self._lib.errors, "msg", "")
                raise EngineUnavailableError(f"pgh_create(device={device}) failed: {msg}")
        self._h = h
        self.devices = devs
        self.device = devs[0]
        self.numel: Tuple[int, ...] = ()
        self.P = 0
        self.lo = 0
        self.hi = 0
        self.dtype = F32
        self.parties = 1
        self.max_clients = 0
        # Who put the current resident checkpoint in HBM (CycleAggregator / IncrementalCycle): any
        # call that overwrites it resets this, so a holder re-uploads instead of trusting stale bytes.
        self.ckpt_owner = None
        # The bytes object the resident checkpoint was produced as (valid while ckpt_owner is set):
        # the next cycle, handed those very bytes, skips the upload.
        self.ckpt_bytes = None

    # ---- plumbing ----------------------------------------------------------------------------
    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = getattr(self._lib.errors, "msg", "")
            cls = StateParseError if rc == -5 else AggregationError
            raise cls(f"{what}: {_lib.STATUS_NAMES.get(rc, rc)}: {msg}", status=rc)

    def close(self):
        if getattr(self, "_h", None):
            if getattr(self, "_owned", True):
                self._lib.pgh_destroy(self._h)
            self._h = None

    # ---- multi-GPU group ----------------------------------------------------------------------
    @property
    def n_gpus(self) -> int:
        n = C.c_int(0)
        self._check(self._lib.pgh_group_size(self._h, C.byref(n)), "group_size")
        return n.value

    def child(self, i: int) -> "Engine":
        """GPU i's context of a group (borrowed: valid while this engine lives), for the entry points
        that take device pointers.  A single-GPU engine is its own child 0."""
        k = C.c_void_p()
        self._check(self._lib.pgh_group_child(self._h, int(i), C.byref(k)), "group_child")
        e = Engine(self.devices[i] if i < len(self.devices) else self.device, _borrowed=(k, self._lib))
        e.numel, e.P = self.numel, self.P
        return e

    def set_client_sharding(self, on: bool = True):
        """Group + int64 shares: split the CLIENTS across the GPUs (ncclReduceScatter of the sums)."""
        self._check(self._lib.pgh_set_client_sharding(self._h, 1 if on else 0), "set_client_sharding")

    def allgather_resident(self):
        """All-gather the resident checkpoint into a full copy on every GPU; returns the device
        pointers (GPU g holds shard r at [r * S, r * S + len_r))."""
        ptrs = (C.c_void_p * len(self.devices))()
        self._check(self._lib.pgh_group_allgather_resident(self._h, ptrs), "allgather_resident")
        return [p or 0 for p in ptrs]

    def group_backend(self) -> int:
        """1: RCCL, 0: peer copies, -1: no collective yet (or a single GPU)."""
        b = C.c_int(-1)
        self._check(self._lib.pgh_group_backend(self._h, C.byref(b)), "group_backend")
        return b.value

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- layout --------------------------------------------------------------------------------
    @property
    def p_shard(self) -> int:
        return self.hi - self.lo

    def set_layout(self, numel: Sequence[int]):
        arr = (C.c_int64 * len(numel))(*[int(n) for n in numel])
        self._check(self._lib.pgh_set_layout(self._h, len(numel), arr), "set_layout")
        self.numel = tuple(int(n) for n in numel)
        self.P = sum(self.numel)
        self.lo, self.hi = 0, self.P
        self.max_clients = 0  # the slab was freed
        self.ckpt_owner = None

    def set_shard(self, lo: int, hi: int):
        self._check(self._lib.pgh_set_shard(self._h, int(lo), int(hi)), "set_shard")
        self.lo, self.hi = int(lo), int(hi)
        self.max_clients = 0
        self.ckpt_owner = None

    def reserve(self, max_clients: int, dtype: int = F32, n_parties: int = 1):
        self._check(self._lib.pgh_reserve(self._h, int(max_clients), int(dtype), int(n_parties)), "reserve")
        self.dtype = dtype
        self.parties = 1 if dtype == F32 else int(n_parties)
        self.max_clients = int(max_clients)
        self.ckpt_owner = None

    def reset(self):
        self._check(self._lib.pgh_reset(self._h), "reset")

    # ---- ingest --------------------------------------------------------------------------------
    def ingest(self, client: int, flat: np.ndarray):
        """Client diff: float32 [P] (dtype F32) or int64 [parties][P] shares (dtype I64)."""
        if self.dtype == F32:
            a = np.ascontiguousarray(flat, dtype=np.float32).reshape(-1)
        else:
            a = np.ascontiguousarray(flat, dtype=np.int64).reshape(-1)
        self._check(self._lib.pgh_ingest_raw(self._h, int(client), _ptr(a), a.nbytes, self.dtype),
                    f"ingest client {client}")

    def ingest_state(self, client: int, pb):
        """``pb``: State bytes, or any buffer over them (a page-locked report buffer is DMA'd as it
        lies: ``report.PinnedPool``)."""
        keep, arg = _lib.buf_arg(pb)
        self._check(self._lib.pgh_ingest_state(self._h, int(client), arg, len(keep)),
                    f"ingest_state client {client}")

    def ingest_state_shares(self, client: int, messages: Sequence[bytes]):
        """One client's secure-aggregation shares, one State message per party (packed-varint
        int64 payloads, decoded on the GPU; ``pgh_ingest_state_shares``)."""
        n = len(messages)
        ptrs = (C.c_char_p * max(n, 1))(*messages)
        lens = (C.c_size_t * max(n, 1))(*[len(m) for m in messages])
        self._check(self._lib.pgh_ingest_state_shares(self._h, int(client), n, ptrs, lens),
                    f"ingest_state_shares client {client}")

    def set_synth_kind(self, kind: int):
        """0: Irwin-Hall(4 x u16) per param (default); 1: fast, one hash word per 4 params."""
        self._check(self._lib.pgh_set_synth_kind(self._h, int(kind)), "set_synth_kind")

    def synth_fill(self, seed: int, n_clients: int):
        self._check(self._lib.pgh_synth_fill(self._h, C.c_uint64(seed), int(n_clients)), "synth_fill")

    def synth_ingest(self, seed: int, client0: int, n: int):
        self._check(self._lib.pgh_synth_ingest(self._h, C.c_uint64(seed), int(client0), int(n)), "synth_ingest")

    def set_weights(self, w: Sequence[float]):
        a = np.ascontiguousarray(w, dtype=np.float32)
        self._check(self._lib.pgh_set_weights(self._h, a.ctypes.data_as(C.POINTER(C.c_float)), a.size),
                    "set_weights")

    # ---- reduction -----------------------------------------------------------------------------
    def fedavg(self, mode: int, ckpt: np.ndarray) -> np.ndarray:
        """``ckpt - avg(diffs)`` over this shard (host arrays of p_shard floats)."""
        c = np.ascontiguousarray(ckpt, dtype=np.float32).reshape(-1)
        if c.size != self.p_shard:
            raise AggregationError(f"checkpoint has {c.size} params, shard has {self.p_shard}")
        out = np.empty_like(c)
        self.ckpt_owner = None  # the host checkpoint is staged through the resident one
        self._check(self._lib.pgh_fedavg(self._h, int(mode), _ptr(c), _ptr(out)), "fedavg")
        return out

    def fedavg_device(self, mode: int, d_ckpt: int, d_out: int, stream: int = 0):
        self._check(self._lib.pgh_fedavg_device(self._h, int(mode), C.c_void_p(d_ckpt), C.c_void_p(d_out),
                                                C.c_void_p(stream or None)), "fedavg_device")

    def fedavg_device_range(self, mode: int, off: int, length: int, d_ckpt: int, d_out: int, stream: int = 0):
        """Fold only the shard-relative param range [off, off + length) (off % 4 == 0)."""
        self._check(self._lib.pgh_fedavg_device_range(self._h, int(mode), int(off), int(length), C.c_void_p(d_ckpt),
                                                      C.c_void_p(d_out), C.c_void_p(stream or None)),
                    "fedavg_device_range")

    # ---- resident checkpoint ---------------------------------------------------------------------
    def ckpt_upload(self, ckpt: np.ndarray):
        a = np.ascontiguousarray(ckpt, dtype=np.float32).reshape(-1)
        self.ckpt_owner = None
        self._check(self._lib.pgh_ckpt_upload(self._h, _ptr(a), a.nbytes), "ckpt_upload")

    def ckpt_upload_state(self, pb):
        self.ckpt_owner = None
        keep, arg = _lib.buf_arg(pb)
        self._check(self._lib.pgh_ckpt_upload_state(self._h, arg, len(keep)), "ckpt_upload_state")

    def fedavg_resident(self, mode: int):
        """Fold into the resident checkpoint: afterwards it IS the new checkpoint."""
        self._check(self._lib.pgh_fedavg_resident(self._h, int(mode)), "fedavg_resident")

    def fold_slots(self, mode: int, slots: Sequence[int]):
        """Fold the diffs in ``slots`` (in this order) into the running state; frees the slots."""
        a = np.ascontiguousarray(slots, dtype=np.int32)
        self._check(self._lib.pgh_fold_slots(self._h, int(mode), a.ctypes.data_as(C.POINTER(C.c_int32)), a.size),
                    "fold_slots")

    def fold_slots_finish_resident(self, mode: int, slots: Sequence[int] = ()):
        """Fold ``slots`` and finish into the resident checkpoint (it IS the new checkpoint then)."""
        a = np.ascontiguousarray(slots, dtype=np.int32)
        self._check(self._lib.pgh_fold_slots_finish_resident(self._h, int(mode),
                                                             a.ctypes.data_as(C.POINTER(C.c_int32)), a.size),
                    "fold_slots_finish_resident")

    def fold_restart(self):
        """Forget the slot folds of this cycle so far (``pgh_fold_slots_restart``); unfolded slots
        keep their diffs, weights must be set again."""
        self._check(self._lib.pgh_fold_slots_restart(self._h), "fold_slots_restart")

    def ckpt_download(self) -> np.ndarray:
        out = np.empty(self.p_shard, dtype=np.float32)
        self._check(self._lib.pgh_ckpt_download(self._h, _ptr(out)), "ckpt_download")
        return out

    def ckpt_patch_state(self, template: bytes) -> bytes:
        """``template`` (State bytes) with this shard's payload slices taken from the resident checkpoint."""
        out, ptr = _lib.fresh_bytes(len(template))  # the library copies the template in, then patches
        self._check(self._lib.pgh_ckpt_patch_state(self._h, template, len(template), ptr), "ckpt_patch_state")
        return out

    def ckpt_patch_into(self, ptr: int, n: int):
        """Patch in place: the n bytes at host address ``ptr`` hold a State whose framing is final;
        its payload slices are written from the resident checkpoint (``state.fresh_checkpoint``)."""
        self._check(self._lib.pgh_ckpt_patch_state(self._h, C.c_char_p(ptr), n, C.c_void_p(ptr)),
                    "ckpt_patch_state (in place)")

    def secagg(self, base: int = 10, prec: int = 3, want_sum: bool = True, want_dec: bool = True,
               out_sum: Optional[np.ndarray] = None,
               out_dec: Optional[np.ndarray] = None) -> Tuple[Optional[np.ndarray], Optional[np.ndarray]]:
        """Z_2^64 share sum + decode into host arrays (fresh ones, or ``out_sum`` / ``out_dec``, e.g.
        page-locked PinnedBuffer arrays that the result is DMA'd into directly)."""
        s = out_sum if out_sum is not None else (np.empty(self.p_shard, dtype=np.int64) if want_sum else None)
        d = out_dec if out_dec is not None else (np.empty(self.p_shard, dtype=np.float32) if want_dec else None)
        for a, dt in ((s, np.int64), (d, np.float32)):
            if a is not None and (a.dtype != dt or a.size != self.p_shard or not a.flags.c_contiguous):
                raise AggregationError(f"secagg output must be a contiguous {np.dtype(dt).name}[{self.p_shard}]")
        self._check(self._lib.pgh_secagg(self._h, int(base), int(prec), _ptr(s) if s is not None else None,
                                         _ptr(d) if d is not None else None), "secagg")
        return s, d

    def secagg_device(self, d_sum: int, d_dec: int, base: int = 10, prec: int = 3, stream: int = 0):
        self._check(self._lib.pgh_secagg_device(self._h, int(base), int(prec), C.c_void_p(d_sum or None),
                                                C.c_void_p(d_dec or None), C.c_void_p(stream or None)),
                    "secagg_device")

    def secagg_device_range(self, off: int, length: int, d_sum: int, d_dec: int, base: int = 10, prec: int = 3,
                            stream: int = 0):
        """Share sum + decode of the shard-relative param range [off, off + length) (off % 4 == 0)."""
        self._check(self._lib.pgh_secagg_device_range(self._h, int(base), int(prec), int(off), int(length),
                                                      C.c_void_p(d_sum or None), C.c_void_p(d_dec or None),
                                                      C.c_void_p(stream or None)), "secagg_device_range")

    def secagg_decode_device(self, d_sum: int, n: int, d_dec: int, base: int = 10, prec: int = 3, stream: int = 0):
        """d_dec[:n] = float32(int64 d_sum[:n]) / base**prec (client-sharded secagg, after the
        cross-rank reduce-scatter of the share sums)."""
        self._check(self._lib.pgh_secagg_decode_device(self._h, int(base), int(prec), C.c_void_p(d_sum or None),
                                                       int(n), C.c_void_p(d_dec or None),
                                                       C.c_void_p(stream or None)), "secagg_decode_device")

    def synth_ckpt_device(self, seed: int, d_ckpt: int, stream: int = 0):
        self.ckpt_owner = None  # may stage through the resident checkpoint
        self._check(self._lib.pgh_synth_ckpt_device(self._h, C.c_uint64(seed), C.c_void_p(d_ckpt),
                                                    C.c_void_p(stream or None)), "synth_ckpt_device")

    # ---- stream use: fold clients in order as they arrive -----------------------------------------
    def stream_begin(self, kind: int, fold_batch: int = 0):
        self._check(self._lib.pgh_stream_begin(self._h, int(kind), int(fold_batch)), "stream_begin")

    def stream_flush(self):
        self._check(self._lib.pgh_stream_flush(self._h), "stream_flush")

    def stream_finish(self, ckpt: np.ndarray) -> np.ndarray:
        c = np.ascontiguousarray(ckpt, dtype=np.float32).reshape(-1)
        if c.size != self.p_shard:
            raise AggregationError(f"checkpoint has {c.size} params, shard has {self.p_shard}")
        out = np.empty_like(c)
        self.ckpt_owner = None
        self._check(self._lib.pgh_stream_finish(self._h, _ptr(c), _ptr(out)), "stream_finish")
        return out

    def stream_finish_device(self, d_ckpt: int, d_out: int, stream: int = 0):
        self._check(self._lib.pgh_stream_finish_device(self._h, C.c_void_p(d_ckpt), C.c_void_p(d_out),
                                                       C.c_void_p(stream or None)), "stream_finish_device")

    def stream_finish_resident(self):
        """Finish the stream into the resident checkpoint (``ckpt_upload*`` earlier, possibly while
        clients were still arriving): afterwards it IS the new checkpoint."""
        self._check(self._lib.pgh_stream_finish_resident(self._h), "stream_finish_resident")

    def stream_finish_secagg(self, base: int = 10, prec: int = 3):
        s = np.empty(self.p_shard, dtype=np.int64)
        d = np.empty(self.p_shard, dtype=np.float32)
        self._check(self._lib.pgh_stream_finish_secagg(self._h, int(base), int(prec), _ptr(s), _ptr(d)),
                    "stream_finish_secagg")
        return s, d

    def stream_finish_secagg_device(self, d_sum: int, d_dec: int, base: int = 10, prec: int = 3, stream: int = 0):
        self._check(self._lib.pgh_stream_finish_secagg_device(
            self._h, int(base), int(prec), C.c_void_p(d_sum or None), C.c_void_p(d_dec or None),
            C.c_void_p(stream or None)), "stream_finish_secagg_device")

    def sync(self):
        self._check(self._lib.pgh_sync(self._h), "sync")

    # ---- observability -------------------------------------------------------------------------
    def set_ingest_ranges(self, on: bool):
        """Report-time ingest (pgh_set_ingest_ranges): each State diff goes to HBM in param ranges
        with an event each, so the close's fold starts on the last report's ranges as they land."""
        self._check(self._lib.pgh_set_ingest_ranges(self._h, int(bool(on))), "set_ingest_ranges")

    def set_variant(self, v: int):
        """Kernel variant (csrc/pgh_kernels.hip table); -1 restores the default."""
        self._check(self._lib.pgh_set_variant(self._h, int(v)), "set_variant")

    def effective_variant(self, mode: int = MEAN) -> int:
        """Kernel variant the next fold runs for ``mode`` (MEAN / ITERATIVE_MEAN / WEIGHTED_MEAN /
        STREAM_SECAGG)."""
        v = self._lib.pgh_effective_variant(self._h, int(mode))
        self._check(min(v, 0), "effective_variant")
        return v

    def stats(self) -> dict:
        st = _lib.Stats()
        self._check(self._lib.pgh_stats(self._h, C.byref(st)), "stats")
        return {name: getattr(st, name) for name, _ in _lib.Stats._fields_}

    def reset_stats(self):
        self._check(self._lib.pgh_reset_stats(self._h), "reset_stats")

    def slab(self) -> Tuple[int, int, int]:
        """(device pointer, ld, block_pitch): element (row r, shard param i) is at
        ``(i // ld) * block_pitch + r * ld + i % ld`` (include/pgh_api.h)."""
        p = C.c_void_p()
        ld = C.c_int64()
        bp = C.c_int64()
        self._check(self._lib.pgh_slab(self._h, C.byref(p), C.byref(ld), C.byref(bp)), "slab")
        return p.value or 0, ld.value, bp.value
