"""syft State codec, host side: the replacement for ``ModelManager.serialize_model_params`` /
``unserialize_model_params`` (``apps/node/src/app/main/model_centric/models/model_manager.py:79-103``)
on the cycle-close path.

The byte work is done in C++ (``pgh_state_scan`` / ``pgh_state_patch`` in libpygrid_hip):

* unserialize = locate each tensor's packed float32 payload and view it (no per-element
  Python work, unlike syft's ``_unbufferize``);
* serialize of the new checkpoint = a FRESH State, framed like ``serialize_model_params``
  (``model_manager.py:82-90``: new placeholder and tensor ids from syft's id space, plain
  ``torch_tensor`` entries, no tags), its float payloads written straight from HBM
  (``fresh_checkpoint``); or, on request, the current checkpoint's bytes with every payload
  overwritten (``serialize_model_params`` below / ``pgh_ckpt_patch_state``: ids and tags kept).

Schema: build-owned restatement of syft-proto 0.5.2 (``state_schema.py``); parity unpinned
until checked against real client bytes (DESIGN.md "State codec").
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from .exceptions import StateParseError


def scan(pb: bytes) -> List[Tuple[int, int]]:
    """(byte offset, float count) of every tensor payload, in State order."""
    lib = _lib.load()
    n = C.c_int(0)
    keep, arg = _lib.buf_arg(pb)
    rc = lib.pgh_state_scan(arg, len(keep), 0, None, None, C.byref(n))
    if rc != 0:
        raise StateParseError(f"malformed State message ({_lib.STATUS_NAMES.get(rc, rc)})", status=rc)
    k = n.value
    offs = (C.c_int64 * max(k, 1))()
    cnts = (C.c_int64 * max(k, 1))()
    rc = lib.pgh_state_scan(arg, len(keep), k, offs, cnts, C.byref(n))
    if rc != 0:
        raise StateParseError("malformed State message", status=rc)
    return [(offs[i], cnts[i]) for i in range(k)]


def scan_shares(pb: bytes) -> List[Tuple[int, int, int]]:
    """(payload byte offset, payload bytes, int64 value count) of every tensor of a secure-
    aggregation share State (packed-varint contents_int64), validated like protobuf's parser."""
    lib = _lib.load()
    n = C.c_int(0)
    rc = lib.pgh_state_scan_i64(pb, len(pb), 0, None, None, None, C.byref(n))
    if rc != 0:
        raise StateParseError(f"malformed share State message ({_lib.STATUS_NAMES.get(rc, rc)})", status=rc)
    k = n.value
    offs, nbs, cnts = ((C.c_int64 * max(k, 1))() for _ in range(3))
    rc = lib.pgh_state_scan_i64(pb, len(pb), k, offs, nbs, cnts, C.byref(n))
    if rc != 0:
        raise StateParseError("malformed share State message", status=rc)
    return [(offs[i], nbs[i], cnts[i]) for i in range(k)]


def tensor_numels(pb: bytes) -> List[int]:
    return [c for _, c in scan(pb)]


def unserialize_model_params(pb: bytes, shapes: Sequence[Sequence[int]] = None) -> List[np.ndarray]:
    """float32 copies of every tensor, flat (or reshaped to ``shapes``)."""
    buf = np.frombuffer(pb, dtype=np.uint8)
    out = []
    for t, (off, cnt) in enumerate(scan(pb)):
        a = buf[off:off + 4 * cnt].view("<f4").astype(np.float32)
        out.append(a.reshape(shapes[t]) if shapes is not None else a)
    return out


def flat_params(pb: bytes) -> np.ndarray:
    parts = unserialize_model_params(pb)
    return np.concatenate(parts) if parts else np.empty(0, np.float32)


def serialize_model_params(template: bytes, values: np.ndarray) -> bytes:
    """New State bytes: ``template`` with all payloads replaced by ``values`` (P floats)."""
    lib = _lib.load()
    v = np.ascontiguousarray(values, dtype="<f4").reshape(-1)
    out, ptr = _lib.fresh_bytes(len(template))  # pgh_state_patch writes all n bytes (copy + patch)
    rc = lib.pgh_state_patch(template, len(template), v.ctypes.data, v.size, ptr)
    if rc != 0:
        raise StateParseError(f"cannot patch State ({_lib.STATUS_NAMES.get(rc, rc)}): "
                              f"{v.size} values for this checkpoint?", status=rc)
    return out


def fresh_frame_bytes(template: bytes, ids=None):
    """(uninitialised-payload bytes of the fresh checkpoint framed by ``pgh_state_fresh``, its host
    address).  ``ids``: 2 per tensor (placeholder, tensor), syft's id space by default."""
    from . import state_schema

    lib = _lib.load()
    n = C.c_int(0)
    rc = lib.pgh_state_scan(template, len(template), 0, None, None, C.byref(n))
    if rc != 0:
        raise StateParseError(f"malformed checkpoint State ({_lib.STATUS_NAMES.get(rc, rc)})", status=rc)
    ids = list(ids) if ids is not None else state_schema.syft_ids(2 * n.value)
    arr = (C.c_int64 * max(len(ids), 1))(*ids)
    need = C.c_size_t(0)
    rc = lib.pgh_state_fresh(template, len(template), arr, len(ids), None, 0, C.byref(need))
    if rc != 0:
        raise StateParseError(f"cannot frame a fresh checkpoint ({_lib.STATUS_NAMES.get(rc, rc)})", status=rc)
    out, ptr = _lib.fresh_bytes(need.value)
    rc = lib.pgh_state_fresh(template, len(template), arr, len(ids), ptr, need.value, C.byref(need))
    if rc != 0:
        raise StateParseError(f"cannot frame a fresh checkpoint ({_lib.STATUS_NAMES.get(rc, rc)})", status=rc)
    return out, ptr


def prefault(frame):
    """Fault in the pages of a ``fresh_frame_bytes`` result (``pgh_host_prefault``)."""
    out, ptr = frame
    if ptr:
        _lib.load().pgh_host_prefault(C.c_void_p(ptr), len(out))


def prepared_fresh_frame(template: bytes, ids=None):
    """``fresh_frame_bytes`` with the payload pages already faulted in (``pgh_host_prefault``): made
    while a cycle is still open, so the close copies the new checkpoint into resident pages instead
    of faulting ~11 K of them in while the D2H waits."""
    frame = fresh_frame_bytes(template, ids)
    prefault(frame)
    return frame


def fresh_checkpoint(engine, template: bytes, ids=None, prepared=None) -> bytes:
    """The new checkpoint as ``serialize_model_params`` emits it (model_manager.py:79-92): a fresh
    State whose framing ``pgh_state_fresh`` builds from the template's tensor shapes and fresh ids
    (restated in ``state_schema.fresh_frame``) and whose payloads the engine writes in place from
    the resident checkpoint in HBM (``pgh_ckpt_patch_state`` with out == tmpl).  ``prepared``: a
    ``prepared_fresh_frame(template)`` not handed out yet."""
    out, ptr = prepared if prepared is not None else fresh_frame_bytes(template, ids)
    engine.ckpt_patch_into(ptr, len(out))
    return out


def serialize_fresh(shapes, values: np.ndarray, ids=None) -> bytes:
    """Host-only fresh State of float32 ``values`` (P floats) with ``shapes`` (no GPU involved)."""
    from . import state_schema

    v = np.ascontiguousarray(values, dtype="<f4").reshape(-1)
    ids = list(ids) if ids is not None else state_schema.syft_ids(2 * len(shapes))
    total, pieces, spans = state_schema.fresh_frame(shapes, ids)
    buf = bytearray(total)
    for off, b in pieces:
        buf[off:off + len(b)] = b
    at = 0
    for off, n in spans:
        buf[off:off + n] = v[at:at + n // 4].tobytes()
        at += n // 4
    if at != v.size:
        raise StateParseError(f"{v.size} values for tensors of {at} floats")
    return bytes(buf)
