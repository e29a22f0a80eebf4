"""ctypes binding of libpygrid_hip.so (the C ABI of ``include/pgh_api.h``).

``ctypes.CDLL`` releases the GIL around every call, so a cycle close on the node's
Flask-Executor thread (``apps/node/src/app/__init__.py:29,197-199``) does not block the
request threads.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

from .exceptions import EngineUnavailableError

LIB_PATH = Path(__file__).resolve().with_name("libpygrid_hip.so")

PGH_OK = 0
STATUS_NAMES = {-1: "PGH_E_ARG", -2: "PGH_E_HIP", -3: "PGH_E_STATE", -4: "PGH_E_OOM",
                -5: "PGH_E_PARSE", -6: "PGH_E_UNSUPPORTED"}


class Stats(C.Structure):
    _fields_ = [
        ("kernel_ms_last", C.c_double),
        ("kernel_ms_total", C.c_double),
        ("kernel_launches", C.c_uint64),
        ("kernel_bytes_last", C.c_uint64),
        ("kernel_bytes_total", C.c_uint64),
        ("h2d_ms_total", C.c_double),
        ("h2d_bytes_total", C.c_uint64),
        ("close_ms_last", C.c_double),
        ("p_shard", C.c_int64),
        ("ld", C.c_int64),
        ("n_folded", C.c_int64),
        ("n_clients", C.c_int32),
        ("max_clients", C.c_int32),
        ("kernel_busy_ms_total", C.c_double),
        ("h2d_staged_bytes_total", C.c_uint64),
        ("d2h_bytes_total", C.c_uint64),
        ("d2h_kernel_bytes_total", C.c_uint64),
    ]


_new_bytes = C.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = C.py_object
_new_bytes.argtypes = [C.c_void_p, C.c_ssize_t]


def buf_arg(pb):
    """(keep-alive, argument) for a ``void*`` State parameter: a ``bytes`` object is passed as is;
    any other buffer (memoryview, bytearray, numpy) by the address of its first byte -- the
    keep-alive holds the exporting view for the duration of the call."""
    if isinstance(pb, bytes):
        return pb, pb
    import numpy as np

    a = np.frombuffer(pb, dtype=np.uint8)
    return a, (a.ctypes.data if a.size else None)


def fresh_bytes(n: int):
    """A new, unshared, UNINITIALISED ``bytes`` object of n bytes and the address of its buffer, for
    the library to write into (no zero-fill and no ``.raw`` copy: a 47 MB checkpoint saves two
    full passes).  The caller must overwrite all n bytes before the object escapes."""
    b = _new_bytes(None, n)
    return b, (C.cast(C.c_char_p(b), C.c_void_p).value if n else None)


_vp, _i, _i64, _u64, _sz = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_size_t
_P64 = C.POINTER(C.c_int64)

# name -> (restype, argtypes); every entry point declared in include/pgh_api.h
SIGNATURES = {
    "pgh_abi_version": (_i, []),
    "pgh_device_count": (_i, [C.POINTER(C.c_int)]),
    "pgh_create": (_i, [_i, _sz, C.POINTER(_vp)]),
    "pgh_destroy": (None, [_vp]),
    "pgh_create_group": (_i, [_i, C.POINTER(C.c_int), _sz, C.POINTER(_vp)]),
    "pgh_group_size": (_i, [_vp, C.POINTER(C.c_int)]),
    "pgh_group_child": (_i, [_vp, _i, C.POINTER(_vp)]),
    "pgh_set_client_sharding": (_i, [_vp, _i]),
    "pgh_group_allgather_resident": (_i, [_vp, C.POINTER(_vp)]),
    "pgh_group_backend": (_i, [_vp, C.POINTER(C.c_int)]),
    "pgh_last_error": (C.c_char_p, [_vp]),
    "pgh_host_alloc": (_i, [_sz, C.POINTER(_vp)]),
    "pgh_host_free": (_i, [_vp]),
    "pgh_host_prefault": (_i, [_vp, _sz]),
    "pgh_host_async": (_i, [_vp, _sz, _i]),
    "pgh_host_wait": (_i, [_vp, _sz]),
    "pgh_set_layout": (_i, [_vp, _i, _P64]),
    "pgh_set_shard": (_i, [_vp, _i64, _i64]),
    "pgh_reserve": (_i, [_vp, _i, _i, _i]),
    "pgh_reset": (_i, [_vp]),
    "pgh_ingest_raw": (_i, [_vp, _i, _vp, _sz, _i]),
    # State bytes: a bytes object, or the address of any buffer (buf_arg: memoryviews of page-locked
    # report buffers, pygrid_amd.report.PinnedPool)
    "pgh_ingest_state": (_i, [_vp, _i, _vp, _sz]),
    "pgh_set_synth_kind": (_i, [_vp, _i]),
    "pgh_set_ingest_ranges": (_i, [_vp, _i]),
    "pgh_ingest_state_shares": (_i, [_vp, _i, _i, C.POINTER(C.c_char_p), C.POINTER(_sz)]),
    "pgh_synth_fill": (_i, [_vp, _u64, _i]),
    "pgh_synth_ingest": (_i, [_vp, _u64, _i, _i]),
    "pgh_set_weights": (_i, [_vp, C.POINTER(C.c_float), _i]),
    "pgh_fedavg": (_i, [_vp, _i, _vp, _vp]),
    "pgh_fedavg_device": (_i, [_vp, _i, _vp, _vp, _vp]),
    "pgh_fedavg_device_range": (_i, [_vp, _i, _i64, _i64, _vp, _vp, _vp]),
    "pgh_ckpt_upload": (_i, [_vp, _vp, _sz]),
    "pgh_ckpt_upload_state": (_i, [_vp, _vp, _sz]),
    "pgh_fedavg_resident": (_i, [_vp, _i]),
    "pgh_fold_slots": (_i, [_vp, _i, C.POINTER(C.c_int32), _i]),
    "pgh_fold_slots_finish_resident": (_i, [_vp, _i, C.POINTER(C.c_int32), _i]),
    "pgh_fold_slots_restart": (_i, [_vp]),
    "pgh_ckpt_download": (_i, [_vp, _vp]),
    "pgh_ckpt_patch_state": (_i, [_vp, C.c_char_p, _sz, _vp]),
    "pgh_secagg": (_i, [_vp, _i, _i, _vp, _vp]),
    "pgh_secagg_device": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "pgh_secagg_device_range": (_i, [_vp, _i, _i, _i64, _i64, _vp, _vp, _vp]),
    "pgh_secagg_decode_device": (_i, [_vp, _i, _i, _vp, _i64, _vp, _vp]),
    "pgh_synth_ckpt_device": (_i, [_vp, _u64, _vp, _vp]),
    "pgh_stream_begin": (_i, [_vp, _i, _i]),
    "pgh_stream_flush": (_i, [_vp]),
    "pgh_stream_finish": (_i, [_vp, _vp, _vp]),
    "pgh_stream_finish_device": (_i, [_vp, _vp, _vp, _vp]),
    "pgh_stream_finish_resident": (_i, [_vp]),
    "pgh_stream_finish_secagg": (_i, [_vp, _i, _i, _vp, _vp]),
    "pgh_stream_finish_secagg_device": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "pgh_sync": (_i, [_vp]),
    "pgh_set_variant": (_i, [_vp, _i]),
    "pgh_effective_variant": (_i, [_vp, _i]),
    "pgh_stats": (_i, [_vp, C.POINTER(Stats)]),
    "pgh_reset_stats": (_i, [_vp]),
    "pgh_slab": (_i, [_vp, C.POINTER(_vp), _P64, _P64]),
    "pgh_state_scan": (_i, [_vp, _sz, _i, _P64, _P64, C.POINTER(C.c_int)]),
    "pgh_state_scan_i64": (_i, [C.c_char_p, _sz, _i, _P64, _P64, _P64, C.POINTER(C.c_int)]),
    "pgh_state_patch": (_i, [C.c_char_p, _sz, _vp, _i64, _vp]),
    "pgh_state_fresh": (_i, [C.c_char_p, _sz, _P64, _i, _vp, _sz, C.POINTER(_sz)]),
    "pgh_b64_decoded_cap": (_sz, [_sz]),
    # the text argument is a bytes object or an address (a str's own ASCII buffer: report.py)
    "pgh_b64_decode": (_i, [_vp, _sz, _vp, C.POINTER(_sz), _i]),
    "pgh_b64_clean_size": (_i, [_vp, _sz, C.POINTER(_sz)]),
    "pgh_b64_decode_clean": (_i, [_vp, _sz, _vp, _sz, C.POINTER(_sz), _i]),
}

ABI_VERSION = 10  # include/pgh_api.h PGH_ABI_VERSION (Stats layout above)
_LIB = None


def load() -> C.CDLL:
    """Load the library (once).  Raises EngineUnavailableError if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    try:  # torch bundles libamdhip64.so.7 under the same soname: load it first so that one
        import torch  # noqa: F401  HIP runtime serves torch's allocations and ours
    except ImportError:
        pass
    if not LIB_PATH.exists():
        raise EngineUnavailableError(
            f"{LIB_PATH.name} is not built (run `python -m pygrid_amd.build`); "
            "the aggregation engine has no CPU fallback")
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pgh_abi_version() != ABI_VERSION:
        raise EngineUnavailableError(f"{LIB_PATH.name} has ABI {lib.pgh_abi_version()}, this package needs "
                                     f"{ABI_VERSION}: rebuild it (python -m pygrid_amd.build)")
    _LIB = lib
    return lib
