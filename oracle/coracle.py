"""ctypes handle on oracle/_build/liboracle.so (the scalar C oracle) -- TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists() or LIB.stat().st_mtime < (HERE / "pgh_oracle.c").stat().st_mtime:
            build()
        L = C.CDLL(str(LIB))
        vp, i, i64, u64, f = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_float
        L.or_fedavg_mean.argtypes = [vp, i, i64, i64, vp, vp]
        L.or_fedavg_iterative.argtypes = [vp, i, i64, i64, vp, vp]
        L.or_fedavg_weighted.argtypes = [vp, vp, i, i64, i64, vp, vp]
        L.or_secagg.argtypes = [vp, i, i, i64, i64, f, vp, vp]
        L.or_synth_f32.argtypes = [u64, u64, u64, i64, i64, f, vp]
        L.or_synth_u64.argtypes = [u64, u64, u64, i64, i64, vp]
        L.or_synth_f32_fast.argtypes = [u64, u64, u64, i64, i64, f, vp]
        L.or_weight_total.argtypes = [vp, i]
        L.or_weight_total.restype = f
        L.or_row_key.argtypes = [u64, u64, u64]
        L.or_row_key.restype = u64
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


def fedavg(mode: int, diffs: np.ndarray, ckpt: np.ndarray, weights=None) -> np.ndarray:
    """diffs: float32 [N][ld] (ld >= P), ckpt float32 [P]; mode 0 mean, 1 iterative, 2 weighted."""
    d = np.ascontiguousarray(diffs, dtype=np.float32)
    c = np.ascontiguousarray(ckpt, dtype=np.float32)
    n, ld = d.shape
    out = np.empty_like(c)
    L = lib()
    if mode == 0:
        rc = L.or_fedavg_mean(_p(d), n, ld, c.size, _p(c), _p(out))
    elif mode == 1:
        rc = L.or_fedavg_iterative(_p(d), n, ld, c.size, _p(c), _p(out))
    else:
        w = np.ascontiguousarray(weights, dtype=np.float32)
        rc = L.or_fedavg_weighted(_p(d), _p(w), n, ld, c.size, _p(c), _p(out))
    if rc:
        raise ValueError("oracle rejected the input")
    return out


def secagg(shares: np.ndarray, p: int, divisor: float = 1000.0):
    """shares int64 [N][S][ld] -> (int64 sum [p], float32 decoded [p])."""
    s = np.ascontiguousarray(shares, dtype=np.int64)
    n, S, ld = s.shape
    out_s = np.empty(p, np.int64)
    out_d = np.empty(p, np.float32)
    if lib().or_secagg(_p(s), n, S, ld, p, C.c_float(divisor), _p(out_s), _p(out_d)):
        raise ValueError("oracle rejected the input")
    return out_s, out_d


def synth_f32(seed: int, stream: int, row: int, idx0: int, n: int, scale: float) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().or_synth_f32(seed, stream, row, idx0, n, C.c_float(scale), _p(out))
    return out


def synth_f32_fast(seed: int, stream: int, row: int, idx0: int, n: int, scale: float) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().or_synth_f32_fast(seed, stream, row, idx0, n, C.c_float(scale), _p(out))
    return out


def synth_u64(seed: int, stream: int, row: int, idx0: int, n: int) -> np.ndarray:
    out = np.empty(n, np.uint64)
    lib().or_synth_u64(seed, stream, row, idx0, n, _p(out))
    return out
