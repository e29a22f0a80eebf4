"""Test infrastructure: the engine's slot / resident-checkpoint semantics (include/pgh_api.h) in
numpy, for CPU tests of the host logic that drives it (pygrid_amd.incremental, pygrid_amd.node).
Folds are computed by the C oracle (oracle/pgh_oracle.c) over the diffs in the order the host
logic folded them -- exactly what the GPU kernels compute (bit-exact, tests/test_gpu_*.py).  This
is never a product path: the product's Engine has no CPU fallback."""
from __future__ import annotations

import numpy as np

from oracle import coracle
from pygrid_amd import state
from pygrid_amd.exceptions import AggregationError, StateParseError

F32 = 0


class NumpyEngine:
    def __init__(self):
        self.numel = ()
        self.P = 0
        self.lo = self.hi = 0
        self.dtype = F32
        self.parties = 1
        self.max_clients = 0
        self.ckpt_owner = None
        self.ckpt_bytes = None
        self.slot = {}
        self.ckpt = None
        self.folded = []      # diffs folded into the running state, in order
        self.weights = []
        self.calls = []

    def set_layout(self, numel):
        self.numel = tuple(int(n) for n in numel)
        self.P = sum(self.numel)
        self.lo, self.hi = 0, self.P
        self.max_clients = 0
        self.ckpt_owner = None
        self.ckpt = None
        self.calls.append(("layout",))

    def reserve(self, n, dtype=F32, parties=1):
        self.max_clients = int(n)
        self.dtype = dtype
        self.slot = {}
        self.folded = []
        self.marks = {}
        self.ckpt_owner = None
        self.ckpt = None
        self.calls.append(("reserve", n))

    def reset(self):
        self.slot = {}
        self.folded = []
        self.marks = {}
        self.weights = []
        self.calls.append(("reset",))

    def _flat(self, pb):
        spans = state.scan(pb)  # raises StateParseError like the library's walker
        if tuple(c for _, c in spans) != self.numel:
            raise StateParseError(f"layout mismatch: {[c for _, c in spans]} vs {self.numel}")
        return np.concatenate(state.unserialize_model_params(pb)) if spans else np.empty(0, np.float32)

    def ingest_state(self, k, pb):
        if not 0 <= k < self.max_clients:
            raise AggregationError(f"client {k} outside slab capacity {self.max_clients}")
        self.slot[k] = self._flat(pb)
        self.calls.append(("ingest", k))

    def set_weights(self, w):
        self.weights = [np.float32(x) for x in w]

    def ckpt_upload_state(self, pb):
        self.ckpt_owner = None
        self.ckpt = self._flat(pb)
        self.calls.append(("upload",))

    def _finish(self, mode, diffs):
        if self.ckpt is None:
            raise AggregationError("no resident checkpoint")
        if not diffs:
            raise AggregationError("no diffs folded")
        w = np.array(self.weights[:len(diffs)], np.float32) if mode == 2 else None
        self.ckpt = coracle.fedavg(mode, np.stack(diffs), self.ckpt, w)

    def fedavg_resident(self, mode):
        n = 0
        while n in self.slot:
            n += 1
        if n == 0 or len(self.slot) != n:
            raise AggregationError("resident fold needs clients 0..n-1")
        self._finish(mode, [self.slot[k] for k in range(n)])
        self.calls.append(("fedavg_resident", n))

    def fold_slots(self, mode, slots):
        self.folded.extend(self.slot.pop(s) for s in slots)
        self.calls.append(("fold", len(slots)))

    def fold_slots_finish_resident(self, mode, slots=()):
        self.folded.extend(self.slot.pop(s) for s in slots)
        self._finish(mode, self.folded)
        self.calls.append(("finish", len(self.folded)))
        self.folded = []

    def fold_restart(self):
        self.folded = []
        self.weights = []
        self.calls.append(("restart",))

    def ckpt_patch_state(self, template):
        return state.serialize_model_params(template, self.ckpt)

    def ckpt_download(self):
        return self.ckpt.copy()
