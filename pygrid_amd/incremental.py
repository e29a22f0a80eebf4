"""Fold diffs into HBM as they are reported.

The reference stores every reported diff in the DB (``submit_worker_diff``,
``cycle_manager.py:151-178``) and reads them all back at cycle close
(``_average_plan_diffs``, ``:243-250``) in the order of the completed-WorkerCycle query
(``self._worker_cycles.query(cycle_id=..., is_completed=True)``: row-id order, i.e. the order in
which workers were assigned, ``cycle_manager.assign``).  The fp32 fold depends on that order, so a
diff can be folded early only once its position is certain: when every worker assigned before it
has already reported.  ``IncrementalCycle`` keeps that rule:

* ``assigned(wid)`` records assignment order (WorkerCycle id order);
* ``reported(wid, diff)`` folds the longest prefix of assigned workers that have all reported
  (engine STREAM use: H2D of later diffs overlaps the folds) and parks the rest on the host;
* ``close(checkpoint)`` drops the workers that never reported (the reference's query skips
  incomplete rows), folds the parked diffs in id order, and returns the new checkpoint bytes --
  bit-identical to folding everything at close time.

Thread safety: the node calls ``reported`` from request handlers and ``close`` from its executor
thread (``tasks/cycle.py``), so every method holds the cycle's lock (the engine context itself is
single-owner).  A report that arrives after ``close`` started raises ``AggregationError`` -- the
reference likewise averages only the diffs its query saw (``cycle_manager.py:243-245``).

The checkpoint can be handed over when the cycle starts (``checkpoint=``): its payloads are then
uploaded into HBM while clients report, and ``close`` only folds the last partial batch into it
and patches the new State bytes from HBM -- O(P) work after the last report instead of the
reference's N + 1 unserializations and N-way fold.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional

from .engine import F32, MEAN, Engine
from .exceptions import AggregationError


class IncrementalCycle:
    def __init__(self, engine: Engine, numel, mode: int = MEAN, ring_slots: int = 64, fold_batch: int = 0,
                 weights_by_worker: Optional[Dict[object, float]] = None, checkpoint: Optional[bytes] = None):
        self.engine = engine
        self.mode = mode
        self._order: List[object] = []      # assigned workers, assignment order
        self._pos: Dict[object, int] = {}
        self._parked: Dict[object, bytes] = {}
        self._reported = set()
        self._front = 0                     # next assigned position not yet folded / skipped
        self._next_client = 0               # next engine client index (fold order)
        self._weights_by_worker = weights_by_worker
        self._weights: List[float] = []
        self.folded_early = 0
        self._lock = threading.Lock()
        self._closed = False
        # keep the engine's ring when a cycle of the same model follows (no re-allocation)
        if tuple(getattr(engine, "numel", ())) != tuple(int(n) for n in numel) or \
                getattr(engine, "max_clients", 0) != ring_slots or getattr(engine, "dtype", None) != F32:
            engine.set_layout(list(numel))
            engine.reserve(ring_slots)
        engine.stream_begin(mode, fold_batch)
        self._ckpt: Optional[bytes] = None  # checkpoint bytes whose payloads are resident in HBM
        if checkpoint is not None:
            engine.ckpt_upload_state(checkpoint)
            engine.ckpt_owner = self
            self._ckpt = checkpoint

    def assigned(self, worker):
        with self._lock:
            if worker in self._pos:
                return
            self._pos[worker] = len(self._order)
            self._order.append(worker)

    def reported(self, worker, diff: bytes):
        with self._lock:
            if self._closed:
                raise AggregationError(f"worker {worker!r} reported after the cycle closed")
            if worker not in self._pos:
                raise AggregationError(f"worker {worker!r} reported without being assigned to the cycle")
            if worker in self._reported:
                raise AggregationError(f"worker {worker!r} reported twice")
            self._reported.add(worker)
            self._parked[worker] = diff
            self._advance(final=False)

    def _ingest(self, worker):
        if self._weights_by_worker is not None:
            self._weights.append(float(self._weights_by_worker[worker]))
            self.engine.set_weights(self._weights)
        self.engine.ingest_state(self._next_client, self._parked.pop(worker))
        self._next_client += 1

    def _advance(self, final: bool):
        while self._front < len(self._order):
            w = self._order[self._front]
            if w in self._reported:
                if not final:
                    self.folded_early += 1
                self._ingest(w)
            elif not final:
                return  # an earlier worker may still report: later positions are not certain yet
            self._front += 1  # at close, a worker that never reported is dropped

    def close(self, checkpoint: bytes) -> bytes:
        """New checkpoint bytes (``cycle_manager.py:293-303``)."""
        with self._lock:
            if self._closed:
                raise AggregationError("cycle already closed")
            self._closed = True
            self._advance(final=True)
            if self._next_client == 0:
                raise AggregationError("no diffs to average")
            if checkpoint is not self._ckpt or getattr(self.engine, "ckpt_owner", None) is not self:
                self.engine.ckpt_upload_state(checkpoint)  # scan + staged H2D of the payload spans
            self.engine.stream_finish_resident()
            self.engine.ckpt_owner = self
            self._ckpt = None  # HBM now holds the NEW checkpoint
            return self.engine.ckpt_patch_state(checkpoint)

    @property
    def n_folded(self) -> int:
        return self._next_client
