"""Fold diffs into HBM as they are reported.

The reference stores every reported diff in the DB (``submit_worker_diff``,
``cycle_manager.py:151-178``) and reads them all back at cycle close (``_average_plan_diffs``,
``:243-250``) in the order of the completed-WorkerCycle query
(``self._worker_cycles.query(cycle_id=..., is_completed=True)``: row-id order, i.e. the order in
which workers were assigned, ``cycle_manager.assign``), skipping the workers that never reported
(the reference expects ~20 % of them not to: ``routes.py:314``).  The fp32 fold depends on that
order, so ``IncrementalCycle`` separates WHERE a diff lives from WHEN it is folded:

* ``reported(wid, diff)`` copies the diff into HBM at once, into whichever slab slot is free
  (``pgh_ingest_state``: PCIe + host copy happen while the report is handled, in any arrival
  order);
* the fold follows assignment order: a diff's position is certain once every worker assigned
  before it has reported, and the certain prefix is folded from its scattered slots
  (``pgh_fold_slots``: the kernel reads the slots through a row table), freeing them;
* ``close(checkpoint)`` drops the workers that never reported and folds the remaining reporters'
  slots in id order into the resident checkpoint (``pgh_fold_slots_finish_resident``), then patches
  the new State bytes from HBM -- bit-identical to folding everything at close time.

So a missing early worker no longer parks later diffs on the host: they wait in HBM, and close
costs the fold of the not-yet-folded rows (HBM-bound, ~6.8 TB/s) plus the patch.  Only when every
slot is taken does a diff wait on the host (``slots`` is the HBM budget in diffs); one slot is
always kept for the fold front, so the front can never be starved by later diffs.

Thread safety: the node calls ``reported`` from request handlers and ``close`` from its executor
thread (``tasks/cycle.py``), so every method holds the cycle's lock (the engine context itself is
single-owner).  A report that arrives after ``close`` started raises ``AggregationError`` -- the
reference likewise averages only the diffs its query saw (``cycle_manager.py:243-245``).  A
malformed diff is rejected in its own ``reported`` call (``StateParseError``, nothing recorded),
so one bad client cannot break the cycle for the others.  A well-formed diff holding non-float32
tensors is accepted (the reference would average it with torch's type promotion): the cycle is
then declined as a whole -- later reports are only recorded, and ``close`` raises
``ModelNotAcceleratedError`` so the node averages the cycle with its own code, from its DB.

The checkpoint can be handed over when the cycle starts (``checkpoint=``): its payloads are then
uploaded into HBM while clients report, and ``close`` touches only the rows not folded yet.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional

from . import state as state_codec
from .engine import F32, MEAN, Engine
from .exceptions import AggregationError, ModelNotAcceleratedError, StateParseError

DEFAULT_HBM_BUDGET = 64 << 30  # bytes of diffs kept in HBM per cycle when `slots` is not given
MAX_DEFAULT_SLOTS = 4096


def default_slots(P: int, budget: int = DEFAULT_HBM_BUDGET) -> int:
    return int(max(4, min(MAX_DEFAULT_SLOTS, budget // max(4 * P, 1))))


class IncrementalCycle:
    def __init__(self, engine: Engine, numel, mode: int = MEAN, slots: Optional[int] = None, fold_batch: int = 8,
                 weights_by_worker: Optional[Dict[object, float]] = None, checkpoint: Optional[bytes] = None):
        self.engine = engine
        self.mode = mode
        self._numel = tuple(int(n) for n in numel)
        self.slots = int(slots) if slots else default_slots(sum(self._numel))
        if self.slots < 2:
            raise AggregationError("report-time aggregation needs at least 2 HBM slots")
        self.fold_batch = max(1, int(fold_batch))
        self._order: List[object] = []      # assigned workers, assignment order
        self._pos: Dict[object, int] = {}
        self._reported = set()
        self._slot_of: Dict[object, int] = {}  # reported, in HBM, not folded
        self._parked: Dict[object, bytes] = {}  # reported, no free slot yet (host)
        self._free: List[int] = list(range(self.slots - 1, -1, -1))
        self._ready: List[object] = []      # position certain, in HBM, not folded yet (fold order)
        self._front = 0                     # next assigned position not yet certain
        self._n_folded = 0
        self._weights_by_worker = weights_by_worker
        self._weights: List[float] = []     # fold order
        self.folded_early = 0
        self._lock = threading.Lock()
        self._closed = False
        self._declined: Optional[str] = None  # why the engine cannot average this cycle
        # keep the engine's slab when a cycle of the same model follows (no re-allocation)
        if tuple(getattr(engine, "numel", ())) != self._numel or getattr(engine, "max_clients", 0) != self.slots \
                or getattr(engine, "dtype", None) != F32:
            engine.set_layout(list(self._numel))
            engine.reserve(self.slots)
        else:
            engine.reset()
        self._ckpt: Optional[bytes] = None  # checkpoint bytes whose payloads are resident in HBM
        if checkpoint is not None:
            engine.ckpt_owner = None
            try:
                engine.ckpt_upload_state(checkpoint)
            except StateParseError:
                _raise_if_not_float32(checkpoint, "the checkpoint")
                raise
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
            if self._declined:
                self._reported.add(worker)  # the node averages this cycle itself
                return
            if self._weights_by_worker is not None and worker not in self._weights_by_worker:
                # refused to its sender now, not when a later report folds it (that would leave
                # the fold half done and blame another worker)
                raise AggregationError(f"worker {worker!r} reported but has no aggregation weight")
            front = self._pos[worker] == self._front
            try:
                # a diff that cannot fold yet leaves one slot free for the fold front
                if self._free and (front or len(self._free) > 1):
                    self._to_hbm(worker, diff)  # raises StateParseError on a malformed diff: nothing recorded
                else:
                    self._check_layout(worker, diff)
                    self._parked[worker] = diff
            except StateParseError:
                try:
                    _raise_if_not_float32(diff, f"worker {worker!r}'s diff")
                except ModelNotAcceleratedError as e:
                    self._declined = str(e)
                    self._parked.clear()
                    self._reported.add(worker)
                    return
                raise
            self._reported.add(worker)
            self._advance(final=False)

    def _check_layout(self, worker, diff: bytes):
        got = tuple(state_codec.tensor_numels(diff))
        if got != self._numel:
            raise StateParseError(f"worker {worker!r}: diff holds tensors of {got} floats, the model {self._numel}")

    def _to_hbm(self, worker, diff: bytes):
        slot = self._free.pop()
        try:
            self.engine.ingest_state(slot, diff)
        except Exception:
            self._free.append(slot)
            raise
        self._slot_of[worker] = slot

    def _fold_ready(self, final: bool):
        ws = self._ready
        self._ready = []
        slots = [self._slot_of.pop(w) for w in ws]
        if self._weights_by_worker is not None and ws:
            self._weights.extend(float(self._weights_by_worker[w]) for w in ws)
            self.engine.set_weights(self._weights)
        if final:
            self.engine.fold_slots_finish_resident(self.mode, slots)
        else:
            self.engine.fold_slots(self.mode, slots)
            self.folded_early += len(slots)
        self._free.extend(reversed(slots))
        self._n_folded += len(slots)

    def _advance(self, final: bool):
        while self._front < len(self._order):
            w = self._order[self._front]
            if w in self._reported:
                if w in self._parked:  # its turn: it needs a slot now
                    if not self._free:
                        self._fold_ready(final=False)  # frees >= 1 slot (see the invariant above)
                    self._to_hbm(w, self._parked.pop(w))
                self._ready.append(w)
            elif not final:
                break  # an earlier worker may still report: later positions are not certain yet
            self._front += 1  # at close, a worker that never reported is dropped
            if not final and len(self._ready) >= self.fold_batch:
                self._fold_ready(final=False)

    def close(self, checkpoint: bytes, framing: str = "fresh") -> bytes:
        """New checkpoint bytes (``cycle_manager.py:293-303``), framed like ``serialize_model_params``
        (``framing="fresh"``) or as the old checkpoint (``"template"``; see CycleAggregator)."""
        with self._lock:
            if self._closed:
                raise AggregationError("cycle already closed")
            self._closed = True
            if self._declined:
                raise ModelNotAcceleratedError(self._declined)
            self._advance(final=True)
            if self._n_folded + len(self._ready) == 0:
                raise AggregationError("no diffs to average")
            if checkpoint is not self._ckpt or getattr(self.engine, "ckpt_owner", None) is not self:
                self.engine.ckpt_owner = None
                self.engine.ckpt_upload_state(checkpoint)  # scan + staged H2D of the payload spans
            # from the fold on, HBM holds the NEW checkpoint: nobody may take it for `checkpoint`
            self.engine.ckpt_owner = None
            self._ckpt = None
            self._fold_ready(final=True)
            new = (state_codec.fresh_checkpoint(self.engine, checkpoint) if framing == "fresh"
                   else self.engine.ckpt_patch_state(checkpoint))
            self.engine.ckpt_owner = self
            return new

    @property
    def declined(self) -> Optional[str]:
        """Why the engine will not average this cycle (``close`` raises ``ModelNotAcceleratedError``),
        or None."""
        return self._declined

    @property
    def n_folded(self) -> int:
        return self._n_folded

    @property
    def n_parked(self) -> int:
        """Reported diffs waiting on the host because every HBM slot was taken."""
        return len(self._parked)


def _raise_if_not_float32(pb: bytes, what: str):
    from .cycle import _decline_non_float32

    _decline_non_float32(pb, what)
