"""Fold diffs into HBM as they are reported, with the reference's report
semantics.

The reference stores every reported diff in its DB (``submit_worker_diff``,
``cycle_manager.py:151-178``: find the worker's WorkerCycle row, set ``diff``, ``is_completed``)
and reads them all back at cycle close (``_average_plan_diffs``, ``:243-250``) in the order of the
completed-WorkerCycle query (``self._worker_cycles.query(cycle_id=..., is_completed=True)``: a
plain ``filter_by().all()``, no ORDER BY -- row order, in practice the order in which workers were
assigned), skipping the workers that never reported (the reference expects ~20 % of them not to:
``routes.py:314``).  The fp32 fold depends on that order, so ``IncrementalCycle`` separates WHERE a
diff lives from WHEN it is folded:

* ``reported(w, diff)`` copies the diff into HBM at once, into whichever slab slot is free
  (``pgh_ingest_state``: PCIe + host copy happen while the report is handled, in any arrival
  order);
* the fold follows the assignment order (``assigned(w, key)``, ``key`` = the WorkerCycle row id),
  reporters only, through the slots where the diffs landed (the kernel reads them through a row
  table).  A position is CERTAIN once every worker assigned before it has reported.  Certain-only
  folds (default): the certain prefix is folded ``fold_batch`` at a time and freed
  (``pgh_fold_slots``).  Speculative folds (opt-in, ``speculate=True``: under the reference's
  trigger, a close right after the last report, they measured slower, profiles/r04b): every
  reported diff is folded at once (``pgh_fold_slots_keep``: its slot is kept)
  and the fold state is saved every ``mark_every`` rows and at the certain point
  (``pgh_fold_mark``); when an earlier worker reports after all, or a kept one re-reports, the fold
  goes back to the last saved state before its position (``pgh_fold_rewind``) and continues; slots
  before the last saved state at the certain point are freed.  While the GPU is still busy with the
  previous fold (``pgh_fold_busy``), or reports arrive less than ``min_gap_ms`` apart, a report is
  folded with a later one -- or by a timer once no report has come for ``settle_ms``;
* ``close(checkpoint, order=..., fetch=...)`` takes the AUTHORITATIVE order -- the keys of the
  completed-WorkerCycle query, as the node's DB returns them -- keeps the early fold up to the last
  saved state inside its common prefix with that order, and folds the rest of the order from HBM
  (slots), the host (parked diffs) or the DB (``fetch(w)``: diffs this process never saw, e.g.
  reported before a restart).  When even that is impossible (the order differs inside the freed
  prefix, a freed worker re-reported, an assignment arrived behind it) the fold restarts
  (``pgh_fold_slots_restart``) and re-folds the whole order, the folded diffs fetched from the DB:
  bit-identical to the reference in every case, early folding is only ever a speedup;
* speculative close (with speculative folds, ``peek=True``): whenever every reporter is folded, the close's FINAL pass,
  its D2H and the copy of the payloads into the cycle's prepared output bytes run ahead
  (``pgh_fold_peek_into``); a close whose order and fold state match that peek only commits it
  (``pgh_peek_patch_state``), any other close folds and copies as usual.

Report semantics (``cycle_manager.py:162-174``, ``fl_events.py:257-263``):

* **re-report** before the worker's diff was folded: the new diff replaces the old one (same slot,
  or the parked copy); after it was folded: the fold goes back to before it if its slot is still
  kept, else the early fold is stale and ``close`` re-folds from the DB (the reference averages the
  LATEST diff at the worker's original row position);
* **late report** (after ``close``): accepted and ignored -- the reference stores it and its
  ``complete_cycle`` returns early for a completed cycle (``:186-188``);
* **a report from a worker this object was not told about** (assigned before a restart):
  kept in a slot, folded at close at the position the DB order gives it;
* **malformed diff**: ``reported`` raises ``StateParseError`` (the caller decides what the client
  sees; the node wiring keeps the reference's response) and any older diff of that worker is
  dropped -- the DB now holds the malformed bytes, so ``close`` fetches them and fails the way the
  reference's close does (its ``unserialize_model_params`` raises).

Thread safety: the node calls ``reported`` from request handlers and ``close`` from its executor
thread (``tasks/cycle.py``), and the deferred fold runs on a timer thread, so every method holds
the cycle's lock (the engine context itself is single-owner) -- except that once ``seal`` (the
first half of ``close``) has run, ``reported`` / ``assigned`` return without taking it: a handler
never waits for the close's fold.  A well-formed diff holding non-float32 tensors is accepted (the reference would
average it with torch's type promotion): the cycle is then declined as a whole -- later reports
are only recorded, and ``close`` raises ``ModelNotAcceleratedError`` so the node averages the cycle
with its own code, from its DB.

The checkpoint can be handed over when the cycle starts (``checkpoint=``): its payloads are then
uploaded into HBM while clients report, and ``close`` touches only the rows not folded yet.
"""
from __future__ import annotations

import bisect
import itertools
import logging
import threading
import time
from typing import Callable, Dict, Hashable, List, Optional, Sequence

from . import state as state_codec
from .engine import F32, MEAN, WEIGHTED_MEAN, Engine
from .exceptions import AggregationError, ModelNotAcceleratedError, StateParseError

DEFAULT_HBM_BUDGET = 64 << 30  # bytes of diffs kept in HBM per cycle when `slots` is not given
MAX_DEFAULT_SLOTS = 4096
DEFAULT_SPECULATION_BUDGET = 16 << 30  # bytes of HBM for saved fold states (speculative folds)
MAX_MARKS = 256
DEFER_LIMIT = 200  # timer re-arms after a report (settle_ms each) before the close is left to fold

log = logging.getLogger(__name__)


def default_slots(P: int, budget: int = DEFAULT_HBM_BUDGET) -> int:
    return int(max(4, min(MAX_DEFAULT_SLOTS, budget // max(4 * P, 1))))


class IncrementalCycle:
    def __init__(self, engine: Engine, numel, mode: int = MEAN, slots: Optional[int] = None, fold_batch: int = 8,
                 weights_by_worker: Optional[Dict[object, float]] = None, checkpoint: Optional[bytes] = None,
                 early_fold: bool = True, speculate: Optional[bool] = None,
                 speculation_budget: int = DEFAULT_SPECULATION_BUDGET, mark_every: int = 8, lazy: bool = True,
                 min_gap_ms: float = 2.0, peek: bool = True, settle_ms: float = 5.0):
        self.engine = engine
        self.mode = mode
        self._numel = tuple(int(n) for n in numel)
        P = sum(self._numel)
        self.slots = int(slots) if slots else default_slots(P)
        if self.slots < 2:
            raise AggregationError("report-time aggregation needs at least 2 HBM slots")
        self.fold_batch = max(1, int(fold_batch))
        self.early_fold = bool(early_fold)
        # saved fold states the speculation may hold in HBM (each P floats); < 2 turns it off
        self.max_marks = int(min(MAX_MARKS, speculation_budget // max(4 * P, 1)))
        can = all(hasattr(engine, f) for f in ("fold_slots_keep", "fold_mark", "fold_rewind", "fold_unmark"))
        # opt-in (r04): under the reference's trigger -- the close right after the last report -- a
        # certain-only close was faster (profiles/r04b: 2.09 vs 3.7-4.0 ms with the peek, 2.5 without)
        self.speculate = bool(can and self.max_marks >= 2 and speculate)
        self.mark_every = max(1, int(mark_every))
        # speculative folds wait while the GPU is still busy with the previous one (reports arriving
        # back to back would otherwise queue re-folds that the next report discards)
        self._lazy = bool(lazy) and hasattr(engine, "fold_busy")
        self.min_gap_s = max(0.0, float(min_gap_ms)) / 1e3
        # the timer that folds what lazy skips left waits this long after a report (a close that
        # follows the last report at once should find the cycle lock free, not a fold in progress)
        self.settle_s = max(self.min_gap_s, float(settle_ms) / 1e3, 1e-3)
        # speculative close: the FINAL pass of the fold state peeked ahead (pgh_fold_peek) whenever
        # every reporter is folded; a close that finds nothing changed commits it
        self._peek = self.speculate and bool(peek) and hasattr(engine, "fold_peek")
        self._peeked = None  # (fold length, rewinds) of the last peek
        self._last_report = None
        self._hurried = False  # the last report came less than min_gap after the one before
        self._timer: Optional[threading.Timer] = None  # folds what a lazy skip left once reports pause
        self._defer_left = 0
        if speculate and not self.speculate:
            raise AggregationError("speculative folds need an engine with fold marks and HBM for >= 2 of them "
                                   f"({self.max_marks} fit in the budget)")
        self._seq = itertools.count()
        self._order: List[object] = []      # assigned workers, sorted by assignment key
        self._keys: List[tuple] = []        # their keys (sorted, parallel to _order)
        self._key_of: Dict[object, tuple] = {}
        self._behind = set()                # assigned behind the freed fold prefix: never folded early
        self._reported = set()              # workers whose latest report we accepted
        self._slot_of: Dict[object, int] = {}  # latest diff in HBM (not folded, or folded and kept)
        self._parked: Dict[object, bytes] = {}  # latest diff on the host (no free slot yet)
        self._bad: Dict[object, str] = {}   # latest report unusable here (malformed / failed ingest)
        self._free: List[int] = list(range(self.slots - 1, -1, -1))
        self._folded: List[object] = []     # in the running fold state, in fold order
        self._folded_set = set()
        self._base = 0                      # _folded[:_base]: certain, slots freed, never re-folded
        self._marks: List[tuple] = []       # (fold length, mark id), increasing; the base's first
        self._mark_ids = itertools.count()
        self._stale: Optional[str] = None   # why the early fold no longer matches the reports
        self._weights_by_worker = weights_by_worker
        self._weights: List[float] = []     # fold order
        self.folded_early = 0
        self.rewinds = 0
        self.last_close: dict = {}
        self._lock = threading.Lock()
        self._closed = False
        self._close_order: Optional[List] = None  # set by seal(), taken by finish()
        self._declined: Optional[str] = None  # why the engine cannot average this cycle
        # one open cycle per engine: a previous one left open (dropped without close) is abandoned
        # here, so that its deferred-fold timer cannot touch this cycle's slots
        prev = getattr(engine, "cycle_owner", None)
        if prev is not None and prev is not self:
            prev.abandon()
        engine.cycle_owner = self
        # keep the engine's slab when a cycle of the same model follows (no re-allocation)
        if tuple(getattr(engine, "numel", ())) != self._numel or getattr(engine, "max_clients", 0) != self.slots \
                or getattr(engine, "dtype", None) != F32:
            engine.set_layout(list(self._numel))
            engine.reserve(self.slots)
        else:
            engine.reset()
        self._ckpt: Optional[bytes] = None  # checkpoint bytes whose payloads are resident in HBM
        if checkpoint is not None and getattr(engine, "ckpt_owner", None) is not None \
                and getattr(engine, "ckpt_bytes", None) is checkpoint:
            # the previous close left exactly these bytes' params in HBM (the cycles are chained)
            engine.ckpt_owner = self
            self._ckpt = checkpoint
        elif checkpoint is not None:
            engine.ckpt_owner = None
            try:
                engine.ckpt_upload_state(checkpoint)
            except StateParseError:
                _raise_if_not_float32(checkpoint, "the checkpoint")
                raise
            engine.ckpt_owner = self
            self._ckpt = checkpoint
        # the new checkpoint's bytes, framed and faulted in while the cycle is open (the close then
        # copies into resident pages: with speculative folds there is little fold left to hide that).
        # The frame is allocated here; certain-only, its page faults (3-5 ms for 47 MB) run on a thread
        # of its own, off the previous close, which creates this cycle (``finish`` joins it).  With
        # the peek, at once: every peek from the first report on copies into it.
        self._prepared = None
        self._prep_thread: Optional[threading.Thread] = None
        if checkpoint is not None and hasattr(engine, "ckpt_patch_into"):
            try:
                frame = state_codec.fresh_frame_bytes(checkpoint)  # allocated and framed here, on this thread
            except StateParseError:
                frame = None
            if frame is not None:
                self._prepared = (checkpoint, frame)
                if self._peek:
                    state_codec.prefault(frame)
                else:
                    self._prep_thread = threading.Thread(target=state_codec.prefault, args=(frame,),
                                                         name="pgh-prefault", daemon=True)
                    self._prep_thread.start()

    # ---- assignment (cycle_manager.assign, fl_controller.py:131-132) ---------------------------
    def assigned(self, worker, key=None):
        """``worker`` was assigned to the cycle.  ``key`` orders the assignments (the WorkerCycle row
        id: the order the completed-WorkerCycle query returns rows in); default: call order."""
        if self._closed:
            return
        with self._lock:
            if worker in self._key_of or self._closed:
                return
            k = (0, key) if key is not None else (1, next(self._seq))
            i = bisect.bisect_right(self._keys, k)
            if self._base and i <= bisect.bisect_left(self._keys, self._key_of[self._folded[self._base - 1]]):
                # behind the freed fold prefix: never folded early; if it reports, close's order
                # check sees the early prefix is not the DB's prefix and re-folds
                self._behind.add(worker)
            self._key_of[worker] = k
            self._keys.insert(i, k)
            self._order.insert(i, worker)
            if worker in self._reported:  # it reported before we heard of it (e.g. a restart)
                self._sync()

    # ---- report (fl_events.py:257-261 -> submit_worker_diff, cycle_manager.py:151-178) ---------
    def reported(self, worker, diff: bytes):
        """The worker's (latest) diff.  Raises ``StateParseError`` for a malformed diff (see the
        module docstring); never raises for a late or repeated report."""
        if self._closed:  # sealed: no waiting for the close's fold (set under the lock, read without)
            log.info("worker %r reported after the cycle closed: ignored (fl_events.py:261-263)", worker)
            return
        with self._lock:
            if self._closed:
                log.info("worker %r reported after the cycle closed: ignored (fl_events.py:261-263)", worker)
                return
            if self._declined:
                self._reported.add(worker)  # the node averages this cycle itself
                return
            if self._weights_by_worker is not None and worker not in self._weights_by_worker:
                # refused to its sender now, not when a later report folds it
                raise AggregationError(f"worker {worker!r} reported but has no aggregation weight")
            now = time.monotonic()
            self._hurried = self._last_report is not None and now - self._last_report < self.min_gap_s
            self._last_report = now
            self._defer_left = DEFER_LIMIT
            if worker in self._folded_set:
                # its earlier diff is in the fold state: go back to before it (its slot is still
                # held), or -- when it was folded for good -- the close re-folds from the DB
                if not self._rewind(self._folded.index(worker)):
                    self._stale = f"worker {worker!r} re-reported after its diff was folded"
                    self._reported.add(worker)
                    return
            try:
                self._take(worker, diff)
            except StateParseError:
                try:
                    _raise_if_not_float32(diff, f"worker {worker!r}'s diff")
                except ModelNotAcceleratedError as e:
                    self._declined = str(e)
                    self._parked.clear()
                    self._reported.add(worker)
                    return
                self._forget(worker, "malformed diff")
                self._sync()
                raise
            self._reported.add(worker)
            self._bad.pop(worker, None)
            self._sync()

    def _take(self, worker, diff: bytes):
        """Store ``diff`` as the worker's latest: over its old slot, in a free slot, or parked."""
        if worker in self._slot_of:  # re-report before the fold: same slot (parse first, then DMA)
            self.engine.ingest_state(self._slot_of[worker], diff)
            return
        # a diff that cannot fold yet leaves one slot free for the fold front
        if self._free and (len(self._free) > 1 or self._is_front(worker)):
            self._to_hbm(worker, diff)  # raises StateParseError on a malformed diff: nothing recorded
            self._parked.pop(worker, None)
        else:
            self._check_layout(worker, diff)
            self._parked[worker] = diff

    def _forget(self, worker, why: str):
        """The worker's latest report is unusable here: drop any older copy (HBM or host)."""
        slot = self._slot_of.pop(worker, None)
        if slot is not None:
            self._free.append(slot)
        self._parked.pop(worker, None)
        self._reported.discard(worker)
        self._bad[worker] = why

    def _is_front(self, worker) -> bool:
        """``worker`` is the first assigned worker whose diff is neither folded nor in HBM (the one
        the fold waits for)."""
        for w in self._order:
            if w in self._folded_set or w in self._slot_of or w in self._behind:
                continue
            return w == worker
        return False

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

    def _held(self, worker) -> bool:
        return worker in self._slot_of or worker in self._parked

    # ---- early folds ---------------------------------------------------------------------------
    def _plan(self):
        """The reporters in the order the close will fold them, as far as known now (assignment
        order, non-reporters skipped), and how many of them are certain: those before the first
        assigned worker that has not reported (a later report can only land behind that point)."""
        plan, certain = [], None
        for w in self._order:
            if w in self._behind:
                continue
            if w in self._reported:
                plan.append(w)
            elif certain is None:
                certain = len(plan)
        return plan, len(plan) if certain is None else certain

    def _sync(self):
        """Bring the fold state up to date with the reports: go back to before the first position
        that changed, then fold what follows -- every reported diff in HBM when speculating (folded
        and kept, a mark after each fold), else only the certain ones, ``fold_batch`` at a time
        (folded and freed).  Slots of certain positions before a mark are freed."""
        if self._stale or self._declined or self._closed or not self.early_fold:
            return
        plan, certain = self._plan()
        target = plan if self.speculate else plan[:certain]
        common = _common_prefix(self._folded, target)
        if common < len(self._folded) and not self._rewind(common):
            return  # the early fold is not the plan's prefix any more: the close re-folds
        if self.speculate and self._lazy and not self._parked and (self._hurried or self.engine.fold_busy()):
            # reports arriving faster than a re-fold takes, or the GPU still folding: fold this
            # report with a later one instead of queueing re-folds the next report throws away;
            # if none comes within min_gap, a timer folds it (before the close, when that is later)
            self._defer()
            return
        run: List = []
        for w in target[len(self._folded):]:
            if w not in self._slot_of:
                if w not in self._parked:
                    break
                if not self._free and run and not self.speculate:
                    self._fold_run(run)  # frees their slots for the parked diff
                    run = []
                if not (len(self._free) > 1 or self._free and self._is_front(w)):
                    break  # the last free slot is the fold front's
                try:
                    self._to_hbm(w, self._parked[w])
                except Exception as e:  # noqa: BLE001 -- not this caller's report
                    log.warning("parked diff of worker %r failed to ingest: %s", w, e)
                    self._forget(w, f"ingest failed: {e}")
                    break
                del self._parked[w]
            run.append(w)
        if run and (self.speculate or len(run) >= self.fold_batch):
            self._fold_run(run, certain)
        if self.speculate:
            self._advance_base(certain)
            if self._peek and self._prepared is not None and self._folded and self._folded == plan \
                    and self._peeked != (len(self._folded), self.rewinds):
                # every reporter so far is folded: take the close's FINAL pass now, in the background
                try:
                    self.engine.fold_peek(self.mode, into=self._prepared[1] if self._prepared[1][1] else None)
                except AggregationError as e:  # e.g. no HBM for the peek buffer: close the usual way
                    log.warning("speculative close disabled for this cycle: %s", e)
                    self._peek = False
                    return
                if not hasattr(self.engine, "peek_valid") or self.engine.peek_valid():
                    self._peeked = (len(self._folded), self.rewinds)
                else:  # skipped (the previous peek's copy still running): try again once reports pause
                    self._defer()

    def _defer(self):
        if self._timer is None and self._defer_left > 0:
            self._defer_left -= 1
            self._timer = threading.Timer(self.settle_s, self._deferred)
            self._timer.daemon = True
            self._timer.start()

    def _deferred(self):
        """Timer thread: the reports paused (no new one within min_gap) -- fold what the lazy skips
        left, as a report arriving then would have; while the GPU is still folding, wait again."""
        with self._lock:
            self._timer = None
            if self._closed or self._stale or self._declined:
                return
            if self._last_report is not None and time.monotonic() - self._last_report < self.settle_s:
                self._defer()  # still arriving
                return
            self._hurried = False
            try:
                self._sync()
            except Exception as e:  # noqa: BLE001 -- nobody to raise to: the close re-folds from the DB
                log.warning("deferred fold failed (%s): the close re-folds this cycle", e)
                self._stale = f"deferred fold failed: {e}"

    def _cancel_timer(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None

    def _fold_run(self, ws: Sequence, certain: int = 0):
        slots = [self._slot_of[w] for w in ws]
        if self.mode == WEIGHTED_MEAN and self._weights_by_worker is not None:
            self._weights.extend(float(self._weights_by_worker[w]) for w in ws)
            self.engine.set_weights(self._weights)
        if self.speculate:
            # a saved state at least every `mark_every` rows (a later rewind goes back no further
            # than that before the position that changed) and one exactly at the certain point,
            # so that the certain diffs' slots are freed at once
            n0 = len(self._folded)
            cuts = sorted({*range(self.mark_every, len(ws), self.mark_every), len(ws)} |
                          ({certain - n0} if 0 < certain - n0 < len(ws) else set()))
            i = 0
            for j in cuts:
                self.engine.fold_slots_keep(self.mode, slots[i:j])
                self._folded.extend(ws[i:j])
                self._folded_set.update(ws[i:j])
                self._mark()
                self._advance_base(certain)
                i = j
            self.folded_early = len(self._folded)
            return
        else:
            self.engine.fold_slots(self.mode, slots)
            for w in ws:
                del self._slot_of[w]
            self._free.extend(reversed(slots))
        self._folded.extend(ws)
        self._folded_set.update(ws)
        self.folded_early = len(self._folded)
        self._base = len(self._folded)

    def _mark(self):
        n = len(self._folded)
        if len(self._marks) >= self.max_marks:
            # first drop the mark whose neighbours are closest (the base's stays), so that at most
            # max_marks states are ever held
            at = [m[0] for m in self._marks] + [n]
            i = min(range(1, len(self._marks)), key=lambda j: at[j + 1] - at[j - 1])
            self.engine.fold_unmark(self._marks.pop(i)[1])
        mid = next(self._mark_ids)
        try:
            self.engine.fold_mark(mid)
        except AggregationError as e:  # no HBM for another saved state: keep fewer from now on
            log.warning("fold state not saved at %d (%s); speculation keeps %d saved states", n, e, len(self._marks))
            self.max_marks = max(2, len(self._marks))
            return
        self._marks.append((n, mid))

    def _advance_base(self, certain: int):
        """Positions before ``certain`` never change again: free their slots up to the last mark
        there, which becomes the base (the earliest point a rewind may go back to)."""
        cert = min(certain, len(self._folded))
        at = [i for i, (n, _) in enumerate(self._marks) if n <= cert]
        if not at or self._marks[at[-1]][0] <= self._base:
            return
        i = at[-1]
        new_base = self._marks[i][0]
        for w in self._folded[self._base:new_base]:
            slot = self._slot_of.pop(w, None)
            if slot is not None:
                self._free.append(slot)
        for _, mid in self._marks[:i]:
            self.engine.fold_unmark(mid)
        del self._marks[:i]
        self._base = new_base

    def _rewind(self, n: int) -> bool:
        """Go back to a fold state of at most ``n`` folded diffs (the latest saved one); False when
        that would need diffs whose slots were freed."""
        if n >= len(self._folded):
            return True
        if n < self._base:
            return False
        keep = [m for m in self._marks if m[0] <= n]
        to = keep[-1][0] if keep else 0
        if keep:
            self.engine.fold_rewind(keep[-1][1])
        else:  # before the first mark: the base is 0 (a mark is the base otherwise)
            self.engine.fold_restart()
        for _, mid in self._marks[len(keep):]:
            self.engine.fold_unmark(mid)
        del self._marks[len(keep):]
        del self._folded[to:]
        self._folded_set = set(self._folded)
        del self._weights[to:]
        self.folded_early = len(self._folded)
        self.rewinds += 1
        return True

    def _drop_marks(self):
        for _, mid in self._marks:
            self.engine.fold_unmark(mid)
        self._marks = []

    # ---- close (cycle_manager.py:217 -> _average_plan_diffs :240-303) ---------------------------
    def close(self, checkpoint: bytes, framing: str = "fresh", order: Optional[Sequence[Hashable]] = None,
              fetch: Optional[Callable[[object], bytes]] = None) -> bytes:
        """New checkpoint bytes (``cycle_manager.py:293-303``), framed like ``serialize_model_params``
        (``framing="fresh"``) or as the old checkpoint (``"template"``; see CycleAggregator).

        ``order``: the workers of the completed-WorkerCycle query in the order the DB returned them
        (``:243-245``); ``fetch(w)``: that row's ``diff`` bytes (read only for diffs not held here).
        Without ``order`` the assignment order of the reporters is taken as the query's.
        ``seal(order)`` then ``finish(checkpoint, ...)``."""
        self.seal(order)
        return self.finish(checkpoint, framing=framing, fetch=fetch)

    def seal(self, order: Optional[Sequence[Hashable]] = None) -> bool:
        """The close's snapshot (``cycle_manager.py:243-245``: the moment the reference's query reads
        the completed rows): from here on reports and assignments are ignored at once, without the
        cycle's lock, so a handler never waits for the fold.  Returns True when ``finish`` will read
        diffs through ``fetch`` (a re-fold, diffs reported before a restart, parked diffs): the
        caller then keeps later re-reports out of the DB rows until ``finish`` returns (the
        reference reads every diff at its query)."""
        with self._lock:
            if self._closed:
                raise AggregationError("cycle already closed")
            self._closed = True
            self._cancel_timer()
            if self._declined:
                raise ModelNotAcceleratedError(self._declined)
            if order is None:
                if self._stale or self._bad:
                    what = self._stale or ", ".join(f"{w!r}: {why}" for w, why in self._bad.items())
                    raise AggregationError(f"cannot close without the DB's rows ({what}): pass order= and fetch=")
                order = [w for w in self._order if w in self._reported and (self._held(w) or w in self._folded_set)]
                floating = [w for w in self._reported if w not in self._key_of and self._held(w)]
                if floating:
                    log.warning("close without the DB order: %d reports of unassigned workers dropped", len(floating))
            order = list(order)
            if len(set(order)) != len(order):
                raise AggregationError("the completed-WorkerCycle order lists a worker twice")
            if not order:
                raise AggregationError("no diffs to average")
            if self._weights_by_worker is not None:
                missing = [w for w in order if w not in self._weights_by_worker]
                if missing:
                    raise AggregationError(f"workers {missing[:8]!r} have no aggregation weight")
            self._close_order = order
            return self._needs_fetch(order)

    def _needs_fetch(self, order: List) -> bool:
        """Whether folding ``order`` reads any diff through ``fetch``: a stale or re-folded early
        fold, or a row whose diff is not in an HBM slot (parked, never seen; a full slab then also
        gives up a later slot and re-reads it).  Rows between a rewind's mark and the common prefix
        keep their slots (speculative folds free slots only before the base)."""
        if self._stale:
            return True
        common = _common_prefix(self._folded, order)
        if common < len(self._folded) and common < self._base:
            return True
        return any(w not in self._slot_of for w in order[common:])

    def finish(self, checkpoint: bytes, framing: str = "fresh",
               fetch: Optional[Callable[[object], bytes]] = None) -> bytes:
        """The rest of ``close`` after ``seal``: fold, FINAL pass, new checkpoint bytes."""
        with self._lock:
            order = self._close_order
            if order is None:
                raise AggregationError("finish() without a successful seal()")
            self._close_order = None
            folded_before = len(self._folded)
            refold = self._stale
            if not refold and not self._rewind(_common_prefix(self._folded, order)):
                refold = f"the DB order's first {len(self._folded)} workers are not the ones folded early"
            k = 0 if refold else len(self._folded)
            rest = order if refold else order[k:]
            if fetch is None:
                unheld = [w for w in rest if not self._held(w)]
                if unheld:
                    raise AggregationError(f"workers {unheld[:8]!r} in the close order have no diff here and there "
                                           "is no fetch= to read them from the DB")
            if checkpoint is not self._ckpt or getattr(self.engine, "ckpt_owner", None) is not self:
                self.engine.ckpt_owner = None
                self.engine.ckpt_upload_state(checkpoint)  # scan + staged H2D of the payload spans
            # from the fold on, HBM holds the NEW checkpoint: nobody may take it for `checkpoint`
            self.engine.ckpt_owner = None
            self._ckpt = None
            if refold:  # the folded diffs are only in the fold state: discarded, re-read from the DB
                log.info("re-folding the cycle in the DB's order: %s", refold)
                self.engine.fold_restart()
                self._weights = []
            if self._prep_thread is not None:  # a few ms of work at most, and less than doing it here
                self._prep_thread.join()
                self._prep_thread = None
            prep = self._prepared[1] if self._prepared and self._prepared[0] is checkpoint else None
            self._prepared = None
            # nothing left to fold and the last peek still matches: its result IS the new checkpoint
            peeked = bool(not refold and not rest and framing == "fresh" and prep is not None and prep[1]
                          and self._peek and self.engine.peek_patch_into(prep[1], len(prep[0])))
            if peeked:
                stats = {"from_hbm": 0, "from_host": 0, "from_db": 0}
                new = prep[0]
            else:
                stats = self._fold_in_order(rest, fetch)
            self._drop_marks()  # after the FINAL pass: it reads a rewound state from its mark in place
            stats.update(refold=bool(refold), reason=refold or None, early=k, n=len(order),
                         folded_before_close=folded_before, rewinds=self.rewinds, peeked=peeked)
            self.last_close = stats
            if not peeked:
                new = (state_codec.fresh_checkpoint(self.engine, checkpoint, prepared=prep) if framing == "fresh"
                       else self.engine.ckpt_patch_state(checkpoint))
            self.engine.ckpt_owner = self
            self.engine.ckpt_bytes = new
            return new

    def _fold(self, ws: Sequence, final: bool):
        slots = [self._slot_of.pop(w) for w in ws]
        if self.mode == WEIGHTED_MEAN and self._weights_by_worker is not None and (ws or final):
            self._weights.extend(float(self._weights_by_worker[w]) for w in ws)
            if self._weights:
                self.engine.set_weights(self._weights)
        if final:
            self.engine.fold_slots_finish_resident(self.mode, slots)
        else:
            self.engine.fold_slots(self.mode, slots)
        self._free.extend(reversed(slots))
        return slots

    def _fold_in_order(self, rest: List, fetch) -> dict:
        """Fold ``rest`` in order and finish into the resident checkpoint, within the slot budget:
        held slots are folded where they stand, other diffs are ingested into free slots; when none
        is free, the pending batch is folded, or -- when the batch is empty and every slot holds a
        later worker's diff -- the slot of the worker needed LAST is given up (its diff is fetched
        from the DB when its turn comes)."""
        pos = {w: i for i, w in enumerate(rest)}
        for w in [w for w in self._slot_of if w not in pos]:  # held (or folded and kept), not needed
            self._free.append(self._slot_of.pop(w))
        batch: List = []
        from_hbm = from_host = from_db = 0
        for i, w in enumerate(rest):
            if w in self._slot_of:
                batch.append(w)
                from_hbm += 1
                continue
            diff = self._parked.get(w)
            if diff is None:
                if fetch is None:
                    raise AggregationError(f"worker {w!r}: no diff held here and no fetch= to read it from the DB")
                diff = fetch(w)
                from_db += 1
            else:
                from_host += 1
            if not self._free:
                if batch:
                    self._fold(batch, final=False)
                    batch = []
                else:
                    later = max((x for x in self._slot_of if pos[x] > i), key=pos.__getitem__)
                    if fetch is None:
                        raise AggregationError(f"slot budget exhausted and no fetch= to re-read {later!r}")
                    self._free.append(self._slot_of.pop(later))
            self._to_hbm(w, diff)
            self._parked.pop(w, None)
            batch.append(w)
        self._fold(batch, final=True)
        return {"from_hbm": from_hbm, "from_host": from_host, "from_db": from_db}

    def abandon(self):
        """Another user takes the engine (its slab is re-laid): nothing held here survives.  Later
        reports are ignored and ``close`` raises; the node closes this cycle from its DB rows."""
        if self._closed:  # sealed or closed: its result may be the resident checkpoint
            return
        with self._lock:
            if self._closed:  # closed (or abandoned) already: its result may be the resident checkpoint
                return
            self._closed = True
            self._cancel_timer()
            self._slot_of.clear()
            self._parked.clear()
            self._marks = []
            if getattr(self.engine, "ckpt_owner", None) is self:
                self.engine.ckpt_owner = None

    @property
    def peek_enabled(self) -> bool:
        """The speculative close (pgh_fold_peek_into) is on for this cycle."""
        return bool(self._peek)

    @property
    def declined(self) -> Optional[str]:
        """Why the engine will not average this cycle (``close`` raises ``ModelNotAcceleratedError``),
        or None."""
        return self._declined

    @property
    def stale(self) -> Optional[str]:
        """Why ``close`` will re-fold from the DB (a folded worker re-reported), or None."""
        return self._stale

    @property
    def n_folded(self) -> int:
        return self.last_close.get("n", len(self._folded))

    @property
    def n_parked(self) -> int:
        """Reported diffs waiting on the host because every HBM slot was taken."""
        return len(self._parked)


def _common_prefix(a: Sequence, b: Sequence) -> int:
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


def _raise_if_not_float32(pb: bytes, what: str):
    from .cycle import _decline_non_float32

    _decline_non_float32(pb, what)
