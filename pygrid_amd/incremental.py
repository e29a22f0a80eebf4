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
  table).  A position is CERTAIN once every worker assigned before it has reported; the certain
  prefix is folded ``fold_batch`` at a time and its slots freed (``pgh_fold_slots``).  Nothing is
  folded past the first worker that has not reported: a diff folded there could land at the wrong
  position, and undoing that costs more than it saves (the speculative folds and peeked close of
  ABI 6-7, retired in r05: under the reference's trigger they closed slower, 2.59-2.85 vs 2.21 ms,
  BENCH_r04 ``cycle_close_report_time.arms``);
* ``close(checkpoint, order=..., fetch=...)`` takes the AUTHORITATIVE order -- the keys of the
  completed-WorkerCycle query, as the node's DB returns them -- keeps the early fold when it is a
  prefix of that order, and folds the rest of the order from HBM (slots), the host (parked diffs)
  or the DB (``fetch(w)``: diffs this process never saw, e.g. reported before a restart).  When
  that is impossible (the order differs inside the folded prefix, a folded worker re-reported, an
  assignment arrived behind it) the fold restarts (``pgh_fold_slots_restart``) and re-folds the
  whole order, the folded diffs fetched from the DB: bit-identical to the reference in every case,
  early folding is only ever a speedup.

Report semantics (``cycle_manager.py:162-174``, ``fl_events.py:257-263``):

* **re-report** before the worker's diff was folded: the new diff replaces the old one (same slot,
  or the parked copy); after it was folded: the early fold is stale and ``close`` re-folds from the
  DB (the reference averages the LATEST diff at the worker's original row position);
* **late report** (after ``close``): accepted and ignored -- the reference stores it and its
  ``complete_cycle`` returns early for a completed cycle (``:186-188``);
* **a report from a worker this object was not told about** (assigned before a restart):
  kept in a slot, folded at close at the position the DB order gives it;
* **malformed diff**: ``reported`` raises ``StateParseError`` (the caller decides what the client
  sees; the node wiring keeps the reference's response) and any older diff of that worker is
  dropped -- the DB now holds the malformed bytes, so ``close`` fetches them and fails the way the
  reference's close does (its ``unserialize_model_params`` raises).

Thread safety: the node calls ``reported`` from request handlers and ``close`` from its executor
thread (``tasks/cycle.py``), so every method holds the cycle's lock (the engine context itself is
single-owner) -- except that once ``seal`` (the first half of ``close``) has run, ``reported`` /
``assigned`` return without taking it: a handler never waits for the close's fold.  A well-formed diff holding non-float32 tensors is accepted (the reference would
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
import os
import threading
from typing import Callable, Dict, Hashable, List, Optional, Sequence

from . import state as state_codec
from .engine import F32, MEAN, WEIGHTED_MEAN, Engine
from .exceptions import AggregationError, ModelNotAcceleratedError, StateParseError

DEFAULT_HBM_BUDGET = 64 << 30  # bytes of diffs kept in HBM per cycle when `slots` is not given
MAX_DEFAULT_SLOTS = 4096

log = logging.getLogger(__name__)


def default_slots(P: int, budget: int = DEFAULT_HBM_BUDGET) -> int:
    return int(max(4, min(MAX_DEFAULT_SLOTS, budget // max(4 * P, 1))))


class IncrementalCycle:
    def __init__(self, engine: Engine, numel, mode: int = MEAN, slots: Optional[int] = None, fold_batch: int = 8,
                 weights_by_worker: Optional[Dict[object, float]] = None, checkpoint: Optional[bytes] = None,
                 early_fold: bool = True):
        self.engine = engine
        self.mode = mode
        self._numel = tuple(int(n) for n in numel)
        P = sum(self._numel)
        self.slots = int(slots) if slots else default_slots(P)
        if self.slots < 2:
            raise AggregationError("report-time aggregation needs at least 2 HBM slots")
        self.fold_batch = max(1, int(fold_batch))
        self.early_fold = bool(early_fold)
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
        self._stale: Optional[str] = None   # why the early fold no longer matches the reports
        self._weights_by_worker = weights_by_worker
        self._weights: List[float] = []     # fold order
        self.folded_early = 0
        self.last_close: dict = {}
        self._lock = threading.Lock()
        self._closed = False
        self._close_order: Optional[List] = None  # set by seal(), taken by finish()
        self._declined: Optional[str] = None  # why the engine cannot average this cycle
        # one open cycle per engine: a previous one left open (dropped without close) is abandoned
        # here, so that nothing of it touches this cycle's slots
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
        if hasattr(engine, "set_ingest_ranges"):
            # the close overlaps the tail of the last report's copy (pgh_set_ingest_ranges)
            engine.set_ingest_ranges(os.environ.get("PGH_INGEST_RANGES", "1") != "0")
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
        # copies into resident pages).  The frame is allocated here; its page faults (3-5 ms for
        # 47 MB) run on a thread of its own, off the previous close, which creates this cycle
        # (``finish`` joins it).
        self._prepared = None
        self._prep_thread: Optional[threading.Thread] = None
        if checkpoint is not None and hasattr(engine, "ckpt_patch_into"):
            try:
                frame = state_codec.fresh_frame_bytes(checkpoint)  # allocated and framed here, on this thread
            except StateParseError:
                frame = None
            if frame is not None:
                self._prepared = (checkpoint, frame)
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
            if self._folded and i <= bisect.bisect_left(self._keys, self._key_of[self._folded[-1]]):
                # behind the folded prefix: never folded early; if it reports, close's order
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
            if worker in self._folded_set:
                # its earlier diff is in the fold state for good: the close re-folds from the DB
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
        """Fold the certain reporters not folded yet, ``fold_batch`` at a time (folded and freed);
        parked diffs move into slots as they free up."""
        if self._stale or self._declined or self._closed or not self.early_fold:
            return
        plan, certain = self._plan()
        target = plan[:certain]
        if _common_prefix(self._folded, target) < len(self._folded):
            return  # the folded prefix is not the plan's prefix any more: the close re-folds
        run: List = []
        for w in target[len(self._folded):]:
            if w not in self._slot_of:
                if w not in self._parked:
                    break
                if not self._free and run:
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
        if len(run) >= self.fold_batch:
            self._fold_run(run)

    def _fold_run(self, ws: Sequence):
        slots = [self._slot_of[w] for w in ws]
        if self.mode == WEIGHTED_MEAN and self._weights_by_worker is not None:
            self._weights.extend(float(self._weights_by_worker[w]) for w in ws)
            self.engine.set_weights(self._weights)
        self.engine.fold_slots(self.mode, slots)
        for w in ws:
            del self._slot_of[w]
        self._free.extend(reversed(slots))
        self._folded.extend(ws)
        self._folded_set.update(ws)
        self.folded_early = len(self._folded)

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
        gives up a later slot and re-reads it).  ``finish`` reads through ``fetch`` exactly when
        this is True (its ``fetch`` guard enforces it)."""
        if self._stale:
            return True
        common = _common_prefix(self._folded, order)
        if common < len(self._folded):
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
            if not refold and _common_prefix(self._folded, order) < len(self._folded):
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
            stats = self._fold_in_order(rest, fetch)
            del stats["db_rows"]
            stats.update(refold=bool(refold), reason=refold or None, early=k, n=len(order),
                         folded_before_close=folded_before)
            self.last_close = stats
            new = (state_codec.fresh_checkpoint(self.engine, checkpoint, prepared=prep) if framing == "fresh"
                   else self.engine.ckpt_patch_state(checkpoint))
            self.engine.ckpt_owner = self
            self.engine.ckpt_bytes = new
            return new

    def fetch_plan(self) -> List:
        """After ``seal``: the workers whose diffs ``finish`` will read through ``fetch``, in the
        order it reads them -- the rows to read while the DB snapshot still holds (the node reads
        exactly these under its report gate).  Empty when ``seal`` returned False."""
        with self._lock:
            order = self._close_order
            if order is None:
                raise AggregationError("fetch_plan() without a successful seal()")
            refold = self._stale or _common_prefix(self._folded, order) < len(self._folded)
            return self._fold_in_order(order if refold else order[len(self._folded):], None, dry=True)["db_rows"]

    def _fold(self, ws: Sequence, final: bool, slot_of: dict, free: list, dry: bool):
        slots = [slot_of.pop(w) for w in ws]
        if not dry:
            if self.mode == WEIGHTED_MEAN and self._weights_by_worker is not None and (ws or final):
                self._weights.extend(float(self._weights_by_worker[w]) for w in ws)
                if self._weights:
                    self.engine.set_weights(self._weights)
            if final:
                self.engine.fold_slots_finish_resident(self.mode, slots)
            else:
                self.engine.fold_slots(self.mode, slots)
        free.extend(reversed(slots))
        return slots

    def _fold_in_order(self, rest: List, fetch, dry: bool = False) -> dict:
        """Fold ``rest`` in order and finish into the resident checkpoint, within the slot budget:
        held slots are folded where they stand, other diffs are ingested into free slots; when none
        is free, the pending batch is folded, or -- when the batch is empty and every slot holds a
        later worker's diff -- the slot of the worker needed LAST is given up (its diff is fetched
        from the DB when its turn comes).  ``dry``: the same decisions on copies of the slot maps,
        no engine call and no fetch -- which rows it would read (``fetch_plan``)."""
        slot_of = dict(self._slot_of) if dry else self._slot_of
        free = list(self._free) if dry else self._free
        pos = {w: i for i, w in enumerate(rest)}
        for w in [w for w in slot_of if w not in pos]:  # held, not needed
            free.append(slot_of.pop(w))
        batch: List = []
        db_rows: List = []
        from_hbm = from_host = 0
        for i, w in enumerate(rest):
            if w in slot_of:
                batch.append(w)
                from_hbm += 1
                continue
            diff = self._parked.get(w)
            if diff is None:
                if fetch is None and not dry:
                    raise AggregationError(f"worker {w!r}: no diff held here and no fetch= to read it from the DB")
                db_rows.append(w)
                if not dry:
                    diff = fetch(w)
            else:
                from_host += 1
            if not free:
                if batch:
                    self._fold(batch, False, slot_of, free, dry)
                    batch = []
                else:
                    later = max((x for x in slot_of if pos[x] > i), key=pos.__getitem__)
                    if fetch is None and not dry:
                        raise AggregationError(f"slot budget exhausted and no fetch= to re-read {later!r}")
                    free.append(slot_of.pop(later))
            if dry:
                slot_of[w] = free.pop()
            else:
                self._to_hbm(w, diff)
                self._parked.pop(w, None)
            batch.append(w)
        self._fold(batch, True, slot_of, free, dry)
        return {"from_hbm": from_hbm, "from_host": from_host, "from_db": len(db_rows), "db_rows": db_rows}

    def abandon(self):
        """Another user takes the engine (its slab is re-laid): nothing held here survives.  Later
        reports are ignored and ``close`` raises; the node closes this cycle from its DB rows."""
        if self._closed:  # sealed or closed: its result may be the resident checkpoint
            return
        with self._lock:
            if self._closed:  # closed (or abandoned) already: its result may be the resident checkpoint
                return
            self._closed = True
            self._slot_of.clear()
            self._parked.clear()
            if getattr(self.engine, "ckpt_owner", None) is self:
                self.engine.ckpt_owner = None

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
