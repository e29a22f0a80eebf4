"""One opt-in patch that wires the engine into a PyGrid Node.

``install(cycle_manager_module, executor=...)`` replaces, on the node's own objects, the call
sites of the cycle-close path; every endpoint keeps the response the reference gives:

==========================================  ==================================================
reference call site                         what it does after ``install``
==========================================  ==================================================
``CycleManager.assign``                     the DB row as before; the engine learns the row id
(``cycle_manager.py:120-125``, called from  (``IncrementalCycle.assigned``: the fold order the
``fl_controller.py:131-132``)               close-time query will return)
``CycleManager.submit_worker_diff``         the DB write as before; then the diff goes into an
(``cycle_manager.py:151-178``, from         HBM slot at once (``IncrementalCycle.reported``),
``fl_events.py:257-261``)                   THEN the close is requested (never before its ingest)
``run_task_once`` in ``cycle_manager.py``   unchanged by default; ``close_trigger="replay"``:
(``tasks/cycle.py:9-25``)                   ``CycleCloseTrigger`` on the node's Flask-Executor
                                            (replays a request that lands mid-close;
                                            ``deadline=True`` also closes at ``cycle.end``)
``CycleManager._average_plan_diffs``        the report-time fold finished in the DB's query
(``cycle_manager.py:219-323``)              order (``IncrementalCycle.close(order=, fetch=)``),
                                            or the close-time fold over the DB rows
                                            (``CycleAggregator``), or -- for a plan or model
                                            the engine does not implement -- the original
``CycleManager.create`` (``:28-54``)        as before; the next cycle's report-time state is
                                            prepared at once (its checkpoint is already in HBM)
``ModelManager.save`` / ``load``            write-through, bounded ``CheckpointStore`` in front
(``model_manager.py:30-60``; ``load``       of the DB: ``/get-model`` and ``/retrieve-model``
serves ``/get-model`` ``routes.py:183``     (``routes.py:163-201, 471-516``) and the next
and ``/retrieve-model`` ``:498``)           cycle read the newest checkpoints from memory
``base64.b64decode`` in ``fl_events.py``    ``report.b64decode`` into a page-locked block
(``:257``, when ``report_module`` given)    (``PinnedPool``): the diff the DB stores and the
                                            engine DMAs to HBM without a staging copy
==========================================  ==================================================

One engine context is single-owner, so one open cycle at a time folds at report time (the first
one prepared; the next cycle of the same FL process takes over when it closes).  Any other
cycle closes through the close-time path over its DB rows -- bit-identical either way.  After a
node restart the open cycle's state is rebuilt from its WorkerCycle rows: the diffs reported
before the restart are read from the DB at close.

Concurrency (the reference serves handlers on a gevent hub -- ``pywsgi.WSGIServer``,
``apps/node/src/__main__.py:85``, or gunicorn's ``flask_sockets.worker``, ``entrypoint.sh:2`` -- and
closes on Flask-Executor's thread, ``tasks/cycle.py:9-25``): a handler never waits for a close.

* the **report gate** (``_Gate``): a report holds it shared across its DB write and the ingest
  (``submit_worker_diff`` + ``on_report``); a close holds it exclusively only while it reads the
  completed rows and seals the cycle (``IncrementalCycle.seal``) -- the moment the reference's
  query at ``cycle_manager.py:243-250`` reads the diffs.  A re-report lands wholly before the
  snapshot (its diff is the one averaged) or wholly after it (ignored, as by the reference's close
  that already read the rows).  A close that must read diffs from the DB (a re-fold, diffs
  reported before a restart) reads exactly the rows its fold will need while it holds the gate
  (``IncrementalCycle.fetch_plan``), then releases it before folding; a fold that asks for any
  other row fails and the cycle closes through the close-time path instead.  Two closes
  requested inline from two reports at once (a node that calls ``complete_cycle`` from inside
  ``submit_worker_diff``) cannot both upgrade their report's shared hold: the second fails at once
  (``GateUpgradeConflict``) instead of waiting for the first, which waits for it -- and so does an
  inline close that finds the engine lock taken while another close waits for the gate (it
  would otherwise block on the lock while holding the very hold that close waits for);
* after the seal, reports and assignments of the closing cycle return at once (no cycle lock);
* the **engine lock** serialises engine users: closes take it (blocking, on the executor); a
  handler that would prepare a cycle's report-time state while a close holds it skips that
  (``_cycle_state`` returns None) -- the diffs are then read from the DB at that cycle's close.

Nothing runs at import: ``install`` is the opt-in, ``uninstall`` restores every patched name.
"""
from __future__ import annotations

import contextlib
import logging
import threading
from typing import Callable, Dict, Optional, Sequence

from . import state as state_codec
from .checkpoints import Checkpoint, CheckpointStore
from .cycle import CycleAggregator, finish_cycle, hosted_plan, make_average_plan_diffs, select_mode
from .exceptions import AggregationError, ModelNotAcceleratedError, PlanNotAcceleratedError, PyGridError, \
    StateParseError
from .incremental import IncrementalCycle
from .trigger import CycleCloseTrigger

log = logging.getLogger(__name__)

_DECLINED = "declined"   # the engine does not average this cycle (plan / model): the node's code runs
_ELSEWHERE = "elsewhere"  # report-time state not kept for this cycle: close-time path over the DB rows
_BUSY = "busy"  # (_cycle_state only) another thread holds the engine: nothing decided for the cycle yet


def completed_rows(cm, cycle_id):
    """The completed WorkerCycles of the cycle in the order ``cycle_manager.py:243-245`` reads them
    (the same ``filter_by(cycle_id=..., is_completed=True)`` query).  With SQLAlchemy the ``diff``
    column is deferred: the blobs are read only for the diffs the engine does not already hold."""
    return _rows(cm, cycle_id=cycle_id, is_completed=True)


def _deferred(cm):
    """``WorkerCycle.query`` with the ``diff`` blob deferred (SQLAlchemy), or None."""
    schema = getattr(cm._worker_cycles, "_schema", None)
    q = getattr(schema, "query", None)
    if q is not None and hasattr(schema, "diff"):
        try:
            from sqlalchemy.orm import defer

            return q.options(defer(schema.diff))
        except ImportError:
            pass
    return None


def _rows(cm, **filters):
    q = _deferred(cm)
    return q.filter_by(**filters).all() if q is not None else cm._worker_cycles.query(**filters)


def _first_row(cm, **filters):
    """``Warehouse.first`` without reading the row's diff back (the handler just wrote it)."""
    q = _deferred(cm)
    return q.filter_by(**filters).first() if q is not None else cm._worker_cycles.first(**filters)


class NodeEngine:
    """What ``install`` wires in (see the module docstring).  Attributes: ``aggregator``
    (close-time path), ``engine``, ``store`` (checkpoint cache), ``trigger`` (or None), ``stats``."""

    def __init__(self, cm_module, executor=None, engine=None, devices: Optional[Sequence[int]] = None,
                 report_time: bool = True, close_trigger: str = "reference", deadline: bool = False,
                 keep_checkpoints: int = 4, slots: Optional[int] = None, fold_batch: int = 8,
                 mean_plans: Optional[str] = None, framing: str = "fresh", report_module=None,
                 pinned_reports: int = 16):
        if close_trigger not in ("reference", "replay"):
            raise AggregationError(f"close_trigger must be 'reference' or 'replay', not {close_trigger!r}")
        if deadline and close_trigger != "replay":
            raise AggregationError("deadline=True needs close_trigger='replay'")
        self.mod = cm_module
        self.model_manager = cm_module.model_manager
        self.process_manager = cm_module.process_manager
        self.plan_manager = cm_module.PlanManager
        self.aggregator = CycleAggregator(engine, devices=devices, mean_plans=mean_plans) if engine is not None \
            or devices is not None else CycleAggregator(mean_plans=mean_plans)
        self.engine = self.aggregator.engine
        self.report_time = report_time
        self.close_trigger = close_trigger
        self.deadline = deadline
        self.slots = slots
        self.fold_batch = fold_batch
        self.framing = framing
        self.store = CheckpointStore(keep=keep_checkpoints) if keep_checkpoints else None
        self.report_module = report_module
        self.pinned = None
        if report_module is not None:
            from .report import PinnedPool

            self.pinned = PinnedPool(max_blocks=pinned_reports) if pinned_reports else None
        self.trigger = CycleCloseTrigger(lambda fn, *a: fn(*a), executor=executor) if close_trigger == "replay" \
            else None
        self._cycles: Dict[object, object] = {}  # cycle id -> IncrementalCycle | _DECLINED | _ELSEWHERE
        # (worker id, request key) -> (WorkerCycle id, cycle id) of the rows assigned through this
        # process: a report finds its row without a DB query (rows assigned before a restart: queried).
        # Kept per cycle (_assigned_keys), dropped when the cycle closes or loses its report-time state.
        self._assigned: Dict[tuple, tuple] = {}
        self._assigned_keys: Dict[object, list] = {}
        # assignments whose handler found the engine busy before the cycle had its state: recorded
        # into the state when it is made (a cycle just created is built without a rows query)
        self._pending_assign: Dict[object, list] = {}
        self._owner = None  # the cycle id whose IncrementalCycle holds the engine
        self._lock = threading.RLock()  # the maps above; held only briefly
        self._gate = _Gate()  # reports (shared) vs a close's snapshot of the rows (exclusive)
        self._engine_lock = threading.RLock()  # closes / cycle preparation vs each other
        self._hold = threading.local()
        self._patched: list = []
        self.stats = {"closes_report_time": 0, "closes_close_time": 0, "closes_declined": 0, "refolds": 0,
                      "diffs_from_db": 0, "report_errors": 0, "gate_conflicts": 0}

    # ---- patching ------------------------------------------------------------------------------
    def _patch(self, owner, name, value):
        """Set ``owner.name`` (a class, a module or an instance), remembering what its own namespace
        held (nothing, for an inherited or class-level attribute: uninstall then deletes ours)."""
        self._patched.append((owner, name, vars(owner).get(name, _MISSING)))
        setattr(owner, name, value)

    def install(self):
        CM = self.mod.CycleManager
        node = self
        orig = {n: getattr(CM, n) for n in ("assign", "submit_worker_diff", "_average_plan_diffs", "create")}
        orig_run = self.mod.run_task_once
        close_time = make_average_plan_diffs(self.aggregator, self.model_manager, self.process_manager,
                                             self.plan_manager, original=orig["_average_plan_diffs"],
                                             gate=self._gate.exclusive, framing=self.framing)

        def assign(cm, worker, cycle, hash_key):
            wc = orig["assign"](cm, worker, cycle, hash_key)
            node.on_assign(cm, cycle, wc, key=(getattr(worker, "id", None), hash_key))
            return wc

        def submit_worker_diff(cm, worker_id, request_key, diff):
            with node._gate.shared(), node._holding_triggers() as held:
                orig["submit_worker_diff"](cm, worker_id, request_key, diff)  # the DB write, :162-174
                node.on_report(cm, worker_id, request_key, diff)
            for name, func, args in held:  # :176-178, after the diff is in HBM
                node.run_task_once(name, func, *args)

        def _average_plan_diffs(cm, server_config, cycle):
            return node.average_plan_diffs(cm, server_config, cycle, close_time, orig["_average_plan_diffs"])

        def create(cm, fl_process_id, version, cycle_time):
            cyc = orig["create"](cm, fl_process_id, version, cycle_time)
            node.on_cycle_created(cm, cyc)
            return cyc

        def run_task_once(name, func, *args):
            if getattr(node._hold, "queue", None) is not None:
                node._hold.queue.append((name, func, args))
                return None
            return node.run_task_once(name, func, *args)

        self._orig_run = orig_run
        self._patch(CM, "_average_plan_diffs", _average_plan_diffs)
        self._patch(CM, "submit_worker_diff", submit_worker_diff)
        self._patch(self.mod, "run_task_once", run_task_once)
        if self.report_time:
            self._patch(CM, "assign", assign)
            self._patch(CM, "create", create)
        if self.store is not None:
            mm = self.model_manager
            orig_save, orig_load = mm.save, mm.load

            def save(model_id, data):
                cp = orig_save(model_id, data)
                node.store.put(_as_checkpoint(cp, model_id, data))
                return cp

            def load(**kwargs):
                hit = node.store.lookup(**kwargs)
                if hit is not None:
                    return hit
                cp = orig_load(**kwargs)
                if set(kwargs) <= {"model_id", "alias"} and kwargs.get("alias", "latest") == "latest":
                    node.store.seed(_as_checkpoint(cp, kwargs["model_id"], cp.value))  # newest of the model
                return cp

            self._patch(mm, "save", save)
            self._patch(mm, "load", load)
        if self.report_module is not None:
            self._patch(self.report_module, "base64", _Base64(self.pinned))
        return self

    def uninstall(self):
        with self._lock:
            self._abandon_others()  # nothing of theirs touches the engine after this
        for owner, name, old in reversed(self._patched):
            if old is _MISSING:
                delattr(owner, name)
            else:
                setattr(owner, name, old)
        self._patched.clear()
        if self.trigger is not None:
            self.trigger.shutdown()
        if self.pinned is not None:
            self.pinned.close()

    # ---- run_task_once ---------------------------------------------------------------------------
    @contextlib.contextmanager
    def _holding_triggers(self):
        """run_task_once calls made inside are queued, and dispatched by the caller afterwards."""
        prev = getattr(self._hold, "queue", None)
        self._hold.queue = []
        try:
            yield self._hold.queue
        finally:
            self._hold.queue = prev

    def run_task_once(self, name, func, *args):
        if self.trigger is not None and name == "complete_cycle":
            return self.trigger.request(func, *args)
        return self._orig_run(name, func, *args)

    # ---- report-time state -------------------------------------------------------------------
    def _cycle_state(self, cm, cycle, create: bool = True, fresh: bool = False):
        """The cycle's IncrementalCycle (made on first use, from its DB rows after a restart), or a
        marker saying why there is none.  _BUSY (nothing recorded, retried on the next call) while
        another thread holds the engine -- a close, or this cycle's state being built: a handler
        does not wait for it."""
        got = self._cycles.get(cycle.id)
        if got is not None or not create:
            return got
        if not self.report_time or getattr(cycle, "is_completed", False):
            return None
        if not self._engine_lock.acquire(blocking=False):
            return _BUSY
        try:  # the engine lock keeps builders and closes apart; self._lock is held only briefly
            with self._lock:
                got = self._cycles.get(cycle.id)
                if got is not None:
                    return got
                if self._owner is not None and self._owner != cycle.id and \
                        isinstance(self._cycles.get(self._owner), IncrementalCycle):
                    self._set_elsewhere(cycle.id)  # the engine serves another open cycle
                    return _ELSEWHERE
            try:
                inc = self._new_cycle(cm, cycle, fresh)
            except PlanNotAcceleratedError as e:
                log.info("cycle %s: %s -- the node averages it", cycle.id, e)
                with self._lock:
                    self._cycles[cycle.id] = _DECLINED
                    self._drop_assigned(cycle.id)
                return _DECLINED
            with self._lock:
                self._cycles[cycle.id] = inc
                self._owner = cycle.id
                for row_id, key in self._pending_assign.pop(cycle.id, ()):
                    self._record_assign(inc, cycle.id, row_id, key)
                return inc
        finally:
            self._engine_lock.release()

    def _new_cycle(self, cm, cycle, fresh: bool = False) -> IncrementalCycle:
        server_config, _ = self.process_manager.get_configs(id=cycle.fl_process_id)
        avg_plan, plan_key = hosted_plan(server_config, cycle, self.process_manager, self.plan_manager,
                                         self.aggregator.mean_plans)
        model = self.model_manager.get(fl_process_id=cycle.fl_process_id)
        ckpt = self.model_manager.load(model_id=model.id).value
        try:
            numel = state_codec.tensor_numels(ckpt)
        except StateParseError:
            from .cycle import _decline_non_float32

            _decline_non_float32(ckpt, "the checkpoint")
            raise
        mode = select_mode(server_config, avg_plan, plan_key=plan_key, mean_plans=self.aggregator.mean_plans,
                           shapes=lambda: _shapes(ckpt))
        self.aggregator._resident = None  # the report-time cycle takes over the engine's slab
        inc = IncrementalCycle(self.engine, numel, mode=mode, slots=self.slots, fold_batch=self.fold_batch,
                               checkpoint=ckpt)
        if not fresh:  # after a restart: the rows assigned before it (a cycle just created has none;
            # an assignment that lands while this state is built is recorded from _pending_assign)
            for row in _rows(cm, cycle_id=cycle.id):
                inc.assigned(row.id, key=row.id)
        return inc

    def on_cycle_created(self, cm, cycle):
        if self.trigger is not None and self.deadline:
            self.trigger.schedule_deadline(cycle.id, getattr(cycle, "end", None),
                                           args=(self._task_fn(), cm, cycle.id))
        try:
            self._cycle_state(cm, cycle, fresh=True)
        except Exception as e:  # noqa: BLE001 -- preparing early is an optimisation only
            log.warning("cycle %s: report-time state not prepared (%s); close-time path", cycle.id, e)
            with self._lock:
                self._set_elsewhere(cycle.id)

    def _task_fn(self):
        """The task ``submit_worker_diff`` hands to ``run_task_once`` (``tasks/cycle.py:28-37``,
        imported into ``cycle_manager.py:18``)."""
        return self.mod.complete_cycle

    def on_assign(self, cm, cycle, wc, key=None):
        """After the reference's DB write of the assignment.  Never raises: the response stays the
        reference's (a cycle whose report-time state cannot be made closes from its DB rows)."""
        try:
            st = self._cycle_state(cm, cycle)
        except Exception as e:  # noqa: BLE001
            log.warning("cycle %s: report-time state not prepared at an assignment (%s); close-time path",
                        cycle.id, e)
            with self._lock:
                self._set_elsewhere(cycle.id)
            return
        if st is _BUSY:
            with self._lock:
                st = self._cycles.get(cycle.id)
                if st is None:  # its state is not made yet: recorded into it when it is
                    self._pending_assign.setdefault(cycle.id, []).append((wc.id, key))
                    return
        if isinstance(st, IncrementalCycle):
            with self._lock:
                if self._cycles.get(cycle.id) is st:  # not closed or abandoned meanwhile
                    self._record_assign(st, cycle.id, wc.id, key)

    def _record_assign(self, inc, cycle_id, row_id, key):
        """(under self._lock) the engine learns the row; the report finds it without a query."""
        inc.assigned(row_id, key=row_id)
        if key is not None and key[0] is not None:
            self._assigned[key] = (row_id, cycle_id)
            self._assigned_keys.setdefault(cycle_id, []).append(key)

    def on_report(self, cm, worker_id, request_key, diff):
        """After the reference's DB write.  Never raises: the response stays the reference's, and a
        diff the engine could not take is read from the DB at close."""
        try:
            hit = self._assigned.get((worker_id, request_key))
            if hit is None:
                wc = _first_row(cm, worker_id=worker_id, request_key=request_key)
                hit = (wc.id, wc.cycle_id)
            row_id, cycle_id = hit
            st = self._cycles.get(cycle_id)
            if st is None and self.report_time:
                cycle = cm._cycles.first(id=cycle_id)
                st = self._cycle_state(cm, cycle) if cycle is not None else None
            if isinstance(st, IncrementalCycle):
                st.reported(row_id, diff)
        except (PyGridError, StateParseError) as e:
            self.stats["report_errors"] += 1
            log.warning("report of worker %s kept for the close-time read (%s)", worker_id, e)
        except Exception as e:  # noqa: BLE001 -- never change the report's response
            self.stats["report_errors"] += 1
            log.error("report of worker %s: engine error %s; the close reads it from the DB", worker_id, e)

    # ---- close ---------------------------------------------------------------------------------
    def average_plan_diffs(self, cm, server_config, cycle, close_time: Callable, original: Callable):
        """The close (executor thread).  Holds the engine lock throughout, the report gate only for
        the snapshot of the completed rows (see the module docstring)."""
        with self._engine_for_close():
            model = ckpt = None
            if isinstance(self._cycles.get(cycle.id), IncrementalCycle):
                model = self.model_manager.get(fl_process_id=cycle.fl_process_id)
                ckpt = self.model_manager.load(model_id=model.id)
            try:
                self._gate.acquire_exclusive()  # no report is between its DB write and its ingest now
            except GateUpgradeConflict as e:
                self.stats["gate_conflicts"] += 1
                log.warning("close of cycle %s not run: %s", cycle.id, e)
                raise
            try:
                with self._lock:
                    st = self._cycles.pop(cycle.id, None)
                    self._drop_assigned(cycle.id)
                    if self._owner == cycle.id:
                        self._owner = None
                    if not isinstance(st, IncrementalCycle) and st != _DECLINED:
                        self._abandon_others()  # the close-time path re-lays the engine's slab
            except BaseException:
                self._gate.release_exclusive()
                raise
            if not isinstance(st, IncrementalCycle):
                self._gate.release_exclusive()  # the close-time path takes it for its own query
                if st == _DECLINED:
                    self.stats["closes_declined"] += 1
                    return original(cm, server_config, cycle)
                self.stats["closes_close_time"] += 1
                return close_time(cm, server_config, cycle)
            gated, fallback = True, None
            try:
                if ckpt is None:
                    model = self.model_manager.get(fl_process_id=cycle.fl_process_id)
                    ckpt = self.model_manager.load(model_id=model.id)
                rows = completed_rows(cm, cycle.id)
                blobs = {}
                if st.seal(order=[r.id for r in rows]):
                    # the diffs the fold will read from the DB, read now -- as the reference's query
                    # reads every diff -- so that no re-report lands between the snapshot and them
                    by_id = {r.id: r for r in rows}
                    blobs = {rid: by_id[rid].diff for rid in st.fetch_plan()}
                self._gate.release_exclusive()  # the fold needs no DB row beyond `blobs`
                gated = False
                new = st.finish(ckpt.value, framing=self.framing, fetch=_only(blobs))
            except PlanNotAcceleratedError as e:  # incl. ModelNotAcceleratedError: a non-float32 diff
                log.info("engine declined cycle %s (%s): running the reference averaging", cycle.id, e)
                fallback = "original"
            except AggregationError as e:
                log.warning("report-time close of cycle %s failed (%s): close-time path over the DB rows",
                            cycle.id, e)
                fallback = "close_time"
            finally:
                if gated:
                    self._gate.release_exclusive()
            # the fallbacks run outside the try: their own errors reach complete_cycle's log, once
            if fallback == "original":
                self.stats["closes_declined"] += 1
                return original(cm, server_config, cycle)
            if fallback == "close_time":
                self.aggregator._resident = None
                self.stats["closes_close_time"] += 1
                return close_time(cm, server_config, cycle)
            self.stats["closes_report_time"] += 1
            self.stats["refolds"] += int(st.last_close.get("refold", False))
            self.stats["diffs_from_db"] += st.last_close.get("from_db", 0)
            self.aggregator._resident = None
            finish_cycle(cm, server_config, cycle, self.model_manager, model.id, new)

    @contextlib.contextmanager
    def _engine_for_close(self):
        """The engine lock for a close.  A close on the executor waits for it.  A close run inline
        inside a report holds that report's shared gate hold: blocking on the engine lock there
        deadlocks against a close that holds the lock and waits for the exclusive gate -- i.e. for
        this very hold.  So an inline close polls the lock and gives up (``GateUpgradeConflict``)
        as soon as another close is waiting for the gate; its handler then ends and lets that close
        run."""
        if not self._gate.held_here():
            with self._engine_lock:
                yield
            return
        while not self._engine_lock.acquire(timeout=0.002):
            if self._gate.exclusive_wanted():
                self.stats["gate_conflicts"] += 1
                raise GateUpgradeConflict("another close holds the engine and waits for this report's hold on "
                                          "the report gate")
        try:
            yield
        finally:
            self._engine_lock.release()

    def _abandon_others(self):
        for cid, st in list(self._cycles.items()):
            if isinstance(st, IncrementalCycle):
                st.abandon()
                self._set_elsewhere(cid)
        self._owner = None

    def _set_elsewhere(self, cycle_id):
        self._cycles[cycle_id] = _ELSEWHERE
        self._drop_assigned(cycle_id)

    def _drop_assigned(self, cycle_id):
        """Forget the row lookups of a cycle that closes or has no report-time state (its reports
        then find their row with one query, as after a restart)."""
        self._pending_assign.pop(cycle_id, None)
        for k in self._assigned_keys.pop(cycle_id, ()):
            if self._assigned.get(k, (None, None))[1] == cycle_id:
                del self._assigned[k]


def _only(blobs: dict):
    """``fetch`` for a finish after the gate was released: the rows read under it, nothing else."""
    def fetch(rid):
        try:
            return blobs[rid]
        except KeyError:
            raise AggregationError(f"the fold asked for row {rid!r}, which was not read under the report gate") \
                from None
    return fetch


class GateUpgradeConflict(AggregationError):
    """A second close tried to upgrade its report's shared hold while another upgrade was pending."""


class _Gate:
    """Shared (reports: DB write + ingest) / exclusive (a close's snapshot of the rows) lock.  A
    waiting close keeps new reports out, so it waits only for the reports already in flight.  A
    close requested synchronously from inside a report (a node that runs ``complete_cycle`` inline
    instead of through the patched ``run_task_once``) upgrades: it waits for the OTHER reports in
    flight, never for its own handler.  One upgrade at a time: two upgraders would each wait for
    the other's shared hold, so a second one raises ``GateUpgradeConflict`` at once."""

    def __init__(self):
        self._cv = threading.Condition(threading.Lock())
        self._shared = 0
        self._exclusive = False
        self._waiting = 0
        self._upgrading = False  # an upgrade is waiting for, or holds, the exclusive side
        self._held_by_upgrade = False
        self._mine = threading.local()  # shared holds of this thread

    @contextlib.contextmanager
    def shared(self):
        with self._cv:
            while (self._exclusive or self._waiting) and not getattr(self._mine, "n", 0):
                self._cv.wait()
            self._shared += 1
        self._mine.n = getattr(self._mine, "n", 0) + 1
        try:
            yield
        finally:
            self._mine.n -= 1
            with self._cv:
                self._shared -= 1
                if not self._shared:
                    self._cv.notify_all()
                elif self._waiting:
                    self._cv.notify_all()

    def held_here(self) -> bool:
        """Whether this thread holds the gate shared (a report handler, or a close run inside one)."""
        return getattr(self._mine, "n", 0) > 0

    def exclusive_wanted(self) -> bool:
        """Whether a close waits for (or holds) the exclusive side."""
        with self._cv:
            return bool(self._waiting or self._exclusive)

    def acquire_exclusive(self):
        mine = getattr(self._mine, "n", 0)
        with self._cv:
            if mine:
                if self._upgrading:
                    raise GateUpgradeConflict("another close is upgrading its report's hold on the report gate")
                self._upgrading = True
            self._waiting += 1
            try:
                while self._exclusive or self._shared - mine:
                    self._cv.wait()
            except BaseException:
                self._upgrading = self._upgrading and not mine
                raise
            finally:
                self._waiting -= 1
            self._exclusive = True
            self._held_by_upgrade = bool(mine)

    def release_exclusive(self):
        with self._cv:
            self._exclusive = False
            if self._held_by_upgrade:
                self._upgrading = self._held_by_upgrade = False
            self._cv.notify_all()

    @contextlib.contextmanager
    def exclusive(self):
        self.acquire_exclusive()
        try:
            yield
        finally:
            self.release_exclusive()


class _Base64:
    """Stands for the ``base64`` module inside ``fl_events``: ``b64decode(text)`` (``:257``) decodes
    natively, into a page-locked block when the pool has one; everything else is ``base64``'s."""

    def __init__(self, pool):
        self._pool = pool

    def b64decode(self, s, *args, **kwargs):
        if args or kwargs:  # altchars / validate: not what the report handler uses
            import base64

            return base64.b64decode(s, *args, **kwargs)
        from .report import b64decode

        return b64decode(s, into=self._pool)

    def __getattr__(self, name):
        import base64

        return getattr(base64, name)


class _Missing:
    pass


_MISSING = _Missing()


def _as_checkpoint(cp, model_id, value) -> Checkpoint:
    state = getattr(cp, "_sa_instance_state", None)
    if state is not None and state.key is not None and state.session is not None and "number" not in cp.__dict__:
        # A ModelCheckPoint the save's commit expired (expire_on_commit): reading any attribute would
        # reload the whole row, its 47 MB blob included -- 55-60 ms per close for a value we hold.
        # Read the small columns alone; the id is the identity key (no query).
        cls = type(cp)
        ident = state.key[1][0]
        number, alias, mid = state.session.query(cls.number, cls.alias, cls.model_id).filter(cls.id == ident).one()
        return Checkpoint(id=ident, model_id=mid, number=number, alias=alias, value=value)
    return Checkpoint(id=getattr(cp, "id", 0), model_id=getattr(cp, "model_id", model_id),
                      number=getattr(cp, "number", 0), alias=getattr(cp, "alias", "latest"), value=value)


def _shapes(pb: bytes):
    from .state_schema import tensor_shapes

    return tensor_shapes(pb)


def install(cycle_manager_module, executor=None, **options) -> NodeEngine:
    """Wire the engine into the node whose ``cycle_manager`` module is given (it holds
    ``CycleManager``, ``run_task_once``, and the ``model_manager`` / ``process_manager`` /
    ``PlanManager`` singletons it uses).  ``executor``: the node's Flask-Executor (for
    ``close_trigger="replay"``).  Options: see ``NodeEngine``.  Returns the NodeEngine
    (``.uninstall()`` undoes it)."""
    return NodeEngine(cycle_manager_module, executor=executor, **options).install()


def install_into_node(package: str = "src.app", **options) -> NodeEngine:
    """``install`` for the node app as shipped (``apps/node``: ``python -m src`` imports it as
    ``src.app``)."""
    from importlib import import_module

    cm_module = import_module(f"{package}.main.model_centric.cycles.cycle_manager")
    fl_events = import_module(f"{package}.main.events.model_centric.fl_events")
    app = import_module(package)
    options.setdefault("report_module", fl_events)
    return install(cm_module, executor=getattr(app, "executor", None), **options)
