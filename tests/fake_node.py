"""Test infrastructure: an in-memory stand-in for the PyGrid Node pieces the engine's wiring
touches.  The reference node itself is not importable here (syft, flask_sqlalchemy, flask_executor,
gevent are absent; flask and sqlalchemy are present): tests/sql_node.py puts the same bookkeeping
on real SQLAlchemy tables (``make_node(warehouse=...)``).

* ``Warehouse`` -- ``core/warehouse.py`` over a list of rows: ``register`` (autoincrement id),
  ``query`` / ``first`` / ``count`` / ``last`` / ``modify`` / ``update``.  ``query`` returns rows
  in ``row_order`` (default: id order, what SQLite returns for ``filter_by().all()``; a test can
  hand another order to stand for a DB that returns rows in another physical order).
* ``CycleManager`` -- the reference's cycle bookkeeping (``cycle_manager.py:28-54, 109-125,
  151-217``) and its ``_average_plan_diffs`` (``:219-323``) with the arithmetic done the
  reference's way in torch (``reduce(th.add)``, ``th.div`` by the python int, ``model_param -
  diff_param``; iterative: the hosted plan called as at ``:266-269``) over the build's State
  codec (syft is absent; ``pygrid_amd.state_schema``).  The new checkpoint is serialized with the
  checkpoint's framing (``state.serialize_model_params``) so that an engine run with
  ``framing="template"`` must produce the SAME BYTES.
* ``ModelManager`` -- ``model_manager.py:19-77`` (create / save numbering + ``latest`` alias /
  load = ``Warehouse.last`` / get).
* ``run_task_once`` runs the task at once (the executor's thread is not needed for the order of
  events these tests drive).
"""
from __future__ import annotations

import threading
import types
from datetime import datetime, timedelta
from functools import reduce

import numpy as np


class Row(types.SimpleNamespace):
    pass


class Warehouse:
    def __init__(self, name):
        self.name = name
        self.rows = []
        self.next_id = 1
        self.row_order = None  # callable(list of rows) -> list in "physical" order, or None (id order)
        self._lock = threading.Lock()  # autoincrement ids under concurrent handlers

    def register(self, **kw):
        with self._lock:
            r = Row(id=self.next_id, **kw)
            self.next_id += 1
            self.rows.append(r)
        return r

    def _match(self, kw):
        return [r for r in list(self.rows) if all(getattr(r, k, None) == v for k, v in kw.items())]

    def query(self, **kw):
        got = self._match(kw)
        return self.row_order(got) if self.row_order else got

    def first(self, **kw):
        got = self.query(**kw)
        return got[0] if got else None

    def last(self, **kw):
        got = sorted(self._match(kw), key=lambda r: r.id)
        return got[-1] if got else None

    def count(self, **kw):
        return len(self._match(kw))

    def modify(self, query, values):
        for r in self._match(query):
            for k, v in values.items():
                setattr(r, k, v)

    def update(self):
        pass


class ModelNotFoundError(Exception):
    pass


class ModelManager:
    def __init__(self, warehouse=Warehouse):
        self._models = warehouse("model")
        self._model_checkpoints = warehouse("checkpoint")
        self.db_loads = 0

    def create(self, model, process):  # model_manager.py:19-28
        m = self._models.register(fl_process_id=process.id)
        self._model_checkpoints.register(value=model, model_id=m.id, number=1, alias="latest")
        return m

    def save(self, model_id, data):  # :30-51
        n = self._model_checkpoints.count(model_id=model_id)
        self._model_checkpoints.modify({"model_id": model_id, "alias": "latest"}, {"alias": ""})
        return self._model_checkpoints.register(model_id=model_id, value=data, number=n + 1, alias="latest")

    def load(self, **kw):  # :53-60
        self.db_loads += 1
        cp = self._model_checkpoints.last(**kw)
        if not cp:
            raise ModelNotFoundError
        return cp

    def get(self, **kw):  # :62-77
        m = self._models.last(**kw)
        if not m:
            raise ModelNotFoundError
        return m


class ProcessManager:
    def __init__(self):
        self.procs = {}
        self.plans = {}

    def create(self, server_config, avg_plan_bytes=None):
        pid = len(self.procs) + 1
        self.procs[pid] = server_config
        if avg_plan_bytes:
            self.plans[pid] = Row(value=avg_plan_bytes)
        return Row(id=pid, version="1.0")

    def get_configs(self, id=None, **kw):
        return self.procs[id], {}

    def get_plan(self, fl_process_id=None, is_avg_plan=True):
        return self.plans.get(fl_process_id)


def canonical_plan(avg, item, num):  # 01-Create-plan.ipynb:450-454
    return [(a * num + i) / (num + 1) for a, i in zip(avg, item)]


class PlanManager:
    PLANS = {b"ITERATIVE_AVG_PLAN": canonical_plan}

    @staticmethod
    def deserialize_plan(b):
        return PlanManager.PLANS[bytes(b)]


def run_task_once(name, func, *args):  # tasks/cycle.py:9-25, synchronously
    func(*args)


def complete_cycle(cycle_manager, cycle_id):  # tasks/cycle.py:28-37
    try:
        cycle_manager.complete_cycle(cycle_id)
        return True
    except Exception as e:  # noqa: BLE001
        cycle_manager.task_errors.append(e)
        return e


def make_node(warehouse=Warehouse, mod=None):
    """A fresh node: a module-like namespace holding what cycle_manager.py holds (CycleManager,
    run_task_once, complete_cycle, model_manager, process_manager, PlanManager).  ``warehouse(name)``
    makes the tables ("model", "checkpoint", "cycle", "worker_cycle"); ``mod``: fill this object
    (e.g. a module) instead of a new namespace -- its ``run_task_once`` is what submit_worker_diff
    calls, as the reference's module global is."""
    mod = types.SimpleNamespace() if mod is None else mod
    mod.model_manager = ModelManager(warehouse)
    mod.process_manager = ProcessManager()
    mod.PlanManager = PlanManager
    mod.run_task_once = run_task_once
    mod.complete_cycle = complete_cycle

    class CycleManager:
        def __init__(self):
            self._cycles = warehouse("cycle")
            self._worker_cycles = warehouse("worker_cycle")
            self.task_errors = []

        def create(self, fl_process_id, version, cycle_time):  # :28-54
            seq = len(self._cycles.query(fl_process_id=fl_process_id, version=version))
            now = datetime.now()
            end = now + timedelta(seconds=cycle_time) if cycle_time is not None else None
            return self._cycles.register(start=now, end=end, sequence=seq + 1, version=version,
                                         fl_process_id=fl_process_id, is_completed=False)

        def last(self, fl_process_id):
            return self._cycles.last(fl_process_id=fl_process_id, is_completed=False)

        def assign(self, worker, cycle, hash_key):  # :120-125
            return self._worker_cycles.register(worker_id=worker.id, cycle_id=cycle.id, request_key=hash_key,
                                                is_completed=False, diff=None)

        def submit_worker_diff(self, worker_id, request_key, diff):  # :151-178
            wc = self._worker_cycles.first(worker_id=worker_id, request_key=request_key)
            if not wc:
                raise ProcessLookupError
            wc.is_completed = True
            wc.completed_at = datetime.utcnow()
            wc.diff = diff
            self._worker_cycles.update()
            mod.run_task_once("complete_cycle", mod.complete_cycle, self, wc.cycle_id)

        def complete_cycle(self, cycle_id):  # :180-217
            from pygrid_amd.cycle import ready_to_average

            cycle = self._cycles.first(id=cycle_id)
            if cycle.is_completed:
                return
            server_config, _ = mod.process_manager.get_configs(id=cycle.fl_process_id)
            received = self._worker_cycles.count(cycle_id=cycle_id, is_completed=True)
            if ready_to_average(server_config, received, cycle.end, datetime.now()):
                self._average_plan_diffs(server_config, cycle)

        def _average_plan_diffs(self, server_config, cycle):  # :219-323, arithmetic in torch
            import torch as th

            from pygrid_amd import state

            _model = mod.model_manager.get(fl_process_id=cycle.fl_process_id)
            _checkpoint = mod.model_manager.load(model_id=_model.id)
            shapes = [tuple(s) for s in _shapes(_checkpoint.value)]
            model_params = [th.from_numpy(a.copy()) for a in state.unserialize_model_params(_checkpoint.value, shapes)]
            reports = self._worker_cycles.query(cycle_id=cycle.id, is_completed=True)
            diffs = [[th.from_numpy(a.copy()) for a in state.unserialize_model_params(r.diff, shapes)]
                     for r in reports]
            rec = mod.process_manager.get_plan(fl_process_id=cycle.fl_process_id, is_avg_plan=True)
            if rec and rec.value:
                avg_plan = mod.PlanManager.deserialize_plan(rec.value)
                if server_config.get("iterative_plan", False):
                    diff_avg = diffs[0]
                    for i, diff in enumerate(diffs[1:]):
                        diff_avg = avg_plan(list(diff_avg), diff, th.tensor([i + 1]))
                else:
                    diff_avg = avg_plan(diffs)
            else:
                raw = [[d[j] for d in diffs] for j in range(len(model_params))]
                sums = [reduce(th.add, p) for p in raw]
                diff_avg = [th.div(p, len(diffs)) for p in sums]
            new = [m - d for m, d in zip(model_params, diff_avg)]
            flat = np.concatenate([t.numpy().reshape(-1) for t in new]).astype(np.float32)
            mod.model_manager.save(_model.id, state.serialize_model_params(_checkpoint.value, flat))
            cycle.is_completed = True
            self._cycles.update()
            done = self._cycles.count(fl_process_id=cycle.fl_process_id, is_completed=True)
            max_cycles = server_config.get("num_cycles", 0)
            if done < max_cycles or max_cycles == 0:
                self.create(cycle.fl_process_id, cycle.version, server_config.get("cycle_length"))

    mod.CycleManager = CycleManager
    mod.cycle_manager = CycleManager()
    return mod


def _shapes(pb):
    from pygrid_amd.state_schema import tensor_shapes

    return tensor_shapes(pb)


def host_process(mod, server_config, checkpoint: bytes, avg_plan_bytes=None):
    """fl_controller.create_process (fl_controller.py:23-67): process, model + checkpoint #1, cycle."""
    proc = mod.process_manager.create(server_config, avg_plan_bytes)
    model = mod.model_manager.create(checkpoint, proc)
    cyc = mod.cycle_manager.create(proc.id, proc.version, server_config.get("cycle_length"))
    return proc, model, cyc


def assign(mod, worker_id, proc):
    """fl_controller.assign's accepted branch (:104-132): the current cycle, a request key, the row."""
    cyc = mod.cycle_manager.last(proc.id)
    key = f"key-{worker_id}-{cyc.id}"
    mod.cycle_manager.assign(Row(id=worker_id), cyc, key)
    return key
