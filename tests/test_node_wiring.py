"""CPU: pygrid_amd.node.install wires report-time aggregation, the close trigger and the checkpoint
cache into a node -- and the node then saves BYTE-IDENTICAL checkpoints to
the reference's own close over its DB rows (cycle_manager.py:219-323), whatever the reports do:
re-reports before and after their early fold, late reports, a restart mid-cycle, assignments
announced out of row order, a DB that returns rows in another order, malformed diffs.

The node is tests/fake_node.py (the reference's bookkeeping restated in memory, arithmetic in
torch the reference's way); the engine is tests/fake_engine.py (the library's slot semantics in
numpy, folds by the C oracle).  Every scenario runs twice on fresh nodes -- once as shipped
(reference), once after install() -- and the saved checkpoints are compared byte for byte."""
import threading

import numpy as np
import pytest

from fake_engine import NumpyEngine
from fake_node import assign, host_process, make_node
from pygrid_amd import node as pnode
from pygrid_amd.state_schema import build_state_fast

SHAPES = [(5, 3), (3,), (7,)]
F = np.float32


def ckpt_bytes(seed=0):
    rng = np.random.default_rng(seed)
    return build_state_fast([rng.standard_normal(s).astype(F) for s in SHAPES])


def diff_bytes(worker, version=0):
    import zlib

    rng = np.random.default_rng([version, zlib.crc32(str(worker).encode())])
    return build_state_fast([(rng.standard_normal(s) * 10.0 ** rng.integers(-3, 2)).astype(F) for s in SHAPES])


class Scenario:
    """Drives one node through a script of events; `installed` wires the engine in first."""

    def __init__(self, server_config, installed: bool, plan=None, row_order=None, **opts):
        self.mod = make_node()
        self.cm = self.mod.cycle_manager
        self.installed = installed
        self.opts = {"framing": "template", "fold_batch": 1, **opts}
        self.node = None
        if installed:
            self.node = pnode.install(self.mod, engine=NumpyEngine(), **self.opts)
        if row_order:
            self.cm._worker_cycles.row_order = row_order
        self.proc, self.model, _ = host_process(self.mod, server_config, ckpt_bytes(), plan)
        self.keys = {}

    def assign(self, w):
        self.keys[w] = assign(self.mod, w, self.proc)

    def report(self, w, version=0, payload=None):
        self.cm.submit_worker_diff(w, self.keys[w], payload if payload is not None else diff_bytes(w, version))

    def restart(self):
        """The node process restarts: the engine's state is gone, the DB stays."""
        if self.installed:
            self.node.uninstall()
            self.node = pnode.install(self.mod, engine=NumpyEngine(), **self.opts)

    def checkpoints(self):
        rows = sorted(self.mod.model_manager._model_checkpoints.rows, key=lambda r: r.id)
        return [(r.number, r.alias, r.value) for r in rows]


def both(server_config, script, plan=None, row_order=None, **opts):
    out = []
    for installed in (False, True):
        sc = Scenario(server_config, installed, plan, row_order, **opts)
        script(sc)
        out.append(sc)
    ref, eng = out
    assert len(ref.checkpoints()) >= 2, "the script must close at least one cycle"
    assert eng.checkpoints() == ref.checkpoints()
    assert eng.cm.task_errors == ref.cm.task_errors == []
    return ref, eng


CFG3 = {"min_diffs": 3, "max_diffs": 3, "num_cycles": 0, "cycle_length": None}


def test_plain_cycles_close_at_report_time():
    def script(sc):
        for cyc in range(3):
            for w in range(5):
                sc.assign(f"w{cyc}{w}")
            for w in (3, 0, 1):
                sc.report(f"w{cyc}{w}")
    ref, eng = both(CFG3, script)
    assert eng.node.stats["closes_report_time"] == 3 and eng.node.stats["refolds"] == 0
    assert eng.node.stats["diffs_from_db"] == 0


def test_re_report_before_its_fold_replaces_the_diff():
    def script(sc):
        for w in range(5):
            sc.assign(w)
        sc.report(2)            # not foldable yet (0, 1 outstanding)
        sc.report(2, version=1)  # overwrites the row's diff (cycle_manager.py:173)
        sc.report(0)
        sc.report(1)            # third completed row: close
    ref, eng = both(CFG3, script)
    assert eng.node.stats["refolds"] == 0


def test_re_report_after_its_fold_refolds_from_the_db():
    def script(sc):
        for w in range(5):
            sc.assign(w)
        sc.report(0)            # the fold front: folded at once (fold_batch=1)
        sc.report(0, version=1)  # the DB now holds another diff for row 0
        sc.report(1)
        sc.report(4)
    ref, eng = both(CFG3, script)
    assert eng.node.stats["refolds"] == 1 and eng.node.stats["diffs_from_db"] >= 1


def test_late_report_is_accepted_and_ignored():
    def script(sc):
        for w in range(4):
            sc.assign(w)
        for w in (0, 1, 2):
            sc.report(w)        # closes cycle 1
        sc.report(3)            # late: stored in the DB, complete_cycle returns early (:186-188)
        for w in range(10, 14):
            sc.assign(w)
        for w in (13, 11, 10):
            sc.report(w)        # cycle 2 closes normally
    ref, eng = both(CFG3, script)
    assert len(ref.checkpoints()) == 3


def test_restart_mid_cycle_reads_earlier_reports_from_the_db():
    def script(sc):
        for w in range(6):
            sc.assign(w)
        sc.report(1)
        sc.report(0)            # folded early before the restart
        sc.restart()
        sc.assign(6)
        sc.report(5)            # third completed row: close on the new engine state
    ref, eng = both(CFG3, script)
    assert eng.node.stats["diffs_from_db"] == 2


def test_assignments_announced_out_of_row_order():
    """Two cycle_request handlers: row A is inserted before row B, but the engine hears of B first
    (and B reports and is folded early): the DB order still wins."""
    def script(sc):
        cyc = sc.cm.last(sc.proc.id)
        if sc.installed:  # A's row exists, the engine is not told yet
            row_a = sc.cm._worker_cycles.register(worker_id="A", cycle_id=cyc.id, request_key="kA",
                                                  is_completed=False, diff=None)
            sc.keys["A"] = "kA"
        else:
            sc.assign("A")
        sc.assign("B")
        sc.report("B")
        if sc.installed:
            sc.node.on_assign(sc.cm, cyc, row_a)
        sc.assign("C")
        sc.report("C")
        sc.report("A")
    ref, eng = both(CFG3, script)
    assert eng.node.stats["refolds"] == 1


@pytest.mark.parametrize("order", ["reversed", "scrambled"])
def test_db_returning_rows_in_another_order(order):
    """cycle_manager.py:243-245 has no ORDER BY: whatever order the DB returns is the fold order
    (a DB returning updated rows in their new physical place, say)."""
    def row_order(rows):
        return rows[::-1] if order == "reversed" else sorted(rows, key=lambda r: (r.id * 5) % 7)

    def script(sc):
        for w in range(6):
            sc.assign(w)
        for w in (0, 1, 4):
            sc.report(w)
    ref, eng = both(CFG3, script, row_order=row_order)
    assert eng.node.stats["refolds"] == 1


def test_iterative_plan_and_slot_pressure():
    cfg = {"min_diffs": 6, "max_diffs": 6, "num_cycles": 0, "cycle_length": None, "iterative_plan": True}

    def script(sc):
        for w in range(9):
            sc.assign(w)
        for w in (8, 6, 5, 0, 2, 1):
            sc.report(w)
    ref, eng = both(cfg, script, plan=b"ITERATIVE_AVG_PLAN", slots=2)
    assert eng.node.stats["closes_report_time"] == 1


def test_malformed_diff_fails_the_close_like_the_reference():
    """The reference stores a malformed diff and its close raises in unserialize (the task logs it,
    the cycle stays open); the engine path reads the same bytes from the DB and raises too."""
    errs = []
    for installed in (False, True):
        sc = Scenario(CFG3, installed)
        for w in range(3):
            sc.assign(w)
        sc.report(0)
        sc.report(1, payload=b"\x0a\xff\xff")  # truncated
        sc.report(2)
        errs.append(len(sc.cm.task_errors))
        assert len(sc.checkpoints()) == 1  # no new checkpoint
    assert errs == [1, 1]


def test_randomised_report_sequences():
    """Random assignment / report / re-report / late-report / restart scripts, random DB orders:
    the installed node (certain-only report-time folds) saves the shipped node's checkpoints."""
    totals = {"closes_report_time": 0, "refolds": 0, "diffs_from_db": 0}
    for trial in range(40):
        rng = np.random.default_rng(100 + trial)
        n = int(rng.integers(3, 9))
        need = int(rng.integers(1, n + 1))
        cfg = {"min_diffs": need, "max_diffs": need, "num_cycles": 0, "cycle_length": None}
        ops = []
        for cyc in range(int(rng.integers(1, 4))):
            ws = [f"c{cyc}w{i}" for i in range(n)]
            ops += [("assign", w) for w in ws]
            reporters = list(rng.permutation(ws))
            for w in reporters[:need + 1]:
                ops.append(("report", w, 0))
                if rng.random() < 0.3:
                    ops.append(("report", w, 1))
                if rng.random() < 0.1:
                    ops.append(("restart",))
        reverse = rng.random() < 0.3
        fb = int(rng.integers(1, 4))
        slots = int(rng.integers(2, n + 2))

        def script(sc):
            for op in ops:
                if op[0] == "assign":
                    sc.assign(op[1])
                elif op[0] == "report":
                    sc.report(op[1], op[2])
                else:
                    sc.restart()
        res = []
        for installed in (False, True):
            sc = Scenario(cfg, installed, row_order=(lambda r: r[::-1]) if reverse else None,
                          **({"fold_batch": fb, "slots": slots} if installed else {}))
            script(sc)
            res.append(sc.checkpoints())
        assert len(res[0]) >= 2 and res[0] == res[1], trial
        for k in totals:
            totals[k] += sc.node.stats[k]
    # the scripts did exercise every path
    assert totals["closes_report_time"] >= 40 and totals["refolds"] >= 3 and totals["diffs_from_db"] >= 3, totals


def test_checkpoint_cache_serves_get_model_and_stays_bounded():
    sc = Scenario(CFG3, True, keep_checkpoints=2)
    for cyc in range(5):
        for w in range(3):
            sc.assign(f"{cyc}-{w}")
        for w in range(3):
            sc.report(f"{cyc}-{w}")
    mm = sc.mod.model_manager
    db = mm._model_checkpoints
    newest = db.last(model_id=sc.model.id)
    loads = mm.db_loads
    got = mm.load(model_id=sc.model.id)                   # /get-model (routes.py:183)
    assert got.value is newest.value and got.number == newest.number == 6
    assert mm.load(model_id=sc.model.id, alias="latest").value is newest.value  # /retrieve-model
    assert mm.load(model_id=sc.model.id, number=5).value == db.last(model_id=sc.model.id, number=5).value
    assert mm.db_loads == loads                           # all three from memory
    assert mm.load(model_id=sc.model.id, number=1).value == ckpt_bytes()  # older than the cache: the DB
    assert mm.db_loads == loads + 1
    assert len(sc.node.store._by_model[sc.model.id]) == 2
    sc.node.uninstall()
    assert mm.load(model_id=sc.model.id).value is newest.value and mm.db_loads == loads + 2


def test_replay_trigger_runs_on_the_executor():
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(1, thread_name_prefix="executor") as ex:
        sc = Scenario(CFG3, False)
        seen = []
        orig = sc.mod.complete_cycle

        def task(cm, cid):
            seen.append(threading.current_thread().name)
            return orig(cm, cid)
        sc.mod.complete_cycle = task
        sc.node = pnode.install(sc.mod, engine=NumpyEngine(), executor=ex, close_trigger="replay", framing="template")
        for w in range(3):
            sc.assign(w)
        for w in range(3):
            sc.report(w)
        assert sc.node.trigger.wait_idle(5)
        assert len(sc.checkpoints()) == 2 and all(n.startswith("executor") for n in seen)
    with pytest.raises(Exception):
        pnode.install(make_node(), engine=NumpyEngine(), deadline=True)  # deadline needs replay


def test_uninstall_restores_the_node():
    mod = make_node()
    before = (dict(vars(mod.CycleManager)), mod.run_task_once, vars(mod.model_manager).copy())
    n = pnode.install(mod, engine=NumpyEngine())
    assert mod.CycleManager._average_plan_diffs is not before[0]["_average_plan_diffs"]
    n.uninstall()
    assert dict(vars(mod.CycleManager)) == before[0] and mod.run_task_once is before[1]
    assert vars(mod.model_manager) == before[2]


def test_a_failing_close_time_fallback_runs_once():
    """The report-time close fails (AggregationError) -> the close-time path over the DB rows; when
    that fails too, its error reaches complete_cycle's log once -- it is not retried by the close's
    own error handling."""
    from pygrid_amd.exceptions import AggregationError
    from pygrid_amd.incremental import IncrementalCycle

    sc = Scenario(CFG3, True)
    calls = []

    def failing(*a, **k):
        calls.append(1)
        raise AggregationError("engine failure (test)")
    sc.node.aggregator.average_plan_diffs = failing
    orig_finish = IncrementalCycle.finish
    IncrementalCycle.finish = lambda self, *a, **k: (_ for _ in ()).throw(AggregationError("finish failed (test)"))
    try:
        for w in range(3):
            sc.assign(w)
        for w in range(3):
            sc.report(w)
    finally:
        IncrementalCycle.finish = orig_finish
    assert len(calls) == 1
    assert len(sc.cm.task_errors) == 1 and "engine failure" in str(sc.cm.task_errors[0])
    sc.node.uninstall()
