"""CPU: ``pygrid_amd.node.install`` against the reference node's real storage types and report
handler code.

The node's tables live in SQLAlchemy on a SQLite file (tests/sql_node.py: the reference's columns,
``WorkerCycle.diff`` a ``LargeBinary``, ``Model.query`` from a thread-scoped session, the
reference's ``Warehouse``); clients report through the reference's handler restated
(tests/ref_fl_events.py: ``base64.b64decode(data.get(CYCLE.DIFF).encode())``, fl_events.py:257).
Each script runs on two fresh nodes -- as shipped, and after ``install(..., report_module=
ref_fl_events)`` -- and the saved ``ModelCheckPoint`` rows, read back through a session of their
own, must be byte-identical.  Also checked:

* the installed handler's decoded diffs are read-only memoryviews over pool blocks, SQLAlchemy binds
  them into the ``LargeBinary`` column, and every row reads back byte-identical to the decoded diff
  after commit (and expire-on-commit) -- and every block comes back to the pool;
* the close reads the completed rows with ``defer(WorkerCycle.diff)`` (``node._rows``): the blobs
  of diffs already in HBM are never loaded;
* the close running on an executor thread (its own session) reads what the handler threads
  committed.

Engine: tests/fake_engine.py (folds by the C oracle); the GPU version of this test is
tests/test_gpu_node_sql.py."""
import base64
import collections
import gc
import types

import pytest
import sqlalchemy.orm
from sqlalchemy import inspect

import ref_fl_events
from fake_engine import NumpyEngine
from fake_node import assign, host_process
from pygrid_amd import node as pnode
from sql_node import HeapPool, make_sql_node
from test_node_concurrency import NamedExecutor
from test_node_wiring import ckpt_bytes, diff_bytes

CFG = {"min_diffs": 3, "max_diffs": 4, "num_cycles": 3}


class SqlScenario:
    def __init__(self, path, installed: bool, threaded: bool = False, pool: bool = False, engine=None,
                 cfg=CFG, ckpt=None, diff_fn=diff_bytes, **opts):
        self.mod, self.store = make_sql_node(f"sqlite:///{path}")
        self.ex = NamedExecutor() if threaded else None
        if self.ex:
            self.mod.run_task_once = self.ex.run_task_once
        self.installed = installed
        self.engine_factory = engine or NumpyEngine
        self.opts = {"framing": "template", "report_module": ref_fl_events, "pinned_reports": 0, **opts}
        self.use_pool = pool
        self.pools = []  # one per (re)start of the node process
        self.node = None
        self.before_restart = collections.Counter()
        self.sent = {}  # (worker) -> the latest diff bytes it reported
        self.diff_fn = diff_fn
        if installed:
            self._install()
        ref_fl_events.processes = types.SimpleNamespace(
            submit_diff=lambda *a: self.mod.cycle_manager.submit_worker_diff(*a))
        self.proc, _, _ = host_process(self.mod, cfg, ckpt if ckpt is not None else ckpt_bytes())
        self.keys = {}

    def _install(self):
        self.node = pnode.install(self.mod, engine=self.engine_factory(), **self.opts)
        if self.use_pool:  # the handler's pool: ordinary memory on a CPU box
            self.node.pinned = HeapPool(max_blocks=4)
            ref_fl_events.base64._pool = self.node.pinned
        if self.node.pinned is not None:
            self.pools.append(self.node.pinned)

    @property
    def pool(self):
        return self.pools[-1]

    def restart(self):
        if self.installed:
            self.node.uninstall()
            self.before_restart.update(self.node.stats)
            self._install()

    @property
    def stats(self):
        """The node's counters summed over its restarts."""
        return self.before_restart + collections.Counter(self.node.stats)

    def assign(self, *workers):
        for w in workers:
            self.keys[w] = assign(self.mod, w, self.proc)

    def report(self, w, version=0, payload=None):
        diff = payload if payload is not None else self.diff_fn(w, version)
        msg = {"data": {"worker_id": w, "request_key": self.keys[w], "diff": base64.b64encode(diff).decode()}}
        resp = ref_fl_events.report(msg)
        assert resp["data"] == {"status": "success"}, resp
        self.sent[w] = diff
        if self.ex:
            self.ex.wait()
        return resp

    def checkpoints(self):
        s = self.store.fresh_session()
        try:
            rows = s.query(self.store.ModelCheckPoint).order_by(self.store.ModelCheckPoint.id).all()
            return [(r.number, r.alias, bytes(r.value)) for r in rows]
        finally:
            s.close()

    def diffs_in_db(self):
        s = self.store.fresh_session()
        try:
            return {(r.cycle_id, r.worker_id): r.diff for r in s.query(self.store.WorkerCycle).all()
                    if r.diff is not None}
        finally:
            s.close()

    def finish(self):
        if self.node is not None:
            self.node.uninstall()
        self.store.close()


def script_three_cycles(sc: SqlScenario):
    """Re-report, late report, a restart mid-cycle, workers that never report."""
    sc.assign("w1", "w2", "w3", "w4", "w5", "w6")
    sc.report("w2")
    sc.report("w1")
    sc.report("w5")
    sc.report("w2", version=1)  # re-report: the latest diff is averaged at w2's row position
    sc.report("w6")  # 4 = max_diffs: the close
    sc.report("w3")  # late: stored, ignored (cycle_manager.py:186-188)
    sc.assign("w1", "w2", "w3", "w4", "w5")
    for w in ("w5", "w4", "w3", "w1"):
        sc.report(w, version=2)
    sc.assign("w1", "w2", "w3", "w4")
    sc.report("w1", version=3)
    sc.report("w2", version=3)
    sc.restart()  # the node process restarts: the DB stays
    sc.report("w3", version=3)
    sc.report("w4", version=3)


def run_both(tmp_path, script, **kw):
    tmp_path.mkdir(parents=True, exist_ok=True)
    out = []
    for installed in (False, True):
        sc = SqlScenario(tmp_path / f"node_{int(installed)}.db", installed, **kw)
        try:
            script(sc)
            out.append((sc.checkpoints(), sc.diffs_in_db(), sc))
        finally:
            sc.finish()
    (ref_ck, ref_db, _), (eng_ck, eng_db, eng) = out
    assert len(ref_ck) == 4  # the initial checkpoint + three closed cycles
    assert eng_ck == ref_ck
    assert eng_db == ref_db
    return eng


@pytest.mark.parametrize("threaded", [False, True], ids=["sync", "executor"])
@pytest.mark.parametrize("pool", [False, True], ids=["bytes", "pooled-views"])
def test_installed_sql_node_saves_the_reference_bytes(tmp_path, monkeypatch, threaded, pool):
    deferred = []
    real_defer = sqlalchemy.orm.defer
    monkeypatch.setattr(sqlalchemy.orm, "defer", lambda *a, **k: deferred.append(a) or real_defer(*a, **k))
    eng = run_both(tmp_path, script_three_cycles, threaded=threaded, pool=pool)
    st = eng.stats
    assert st["closes_report_time"] == 3 and st["closes_close_time"] == 0, st
    assert st["report_errors"] == 0
    assert st["diffs_from_db"] >= 2  # the two cycle-3 reports made before the restart
    assert deferred, "the close never read the completed rows with defer(WorkerCycle.diff)"
    if pool:
        gc.collect()
        hits = [(p.hits, p.misses, p.outstanding) for p in eng.pools]
        assert hits == [(12, 0, 0), (2, 0, 0)], hits  # every report decoded into a block, all given back


def test_pooled_view_binds_into_largebinary_and_reads_back(tmp_path):
    """The installed handler's diff: a read-only memoryview over a pool block, stored by
    submit_worker_diff into WorkerCycle.diff; after the commit the row reads back (this session,
    after expire-on-commit, and a fresh one) byte-identical."""
    sc = SqlScenario(tmp_path / "n.db", installed=True, pool=True)
    try:
        seen = []
        orig = sc.mod.CycleManager.submit_worker_diff

        def spy(cm, worker_id, request_key, diff):
            seen.append(diff)
            return orig(cm, worker_id, request_key, diff)
        sc.mod.CycleManager.submit_worker_diff = spy
        sc.assign("a", "b")
        wc = sc.mod.cycle_manager._worker_cycles.first(worker_id="a")  # the handler's session's row
        sc.report("a", version=4)
        assert isinstance(seen[0], memoryview) and seen[0].readonly
        assert bytes(seen[0]) == sc.sent["a"]
        # expired on commit; the reference's own ``_worker_cycle.cycle_id`` (cycle_manager.py:178)
        # then refreshed the row: what the session holds now is the DB's copy, not the view
        assert isinstance(inspect(wc).dict.get("diff"), bytes)
        assert wc.diff == sc.sent["a"]
        assert sc.diffs_in_db()[(wc.cycle_id, "a")] == sc.sent["a"]
        del seen[:], wc
        gc.collect()
        assert sc.pool.outstanding == 0
    finally:
        sc.finish()


def test_completed_rows_defer_the_diff_blobs(tmp_path):
    sc = SqlScenario(tmp_path / "n.db", installed=True)
    try:
        sc.assign("a", "b", "c")
        sc.report("b")
        sc.report("a")
        cm = sc.mod.cycle_manager
        sc.store.session.expire_all()
        rows = pnode.completed_rows(cm, sc.mod.cycle_manager.last(sc.proc.id).id)
        assert [r.worker_id for r in rows] == ["a", "b"]  # row (assignment) order, not report order
        assert all("diff" not in inspect(r).dict for r in rows)
        assert [r.diff for r in rows] == [sc.sent["a"], sc.sent["b"]]  # loaded on access
    finally:
        sc.finish()


def test_malformed_report_answers_like_the_reference(tmp_path):
    """A bad base64 body: the installed decoder raises binascii.Error as base64 does, so the
    handler's error response (its text up to the traceback) is the reference's."""
    answers = []
    for installed in (False, True):
        sc = SqlScenario(tmp_path / f"m{int(installed)}.db", installed, pool=installed)
        try:
            sc.assign("a")
            resp = ref_fl_events.report({"data": {"worker_id": "a", "request_key": sc.keys["a"], "diff": "QUJ"}})
            answers.append(resp["data"]["error"].split("\n")[0])
        finally:
            sc.finish()
    assert answers[0] == answers[1] and answers[0]


def test_install_into_node_by_package_name(tmp_path, monkeypatch):
    """``install_into_node("src.app")`` imports the node's modules by the reference's layout
    (``src/app/main/model_centric/cycles/cycle_manager.py``, ``src/app/main/events/model_centric/
    fl_events.py``, ``src/app.executor``): here a throwaway package with that layout over
    tests/fake_node.py and the restated handler.  The handler's ``base64`` is replaced, the close
    runs on the engine, and uninstall restores both."""
    import importlib
    import shutil
    import sys

    pkg = tmp_path / "nodepkg"
    (pkg / "main" / "model_centric" / "cycles").mkdir(parents=True)
    (pkg / "main" / "events" / "model_centric").mkdir(parents=True)
    for d in (pkg, pkg / "main", pkg / "main" / "model_centric", pkg / "main" / "model_centric" / "cycles",
              pkg / "main" / "events", pkg / "main" / "events" / "model_centric"):
        (d / "__init__.py").write_text("")
    (pkg / "__init__.py").write_text("executor = None\n")
    (pkg / "main" / "model_centric" / "cycles" / "cycle_manager.py").write_text(
        "import sys\nimport fake_node\nfake_node.make_node(mod=sys.modules[__name__])\n")
    shutil.copy(ref_fl_events.__file__, pkg / "main" / "events" / "model_centric" / "fl_events.py")
    monkeypatch.syspath_prepend(str(tmp_path))
    try:
        node = pnode.install_into_node("nodepkg", engine=NumpyEngine(), framing="template", pinned_reports=0)
        cmm = importlib.import_module("nodepkg.main.model_centric.cycles.cycle_manager")
        fle = importlib.import_module("nodepkg.main.events.model_centric.fl_events")
        assert isinstance(fle.base64, pnode._Base64)
        fle.processes = types.SimpleNamespace(submit_diff=lambda *a: cmm.cycle_manager.submit_worker_diff(*a))
        proc, _, _ = host_process(cmm, {"min_diffs": 2, "max_diffs": 2}, ckpt_bytes())
        keys = {w: assign(cmm, w, proc) for w in ("a", "b")}
        for w in ("a", "b"):
            msg = {"data": {"worker_id": w, "request_key": keys[w], "diff": base64.b64encode(diff_bytes(w)).decode()}}
            assert fle.report(msg)["data"] == {"status": "success"}
        assert node.stats["closes_report_time"] == 1
        node.uninstall()
        assert fle.base64 is base64
    finally:
        for m in [m for m in sys.modules if m == "nodepkg" or m.startswith("nodepkg.")]:
            del sys.modules[m]


def random_script(seed: int, prefix: str):
    """Three cycles (CFG: max_diffs 4) of a fresh set of 5-8 workers each, reports in random order with
    re-reports, a fifth report arriving after the close (late), and restarts of the node process."""
    import numpy as np

    rng = np.random.default_rng(seed)
    n = int(rng.integers(5, 9))
    ops = []
    for cyc in range(3):
        ws = [f"{prefix}c{cyc}w{i}" for i in range(n)]
        ops.append(("assign", ws))
        for w in list(rng.permutation(ws))[:5]:
            ops.append(("report", w, 0))
            if rng.random() < 0.25:
                ops.append(("report", w, 1))
            if rng.random() < 0.1:
                ops.append(("restart",))

    def script(sc):
        for op in ops:
            if op[0] == "assign":
                sc.assign(*op[1])
            elif op[0] == "report":
                sc.report(op[1], version=op[2])
            else:
                sc.restart()
    return script, int(rng.integers(2, 7))


@pytest.mark.parametrize("threaded", [False, True], ids=["sync", "executor"])
def test_randomised_scripts_on_the_sql_node(tmp_path, threaded):
    """Random scripts (``random_script``) through the reference's storage and handler, random slot
    budgets: installed and shipped nodes save identical checkpoints and hold identical diff blobs."""
    totals = collections.Counter()
    for trial in range(8):
        script, slots = random_script(500 + trial, f"t{trial}")
        eng = run_both(tmp_path / f"t{trial}", script, threaded=threaded, slots=slots)
        totals.update(eng.stats)
    assert totals["report_errors"] == 0, totals
    assert totals["closes_report_time"] == 24 and totals["diffs_from_db"] >= 1, totals  # restarts read the DB


def test_installed_close_reads_no_checkpoint_blob(tmp_path):
    """After the first cycle, no close of the installed node SELECTs a checkpoint's ``value``: the
    input checkpoint is resident (HBM + the write-through cache), and caching the saved one reads
    its small columns only -- touching the ``ModelCheckPoint`` the save's commit expired would
    reload its 47 MB blob (55-60 ms per close at ResNet-18 size)."""
    from sqlalchemy import event

    sc = SqlScenario(tmp_path / "node.db", True)
    try:
        blob_selects = []

        def seen(conn, cursor, statement, params, context, executemany):
            s = statement.lower()
            if s.lstrip().startswith("select") and "model_centric_model_checkpoint.value" in s:
                blob_selects.append(statement)
        sc.assign("w1", "w2", "w3", "w4")
        for w in ("w2", "w1", "w4", "w3"):
            sc.report(w)  # first close: the checkpoint is read from the DB once
        event.listen(sc.store.engine, "before_cursor_execute", seen)
        for cyc in (1, 2):
            sc.assign("w1", "w2", "w3", "w4")
            for w in ("w3", "w1", "w2", "w4"):
                sc.report(w, version=cyc)
        assert sc.stats["closes_report_time"] == 3, sc.stats
        assert not blob_selects, blob_selects
        cached = sc.node.store.lookup(model_id=sc.proc.id if hasattr(sc.proc, "id") else 1, alias="latest")
        rows = sc.checkpoints()
        assert cached is not None and (cached.number, cached.alias, cached.value) == rows[-1]
    finally:
        sc.finish()


def test_reports_find_their_rows_without_a_query(tmp_path, monkeypatch):
    """A report of a row assigned through the installed node finds its WorkerCycle id and cycle from
    the assignment (no query after the handler's DB write); rows assigned before a restart are
    looked up in the DB -- the checkpoints stay the reference's."""
    calls = []
    real = pnode._first_row
    monkeypatch.setattr(pnode, "_first_row", lambda *a, **k: calls.append(k) or real(*a, **k))
    eng = run_both(tmp_path, script_three_cycles)
    # script_three_cycles: cycle 1's late report (its cycle closed: the rows are forgotten) and the
    # two reports of cycle 3 that follow the restart
    assert [(c["worker_id"], c["request_key"]) for c in calls] == [("w3", "key-w3-1"), ("w3", "key-w3-3"),
                                                                  ("w4", "key-w4-3")], calls
    assert eng.stats["closes_report_time"] == 3
