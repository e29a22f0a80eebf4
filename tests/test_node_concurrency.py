"""CPU: the installed node under concurrency.

The reference runs report handlers on a gevent hub (``apps/node/src/__main__.py:85``,
``entrypoint.sh:2``) and the close on Flask-Executor's thread (``tasks/cycle.py:9-25``): a handler
that waits for a close stalls every client.  These tests run the close on a real executor thread,
block it inside the fold, and check that

* a late report, a re-report and an assignment of the closing cycle, and a report of another FL
  process's cycle, each return within milliseconds while the close is blocked;
* a re-report whose DB write is in flight when the close starts is averaged (its DB write and its
  ingest are atomic with respect to the close's snapshot of the rows), and a re-report that lands
  after the snapshot is ignored -- in both cases the saved checkpoints are byte-identical to the
  reference node run with the same events in the equivalent serial order.

Node: tests/fake_node.py; engine: tests/fake_engine.py (folds by the C oracle)."""
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from fake_engine import NumpyEngine
from fake_node import assign, host_process, make_node
from pygrid_amd import node as pnode
from test_node_wiring import ckpt_bytes, diff_bytes

CFG3 = {"min_diffs": 3, "max_diffs": 3, "num_cycles": 0}
FAST_S = 0.25  # "returns at once": generous for a loaded CI box, far below a blocked close


class NamedExecutor:
    """``run_task_once`` as the reference has it (``tasks/cycle.py:9-25``): one named future; a
    request while it runs is skipped."""

    def __init__(self):
        self.pool = ThreadPoolExecutor(1, thread_name_prefix="executor")
        self.futures = {}

    def run_task_once(self, name, func, *args):
        f = self.futures.get(name)
        if f is None or f.done():
            self.futures[name] = self.pool.submit(func, *args)

    def wait(self, timeout=10):
        for f in list(self.futures.values()):
            f.result(timeout)


class BlockingEngine(NumpyEngine):
    """The fold's FINAL pass waits for ``release`` (a close stuck on the GPU)."""

    def __init__(self):
        super().__init__()
        self.entered = threading.Event()
        self.release = threading.Event()

    def fold_slots_finish_resident(self, mode, slots=()):
        self.entered.set()
        assert self.release.wait(20), "test never released the close"
        return super().fold_slots_finish_resident(mode, slots)


def checkpoints(mod):
    rows = sorted(mod.model_manager._model_checkpoints.rows, key=lambda r: r.id)
    return [(r.number, r.alias, r.value) for r in rows]


def timed(fn, *a):
    t0 = time.perf_counter()
    fn(*a)
    return time.perf_counter() - t0


def test_handlers_never_wait_for_a_blocked_close():
    ex = NamedExecutor()
    mod = make_node()
    mod.run_task_once = ex.run_task_once
    eng = BlockingEngine()
    node = pnode.install(mod, engine=eng, framing="template", fold_batch=1)
    cm = mod.cycle_manager
    proc, _, _ = host_process(mod, CFG3, ckpt_bytes())
    other, _, _ = host_process(mod, CFG3, ckpt_bytes(1))  # a second FL process on the same node
    keys = {w: assign(mod, w, proc) for w in range(1, 5)}
    okey = assign(mod, 9, other)
    for w in (1, 2, 3):
        cm.submit_worker_diff(w, keys[w], diff_bytes(w))
    assert eng.entered.wait(10), "the close never reached the fold"
    try:
        took = {
            "late report": timed(cm.submit_worker_diff, 4, keys[4], diff_bytes(4)),
            "re-report": timed(cm.submit_worker_diff, 1, keys[1], diff_bytes(1, version=7)),
            "assign": timed(assign, mod, 5, proc),
            "other process": timed(cm.submit_worker_diff, 9, okey, diff_bytes(9)),
        }
        assert all(t < FAST_S for t in took.values()), took
        assert not ex.futures["complete_cycle"].done()  # the close really was blocked meanwhile
    finally:
        eng.release.set()
    ex.wait()
    node.uninstall()

    # the reference with the same events, serially: the close read the rows before the late ones
    ref = make_node()
    rproc, _, _ = host_process(ref, CFG3, ckpt_bytes())
    host_process(ref, CFG3, ckpt_bytes(1))
    rkeys = {w: assign(ref, w, rproc) for w in range(1, 5)}
    for w in (1, 2, 3):
        ref.cycle_manager.submit_worker_diff(w, rkeys[w], diff_bytes(w))
    assert checkpoints(mod) == checkpoints(ref)
    assert len(checkpoints(mod)) == 3  # 2 initial + the closed cycle of process 1
    assert node.stats["closes_report_time"] == 1


class SlowUpdateWarehouse:
    """Wraps the worker-cycle warehouse: ``update`` (the commit of ``submit_worker_diff``,
    ``cycle_manager.py:174``) of a chosen thread blocks until released."""

    def __init__(self, wh):
        self.wh = wh
        self.block_thread = None
        self.in_update = threading.Event()
        self.release = threading.Event()

    def __getattr__(self, name):
        return getattr(self.wh, name)

    def update(self):
        if threading.current_thread() is self.block_thread:
            self.in_update.set()
            assert self.release.wait(20)
        return self.wh.update()


def test_rereport_in_flight_at_the_close_is_averaged():
    """the re-report's DB write has landed (the row holds the new diff) but its
    ingest has not, when the last report triggers the close.  The close must average the new diff,
    as the reference's query at :243-250 -- which reads the committed row -- does."""
    ex = NamedExecutor()
    mod = make_node()
    mod.run_task_once = ex.run_task_once
    node = pnode.install(mod, engine=NumpyEngine(), framing="template", fold_batch=1)
    cm = mod.cycle_manager
    slow = SlowUpdateWarehouse(cm._worker_cycles)
    cm._worker_cycles = slow
    proc, _, _ = host_process(mod, CFG3, ckpt_bytes())
    keys = {w: assign(mod, w, proc) for w in range(1, 4)}
    cm.submit_worker_diff(1, keys[1], diff_bytes(1))
    cm.submit_worker_diff(2, keys[2], diff_bytes(2))

    t = threading.Thread(target=cm.submit_worker_diff, args=(1, keys[1], diff_bytes(1, version=5)))
    slow.block_thread = t
    t.start()
    assert slow.in_update.wait(10)
    cm.submit_worker_diff(3, keys[3], diff_bytes(3))  # triggers the close on the executor
    deadline = time.monotonic() + 10
    while node._gate._waiting == 0 and time.monotonic() < deadline:  # the close waits for the gate
        time.sleep(0.005)
    assert node._gate._waiting == 1
    slow.release.set()
    t.join(10)
    ex.wait()
    node.uninstall()

    ref = make_node()
    rproc, _, _ = host_process(ref, CFG3, ckpt_bytes())
    rkeys = {w: assign(ref, w, rproc) for w in range(1, 4)}
    rcm = ref.cycle_manager
    rcm.submit_worker_diff(1, rkeys[1], diff_bytes(1))
    rcm.submit_worker_diff(2, rkeys[2], diff_bytes(2))
    rcm.submit_worker_diff(1, rkeys[1], diff_bytes(1, version=5))
    rcm.submit_worker_diff(3, rkeys[3], diff_bytes(3))
    assert checkpoints(mod) == checkpoints(ref)
    assert len(checkpoints(mod)) == 2


def test_gate_close_waits_only_for_reports_in_flight():
    g = pnode._Gate()
    order = []
    entered = threading.Event()
    go = threading.Event()

    def report():
        with g.shared():
            entered.set()
            go.wait(10)
            order.append("report")

    t = threading.Thread(target=report)
    t.start()
    entered.wait(10)

    def close():
        with g.exclusive():
            order.append("close")

    c = threading.Thread(target=close)
    c.start()
    while g._waiting == 0:
        time.sleep(0.001)
    late = threading.Thread(target=lambda: (g.shared().__enter__(), order.append("late")))
    late.start()
    time.sleep(0.05)
    assert order == []  # the late report queues behind the waiting close
    go.set()
    for th in (t, c, late):
        th.join(10)
    assert order == ["report", "close", "late"]


class JitterWarehouse(SlowUpdateWarehouse):
    """Every commit of submit_worker_diff takes 0-2 ms (a DB write), so a close's snapshot often
    lands between a report's DB write and its ingest -- where only the report gate keeps them
    consistent."""

    def __init__(self, wh):
        super().__init__(wh)
        import random

        self.rng = random.Random(7)

    def update(self):
        time.sleep(self.rng.random() * 0.002)
        return self.wh.update()


def test_concurrent_handlers_and_closes_equal_the_reference_over_each_snapshot(monkeypatch):
    """Linearizability under load: 4 handler threads assign, report and re-report workers of
    whatever cycle is open (late reports included) while closes run on the executor.  Each close's
    snapshot of the completed rows (taken under the report gate) is recorded with the diffs the
    rows held then; the reference node, replayed serially over exactly those rows, must save the
    same checkpoint bytes, cycle after cycle."""
    import random

    ex = NamedExecutor()
    mod = make_node()
    mod.run_task_once = ex.run_task_once
    node = pnode.install(mod, engine=NumpyEngine(), framing="template", fold_batch=1)
    cm = mod.cycle_manager
    cm._worker_cycles = JitterWarehouse(cm._worker_cycles)  # widen the write -> ingest window
    cfg = {"min_diffs": 5, "max_diffs": 5, "num_cycles": 4}
    snaps = []
    real_rows = pnode.completed_rows

    def recording_rows(cm_, cycle_id):
        rows = real_rows(cm_, cycle_id)
        snaps.append([(r.id, r.diff) for r in rows])  # under the exclusive gate: the DB as read
        return rows
    monkeypatch.setattr(pnode, "completed_rows", recording_rows)
    proc, _, _ = host_process(mod, cfg, ckpt_bytes())
    stop = threading.Event()
    errors = []

    def handler(seed):
        rng = random.Random(seed)
        v = 0
        try:
            while not stop.is_set():
                w = f"h{seed}-{rng.randrange(4)}"
                try:
                    key = assign(mod, w, proc)
                except AttributeError:  # every cycle done: cycle_manager.last() found none
                    return
                for _ in range(rng.choice((1, 1, 2))):  # sometimes a re-report
                    v += 1
                    cm.submit_worker_diff(w, key, diff_bytes(w, v))
                    time.sleep(rng.random() * 0.003)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=handler, args=(s,)) for s in range(4)]
    for t in threads:
        t.start()
    deadline = time.monotonic() + 60
    while len(checkpoints(mod)) < 5 and time.monotonic() < deadline:
        time.sleep(0.01)
    stop.set()
    for t in threads:
        t.join(10)
    ex.wait()
    node.uninstall()
    assert not errors, errors
    assert cm.task_errors == []
    saved = checkpoints(mod)
    assert len(saved) == 5 and len(snaps) == 4, (len(saved), len(snaps))
    # replay each close on a fresh reference node: the previous checkpoint, the snapshot's rows
    for k, rows in enumerate(snaps):
        ref = make_node()
        rp, _, _ = host_process(ref, {"min_diffs": len(rows), "max_diffs": len(rows), "num_cycles": 1}, saved[k][2])
        keys = [assign(ref, i, rp) for i in range(len(rows))]
        for i, (_, d) in enumerate(rows):
            ref.cycle_manager.submit_worker_diff(i, keys[i], d)
        assert checkpoints(ref)[-1][2] == saved[k + 1][2], f"close {k}"


def test_close_run_inline_from_a_report_does_not_deadlock():
    """A node whose submit_worker_diff runs complete_cycle inline (not through the patched
    run_task_once): the close's exclusive gate upgrades the report's shared hold instead of waiting
    for it forever; the close reads the triggering diff from the DB (its ingest has not run yet)."""
    mod = make_node()
    node = pnode.install(mod, engine=NumpyEngine(), framing="template", fold_batch=1)
    mod.run_task_once = lambda name, func, *args: func(*args)  # bypasses install's hold-and-dispatch
    proc, _, _ = host_process(mod, CFG3, ckpt_bytes())
    keys = {w: assign(mod, w, proc) for w in range(1, 4)}
    t = threading.Thread(target=lambda: [mod.cycle_manager.submit_worker_diff(w, keys[w], diff_bytes(w))
                                         for w in (1, 2, 3)])
    t.start()
    t.join(10)
    assert not t.is_alive(), "deadlock: the inline close waited for its own report's gate"
    node.uninstall()
    ref = make_node()
    rproc, _, _ = host_process(ref, CFG3, ckpt_bytes())
    rkeys = {w: assign(ref, w, rproc) for w in range(1, 4)}
    for w in (1, 2, 3):
        ref.cycle_manager.submit_worker_diff(w, rkeys[w], diff_bytes(w))
    assert checkpoints(mod) == checkpoints(ref) and len(checkpoints(mod)) == 2


def test_two_inline_closers_do_not_deadlock_the_gate():
    """two reports holding the gate shared both run a close inline and upgrade.  Each
    would wait for the other's shared hold forever; the second upgrader fails at once instead
    (GateUpgradeConflict), its handler goes on and releases its hold, and the first upgrade
    completes."""
    g = pnode._Gate()
    both_in = threading.Barrier(2)
    first_waiting = threading.Event()
    got, errors = [], []

    def handler(name, delay):
        with g.shared():
            both_in.wait(10)
            time.sleep(delay)
            try:
                if name == "a":
                    first_waiting.set()
                else:
                    first_waiting.wait(10)
                    while not g._upgrading:
                        time.sleep(0.001)
                g.acquire_exclusive()
            except pnode.GateUpgradeConflict:
                errors.append(name)
                return
            try:
                got.append(name)
            finally:
                g.release_exclusive()

    ts = [threading.Thread(target=handler, args=("a", 0.0)), threading.Thread(target=handler, args=("b", 0.01))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert not any(t.is_alive() for t in ts), "deadlock: two upgraders waited for each other"
    assert got == ["a"] and errors == ["b"]
    # the gate is whole again: a plain close and a later upgrade both get it
    with g.exclusive():
        pass
    with g.shared():
        g.acquire_exclusive()
        g.release_exclusive()
    assert not g._upgrading and not g._exclusive


class BarrierWarehouse(SlowUpdateWarehouse):
    """``update`` (the report's DB write, under its shared gate hold) of the named threads waits
    until all of them are there, so every report holds the gate shared before any close starts."""

    def __init__(self, wh, parties):
        super().__init__(wh)
        self.barrier = threading.Barrier(parties)
        self.threads = set()

    def update(self):
        if threading.current_thread().name in self.threads:
            self.threads.discard(threading.current_thread().name)
            self.barrier.wait(10)
        return self.wh.update()


def test_two_inline_closes_on_the_node_do_not_deadlock():
    """two reports of two FL processes each complete their cycle and run
    complete_cycle inline, both while holding the report gate shared.  The first close takes the
    engine lock and waits for the exclusive gate -- for the other report's hold; the other close
    must not block on the engine lock behind it.  It gives up (GateUpgradeConflict, logged by
    complete_cycle as the reference logs a failed close), its handler ends, the first close
    finishes; a re-report then closes the second cycle, and the saved checkpoints equal the
    reference node's."""
    cfg1 = {"min_diffs": 1, "max_diffs": 1, "num_cycles": 0}
    mod = make_node()
    node = pnode.install(mod, engine=NumpyEngine(), framing="template", fold_batch=1)
    mod.run_task_once = lambda name, func, *args: func(*args)  # complete_cycle inline, in the handler
    cm = mod.cycle_manager
    bw = BarrierWarehouse(cm._worker_cycles, 2)
    cm._worker_cycles = bw
    pa, _, _ = host_process(mod, cfg1, ckpt_bytes())
    pb, _, _ = host_process(mod, cfg1, ckpt_bytes(1))
    ka, kb = assign(mod, "a", pa), assign(mod, "b", pb)
    ts = [threading.Thread(target=cm.submit_worker_diff, args=("a", ka, diff_bytes("a")), name="report-a"),
          threading.Thread(target=cm.submit_worker_diff, args=("b", kb, diff_bytes("b")), name="report-b")]
    bw.threads = {t.name for t in ts}
    for t in ts:
        t.start()
    for t in ts:
        t.join(15)
    assert not any(t.is_alive() for t in ts), "deadlock: an inline close waited on the engine lock"
    assert len(cm.task_errors) == 1 and isinstance(cm.task_errors[0], pnode.GateUpgradeConflict), cm.task_errors
    assert node.stats["gate_conflicts"] == 1
    assert len(checkpoints(mod)) == 3  # 2 initial + exactly one closed cycle
    # the gate and the engine lock are free again: the cycle left open closes on the next report
    done = {r[2] for r in checkpoints(mod)}
    for w, k, p in (("a", ka, pa), ("b", kb, pb)):
        cm.submit_worker_diff(w, k, diff_bytes(w))
    assert len(checkpoints(mod)) == 4 and len(cm.task_errors) == 1
    assert done <= {r[2] for r in checkpoints(mod)}
    node.uninstall()

    ref = make_node()
    ra, _, _ = host_process(ref, cfg1, ckpt_bytes())
    rb, _, _ = host_process(ref, cfg1, ckpt_bytes(1))
    rka, rkb = assign(ref, "a", ra), assign(ref, "b", rb)
    ref.cycle_manager.submit_worker_diff("a", rka, diff_bytes("a"))
    ref.cycle_manager.submit_worker_diff("b", rkb, diff_bytes("b"))
    assert sorted(r[2] for r in checkpoints(mod)) == sorted(r[2] for r in checkpoints(ref))


def test_assignment_while_the_cycle_state_is_built_is_recorded(monkeypatch):
    """a cycle the node just created is prepared under the engine lock without a rows
    query; an assign handler that runs meanwhile finds the lock taken.  Its assignment is recorded
    into the state when the state is made (fold order, and the report's row lookup without a
    query) -- then the cycle closes byte-identical to the reference."""
    mod = make_node()
    node = pnode.install(mod, engine=NumpyEngine(), framing="template", fold_batch=1)
    real = node._new_cycle
    built = []

    def build_with_an_assign_racing(cm, cycle, fresh=False):
        inc = real(cm, cycle, fresh)
        if not built:  # the first cycle: a worker is assigned (DB row written) while this runs
            t = threading.Thread(target=lambda: built.append(("key", assign(mod, 1, proc_box[0]))))
            t.start()
            t.join(10)
            assert not t.is_alive()
            assert not inc._key_of  # not recorded yet: the handler found the engine lock taken
        return inc

    proc_box = []
    monkeypatch.setattr(node, "_new_cycle", build_with_an_assign_racing)
    orig_create = mod.CycleManager.create

    def create_after_the_process_exists(cm, *a):
        if not proc_box:
            import types

            proc_box.append(types.SimpleNamespace(id=a[0]))
        return orig_create(cm, *a)
    monkeypatch.setattr(mod.CycleManager, "create", create_after_the_process_exists)
    proc, _, _ = host_process(mod, CFG3, ckpt_bytes())
    inc = next(st for st in node._cycles.values() if isinstance(st, pnode.IncrementalCycle))
    assert len(inc._key_of) == 1 and not node._pending_assign  # recorded when the state was made
    keys = {1: built[0][1]}
    keys.update({w: assign(mod, w, proc) for w in (2, 3)})
    for w in (1, 2, 3):
        mod.cycle_manager.submit_worker_diff(w, keys[w], diff_bytes(w))
    assert node.stats["closes_report_time"] == 1 and node.stats["diffs_from_db"] == 0, node.stats
    node.uninstall()
    ref = make_node()
    rproc, _, _ = host_process(ref, CFG3, ckpt_bytes())
    rkeys = {w: assign(ref, w, rproc) for w in (1, 2, 3)}
    for w in (1, 2, 3):
        ref.cycle_manager.submit_worker_diff(w, rkeys[w], diff_bytes(w))
    assert checkpoints(mod) == checkpoints(ref)


def test_assignment_never_raises_when_the_cycle_state_cannot_be_made(monkeypatch):
    """A cycle that existed before install (a restart) gets its report-time state at its first
    assignment; if making it fails, the assign handler still returns the reference's result and
    the cycle closes through the close-time path over its DB rows, byte-identical."""
    mod = make_node()
    proc, _, _ = host_process(mod, CFG3, ckpt_bytes())  # created before install: no state yet
    node = pnode.install(mod, engine=NumpyEngine(), framing="template", fold_batch=1)

    def broken(cm, cycle, fresh=False):
        raise RuntimeError("model load failed")
    monkeypatch.setattr(node, "_new_cycle", broken)
    keys = {w: assign(mod, w, proc) for w in (1, 2, 3)}  # no exception reaches the handler
    for w in (1, 2, 3):
        mod.cycle_manager.submit_worker_diff(w, keys[w], diff_bytes(w))
    assert node.stats["closes_close_time"] == 1 and node.stats["closes_report_time"] == 0, node.stats
    node.uninstall()
    ref = make_node()
    rproc, _, _ = host_process(ref, CFG3, ckpt_bytes())
    rkeys = {w: assign(ref, w, rproc) for w in (1, 2, 3)}
    for w in (1, 2, 3):
        ref.cycle_manager.submit_worker_diff(w, rkeys[w], diff_bytes(w))
    assert checkpoints(mod) == checkpoints(ref)
