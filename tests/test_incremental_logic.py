"""CPU: fold order of report-time aggregation (pygrid_amd/incremental.py) with a recording
engine.  Every reported diff must reach HBM at once (any arrival order), and the engine must fold
the clients in WorkerCycle-id order with non-reporters dropped (cycle_manager.py:243-245),
folding early only what is certain."""
import numpy as np
import pytest

from pygrid_amd.exceptions import AggregationError, StateParseError
from pygrid_amd.incremental import IncrementalCycle
from pygrid_amd.state_schema import build_state_fast


class RecordingEngine:
    """Slots hold payloads; folds are recorded as payload lists in fold order."""

    def __init__(self, fail_on=None):
        self.calls = []
        self.weights = []
        self.slot = {}
        self.folds = []  # (final, [payload, ...])
        self.fail_on = fail_on

    def set_layout(self, numel):
        self.calls.append(("layout", tuple(numel)))

    def reserve(self, n):
        self.calls.append(("reserve", n))
        self.max_slots = n

    def reset(self):
        self.calls.append(("reset",))

    def set_weights(self, w):
        self.weights = list(w)

    def ingest_state(self, k, pb):
        if self.fail_on is not None and pb == self.fail_on:
            raise StateParseError("malformed diff")
        assert 0 <= k < self.max_slots, (k, self.slot)
        self.slot[k] = pb  # an occupied slot is overwritten (a re-report, pgh_ingest_state RESIDENT)
        self.calls.append(("ingest", k, pb))

    def fold_slots(self, mode, slots):
        self.folds.append((False, [self.slot.pop(s) for s in slots]))
        self.calls.append(("fold", len(slots)))

    def fold_slots_finish_resident(self, mode, slots):
        self.folds.append((True, [self.slot.pop(s) for s in slots]))
        self.calls.append(("finish",))

    def fold_restart(self):
        self.folds.append(("restart", []))
        self.calls.append(("restart",))

    def ckpt_upload_state(self, pb):
        self.calls.append(("upload", pb))

    def ckpt_patch_state(self, pb):
        self.calls.append(("patch", pb))
        return pb


def folded(eng):
    """Payloads in the fold state, in fold order (a restart discards what came before it)."""
    out = []
    for kind, ps in eng.folds:
        out = [] if kind == "restart" else out + ps
    return out


def mk(w: int) -> bytes:
    """A valid 3-float State diff that identifies worker w (parked diffs are scanned)."""
    return build_state_fast([np.full(3, w, np.float32)])


def test_in_order_reports_fold_in_batches():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [10], fold_batch=2, slots=8)
    for w in ("a", "b", "c"):
        inc.assigned(w)
    for w in ("a", "b", "c"):
        inc.reported(w, w.encode())
    assert folded(eng) == [b"a", b"b"]  # c waits for a full batch (or close)
    assert inc.folded_early == 2
    inc.close(b"ck", framing="template")
    assert folded(eng) == [b"a", b"b", b"c"] and eng.folds[-1] == (True, [b"c"])


def test_out_of_order_reports_go_to_hbm_at_once_and_fold_in_id_order():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [10], fold_batch=1, slots=8)
    for w in range(5):
        inc.assigned(w)
    inc.reported(2, b"2")
    inc.reported(1, b"1")
    assert sorted(eng.slot.values()) == [b"1", b"2"]  # in HBM although worker 0 may still report
    assert folded(eng) == []
    inc.reported(0, b"0")
    assert folded(eng) == [b"0", b"1", b"2"]
    inc.reported(4, b"4")
    assert len(folded(eng)) == 3 and b"4" in eng.slot.values()  # worker 3 outstanding


def test_close_drops_non_reporters_and_keeps_id_order():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=8)
    for w in range(6):
        inc.assigned(w)
    for w in (5, 1, 4, 2):
        inc.reported(w, bytes([w]))
    assert folded(eng) == []            # worker 0 never reports
    assert sorted(eng.slot.values()) == [bytes([w]) for w in (1, 2, 4, 5)]
    ck = build_state_fast([np.array([1.0, 2.0, 3.0], np.float32)])
    assert inc.close(ck, framing="template") == ck
    assert eng.folds == [(True, [b"\x01", b"\x02", b"\x04", b"\x05"])]
    assert inc.n_folded == 4 and inc.folded_early == 0
    assert [c[0] for c in eng.calls[-3:]] == ["upload", "finish", "patch"]


def test_twenty_percent_dropouts_shuffled_arrival():
    """The reference's expected failure rate (routes.py:314), reports in random order: every
    reporter is in HBM before close, and the close folds exactly the reporters in id order."""
    rng = np.random.default_rng(5)
    eng = RecordingEngine()
    n = 100
    inc = IncrementalCycle(eng, [3], slots=n, fold_batch=4)
    for w in range(n):
        inc.assigned(w)
    reporters = [w for w in range(n) if rng.random() >= 0.2]
    order = list(rng.permutation(reporters))
    for w in order:
        inc.reported(int(w), int(w).to_bytes(2, "little"))
        assert inc.n_parked == 0
    inc.close(b"ck", framing="template")
    assert folded(eng) == [w.to_bytes(2, "little") for w in sorted(reporters)]


def test_slot_pressure_parks_on_host_but_never_starves_the_front():
    """Fewer slots than reporters: later diffs wait on the host, one slot stays for the fold front,
    and the fold order is still the id order."""
    rng = np.random.default_rng(6)
    for trial in range(20):
        eng = RecordingEngine()
        n, slots = 40, int(rng.integers(2, 7))
        inc = IncrementalCycle(eng, [3], slots=slots, fold_batch=int(rng.integers(1, 5)))
        for w in range(n):
            inc.assigned(w)
        reporters = [w for w in range(n) if rng.random() >= 0.25]
        for w in rng.permutation(reporters):
            inc.reported(int(w), mk(int(w)))
            assert len(eng.slot) <= slots
        inc.close(b"ck", framing="template")
        assert folded(eng) == [mk(w) for w in sorted(reporters)], trial


def test_checkpoint_handed_over_at_start_is_uploaded_once():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], checkpoint=b"ck", slots=4)
    assert eng.calls[-1] == ("upload", b"ck")  # before any report: the upload overlaps the cycle
    inc.assigned("a")
    inc.reported("a", b"a")
    assert inc.close(b"ck", framing="template") == b"ck"
    assert [c[0] for c in eng.calls].count("upload") == 1
    assert [c[0] for c in eng.calls[-2:]] == ["finish", "patch"]


def test_weights_follow_fold_order():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], mode=2, slots=4, fold_batch=1,
                           weights_by_worker={"x": 1.0, "y": 2.0, "z": 3.0})
    for w in ("x", "y", "z"):
        inc.assigned(w)
    inc.reported("z", b"z")
    inc.reported("x", b"x")
    inc.reported("y", b"y")
    assert eng.weights == [1.0, 2.0, 3.0]


def test_weightless_report_is_refused_to_its_sender():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], mode=2, slots=4, fold_batch=1, weights_by_worker={"x": 1.0, "z": 3.0})
    for w in ("x", "y", "z"):
        inc.assigned(w)
    with pytest.raises(AggregationError):
        inc.reported("y", b"y")  # nothing recorded: y counts as a non-reporter
    inc.reported("z", b"z")
    inc.reported("x", b"x")
    inc.close(b"ck", framing="template")
    assert folded(eng) == [b"x", b"z"] and eng.weights == [1.0, 3.0]


def test_errors():
    inc2 = IncrementalCycle(RecordingEngine(), [3], slots=4)
    inc2.assigned("b")
    with pytest.raises(AggregationError):
        inc2.close(b"", framing="template")  # nobody reported
    inc3 = IncrementalCycle(RecordingEngine(), [3], slots=4)
    inc3.assigned("c")
    inc3.reported("c", b"c")
    with pytest.raises(AggregationError):
        inc3.close(b"ck", framing="template", order=["c", "c"])  # a row twice
    inc4 = IncrementalCycle(RecordingEngine(), [3], slots=4)
    with pytest.raises(AggregationError):
        inc4.close(b"ck", framing="template", order=["x"])  # no diff here, no fetch=


def test_re_report_before_its_fold_replaces_the_diff():
    """cycle_manager.py:162-174: a second report overwrites the row's diff; the close folds the
    LATEST diff at the worker's row position."""
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=4, fold_batch=1)
    for w in "abc":
        inc.assigned(w)
    inc.reported("b", b"b1")
    inc.reported("b", b"b2")  # same slot, new bytes
    inc.reported("a", b"a1")  # a, b folded now
    assert folded(eng) == [b"a1", b"b2"]
    inc.reported("c", b"c1")
    inc.close(b"ck", framing="template")
    assert folded(eng) == [b"a1", b"b2", b"c1"] and inc.last_close["refold"] is False


def test_re_report_of_a_parked_diff_replaces_it():
    good = {k: build_state_fast([np.full(3, k, np.float32)]) for k in range(6)}
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=2, fold_batch=4)
    for w in range(4):
        inc.assigned(w)
    inc.reported(2, good[2])
    inc.reported(3, good[3])
    assert inc.n_parked == 1
    inc.reported(3, good[5])  # replaces the parked copy
    for w in (0, 1):
        inc.reported(w, good[w])
    inc.close(b"ck", framing="template")
    assert folded(eng) == [good[0], good[1], good[2], good[5]]


def test_re_report_after_its_fold_refolds_from_the_db():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=4, fold_batch=1)
    for w in "abc":
        inc.assigned(w)
    inc.reported("a", b"a1")
    assert folded(eng) == [b"a1"]
    inc.reported("a", b"a2")  # the fold holds a1, the DB a2
    assert inc.stale
    inc.reported("c", b"c1")
    db = {"a": b"a2", "b": b"b1", "c": b"c1"}
    with pytest.raises(AggregationError):
        inc.close(b"ck", framing="template")  # no DB order: cannot re-fold
    inc = _replay_stale(db)
    assert folded(inc.engine) == [b"a2", b"c1"] and inc.last_close["refold"]


def _replay_stale(db):
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=4, fold_batch=1)
    for w in "abc":
        inc.assigned(w)
    inc.reported("a", b"a1")
    inc.reported("a", b"a2")
    inc.reported("c", b"c1")
    inc.close(b"ck", framing="template", order=["a", "c"], fetch=db.__getitem__)
    return inc


def test_close_follows_the_db_order_and_reads_what_it_lacks():
    """The DB's order is the truth: an early fold that is not its prefix is redone; workers this
    object never heard of (reported before a restart) are read with fetch."""
    db = {w: w.encode() for w in "abcdef"}
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=3, fold_batch=1)
    for w in "abcd":
        inc.assigned(w)
    for w in "abd":
        inc.reported(w, db[w])
    assert folded(eng) == [b"a", b"b"]
    fetched = []

    def fetch(w):
        fetched.append(w)
        return db[w]
    inc.close(b"ck", framing="template", order=list("badf"), fetch=fetch)
    assert folded(eng) == [b"b", b"a", b"d", b"f"] and inc.last_close["refold"]
    assert sorted(fetched) == ["a", "b", "f"]  # d was still in HBM


def test_close_evicts_when_every_slot_holds_a_later_diff():
    """Every slot held by a diff the DB order needs LATER and nothing to fold yet: the slot of the
    diff needed last is given up and that diff is re-read from the DB when its turn comes."""
    db = {w: mk(i) for i, w in enumerate("uxa")}
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=2, fold_batch=4)
    inc.assigned("a")
    inc.reported("x", db["x"])  # unassigned (a restart lost it): held, never folded early
    inc.reported("a", db["a"])  # the fold front takes the last slot, waits for a batch of 4
    fetched = []

    def fetch(w):
        fetched.append(w)
        return db[w]
    inc.close(b"ck", framing="template", order=list("uxa"), fetch=fetch)
    assert folded(eng) == [db["u"], db["x"], db["a"]]
    assert fetched == ["u", "a"]


def test_late_and_unknown_reports_do_not_raise():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=4)
    inc.assigned("a")
    inc.reported("a", b"a")
    inc.reported("ghost", b"g")  # assigned before a restart: held, placed by the DB order at close
    inc.close(b"ck", framing="template")  # no order: only the assigned reporters
    assert folded(eng) == [b"a"]
    inc.reported("a", b"late")  # fl_events.py:261-263 answers success; nothing changes
    assert folded(eng) == [b"a"]


def test_parked_ingest_failure_is_not_blamed_on_another_reporter():
    """a parked diff is ingested when the front reaches it, during ANOTHER worker's
    report; if that fails, that worker gets no error, the parked worker's diff is dropped, and the
    close reads it from the DB."""
    good = {k: build_state_fast([np.full(3, k, np.float32)]) for k in range(4)}

    class FlakyEngine(RecordingEngine):
        fail_once = good[3]

        def ingest_state(self, k, pb):
            if pb is self.fail_once:
                self.fail_once = None
                raise RuntimeError("HIP copy failed")
            super().ingest_state(k, pb)

    eng = FlakyEngine()
    inc = IncrementalCycle(eng, [3], slots=2, fold_batch=4)
    for w in range(4):
        inc.assigned(w)
    inc.reported(2, good[2])
    inc.reported(3, good[3])  # parked
    inc.reported(0, good[0])
    inc.reported(1, good[1])  # the front passes 2 and reaches 3: its ingest fails -- not 1's error
    with pytest.raises(AggregationError):
        inc.close(b"ck", framing="template")  # no DB order: cannot invent worker 3's diff
    inc = IncrementalCycle(FlakyEngine(), [3], slots=2, fold_batch=4)
    inc.engine.fail_once = good[3]
    for w in range(4):
        inc.assigned(w)
    for w in (2, 3, 0, 1):
        inc.reported(w, good[w])
    inc.close(b"ck", framing="template", order=[0, 1, 2, 3], fetch=good.__getitem__)
    assert folded(inc.engine) == [good[k] for k in range(4)]


def test_malformed_diff_is_refused_to_its_sender_only():
    """a bad diff raises in its own report and leaves no trace; the honest workers'
    reports and the close still work (the reference's report only stores the blob)."""
    eng = RecordingEngine(fail_on=b"bad")
    inc = IncrementalCycle(eng, [3], slots=8, fold_batch=1)
    for w in range(4):
        inc.assigned(w)
    with pytest.raises(StateParseError):
        inc.reported(0, b"bad")
    inc.reported(1, b"1")
    inc.reported(0, b"0")  # the worker may retry with a good diff
    inc.reported(3, b"3")
    inc.close(b"ck", framing="template")
    assert folded(eng) == [b"0", b"1", b"3"]


def test_malformed_re_report_drops_the_older_diff():
    """The DB now holds the malformed bytes (cycle_manager.py:173): the older diff must not be
    averaged in their place -- close reads the row from the DB (and fails the way the reference's
    unserialize does)."""
    eng = RecordingEngine(fail_on=b"bad")
    inc = IncrementalCycle(eng, [3], slots=8, fold_batch=4)
    for w in range(3):
        inc.assigned(w)
    inc.reported(1, b"1")
    inc.reported(2, b"2")
    with pytest.raises(StateParseError):
        inc.reported(1, b"bad")
    inc.reported(0, b"0")
    assert folded(eng) == []  # the front stops at worker 1
    with pytest.raises(AggregationError):
        inc.close(b"ck", framing="template")
    eng = RecordingEngine(fail_on=b"bad")
    inc = IncrementalCycle(eng, [3], slots=8, fold_batch=4)
    for w in range(3):
        inc.assigned(w)
    inc.reported(1, b"1")
    with pytest.raises(StateParseError):
        inc.reported(1, b"bad")
    with pytest.raises(StateParseError):  # the DB's bytes for row 1, read at close
        inc.close(b"ck", framing="template", order=[1], fetch=lambda w: b"bad")


def test_malformed_diff_is_refused_when_it_would_park():
    """A diff that cannot go to HBM yet (no spare slot) is validated before it is parked."""
    ck = build_state_fast([np.zeros(3, np.float32)])
    good = build_state_fast([np.ones(3, np.float32)])
    bad = build_state_fast([np.ones(4, np.float32)])
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], slots=2, fold_batch=4)
    for w in range(4):
        inc.assigned(w)
    inc.reported(2, good)       # takes a slot (one stays for the front)
    with pytest.raises(StateParseError):
        inc.reported(3, bad)    # would park: scanned against the layout first
    inc.reported(3, good)
    assert inc.n_parked == 1
    inc.reported(0, good)
    inc.reported(1, good)
    inc.close(ck, framing="template")
    assert len(folded(eng)) == 4


def test_reports_from_many_threads_and_a_late_one():
    """Request threads report concurrently (the node's handlers); folds still follow assignment
    order exactly once each, and a report after close is ignored."""
    import threading

    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], checkpoint=b"ck", slots=16, fold_batch=3)
    workers = list(range(64))
    for w in workers:
        inc.assigned(w)
    rng = np.random.default_rng(4)
    order = [int(w) for w in rng.permutation(workers)]
    threads = [threading.Thread(target=inc.reported, args=(w, mk(w))) for w in order]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    inc.close(b"ck", framing="template")
    assert folded(eng) == [mk(k) for k in range(64)]
    inc.reported(0, b"late")  # accepted and ignored (fl_events.py:261-263)
    with pytest.raises(AggregationError):
        inc.close(b"ck", framing="template")


class ScanningEngine(RecordingEngine):
    """ingest_state / ckpt_upload_state refuse what the real State walker refuses."""

    def ingest_state(self, k, pb):
        from pygrid_amd import state

        state.scan(pb)
        super().ingest_state(k, pb)

    def ckpt_upload_state(self, pb):
        from pygrid_amd import state

        state.scan(pb)
        super().ckpt_upload_state(pb)


def _f64_diff():
    from pygrid_amd.state_schema import classes

    st = classes()["State"]()
    st.ParseFromString(mk(9))
    td = st.tensors[0].torch_tensor.contents_data
    td.ClearField("contents_float32")
    td.dtype = "float64"
    td.contents_float64.extend([9.0, 9.0, 9.0])
    return st.SerializeToString()


@pytest.mark.parametrize("parked", [False, True])
def test_float64_diff_declines_the_cycle_not_the_worker(parked):
    """A well-formed float64 diff (the reference averages it with torch's type promotion) is
    accepted; the cycle is declined as a whole, later reports are only recorded, and close raises
    ModelNotAcceleratedError so the node averages the cycle itself.  A truncated diff is still
    refused to its sender."""
    from pygrid_amd import ModelNotAcceleratedError

    eng = ScanningEngine()
    inc = IncrementalCycle(eng, [3], slots=2 if parked else 8, fold_batch=1)
    for w in range(5):
        inc.assigned(w)
    with pytest.raises(StateParseError):
        inc.reported(0, mk(0)[:-2])
    if parked:  # worker 3's diff waits on the host (no free slot for a non-front diff): scanned there
        inc.reported(2, mk(2))
    inc.reported(3, _f64_diff())
    assert inc.declined and "non-float32" in inc.declined
    n_ingests = sum(c[0] == "ingest" for c in eng.calls)
    inc.reported(4, mk(4))
    assert sum(c[0] == "ingest" for c in eng.calls) == n_ingests  # recorded, not ingested
    with pytest.raises(ModelNotAcceleratedError):
        inc.close(mk(7), framing="template")


def test_float64_checkpoint_declined_at_cycle_start():
    from pygrid_amd import ModelNotAcceleratedError

    with pytest.raises(ModelNotAcceleratedError):
        IncrementalCycle(ScanningEngine(), [3], slots=4, checkpoint=_f64_diff())


# ---- the close's DB reads: exactly fetch_plan (what the node reads under its report gate) --------------

def close_like_the_node(inc, order, db):
    """seal -> fetch_plan -> (the gate released) finish, with a fetch that refuses any row the plan
    did not name: the node's flow (pygrid_amd.node.NodeEngine.average_plan_diffs)."""
    needs = inc.seal(order=order)
    plan = inc.fetch_plan() if needs else []
    assert len(set(plan)) == len(plan)
    read = []

    def fetch(w):
        assert w in plan, f"finish read row {w!r}, which fetch_plan did not name ({plan})"
        read.append(w)
        return db[w]
    new = inc.finish(b"ck", framing="template", fetch=fetch)
    assert read == plan  # the plan is exact: every row it names is read, in its order
    return new


@pytest.mark.parametrize("seed", range(40))
def test_randomised_scripts_fold_the_db_order_and_read_only_the_planned_rows(seed):
    """Random scripts -- assignments (some announced behind the fold), shuffled reports, re-reports,
    malformed re-reports, parked diffs under slot pressure, random DB orders -- fold exactly the DB
    order's latest diffs, and the close reads from the DB exactly the rows ``fetch_plan`` named
    (the node releases its report gate before folding)."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(3, 30))
    slots = int(rng.integers(2, n + 3))
    eng = RecordingEngine(fail_on=b"bad")
    inc = IncrementalCycle(eng, [3], slots=slots, fold_batch=int(rng.integers(1, 4)))
    late = set(int(x) for x in rng.choice(n, size=int(rng.integers(0, n // 3 + 1)), replace=False))
    for w in range(n):
        if w not in late:
            inc.assigned(w, key=w)
    db = {}
    events = [("r", int(w)) for w in rng.permutation(n) if rng.random() >= 0.25]
    events += [("r", int(w)) for w in rng.choice(n, size=int(rng.integers(0, 6)))]   # re-reports
    events += [("a", w) for w in late]
    rng.shuffle(events)
    version = {}
    for kind, w in events:
        if kind == "a":
            inc.assigned(w, key=w)
            continue
        version[w] = version.get(w, 0) + 1
        if rng.random() < 0.05:
            db[w] = b"bad"
            if w in inc._folded_set:  # folded already: the early fold goes stale, the close reads the DB
                inc.reported(w, b"bad")
            else:
                with pytest.raises(StateParseError):
                    inc.reported(w, b"bad")
        else:
            db[w] = mk(100 * version[w] + w)
            inc.reported(w, db[w])
    order = sorted(db)
    if not order:
        return
    if rng.random() < 0.3:
        order = [order[i] for i in rng.permutation(len(order))]
    if any(db[w] == b"bad" for w in order):
        with pytest.raises(StateParseError):
            close_like_the_node(inc, order, db)
        return
    close_like_the_node(inc, order, db)
    assert folded(eng) == [db[w] for w in order]


@pytest.mark.parametrize("slots", [2, 3, 5])
@pytest.mark.parametrize("seed", range(6))
def test_fetch_plan_covers_evictions_under_slot_pressure(slots, seed):
    """Few slots and a DB order unlike the assignment order: the close gives up slots of diffs
    needed later and re-reads them -- fetch_plan names those rows too."""
    rng = np.random.default_rng(70 + seed)
    eng = RecordingEngine()
    n = 16
    inc = IncrementalCycle(eng, [3], slots=slots, fold_batch=2)
    for w in range(n):
        inc.assigned(w, key=w)
    reporters = [w for w in range(n) if w % 5 != 3]
    db = {w: mk(w) for w in reporters}
    for w in rng.permutation(reporters):
        inc.reported(int(w), db[int(w)])
    order = [reporters[i] for i in rng.permutation(len(reporters))]
    close_like_the_node(inc, order, db)
    assert folded(eng) == [db[w] for w in order]


def test_fetch_plan_needs_a_seal():
    inc = IncrementalCycle(RecordingEngine(), [3], slots=4)
    with pytest.raises(AggregationError):
        inc.fetch_plan()


@pytest.mark.parametrize("seed", range(4))
def test_concurrent_reports_never_overlap_engine_calls(seed):
    """Report handlers on several threads with re-reports: every engine call happens under the
    cycle's lock (no two at once), and the close is the reference's order."""
    import threading
    import time as _time

    class GuardedEngine(RecordingEngine):
        def __getattribute__(self, name):
            attr = object.__getattribute__(self, name)
            if callable(attr) and not name.startswith("_"):
                def guarded(*a, **k):
                    lock = object.__getattribute__(self, "_guard")
                    assert lock.acquire(blocking=False), f"engine call {name} overlapped another"
                    try:
                        _time.sleep(0.0002)
                        return attr(*a, **k)
                    finally:
                        lock.release()
                return guarded
            return attr

    rng = np.random.default_rng(300 + seed)
    eng = GuardedEngine()
    object.__setattr__(eng, "_guard", threading.Lock())
    n = 40
    inc = IncrementalCycle(eng, [3], slots=48)
    for w in range(n):
        inc.assigned(w)
    reporters = [w for w in range(n) if rng.random() >= 0.2]
    rereport = set(int(w) for w in rng.choice(reporters, size=4, replace=False))
    order = [int(w) for w in rng.permutation(reporters)]
    chunks = [order[i::4] for i in range(4)]
    errors = []

    def handler(ws, delays):
        try:
            for w, d in zip(ws, delays):
                _time.sleep(d)
                inc.reported(w, mk(w + 1000) if w in rereport else mk(w))
            for w in ws:
                if w in rereport:
                    inc.reported(w, mk(w))  # the latest diff wins
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=handler, args=(c, list(rng.uniform(0, 0.003, len(c))))) for c in chunks]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    # a re-report after its diff was folded is read from the DB (fetch) at close
    inc.close(b"ck", framing="template", order=sorted(reporters), fetch=mk)
    assert folded(eng) == [mk(w) for w in sorted(reporters)]


def test_a_dropped_open_cycle_is_abandoned_by_the_next_one():
    """A cycle dropped without close: the next cycle on the engine abandons it, so nothing of the
    old cycle touches the new one's slots; a cycle that was closed keeps its resident checkpoint for
    the next one."""
    eng = RecordingEngine()
    a = IncrementalCycle(eng, [3], slots=8)
    for w in range(4):
        a.assigned(w)
    for w in (2, 1, 3):
        a.reported(w, mk(w))
    b = IncrementalCycle(eng, [3], slots=8)
    assert a._closed
    for w in range(3):
        b.assigned(w)
    for w in (1, 0, 2):
        b.reported(w, mk(10 + w))
    a.reported(0, mk(0))  # the abandoned cycle ignores it
    b.close(b"ck", framing="template")
    assert folded(eng) == [mk(10), mk(11), mk(12)]
    with pytest.raises(AggregationError):
        a.close(b"ck", framing="template")
    c = IncrementalCycle(eng, [3], slots=8)  # b was closed: abandoning it is a no-op
    assert eng.cycle_owner is c and b.last_close
