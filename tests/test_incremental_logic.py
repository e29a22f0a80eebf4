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


# ---- speculative folds (pgh_fold_slots_keep / pgh_fold_mark / pgh_fold_rewind) ----------------------

class SpecEngine(RecordingEngine):
    """RecordingEngine with the library's saved fold states: `state` is the running fold state as a
    payload list; a kept fold appends the slots' current payloads without freeing them."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.state = []
        self.marks = {}
        self.kept_rows = 0
        self.max_marks_held = 0

    def fold_slots(self, mode, slots):
        self.state += [self.slot[s] for s in slots]
        super().fold_slots(mode, slots)

    def fold_slots_keep(self, mode, slots):
        assert len(set(slots)) == len(slots) and all(s in self.slot for s in slots)
        self.state += [self.slot[s] for s in slots]
        self.kept_rows += len(slots)
        self.calls.append(("keep", len(slots)))

    def fold_mark(self, m):
        self.marks[m] = list(self.state)
        self.max_marks_held = max(self.max_marks_held, len(self.marks))

    def fold_rewind(self, m):
        self.state = list(self.marks[m])
        self.calls.append(("rewind", len(self.state)))

    def fold_unmark(self, m):
        del self.marks[m]

    def fold_restart(self):
        self.state = []
        super().fold_restart()

    def fold_slots_finish_resident(self, mode, slots):
        self.final_rows = len(slots)
        self.state += [self.slot[s] for s in slots]
        self.result = list(self.state)
        self.state = []
        super().fold_slots_finish_resident(mode, slots)


def test_speculation_folds_every_report_and_closes_with_nothing_left():
    """Worker 0 never reports, so nothing is ever certain; every reported diff is folded as it
    arrives anyway (in assignment order), rewound when an earlier worker reports after it, and the
    close only finishes: no rows left to fold."""
    rng = np.random.default_rng(11)
    eng = SpecEngine()
    n = 40
    inc = IncrementalCycle(eng, [3], speculate=True, slots=n, fold_batch=8)
    assert inc.speculate
    for w in range(n):
        inc.assigned(w)
    reporters = [w for w in range(1, n) if rng.random() >= 0.2]
    seen = []
    for w in rng.permutation(reporters):
        inc.reported(int(w), bytes([int(w)]))
        seen.append(int(w))
        assert eng.state == [bytes([x]) for x in sorted(seen)]  # the fold state is the plan so far
    assert eng.marks and any(c[0] == "rewind" for c in eng.calls)
    inc.close(b"ck", framing="template")
    assert eng.result == [bytes([w]) for w in sorted(reporters)]
    assert eng.final_rows == 0 and inc.last_close["early"] == len(reporters) and not inc.last_close["refold"]
    assert eng.marks == {}  # every saved state released at close


def test_speculation_frees_certain_slots_and_rewinds_only_after_the_base():
    eng = SpecEngine()
    inc = IncrementalCycle(eng, [3], speculate=True, slots=6)
    for w in "abcdefgh":
        inc.assigned(w)
    for w in "abd":            # a, b certain; d speculative (c outstanding)
        inc.reported(w, w.encode())
    assert eng.state == [b"a", b"b", b"d"] and inc._base == 2 and len(inc._free) == 6 - 1
    inc.reported("c", b"c")    # lands before d: back to the mark after b, refold c, d
    assert eng.state == [b"a", b"b", b"c", b"d"] and eng.calls[-2][0] == "rewind" or ("rewind", 2) in eng.calls
    assert inc._base == 4 and len(inc._free) == 6
    inc.reported("b", b"b2")   # re-report of a certain (freed) diff: the close re-folds from the DB
    assert inc.stale
    db = {"a": b"a", "b": b"b2", "c": b"c", "d": b"d"}
    inc.close(b"ck", framing="template", order=list("abcd"), fetch=db.__getitem__)
    assert eng.result == [b"a", b"b2", b"c", b"d"] and inc.last_close["refold"]


def test_speculative_re_report_rewinds_and_folds_the_latest_diff():
    eng = SpecEngine()
    inc = IncrementalCycle(eng, [3], speculate=True, slots=8)
    for w in range(6):
        inc.assigned(w)
    for w, v in ((2, b"2a"), (4, b"4a"), (3, b"3a"), (4, b"4b"), (2, b"2b")):
        inc.reported(w, v)
    assert eng.state == [b"2b", b"3a", b"4b"]  # worker 0 outstanding: all speculative, kept
    inc.reported(0, b"0")
    inc.close(b"ck", framing="template", order=[0, 2, 3, 4], fetch=None)
    assert eng.result == [b"0", b"2b", b"3a", b"4b"] and not inc.last_close["refold"]


def test_close_rewinds_to_the_db_order():
    """The DB returns another order than assignment: the close goes back to the last saved state
    inside the common prefix and folds the rest from the kept slots -- no DB reads."""
    eng = SpecEngine()
    inc = IncrementalCycle(eng, [3], speculate=True, slots=8, mark_every=1)
    for w in range(6):
        inc.assigned(w)
    for w in (5, 1, 2, 4):
        inc.reported(w, bytes([w]))
    assert eng.state == [bytes([w]) for w in (1, 2, 4, 5)]
    inc.close(b"ck", framing="template", order=[1, 2, 5, 4], fetch=lambda w: pytest.fail("DB read"))
    assert eng.result == [bytes([w]) for w in (1, 2, 5, 4)]
    assert inc.last_close["early"] == 2 and inc.last_close["from_hbm"] == 2 and not inc.last_close["refold"]


def test_mark_budget_thins_saved_states():
    rng = np.random.default_rng(12)
    eng = SpecEngine()
    n = 60
    inc = IncrementalCycle(eng, [1000], speculate=True, slots=n, speculation_budget=5 * 4000)
    assert inc.max_marks == 5
    for w in range(n):
        inc.assigned(w)
    reporters = [w for w in range(1, n) if rng.random() >= 0.2]
    for w in rng.permutation(reporters):
        inc.reported(int(w), bytes([int(w)]))
    assert eng.max_marks_held <= 5
    inc.close(b"ck", framing="template")
    assert eng.result == [bytes([w]) for w in sorted(reporters)]


def test_no_speculation_without_budget():
    with pytest.raises(AggregationError):  # room for one saved state only
        IncrementalCycle(SpecEngine(), [1000], slots=4, speculation_budget=4000, speculate=True)
    assert not IncrementalCycle(SpecEngine(), [10], slots=4).speculate  # opt-in (r04)
    assert not IncrementalCycle(SpecEngine(), [10], slots=4, speculate=False).speculate
    with pytest.raises(AggregationError):
        IncrementalCycle(RecordingEngine(), [10], slots=4, speculate=True)


@pytest.mark.parametrize("seed", range(30))
def test_randomised_speculation_matches_the_reference_order(seed):
    """Random scripts -- assignments (some announced behind the fold), shuffled reports, re-reports,
    malformed re-reports, parked diffs under slot pressure, thinned marks, random DB orders -- fold
    exactly the DB order's latest diffs, and speculation rewinds instead of reading the DB whenever
    the order was the assignment order."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(3, 30))
    slots = int(rng.integers(2, n + 3))
    eng = SpecEngine(fail_on=b"bad")
    inc = IncrementalCycle(eng, [3], speculate=True, slots=slots, fold_batch=int(rng.integers(1, 4)),
                           speculation_budget=int(rng.integers(2, 12)) * 12)
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
            inc.close(b"ck", framing="template", order=order, fetch=db.__getitem__)
        return
    inc.close(b"ck", framing="template", order=order, fetch=db.__getitem__)
    assert eng.result == [db[w] for w in order]


@pytest.mark.parametrize("slots", [2, 3, 5])
@pytest.mark.parametrize("seed", range(8))
def test_speculation_under_slot_pressure_closes_without_the_db(slots, seed):
    """Few slots: speculative folds keep their slots, so the reserved slot of the fold front must
    still come free (a mark at the certain point frees the certain diffs) -- every diff stays in
    HBM or on the host and the close needs no DB read."""
    rng = np.random.default_rng(50 + seed)
    eng = SpecEngine()
    n = 24
    inc = IncrementalCycle(eng, [3], speculate=True, slots=slots, fold_batch=2, mark_every=3)
    for w in range(n):
        inc.assigned(w)
    reporters = [w for w in range(n) if w % 5 != 3]
    for w in rng.permutation(reporters):
        inc.reported(int(w), mk(int(w)))
        assert len([s for s in eng.slot]) <= slots
    inc.close(b"ck", framing="template")
    assert eng.result == [mk(w) for w in reporters]


class BusySpecEngine(SpecEngine):
    """SpecEngine with pgh_fold_busy: `busy` says whether the GPU is still folding."""

    busy = False

    def fold_busy(self):
        return self.busy


@pytest.mark.parametrize("gap_ms,busy,folds_during_reports", [(5.0, False, True), (0.5, False, False),
                                                              (5.0, True, False)])
def test_lazy_speculation_waits_for_slow_reports_and_an_idle_gpu(monkeypatch, gap_ms, busy, folds_during_reports):
    """Lazy speculation (the default with a real engine): a report is folded at once only when the
    previous one came at least min_gap_ms before and the GPU is idle; otherwise it waits for a later
    report or the close -- the result is the same either way."""
    import pygrid_amd.incremental as inc_mod

    clock = [100.0]
    monkeypatch.setattr(inc_mod.time, "monotonic", lambda: clock[0])
    eng = BusySpecEngine()
    eng.busy = busy
    inc = IncrementalCycle(eng, [3], speculate=True, slots=16)
    assert inc.speculate and inc._lazy
    for w in range(8):
        inc.assigned(w)
    for w in (3, 1, 6, 2, 5, 7, 4):   # worker 0 never reports
        clock[0] += gap_ms / 1e3
        inc.reported(w, bytes([w]))
    assert (len(eng.state) > 1) == folds_during_reports
    inc.close(b"ck", framing="template")
    assert eng.result == [bytes([w]) for w in range(1, 8)]


def test_out_of_hbm_for_saved_states_degrades_not_fails():
    """pgh_fold_mark failing (no HBM for another saved state) keeps speculating with fewer saved
    states; reports never fail for it and the close is still the reference's order."""
    class TightEngine(SpecEngine):
        def fold_mark(self, m):
            if len(self.marks) >= 3:
                raise AggregationError("fold state buffer allocation failed")
            super().fold_mark(m)

    rng = np.random.default_rng(77)
    eng = TightEngine()
    inc = IncrementalCycle(eng, [3], speculate=True, slots=40, mark_every=2)
    for w in range(40):
        inc.assigned(w)
    reporters = [w for w in range(1, 40) if rng.random() >= 0.2]
    for w in rng.permutation(reporters):
        inc.reported(int(w), bytes([int(w)]))
    assert len(eng.marks) <= 3 and inc.max_marks <= 3
    inc.close(b"ck", framing="template")
    assert eng.result == [bytes([w]) for w in sorted(reporters)]


def test_lazy_skips_are_folded_by_a_timer_once_reports_pause(monkeypatch):
    """Reports back to back leave their folds to a later report; when none comes within min_gap (the
    close comes later, e.g. at the cycle's end), a timer folds them -- and waits while the GPU is
    still busy -- so the close finds the fold done.  The result is unchanged."""
    import time as _time

    import pygrid_amd.incremental as inc_mod

    clock = [100.0]
    monkeypatch.setattr(inc_mod.time, "monotonic", lambda: clock[0])
    eng = BusySpecEngine()
    eng.busy = True
    inc = IncrementalCycle(eng, [3], speculate=True, slots=16, min_gap_ms=2.0)
    for w in range(8):
        inc.assigned(w)
    for w in (3, 1, 0, 6, 2, 5, 7, 4):
        clock[0] += 0.5e-3
        inc.reported(w, bytes([w]))
    assert len(eng.state) <= 1  # nothing folded while the reports came back to back
    _time.sleep(0.05)
    assert len(eng.state) <= 1  # the fake clock says the reports are still arriving
    clock[0] += 0.01
    _time.sleep(0.05)
    assert len(eng.state) <= 1  # paused, but the GPU is still busy
    eng.busy = False
    deadline = _time.time() + 5
    while len(eng.state) < 8 and _time.time() < deadline:
        _time.sleep(0.01)
    assert len(eng.state) == 8, eng.state  # folded by the timer
    inc.close(b"ck", framing="template")
    assert inc.last_close["folded_before_close"] == 8
    assert eng.result == [bytes([w]) for w in range(8)]
    assert inc._timer is None


@pytest.mark.parametrize("seed", range(4))
def test_concurrent_reports_and_timer_folds_never_overlap_engine_calls(seed):
    """Report handlers on several threads, the deferred-fold timer and re-reports: every engine call
    happens under the cycle's lock (no two at once), and the close is the reference's order."""
    import threading
    import time as _time

    class GuardedEngine(BusySpecEngine):
        def __getattribute__(self, name):
            attr = object.__getattribute__(self, name)
            if callable(attr) and not name.startswith("_") and name not in ("fold_busy",):
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
    inc = IncrementalCycle(eng, [3], speculate=True, slots=48, min_gap_ms=1.0, mark_every=4)
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
                eng.busy = bool(rng.random() < 0.3)
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
    eng.busy = False
    _time.sleep(0.05)
    assert not errors, errors
    # a re-report after its diff was folded for good is read from the DB (fetch) at close
    inc.close(b"ck", framing="template", order=sorted(reporters), fetch=mk)
    assert eng.result == [mk(w) for w in sorted(reporters)]


def test_a_dropped_open_cycle_is_abandoned_by_the_next_one(monkeypatch):
    """A cycle dropped without close while its deferred-fold timer is armed: the next cycle on the
    engine abandons it (timer cancelled), so nothing of the old cycle touches the new one's slots;
    a cycle that was closed keeps its resident checkpoint for the next one."""
    import time as _time

    eng = BusySpecEngine()
    eng.busy = True
    a = IncrementalCycle(eng, [3], speculate=True, slots=8, min_gap_ms=1.0)
    for w in range(4):
        a.assigned(w)
    for w in (2, 1, 3):
        a.reported(w, mk(w))
    assert a._timer is not None
    b = IncrementalCycle(eng, [3], speculate=True, slots=8, min_gap_ms=1.0)
    assert a._closed and a._timer is None
    eng.busy = False
    for w in range(3):
        b.assigned(w)
    for w in (1, 0, 2):
        b.reported(w, mk(10 + w))
    _time.sleep(0.03)
    b.close(b"ck", framing="template")
    assert eng.result == [mk(10), mk(11), mk(12)]
    with pytest.raises(AggregationError):
        a.close(b"ck", framing="template")
    c = IncrementalCycle(eng, [3], speculate=True, slots=8)  # b was closed: abandoning it is a no-op
    assert eng.cycle_owner is c and b.last_close
