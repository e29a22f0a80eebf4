"""CPU: fold order of report-time aggregation (pygrid_amd/incremental.py) with a recording
engine: the engine must see clients in WorkerCycle-id order with non-reporters dropped, and fold
early only when the position is certain."""
import numpy as np
import pytest

from pygrid_amd.exceptions import AggregationError
from pygrid_amd.incremental import IncrementalCycle


class RecordingEngine:
    def __init__(self):
        self.calls = []
        self.weights = []

    def set_layout(self, numel):
        self.calls.append(("layout", tuple(numel)))

    def reserve(self, n):
        self.calls.append(("reserve", n))

    def stream_begin(self, mode, batch):
        self.calls.append(("begin", mode, batch))

    def set_weights(self, w):
        self.weights = list(w)

    def ingest_state(self, k, pb):
        self.calls.append(("ingest", k, pb))

    def ckpt_upload_state(self, pb):
        self.calls.append(("upload", pb))

    def stream_finish_resident(self):
        self.calls.append(("finish",))

    def ckpt_patch_state(self, pb):
        self.calls.append(("patch", pb))
        return pb


def ingests(eng):
    return [(c[1], c[2]) for c in eng.calls if c[0] == "ingest"]


def test_in_order_reports_fold_immediately():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [10])
    for w in ("a", "b", "c"):
        inc.assigned(w)
    for w in ("a", "b", "c"):
        inc.reported(w, w.encode())
    assert ingests(eng) == [(0, b"a"), (1, b"b"), (2, b"c")]
    assert inc.folded_early == 3


def test_out_of_order_waits_for_earlier_workers():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [10])
    for w in range(5):
        inc.assigned(w)
    inc.reported(2, b"2")
    inc.reported(1, b"1")
    assert ingests(eng) == []            # worker 0 may still report
    inc.reported(0, b"0")
    assert ingests(eng) == [(0, b"0"), (1, b"1"), (2, b"2")]
    inc.reported(4, b"4")
    assert len(ingests(eng)) == 3        # worker 3 outstanding


def test_close_drops_non_reporters_and_keeps_id_order():
    from pygrid_amd.state_schema import build_state_fast

    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3])
    for w in range(6):
        inc.assigned(w)
    for w in (5, 1, 4, 2):
        inc.reported(w, bytes([w]))
    assert ingests(eng) == []            # worker 0 never reports
    ck = build_state_fast([np.array([1.0, 2.0, 3.0], np.float32)])
    assert inc.close(ck) == ck
    assert ingests(eng) == [(0, b"\x01"), (1, b"\x02"), (2, b"\x04"), (3, b"\x05")]
    assert inc.n_folded == 4 and inc.folded_early == 0
    assert [c[0] for c in eng.calls[-3:]] == ["upload", "finish", "patch"]


def test_checkpoint_handed_over_at_start_is_uploaded_once():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], checkpoint=b"ck")
    assert eng.calls[-1] == ("upload", b"ck")  # before any report: the upload overlaps the cycle
    inc.assigned("a")
    inc.reported("a", b"a")
    assert inc.close(b"ck") == b"ck"
    assert [c[0] for c in eng.calls].count("upload") == 1
    assert [c[0] for c in eng.calls[-2:]] == ["finish", "patch"]


def test_weights_follow_fold_order():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], mode=2, weights_by_worker={"x": 1.0, "y": 2.0, "z": 3.0})
    for w in ("x", "y", "z"):
        inc.assigned(w)
    inc.reported("z", b"z")
    inc.reported("x", b"x")
    inc.reported("y", b"y")
    assert eng.weights == [1.0, 2.0, 3.0]


def test_errors():
    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3])
    with pytest.raises(AggregationError):
        inc.reported("ghost", b"")
    inc.assigned("a")
    inc.reported("a", b"a")
    with pytest.raises(AggregationError):
        inc.reported("a", b"a")
    inc2 = IncrementalCycle(RecordingEngine(), [3])
    inc2.assigned("b")
    with pytest.raises(AggregationError):
        inc2.close(b"")


def test_reports_from_many_threads_and_a_late_one():
    """Request threads report concurrently (the node's handlers); folds still follow assignment
    order exactly once each, and a report after close is refused."""
    import threading

    eng = RecordingEngine()
    inc = IncrementalCycle(eng, [3], checkpoint=b"ck")
    workers = list(range(64))
    for w in workers:
        inc.assigned(w)
    rng = np.random.default_rng(4)
    order = [int(w) for w in rng.permutation(workers)]
    threads = [threading.Thread(target=inc.reported, args=(w, bytes([w]))) for w in order]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert ingests(eng) == [(k, bytes([k])) for k in range(64)]
    inc.close(b"ck")
    with pytest.raises(AggregationError):
        inc.reported(0, b"late")
    with pytest.raises(AggregationError):
        inc.close(b"ck")
