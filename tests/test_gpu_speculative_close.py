"""GPU: the speculative close (pgh_fold_peek / pgh_peek_patch_state).  Whenever every reporter is
folded, IncrementalCycle takes the close's FINAL pass ahead (into a buffer of its own, copied to the
host behind it); a close that finds nothing changed commits it -- the new checkpoint bytes come from
that copy and the peeked result becomes the resident checkpoint.  Bit-exact against the oracle in
every mode, on one GPU and on groups, chained over cycles, and when the peek goes stale (a later
report, a DB order that differs, a checkpoint handed over anew)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32
SHAPES = [(300, 41), (41,), (7, 300), (7,)]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def wait_for_peek(eng, timeout_s=5.0):
    import time

    deadline = time.monotonic() + timeout_s
    while not eng.peek_valid():
        assert time.monotonic() < deadline, "no valid peek within 5 s of the last report (retry lost)"
        time.sleep(0.002)


def _want(mode, ckpt, rows, weights=None):
    if mode == 0:
        return O.fedavg_mean(ckpt, rows)
    if mode == 1:
        return O.fedavg_iterative(ckpt, rows)
    return O.fedavg_weighted(ckpt, rows, np.array(weights, F))


@pytest.mark.parametrize("devices", [None, [0, 0]])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_committed_peek_is_bit_exact_and_chains(devices, mode):
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(800 + mode)
    numel = [int(np.prod(s)) for s in SHAPES]
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    ck = build_state_fast(ckpt)
    weights = {w: float(rng.uniform(0.5, 2.0)) for w in range(12)}
    eng = Engine(devices=devices) if devices else Engine(0)
    try:
        want = ckpt
        for cyc in range(3):
            diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for w in range(12)}
            reporters = [w for w in range(12) if w % 4 != 1]
            inc = IncrementalCycle(eng, numel, speculate=True, mode=mode, slots=16, checkpoint=ck, lazy=False,
                                   weights_by_worker=weights if mode == 2 else None)
            for w in range(12):
                inc.assigned(w)
            for w in rng.permutation(reporters):
                inc.reported(int(w), build_state_fast(diffs[int(w)]))
            # the last report's peek is skipped when the previous one's copy is still running (reports
            # back to back); the settle timer takes it once the reports pause -- the regime the
            # committed peek is for
            wait_for_peek(eng)
            new = inc.close(ck)
            assert inc.last_close["peeked"], inc.last_close
            want = _want(mode, want, [diffs[w] for w in reporters], [weights[w] for w in reporters])
            for g, w in zip(parse_state(new), want):
                assert np.array_equal(bits(g), bits(w)), cyc
            ck = new  # the next cycle starts from the committed resident checkpoint, no upload
    finally:
        eng.close()


@pytest.mark.parametrize("case", ["late_report", "db_order", "new_checkpoint", "no_peek"])
def test_stale_peek_falls_back_bit_exact(case):
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(810)
    numel = [int(np.prod(s)) for s in SHAPES]
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    ck = build_state_fast(ckpt)
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for w in range(8)}
    with Engine(0) as eng:
        inc = IncrementalCycle(eng, numel, speculate=True, slots=10, checkpoint=ck, lazy=False, peek=case != "no_peek")
        for w in range(8):
            inc.assigned(w)
        for w in (5, 2, 0, 3):
            inc.reported(w, build_state_fast(diffs[w]))
        order = [0, 2, 3, 5]
        if case == "late_report":  # a report after the last peek: the close folds it (no commit)
            inc._lazy, inc.min_gap_s = True, 10.0  # it arrives "too soon": not folded, not peeked
            inc.reported(7, build_state_fast(diffs[7]))
            order = [0, 2, 3, 5, 7]
        elif case == "db_order":
            order = [0, 3, 2, 5]
        close_ck = ck
        if case == "new_checkpoint":  # the close gets other checkpoint bytes: uploaded, the peek is stale
            close_ck = build_state_fast(ckpt)
        new = inc.close(close_ck, order=order, fetch=lambda w: build_state_fast(diffs[w]))
        assert not inc.last_close["peeked"]
        for g, w in zip(parse_state(new), O.fedavg_mean(ckpt, [diffs[w] for w in order])):
            assert np.array_equal(bits(g), bits(w)), case


def test_abandoned_cycle_peek_copy_finishes_before_the_next_peek():
    """A cycle whose peek copy is still running is dropped without a close (the node fell back to
    the DB path); the next cycle's peek into another output waits for that copy, so the dropped
    output can be freed, and its own close is bit-exact."""
    import gc

    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    shapes = [(2048, 2048), (41,)]
    rng = np.random.default_rng(820)
    numel = [int(np.prod(s)) for s in shapes]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck = build_state_fast(ckpt)
    with Engine(0) as eng:
        for cyc in range(3):
            diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in range(4)}
            inc = IncrementalCycle(eng, numel, speculate=True, slots=6, checkpoint=ck, lazy=False)
            for w in range(4):
                inc.assigned(w)
            for w in (2, 0, 3, 1):
                inc.reported(w, build_state_fast(diffs[w]))
            if cyc < 2:
                del inc  # dropped with its peek copy in flight
                gc.collect()
                continue
            wait_for_peek(eng)
            new = inc.close(ck)
            assert inc.last_close["peeked"], inc.last_close
            want = O.fedavg_mean(ckpt, [diffs[w] for w in range(4)])
            for g, w in zip(parse_state(new), want):
                assert np.array_equal(bits(g), bits(w))


def test_peek_into_another_output_while_a_copy_runs():
    """Engine level: a second peek into another output while the first peek's payload copy may still
    run waits for it, then copies its own; committing the second is bit-exact."""
    from pygrid_amd import Engine
    from pygrid_amd import state as state_codec
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    shapes = [(2048, 2048), (41,)]
    rng = np.random.default_rng(830)
    numel = [int(np.prod(s)) for s in shapes]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck = build_state_fast(ckpt)
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in range(3)}
    with Engine(0) as eng:
        inc = IncrementalCycle(eng, numel, speculate=True, slots=5, checkpoint=ck, lazy=False)
        for w in range(3):
            inc.assigned(w)
        for w in (1, 2, 0):
            inc.reported(w, build_state_fast(diffs[w]))  # the last one peeks into the cycle's output
        other = state_codec.prepared_fresh_frame(ck)
        eng.fold_peek(0, into=other)
        assert eng.peek_patch_into(other[1], len(other[0]))
        want = O.fedavg_mean(ckpt, [diffs[w] for w in range(3)])
        for g, w in zip(parse_state(bytes(other[0])), want):
            assert np.array_equal(bits(g), bits(w))


@pytest.mark.parametrize("devices", [None, [0, 0]])
@pytest.mark.parametrize("mode", [0, 2])
def test_burst_then_pause_is_folded_and_peeked_by_the_timer(mode, devices):
    """Reports back to back (lazy: none folded at once), then a pause before the close: the timer
    folds them and peeks on its own thread, the close commits that peek -- bit-exact."""
    import time

    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(840 + mode)
    numel = [int(np.prod(s)) for s in SHAPES]
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    ck = build_state_fast(ckpt)
    weights = {w: float(rng.uniform(0.5, 2.0)) for w in range(10)}
    diffs = {w: build_state_fast([(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES]) for w in range(10)}
    reporters = [w for w in range(10) if w != 4]
    with (Engine(devices=devices) if devices else Engine(0)) as eng:
        inc = IncrementalCycle(eng, numel, speculate=True, mode=mode, slots=12, checkpoint=ck, min_gap_ms=50.0,
                               weights_by_worker=weights if mode == 2 else None)
        for w in range(10):
            inc.assigned(w)
        for w in rng.permutation(reporters):
            inc.reported(int(w), diffs[int(w)])
        deadline = time.time() + 10
        while (len(inc._folded) < len(reporters) or inc._timer is not None) and time.time() < deadline:
            time.sleep(0.01)
        assert len(inc._folded) == len(reporters)
        new = inc.close(ck)
        assert inc.last_close["peeked"], inc.last_close
        rows = [parse_state(diffs[w]) for w in reporters]
        want = _want(mode, ckpt, rows, [weights[w] for w in reporters])
        for g, w in zip(parse_state(new), want):
            assert np.array_equal(bits(g), bits(w))


@pytest.mark.parametrize("speculate", [False, True])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_report_time_close_of_a_large_shard_pipelines_its_final_pass(mode, speculate):
    """Rows left at close on a shard of >= 1 M params: the FINAL pass of the slot fold runs as 8
    param ranges with the D2H behind each (the default for report-time closes); the new checkpoint
    bytes, the resident checkpoint and a chained second cycle are bit-exact."""
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    shapes = [(1024, 1100), (77,)]
    rng = np.random.default_rng(850 + mode)
    numel = [int(np.prod(s)) for s in shapes]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck = build_state_fast(ckpt)
    weights = {w: float(rng.uniform(0.5, 2.0)) for w in range(6)}
    with Engine(0) as eng:
        want = ckpt
        for cyc in range(2):
            diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in range(6)}
            inc = IncrementalCycle(eng, numel, mode=mode, slots=8, checkpoint=ck, speculate=speculate,
                                   lazy=True, min_gap_ms=1e6, peek=False,
                                   weights_by_worker=weights if mode == 2 else None)
            for w in range(6):
                inc.assigned(w)
            for w in (3, 5, 2, 4, 1):  # worker 0 never reports: nothing is certain before close
                inc.reported(w, build_state_fast(diffs[w]))
            new = inc.close(ck)
            assert not inc.last_close["peeked"]
            rep = [1, 2, 3, 4, 5]
            want = _want(mode, want, [diffs[w] for w in rep], [weights[w] for w in rep])
            for g, w in zip(parse_state(new), want):
                assert np.array_equal(bits(g), bits(w)), cyc
            flat = eng.ckpt_download()
            assert np.array_equal(bits(flat), bits(np.concatenate([w.reshape(-1) for w in want])))
            ck = new


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_peek_valid_tracks_the_fold_state(devices):
    """pgh_peek_valid (ABI 7): true after a peek of the fold state as it stands, false
    once a later fold changed it, true again after the next peek -- for a group only when every
    GPU's peek holds.  IncrementalCycle records a peek only when it was taken (a skipped one is
    retried by the settle timer), so a close after a burst still commits a peek."""
    import time

    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(860)
    numel = [int(np.prod(s)) for s in SHAPES]
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    ck = build_state_fast(ckpt)
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for w in range(4)}
    with (Engine(0) if devices is None else Engine(devices=devices)) as eng:
        inc = IncrementalCycle(eng, numel, speculate=True, slots=6, checkpoint=ck, lazy=False)
        for w in range(4):
            inc.assigned(w)
        inc.reported(0, build_state_fast(diffs[0]))  # folded and peeked at once
        eng.sync()
        assert eng.peek_valid()
        inc.reported(1, build_state_fast(diffs[1]))
        inc.reported(2, build_state_fast(diffs[2]))
        inc.reported(3, build_state_fast(diffs[3]))
        deadline = time.monotonic() + 5
        while not eng.peek_valid() and time.monotonic() < deadline:  # a skipped peek is retried
            time.sleep(0.01)
        assert eng.peek_valid()
        new = inc.close(ck)
        assert inc.last_close["peeked"]
        for g, w in zip(parse_state(new), O.fedavg_mean(ckpt, [diffs[w] for w in range(4)])):
            assert np.array_equal(bits(g), bits(w))
