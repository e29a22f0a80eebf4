"""GPU: report-time aggregation equals the reference's fold over the completed WorkerCycles in
id order, for any report order, with workers that never report."""
import numpy as np
import pytest

from oracle import coracle
from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("slots", [3, 8, 32])
@pytest.mark.parametrize("ckpt_at_start", [False, True])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_incremental_cycle_matches_reference_order(engine, mode, ckpt_at_start, slots):
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(70 + mode)
    shapes = [(33, 17), (17,), (5, 33), (5,)]
    n_assigned = 24
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in range(n_assigned)}
    weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n_assigned)}
    reporters = [w for w in range(n_assigned) if w % 5 != 3]  # workers 3, 8, 13, 18, 23 never report
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ckpt_pb = build_state_fast(ckpt)
    inc = IncrementalCycle(engine, [int(np.prod(s)) for s in shapes], mode=mode, slots=slots, fold_batch=2,
                           weights_by_worker=weights if mode == 2 else None,
                           checkpoint=ckpt_pb if ckpt_at_start else None)
    for w in range(n_assigned):
        inc.assigned(w)
    order = list(reporters)
    rng.shuffle(order)
    for w in order:
        inc.reported(w, build_state_fast(diffs[w]))
    new = inc.close(ckpt_pb if ckpt_at_start else build_state_fast(ckpt))
    ref_diffs = [diffs[w] for w in sorted(reporters)]  # query(cycle_id, is_completed=True) order
    if mode == 0:
        want = O.fedavg_mean(ckpt, ref_diffs)
    elif mode == 1:
        want = O.fedavg_iterative(ckpt, ref_diffs)
    else:
        want = O.fedavg_weighted(ckpt, ref_diffs, np.array([weights[w] for w in sorted(reporters)], F))
    for got, w in zip(parse_state(new), want):
        assert np.array_equal(bits(got), bits(w))
    assert inc.n_folded == len(reporters)


def test_shared_engine_resident_checkpoint_is_not_trusted_after_another_user(engine):
    """CycleAggregator keeps its last output checkpoint in HBM for the next cycle; if another
    user of the same engine (here an IncrementalCycle) replaced it meanwhile, the aggregator must
    upload the checkpoint again instead of folding into someone else's."""
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(90)
    shapes = [(40, 9), (9,)]
    numel = [int(np.prod(s)) for s in shapes]
    mk = lambda scale: [(rng.standard_normal(s) * scale).astype(F) for s in shapes]  # noqa: E731
    agg = CycleAggregator(engine)
    ck0 = mk(1.0)
    d1 = [mk(1e-2) for _ in range(3)]
    new1 = agg.average_plan_diffs({}, build_state_fast(ck0), [build_state_fast(d) for d in d1])
    want1 = O.fedavg_mean(ck0, d1)
    # someone else uses the engine in between
    other_ck = mk(1.0)
    inc = IncrementalCycle(engine, numel, slots=4, fold_batch=2, checkpoint=build_state_fast(other_ck))
    inc.assigned(0)
    inc.reported(0, build_state_fast(mk(1e-2)))
    inc.close(build_state_fast(other_ck))
    # the aggregator's next cycle starts from ITS checkpoint (new1), not the incremental result
    d2 = [mk(1e-2) for _ in range(2)]
    new2 = agg.average_plan_diffs({}, new1, [build_state_fast(d) for d in d2])
    want2 = O.fedavg_mean(want1, d2)
    for got, w in zip(parse_state(new2), want2):
        assert np.array_equal(bits(got), bits(w))


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_dropouts_at_position_zero_shuffled_arrival(engine, mode):
    """routes.py:314: ~20 % of assigned workers never report, here including the very first one,
    so nothing is ever certain before close: every reporter waits in its HBM slot and close folds
    them through the row table (> ROWTAB_MAX rows: several indexed launches), bit-exact."""
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(170 + mode)
    shapes = [(129, 33), (33,)]
    n_assigned = 700
    reporters = [w for w in range(n_assigned) if w != 0 and rng.random() >= 0.2]
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in reporters}
    weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n_assigned)}
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ckpt_pb = build_state_fast(ckpt)
    inc = IncrementalCycle(engine, [int(np.prod(s)) for s in shapes], mode=mode, slots=n_assigned, fold_batch=8,
                           weights_by_worker=weights if mode == 2 else None, checkpoint=ckpt_pb)
    for w in range(n_assigned):
        inc.assigned(w)
    for w in rng.permutation(reporters):
        inc.reported(int(w), build_state_fast(diffs[int(w)]))
    assert inc.n_parked == 0 and inc.n_folded == 0
    new = inc.close(ckpt_pb)
    ref = [diffs[w] for w in sorted(reporters)]
    if mode == 0:
        want = O.fedavg_mean(ckpt, ref)
    elif mode == 1:
        want = O.fedavg_iterative(ckpt, ref)
    else:
        want = O.fedavg_weighted(ckpt, ref, np.array([weights[w] for w in sorted(reporters)], F))
    for got, w in zip(parse_state(new), want):
        assert np.array_equal(bits(got), bits(w))
    assert inc.n_folded == len(reporters)


def test_fold_slots_api_edges(engine):
    """pgh_fold_slots rejects empty / foreign / duplicate slots and a mode change; a finish with no
    new slots after early folds writes the average of what was folded."""
    from pygrid_amd.exceptions import AggregationError

    rng = np.random.default_rng(181)
    P = 1000
    d = (rng.standard_normal((6, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    engine.set_layout([P])
    engine.reserve(8)
    engine.ckpt_upload(c)
    for k, slot in enumerate([5, 2, 7, 0, 3, 1]):
        engine.ingest(slot, d[k])
    with pytest.raises(AggregationError):
        engine.fold_slots(0, [4])          # slot 4 holds nothing
    with pytest.raises(AggregationError):
        engine.fold_slots(0, [5, 5])       # listed twice
    engine.fold_slots(0, [5, 2, 7])
    with pytest.raises(AggregationError):
        engine.fold_slots(1, [0])          # mode changed mid-cycle
    with pytest.raises(AggregationError):
        engine.fold_slots(0, [5])          # already folded (slot freed)
    engine.fold_slots(0, [0, 3])
    engine.fold_slots_finish_resident(0, [])
    want = O.fedavg_mean([c], [[x] for x in d[:5]])[0]
    assert np.array_equal(bits(engine.ckpt_download()), bits(want))


@pytest.mark.parametrize("shapes", [[(1,)], [(3,)], [(64,)], [(65,)], [(1,), (2,), (61,)], [(4, 17), (3,)]])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_slot_folds_tiny_and_ragged_shapes(engine, mode, shapes):
    """The row-table fold (K1r) at shard sizes below one lane group, around the 64-element
    alignment and with tensors of 1-3 params, folded in batches of 1, any arrival order."""
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(90 + mode + 7 * len(shapes))
    n_assigned = 9
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in range(n_assigned)}
    weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n_assigned)}
    reporters = [w for w in range(n_assigned) if w not in (0, 4)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ckpt_pb = build_state_fast(ckpt)
    inc = IncrementalCycle(engine, [int(np.prod(s)) for s in shapes], mode=mode, slots=4, fold_batch=1,
                           weights_by_worker=weights if mode == 2 else None, checkpoint=ckpt_pb)
    for w in range(n_assigned):
        inc.assigned(w)
    order = list(reporters)
    rng.shuffle(order)
    for w in order:
        inc.reported(w, build_state_fast(diffs[w]))
    new = inc.close(ckpt_pb)
    ref = [diffs[w] for w in sorted(reporters)]
    want = (O.fedavg_mean(ckpt, ref) if mode == 0 else O.fedavg_iterative(ckpt, ref) if mode == 1 else
            O.fedavg_weighted(ckpt, ref, np.array([weights[w] for w in sorted(reporters)], F)))
    for got, w in zip(parse_state(new), want):
        assert np.array_equal(bits(got), bits(w))
