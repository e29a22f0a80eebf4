"""GPU: report-time aggregation equals the reference's fold over the completed WorkerCycles in
id order, for any report order, with workers that never report."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("ckpt_at_start", [False, True])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_incremental_cycle_matches_reference_order(engine, mode, ckpt_at_start):
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
    inc = IncrementalCycle(engine, [int(np.prod(s)) for s in shapes], mode=mode, ring_slots=8, fold_batch=2,
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
