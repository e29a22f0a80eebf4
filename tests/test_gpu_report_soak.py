"""GPU soak of report-time aggregation at a size where every mechanism engages: a >= 1 M-param model
(the close's FINAL pass in ranges), reports arriving in random bursts and pauses, certain prefixes
folded early, re-reports before and after their fold (re-folds read through the close's fetch
plan, as the node does under its report gate), dropouts, and closes at once or after a pause, in
the DB's order.
Every cycle's new checkpoint is bit-exact against the oracle's fold in that order (reference:
cycle_manager.py:243-296), chained over cycles through the resident checkpoint."""
import time

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32
SHAPES = [(1024, 1200), (1200,), (33, 17)]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("devices", [None, [0, 0]])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_random_bursts_pauses_and_rereports_stay_bit_exact(mode, devices):
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(900 + mode)
    numel = [int(np.prod(s)) for s in SHAPES]
    n = 24
    weights = {w: float(rng.uniform(0.5, 2.0)) for w in range(n)}
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    ck = build_state_fast(ckpt)
    want = ckpt
    stats = {"folded_early": 0, "from_db": 0, "refold": 0}
    with (Engine(devices=devices) if devices else Engine(0)) as eng:
        for cyc in range(5):
            inc = IncrementalCycle(eng, numel, mode=mode, slots=n + 2, checkpoint=ck, fold_batch=2,
                                   weights_by_worker=weights if mode == 2 else None)
            for w in range(n):
                inc.assigned(w)
            reporters = [w for w in range(n) if w < 6 or rng.random() >= 0.2]  # a certain prefix
            latest = {}
            events = [int(w) for w in rng.permutation(reporters)]
            events += [int(w) for w in rng.choice(reporters, size=3, replace=False)]  # re-reports
            for w in events:
                d = [(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES]
                latest[w] = d
                inc.reported(w, build_state_fast(d))
                time.sleep(float(rng.choice([0.0, 0.0005, 0.003, 0.008])))
            time.sleep(float(rng.choice([0.0, 0.002, 0.012])))
            order = sorted(latest)  # the completed-WorkerCycle rows in row (assignment) order
            plan = inc.fetch_plan() if inc.seal(order=order) else []
            blobs = {w: build_state_fast(latest[w]) for w in plan}  # the rows read under the gate
            new = inc.finish(ck, fetch=blobs.__getitem__)
            stats["folded_early"] += inc.last_close["early"]
            stats["from_db"] += inc.last_close["from_db"]
            stats["refold"] += int(inc.last_close["refold"])
            rows = [latest[w] for w in order]
            want = (O.fedavg_mean(want, rows) if mode == 0 else O.fedavg_iterative(want, rows) if mode == 1
                    else O.fedavg_weighted(want, rows, np.array([weights[w] for w in order], F)))
            for g, w in zip(parse_state(new), want):
                assert np.array_equal(bits(g), bits(w)), (cyc, inc.last_close)
            flat = eng.ckpt_download()
            assert np.array_equal(bits(flat), bits(np.concatenate([w.reshape(-1) for w in want]))), cyc
            want = [np.asarray(w, F) for w in want]
            ck = new
    print("soak", mode, devices, stats)
    assert stats["folded_early"] > 0
