"""GPU: the pipelined close (opt-in, PGH_FINAL_RANGES=4; shards of >= 1 M params): the resident
fold's FINAL pass runs as 4 param ranges alternating over two streams with an event after each,
and the new checkpoint's D2H (patch / download) runs on the copy stream piece by piece behind the
range that wrote it.  The bytes must be exactly what the
one-launch fold gives -- checked against the oracle for every mode, through fedavg_resident,
slot folds (report-time), downloads, template and fresh patches, and chained cycles."""
import numpy as np
import pytest

from oracle import coracle
from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32


@pytest.fixture(scope="module")
def piped():
    """A context created with the pipelined close on (PGH_FINAL_RANGES=4, read at pgh_create)."""
    import os

    from pygrid_amd import Engine

    old = os.environ.get("PGH_FINAL_RANGES")
    os.environ["PGH_FINAL_RANGES"] = "4"
    try:
        eng = Engine(int(os.environ.get("PGH_DEVICE", "0")))
    finally:
        if old is None:
            del os.environ["PGH_FINAL_RANGES"]
        else:
            os.environ["PGH_FINAL_RANGES"] = old
    yield eng
    eng.close()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_resident_fold_ranges_download_and_patch(piped, mode):
    engine = piped
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(400 + mode)
    shapes = [(1024, 1500), (1500,), (7, 1024), (7,)]  # 1.55 M params: 4 ranges
    numel = [int(np.prod(s)) for s in shapes]
    P, N = sum(numel), 5
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.5, 2.0, N).astype(F)
    engine.set_layout(numel)
    engine.reserve(N)
    engine.ckpt_upload(c)
    for k in range(N):
        engine.ingest(k, d[k])
    if mode == 2:
        engine.set_weights(w)
    engine.fedavg_resident(mode)
    want = coracle.fedavg(mode, d, c, w if mode == 2 else None)
    tmpl = build_state_fast([np.zeros(s, F) for s in shapes])
    patched = engine.ckpt_patch_state(tmpl)  # the first consumer right behind the ranged fold
    got = np.concatenate([t.reshape(-1) for t in parse_state(patched)])
    assert np.array_equal(bits(got), bits(want))
    assert np.array_equal(bits(engine.ckpt_download()), bits(want))


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_report_time_close_ranges(piped, mode):
    engine = piped
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(410 + mode)
    shapes = [(1200, 1000), (1000,)]
    n = 12
    reporters = [w for w in range(n) if w not in (0, 5)]
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in reporters}
    weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n)}
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck = build_state_fast(ckpt)
    want = ckpt
    for cyc in range(2):  # chained: the second cycle starts from the first one's resident output
        inc = IncrementalCycle(engine, [int(np.prod(s)) for s in shapes], mode=mode, slots=n, fold_batch=3,
                               weights_by_worker=weights if mode == 2 else None, checkpoint=ck)
        for w_ in range(n):
            inc.assigned(w_)
        for w_ in rng.permutation(reporters):
            inc.reported(int(w_), build_state_fast(diffs[int(w_)]))
        ck = inc.close(ck)
        ref = [diffs[w_] for w_ in sorted(reporters)]
        if mode == 0:
            want = O.fedavg_mean(want, ref)
        elif mode == 1:
            want = O.fedavg_iterative(want, ref)
        else:
            want = O.fedavg_weighted(want, ref, np.array([weights[w_] for w_ in sorted(reporters)], F))
        for g, w_ in zip(parse_state(ck), want):
            assert np.array_equal(bits(g), bits(w_)), cyc


def test_group_pipelined_close(monkeypatch):
    """Two children on GPU 0, each shard >= 1 M params: every child pipelines its own slice (ranges
    alternating over two streams)."""
    from pygrid_amd import Engine

    monkeypatch.setenv("PGH_FINAL_RANGES", "4")
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(420)
    shapes = [(2048, 1100), (1100,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(4)]
    with Engine(devices=[0, 0]) as grp:
        new = CycleAggregator(grp).average_plan_diffs({}, build_state_fast(ckpt), [build_state_fast(x) for x in diffs])
    for g, w in zip(parse_state(new), O.fedavg_mean(ckpt, diffs)):
        assert np.array_equal(bits(g), bits(w))


@pytest.mark.parametrize("mode", [0, 1])
def test_one_d2h_piece_spanning_every_range(monkeypatch, mode):
    """with D2H pieces larger than a fold range, one piece holds floats of ranges that
    ran on BOTH streams; its DMA must wait on every one of them, not only on the range holding its
    last float.  Many clients make each range long enough for an unordered copy to read a
    half-written checkpoint."""
    from pygrid_amd import Engine
    from pygrid_amd.state_schema import build_state_fast, parse_state

    monkeypatch.setenv("PGH_FINAL_RANGES", "4")  # the whole 6.2 MB checkpoint is one 8 MiB D2H piece
    rng = np.random.default_rng(430 + mode)
    shapes = [(1024, 1500), (1500,), (7, 1024), (7,)]
    numel = [int(np.prod(s)) for s in shapes]
    P, N = sum(numel), 256
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    want = coracle.fedavg(mode, d, c, None)
    tmpl = build_state_fast([np.zeros(s, F) for s in shapes])
    with Engine(0) as eng:
        eng.set_layout(numel)
        eng.reserve(N)
        for k in range(N):
            eng.ingest(k, d[k])
        for rep in range(3):
            eng.ckpt_upload(c)
            eng.fedavg_resident(mode)
            got = np.concatenate([t.reshape(-1) for t in parse_state(eng.ckpt_patch_state(tmpl))])
            assert np.array_equal(bits(got), bits(want)), rep
