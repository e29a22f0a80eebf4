"""GPU: report-time ingest in param ranges (pgh_set_ingest_ranges, on in IncrementalCycle): each
State diff of a shard of >= 1 M params goes to HBM chunk by chunk with an event each, and the
close's FINAL ranges wait only on the chunks of the last report they read -- the close runs beside
the tail of that report's copy, and its D2H pieces on the aux stream beside it.  The new checkpoint
must be bit-identical to the oracle's fold of the same diffs, whichever way each diff arrived
(pageable bytes through the pinned staging ring, or page-locked blocks DMA'd as they lie), with
ragged shard sizes (a last chunk shorter than the others), every mode, chained cycles, a copy
issued between the last report and the close (which must fall back to the whole-stream wait), and
a two-child group.  Floats compared as bits: bit-exact, as for every fold path."""
import base64
import gc

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32
# 2 M + 2 M + 1.3 M floats per chunk of 2 Mi params: 3 chunks, the last one short; payload spans
# cross chunk boundaries inside a tensor
SHAPES = [(2100, 2000), (1000,), (3, 333_333), (7,)]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _want(mode, ckpt, diffs_in_order, weights=None):
    if mode == 0:
        return O.fedavg_mean(ckpt, diffs_in_order)
    if mode == 1:
        return O.fedavg_iterative(ckpt, diffs_in_order)
    return O.fedavg_weighted(ckpt, diffs_in_order, np.asarray(weights, F))


@pytest.fixture(scope="module")
def engine():
    import os

    from pygrid_amd import Engine

    eng = Engine(int(os.environ.get("PGH_DEVICE", "0")))
    yield eng
    eng.close()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("pinned", [False, True])
def test_ranged_report_close_is_bit_exact(engine, mode, pinned):
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.report import PinnedPool, b64decode
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(900 + 10 * mode + pinned)
    n = 9
    reporters = [w for w in range(n) if w != 3]
    numel = [int(np.prod(s)) for s in SHAPES]
    assert sum(numel) > 2 * (1 << 21)
    weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n)}
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    ck = build_state_fast(ckpt)
    want = ckpt
    pool = PinnedPool(max_blocks=4) if pinned else None
    try:
        for cyc in range(2):  # chained: cycle 2 starts from cycle 1's resident checkpoint
            diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for w in reporters}
            inc = IncrementalCycle(engine, numel, mode=mode, slots=n, fold_batch=3,
                                   weights_by_worker=weights if mode == 2 else None, checkpoint=ck)
            for w in range(n):
                inc.assigned(w)
            for w in rng.permutation(reporters):
                pb = build_state_fast(diffs[int(w)])
                if pinned:
                    pb = b64decode(base64.b64encode(pb).decode(), into=pool)
                    assert isinstance(pb, memoryview)
                inc.reported(int(w), pb)
                del pb
                gc.collect()
            ck = inc.close(ck)  # right behind the last report's (ranged) copy
            order = sorted(reporters)
            want = _want(mode, want, [diffs[w] for w in order], [weights[w] for w in order])
            for g, w_ in zip(parse_state(ck), want):
                assert np.array_equal(bits(g), bits(w_)), cyc
    finally:
        if pool is not None:
            pool.close()


def test_ranged_off_and_on_agree_and_a_copy_in_between_falls_back(engine, monkeypatch):
    """PGH_INGEST_RANGES=0 (whole-copy ingest) and the default give the same bytes; a checkpoint
    upload issued after the last ranged report (a copy the ranges do not cover) makes the close
    wait on the whole copy stream, still bit-exact."""
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(950)
    numel = [int(np.prod(s)) for s in SHAPES]
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for _ in range(4)]
    want = O.fedavg_mean(ckpt, diffs)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("PGH_INGEST_RANGES", flag)
        ck = build_state_fast(ckpt)
        inc = IncrementalCycle(engine, numel, slots=4, fold_batch=8, checkpoint=ck)
        for w in range(4):
            inc.assigned(w)
        for w in (2, 0, 3, 1):
            inc.reported(w, build_state_fast(diffs[w]))
        outs.append(inc.close(ck))
    for off, on, w_ in zip(parse_state(outs[0]), parse_state(outs[1]), want):  # (fresh ids: not the bytes)
        assert np.array_equal(bits(off), bits(w_)) and np.array_equal(bits(on), bits(w_))
    # the checkpoint re-uploaded between the last report and the close
    monkeypatch.setenv("PGH_INGEST_RANGES", "1")
    ck = build_state_fast(ckpt)
    inc = IncrementalCycle(engine, numel, slots=4, fold_batch=8, checkpoint=ck)
    for w in range(4):
        inc.assigned(w)
    for w in (1, 3, 0, 2):
        inc.reported(w, build_state_fast(diffs[w]))
    engine.ckpt_upload_state(ck)
    new = inc.close(ck)
    for g, w_ in zip(parse_state(new), want):
        assert np.array_equal(bits(g), bits(w_))


def test_ranged_report_close_on_a_group():
    """Two children on GPU 0, each shard >= 1 M params: each child ranges its own slice."""
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(960)
    numel = [int(np.prod(s)) for s in SHAPES]
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for _ in range(5)]
    with Engine(devices=[0, 0]) as grp:
        ck = build_state_fast(ckpt)
        inc = IncrementalCycle(grp, numel, slots=6, fold_batch=2, checkpoint=ck)
        for w in range(5):
            inc.assigned(w)
        for w in (4, 1, 0, 3, 2):
            inc.reported(w, build_state_fast(diffs[w]))
        new = inc.close(ck)
    for g, w_ in zip(parse_state(new), O.fedavg_mean(ckpt, diffs)):
        assert np.array_equal(bits(g), bits(w_))


def _slot_close_setup(engine, rng, n=5, ranges=True):
    """Engine-level report-time close: n State diffs in slots 0..n-1 (ranged or not), the resident
    checkpoint uploaded; returns (ckpt flat, diffs flat [n, P])."""
    from pygrid_amd.state_schema import build_state_fast

    numel = [int(np.prod(s)) for s in SHAPES]
    ck = [rng.standard_normal(s).astype(F) for s in SHAPES]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for _ in range(n)]
    engine.set_layout(numel)
    engine.reserve(n)
    engine.set_ingest_ranges(ranges)
    engine.ckpt_upload_state(build_state_fast(ck))
    for k in range(n):
        engine.ingest_state(k, build_state_fast(diffs[k]))
    flat = lambda ts: np.concatenate([t.reshape(-1) for t in ts])  # noqa: E731
    return flat(ck), np.stack([flat(d) for d in diffs])


def _patched(engine):
    from pygrid_amd.state_schema import build_state_fast, parse_state

    out = engine.ckpt_patch_state(build_state_fast([np.zeros(s, F) for s in SHAPES]))
    return np.concatenate([t.reshape(-1) for t in parse_state(out)])


@pytest.mark.parametrize("ranges", [False, True])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_final_pass_starts_the_d2h_and_the_patch_adopts_it(engine, ranges, mode):
    """The FINAL pass of a slot fold issues the D2H pieces whose ranges are done (pre_d2h); the
    patch right after adopts the ring.  Its bytes, and a download after it (a fresh D2H), are the
    fold's, in every mode, ranged ingest on and off."""
    from oracle import coracle

    rng = np.random.default_rng(970 + mode + 10 * ranges)
    c, d = _slot_close_setup(engine, rng, ranges=ranges)
    w = rng.uniform(0.5, 2.0, 5).astype(F)
    order = [3, 0, 4, 1, 2]
    if mode == 2:
        engine.set_weights(w[order])
    engine.fold_slots_finish_resident(mode, order)
    want = coracle.fedavg(mode, d[order], c, w[order] if mode == 2 else None)
    assert np.array_equal(bits(_patched(engine)), bits(want))
    assert np.array_equal(bits(engine.ckpt_download()), bits(want))


def test_started_d2h_dropped_by_an_upload_or_a_staged_ingest(engine):
    """A D2H the FINAL pass started and nobody adopted must not leak into a later read: after a
    checkpoint upload the download and the patch return the uploaded floats; after one or two
    staged ingests (which take the pinned slots) the patch still returns the fold's result."""
    from oracle import coracle
    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng(980)
    c, d = _slot_close_setup(engine, rng)
    engine.fold_slots_finish_resident(0, [0, 1, 2, 3, 4])
    other = rng.standard_normal(c.size).astype(F)
    engine.ckpt_upload(other)
    assert np.array_equal(bits(engine.ckpt_download()), bits(other))
    assert np.array_equal(bits(_patched(engine)), bits(other))
    for staged in range(2):
        c, d = _slot_close_setup(engine, rng)
        engine.fold_slots_finish_resident(0, [4, 3, 2, 1, 0])
        want = coracle.fedavg(0, d[[4, 3, 2, 1, 0]], c, None)
        for k in range(staged + 1):
            engine.ingest_state(k, build_state_fast([(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES]))
        assert np.array_equal(bits(_patched(engine)), bits(want)), staged
