"""GPU: reports decoded straight into page-locked blocks (report.b64decode(into=PinnedPool)) are
DMA'd to HBM as they lie -- no host staging copy (pgh_stats h2d_staged_bytes_total does not move)
-- and the close is bit-exact against the oracle, on one GPU and on a group (VERDICT r2 next #5;
the report handler is fl_events.py:257-261)."""
import base64
import gc

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32
SHAPES = [(512, 300), (300,), (4096,)]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_pinned_reports_skip_the_staging_copy(devices):
    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.report import PinnedPool, b64decode
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(700)
    ckpt = [rng.standard_normal(s).astype(F) for s in SHAPES]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in SHAPES] for _ in range(10)]
    texts = [base64.b64encode(build_state_fast(d)).decode() for d in diffs]
    pool = PinnedPool(max_blocks=3)
    eng = Engine(devices=devices) if devices else Engine(0)
    try:
        numel = [int(np.prod(s)) for s in SHAPES]
        ck = build_state_fast(ckpt)
        inc = IncrementalCycle(eng, numel, slots=12, fold_batch=3, checkpoint=ck)
        for w in range(10):
            inc.assigned(w, key=w)
        eng.reset_stats()
        staged = []
        for w in (4, 0, 2, 1, 3, 9, 8, 7, 6, 5):
            d = b64decode(texts[w], into=pool)
            assert bytes(d) == base64.b64decode(texts[w])
            before = eng.stats()["h2d_staged_bytes_total"]
            inc.reported(w, d)
            staged.append((isinstance(d, memoryview), eng.stats()["h2d_staged_bytes_total"] - before))
            del d
            gc.collect()
        assert all(mv for mv, _ in staged) and pool.hits == 10 and pool.blocks <= 3
        assert all(n == 0 for _, n in staged)  # every payload DMA'd from the pinned block
        assert eng.stats()["h2d_bytes_total"] >= 10 * 4 * sum(numel)
        new = inc.close(ck, order=list(range(10)), framing="template")
        for g, w in zip(parse_state(new), O.fedavg_mean(ckpt, diffs)):
            assert np.array_equal(bits(g), bits(w))
        # the same diffs as pageable bytes DO go through the staging ring
        inc = IncrementalCycle(eng, numel, slots=12, fold_batch=3, checkpoint=new)
        inc.assigned(0)
        before = eng.stats()["h2d_staged_bytes_total"]
        inc.reported(0, base64.b64decode(texts[0]))
        assert eng.stats()["h2d_staged_bytes_total"] - before >= 4 * sum(numel)
    finally:
        eng.close()
        pool.close()


@pytest.mark.parametrize("gather", ["1", "0"])
@pytest.mark.parametrize("devices", [None, [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("shapes", [[(1,), (3,), (5, 7), (4097,), (2,), (12345,)], [(70001,)], [(1,)],
                                    [(64, 65), (131073,), (3,)]])
def test_pinned_messages_at_any_payload_alignment(monkeypatch, shapes, devices, gather):
    """A page-locked message goes to HBM in one DMA and k_gather_f32 moves every payload into the
    slab row, whatever byte offset protobuf gave it (tensor sizes here put payloads at every
    alignment mod 4), chunks crossing slab blocks, group shards cutting tensors -- bit-exact, and the
    same as the per-piece DMA path (PGH_PINNED_GATHER=0)."""
    import base64

    from pygrid_amd import Engine
    from pygrid_amd.report import PinnedPool, b64decode
    from pygrid_amd.state_schema import build_state_fast

    monkeypatch.setenv("PGH_PINNED_GATHER", gather)
    rng = np.random.default_rng(710 + len(shapes))
    numel = [int(np.prod(s)) for s in shapes]
    N = 5
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(N)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    pbs = [build_state_fast(d) for d in diffs]
    from pygrid_amd import state as st

    offs = [o % 4 for o, _ in st.scan(pbs[0])]
    pool = PinnedPool(max_blocks=2)
    eng = Engine(devices=devices) if devices else Engine(0)
    try:
        eng.set_layout(numel)
        eng.reserve(N)
        eng.ckpt_upload(np.concatenate([c.ravel() for c in ckpt]))
        eng.sync()
        eng.reset_stats()
        for k in range(N):
            mv = b64decode(base64.b64encode(pbs[k]).decode(), into=pool)
            assert isinstance(mv, memoryview)
            eng.ingest_state(k, mv)
            del mv
        eng.fedavg_resident(0)
        got = eng.ckpt_download()
        want = np.concatenate([w.ravel() for w in O.fedavg_mean(ckpt, diffs)])
        assert np.array_equal(bits(got), bits(want)), offs
        assert eng.stats()["h2d_staged_bytes_total"] == 0
    finally:
        eng.close()
        pool.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_one_block_reused_by_every_report_while_dmas_fly(devices):
    """Async page-locked ingest: the ingest returns with the DMA queued, so the pool's single block
    is decoded into again by the next report only after pgh_host_wait -- otherwise the next diff would
    overwrite bytes still in flight.  12 reports through ONE block, bit-exact close."""
    import base64

    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.report import PinnedPool, b64decode
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(730)
    shapes = [(2048, 1024), (1024,)]  # 8 MB per diff: the DMA takes ~0.15 ms
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(12)]
    texts = [base64.b64encode(build_state_fast(d)).decode() for d in diffs]
    pool = PinnedPool(max_blocks=1)
    eng = Engine(devices=devices) if devices else Engine(0)
    try:
        ck = build_state_fast(ckpt)
        inc = IncrementalCycle(eng, [int(np.prod(s)) for s in shapes], slots=16, checkpoint=ck)
        for w in range(12):
            inc.assigned(w)
        for w in (3, 0, 7, 1, 2, 11, 4, 5, 10, 6, 8, 9):
            d = b64decode(texts[w], into=pool)
            assert isinstance(d, memoryview)
            inc.reported(w, d)
            del d
        assert pool.hits == 12 and pool.blocks == 1
        new = inc.close(ck, framing="template")
        for g, w in zip(parse_state(new), O.fedavg_mean(ckpt, diffs)):
            assert np.array_equal(bits(g), bits(w))
    finally:
        eng.close()
        pool.close()
