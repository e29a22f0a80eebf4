"""GPU: STREAM use of the slab (clients folded in order as they arrive, ring of R slots).

Same bar as RESIDENT: bit-exact against the oracle, for any arrival order the ring admits and
any fold batch -- the fold order is always the client order.
"""
import numpy as np
import pytest

from oracle import coracle
from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a)
    return a.shape == b.shape and np.array_equal(nan, np.isnan(b)) and np.array_equal(bits(a)[~nan], bits(b)[~nan])


def arrival_order(n, window, rng):
    """A permutation of range(n) where every client arrives fewer than `window` places after
    the fold front could need it (what a ring of `window` slots admits)."""
    order, pending, nxt = [], [], 0
    while len(order) < n:
        while nxt < n and len(pending) < window and (not pending or nxt - min(pending) < window):
            pending.append(nxt)
            nxt += 1
        k = pending.pop(int(rng.integers(len(pending))))
        order.append(k)
    return order


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("slots,batch", [(5, 1), (5, 0), (8, 3), (64, 64)])
def test_stream_matches_oracle_any_arrival(engine, mode, slots, batch):
    rng = np.random.default_rng(100 * mode + slots + batch)
    N, P = 23, 4099
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.1, 5.0, N).astype(F)
    engine.set_layout([P])
    engine.reserve(slots)
    engine.stream_begin(mode, batch)
    if mode == 2:
        engine.set_weights(w)
    b_eff = max(1, slots // 2) if batch <= 0 else min(batch, slots)
    for k in arrival_order(N, slots - b_eff + 1, rng):  # what the ring admits with this batch
        engine.ingest(k, d[k])
    got = engine.stream_finish(c)
    assert same(got, coracle.fedavg(mode, d, c, w if mode == 2 else None))
    st = engine.stats()
    assert st["n_folded"] == N


def test_stream_equals_resident(engine):
    rng = np.random.default_rng(2)
    N, P = 40, 10_007
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    engine.set_layout([P])
    engine.reserve(N)
    for k in range(N):
        engine.ingest(k, d[k])
    resident = engine.fedavg(1, c)
    engine.reserve(7)
    engine.stream_begin(1, 2)
    for k in range(N):
        engine.ingest(k, d[k])
    assert same(engine.stream_finish(c), resident)


def test_stream_synthetic_beyond_ring(engine):
    """N = 600 clients through a 128-slot ring, generated on the GPU in chunks."""
    import torch

    P, N, R, seed = 300_007, 600, 128, 77
    engine.set_layout([P])
    engine.reserve(R)
    engine.stream_begin(0, 64)
    for c0 in range(0, N, 64):
        engine.synth_ingest(seed, c0, min(64, N - c0))
    ck = torch.empty(P, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    engine.synth_ckpt_device(seed, ck.data_ptr())
    engine.stream_finish_device(ck.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    idx = np.unique(np.concatenate([np.arange(5), np.random.default_rng(0).integers(0, P, 1000), [P - 1]]))
    d = np.stack([O.synth_diff(seed, k, idx.astype(np.uint64)) for k in range(N)])
    want = coracle.fedavg(0, d, O.synth_ckpt(seed, idx.astype(np.uint64)))
    assert same(out.cpu().numpy()[idx], want)


def test_stream_secagg(engine, gold):
    z = np.load(gold / "secagg_wrap.npz")
    sh = z["shares"]  # [3][2][P]
    engine.set_layout([sh.shape[2]])
    engine.reserve(2, 1, 2)
    engine.stream_begin(16, 1)
    for k in (1, 0, 2):
        engine.ingest(k, sh[k])
    s, d = engine.stream_finish_secagg()
    assert np.array_equal(s, z["sum"]) and np.array_equal(bits(d), bits(z["dec"]))


def test_stream_secagg_synthetic(engine):
    import torch

    P, N, S = 200_003, 90, 3
    engine.set_layout([P])
    engine.reserve(32, 1, S)
    engine.stream_begin(16, 16)
    engine.synth_ingest(5, 0, 32)
    engine.synth_ingest(5, 32, 32)
    engine.synth_ingest(5, 64, 26)
    s = torch.empty(P, dtype=torch.int64, device="cuda")
    d = torch.empty(P, dtype=torch.float32, device="cuda")
    engine.stream_finish_secagg_device(s.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    idx = np.arange(0, P, 997, dtype=np.uint64)
    want = np.zeros(idx.size, np.uint64)
    with np.errstate(over="ignore"):
        for k in range(N):
            want += O.secagg_sum(O.synth_shares(5, k, S, idx)[None]).view(np.uint64)
    assert np.array_equal(s.cpu().numpy()[idx.astype(np.int64)], want.view(np.int64))


def test_stream_errors(engine):
    from pygrid_amd import AggregationError

    P = 64
    engine.set_layout([P])
    engine.reserve(4)
    engine.stream_begin(0, 4)
    x = np.ones(P, F)
    for k in (0, 1, 3):
        engine.ingest(k, x)
    with pytest.raises(AggregationError, match="ring full"):
        engine.ingest(4, x)  # slot 0 still holds client 0 (fold front waits for client 2)
    with pytest.raises(AggregationError, match="missing"):
        engine.stream_finish(np.zeros(P, F))
    engine.ingest(2, x)  # completes the run of 4 -> folded
    with pytest.raises(AggregationError, match="already folded"):
        engine.ingest(1, x)
    engine.ingest(4, x)
    out = engine.stream_finish(np.zeros(P, F))
    assert np.all(out == F(-1.0))
    with pytest.raises(AggregationError, match="not streaming"):
        engine.stream_finish(np.zeros(P, F))


def test_pinned_buffer_ingest(engine):
    from pygrid_amd import PinnedBuffer

    rng = np.random.default_rng(4)
    P, N = 1_000_001, 3
    bufs = [PinnedBuffer((P,)) for _ in range(N)]
    for b in bufs:
        b.array[:] = rng.standard_normal(P).astype(F)
    c = rng.standard_normal(P).astype(F)
    engine.set_layout([P])
    engine.reserve(N)
    for k, b in enumerate(bufs):
        engine.ingest(k, b.array)
    got = engine.fedavg(0, c)
    d = np.stack([b.array for b in bufs])
    assert same(got, coracle.fedavg(0, d, c))
    for b in bufs:
        b.free()


@pytest.mark.parametrize("mode", [0, 1])
def test_blocked_ring_small_staging(mode):
    """Column-blocked ring (P = 70,001 -> 9 blocks of 8,192, a partial last block) fed through an
    80 KiB pinned staging slot, so slot fills start and end mid-block: every head / 2-D / tail
    copy shape of h2d_range, pageable arrays and State spans, out-of-order arrival."""
    from pygrid_amd import Engine
    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng(11 + mode)
    shapes = [(3, 7001), (12,), (48_985,), (1,)]  # numel sums to 70,001; spans cross blocks
    numel = [int(np.prod(s)) for s in shapes]
    P, N, R = sum(numel), 9, 4
    assert P == 70_001
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    with Engine(0, pinned_bytes=2 * 81_920) as eng:
        eng.set_layout(numel)
        eng.reserve(R)
        _, ld, bp = eng.slab()
        assert ld == 8192 and bp == R * ld
        eng.stream_begin(mode, 2)
        for k in arrival_order(N, R - 2 + 1, rng):
            if k % 2:
                eng.ingest(k, d[k])
            else:
                parts, o = [], 0
                for s in shapes:
                    n = int(np.prod(s))
                    parts.append(d[k, o:o + n].reshape(s))
                    o += n
                eng.ingest_state(k, build_state_fast(parts))
        got = eng.stream_finish(c)
    assert same(got, coracle.fedavg(mode, d, c))


@pytest.mark.parametrize("mode,kind", [(0, 0), (1, 0), (0, 1)])
def test_config4_shard_full_size_sampled(engine, mode, kind):
    """BASELINE config 4, one GPU's shard at full size: 12.5 M params x 10,000 clients (500 GB of
    diffs) through a 1,000-slot ring, generated on the GPU in 500-client chunks exactly like
    `bench.py --workload c4-stream`; bit-exact on sampled params (block edges included) against
    the oracle folding all 10,000 clients."""
    import torch

    P, N, R, chunk, seed = 12_500_000, 10_000, 1000, 500, 4242
    engine.set_layout([P])
    engine.reserve(R)
    engine.set_synth_kind(kind)  # 1: the fast generator bench.py's c4-stream uses
    try:
        engine.stream_begin(mode, chunk)
        for c0 in range(0, N, chunk):
            engine.synth_ingest(seed, c0, min(chunk, N - c0))
        ck = torch.empty(P, dtype=torch.float32, device="cuda")
        out = torch.empty_like(ck)
        engine.synth_ckpt_device(seed, ck.data_ptr())
        engine.stream_finish_device(ck.data_ptr(), out.data_ptr())
        torch.cuda.synchronize()
    finally:
        engine.set_synth_kind(0)
    edges = np.array([k * 65536 + e for k in (1, 95, 190) for e in (-1, 0)])
    idx = np.unique(np.concatenate([[0, 1], np.random.default_rng(mode).integers(0, P, 300), edges, [P - 1]]))
    u = idx.astype(np.uint64)
    gen = O.synth_diff_fast if kind else O.synth_diff
    d = np.stack([gen(seed, k, u) for k in range(N)])
    want = coracle.fedavg(mode, d, O.synth_ckpt(seed, u))
    assert same(out.cpu().numpy()[idx], want)
    engine.set_layout([1])  # release the ring


def test_config5_shard_full_size_pinned_sampled(engine):
    """BASELINE config 5, one GPU's shard at full size: 125 M params x 64 clients, iterative plan,
    diffs DMA'd from page-locked host memory into an 8-slot ring, folded in pairs while the next
    copies run (`bench.py --workload c5-ingest`); bit-exact on sampled params."""
    import torch

    from pygrid_amd import PinnedBuffer

    P, N, R = 125_000_000, 64, 8
    rng = np.random.default_rng(5)
    bufs = [PinnedBuffer((P,)) for _ in range(4)]
    try:
        for b in bufs:
            b.array[:] = rng.standard_normal(P, dtype=np.float32) * np.float32(1e-2)
        engine.set_layout([P])
        engine.reserve(R)
        engine.stream_begin(1, 2)
        for k in range(N):
            engine.ingest(k, bufs[k % 4].array)
        c = rng.standard_normal(P, dtype=np.float32)
        ck = torch.from_numpy(c).cuda()
        out = torch.empty_like(ck)
        engine.stream_finish_device(ck.data_ptr(), out.data_ptr())
        torch.cuda.synchronize()
        idx = np.unique(np.concatenate([[0], rng.integers(0, P, 2000), [P - 1]]))
        d = np.stack([bufs[k % 4].array[idx] for k in range(N)])
        assert same(out.cpu().numpy()[idx], coracle.fedavg(1, d, c[idx]))
    finally:
        for b in bufs:
            b.free()
        engine.set_layout([1])


@pytest.mark.parametrize("lo", [0, 70_001])
def test_fast_generator_matches_oracle(engine, lo):
    """Generator kind 1 on a shard starting anywhere (lo % 4 != 0: per-param words), resident."""
    import torch

    P, N, seed = 300_007, 40, 9
    engine.set_layout([P])
    engine.set_shard(lo, P)
    pg = P - lo
    try:
        engine.reserve(N)
        engine.set_synth_kind(1)
        engine.synth_fill(seed, N)
        ck = torch.empty(pg, dtype=torch.float32, device="cuda")
        out = torch.empty_like(ck)
        engine.synth_ckpt_device(seed, ck.data_ptr())
        engine.fedavg_device(0, ck.data_ptr(), out.data_ptr())
        torch.cuda.synchronize()
    finally:
        engine.set_synth_kind(0)
        engine.set_layout([P])
    u = np.arange(lo, P, dtype=np.uint64)
    d = np.stack([O.synth_diff_fast(seed, k, u) for k in range(N)])
    want = coracle.fedavg(0, d, O.synth_ckpt(seed, u))
    assert same(out.cpu().numpy(), want)
