"""GPU soak: random sequences of engine calls (layouts on and off the 256 KiB block grid, shards,
resident / range / stream / secagg folds, folds on two caller streams, overwrites right after
asynchronous folds) checked against the oracle after every fold.  Model-based: the test keeps
its own copy of what each slot should hold."""
import numpy as np
import pytest

from oracle import coracle
from oracle import oracle as O

pytestmark = pytest.mark.gpu
F = np.float32
SIZES = [1, 3, 64, 4_099, 65_537, 70_001, 131_077, 300_007]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a)
    return a.shape == b.shape and np.array_equal(nan, np.isnan(b)) and np.array_equal(bits(a)[~nan], bits(b)[~nan])


def _ranges(p, k):
    c = -(-p // k)
    c = -(-c // 4) * 4
    return [(o, min(c, p - o)) for o in range(0, p, c)]


@pytest.mark.parametrize("seed", range(24))
def test_random_resident_sequences(engine, seed):
    import torch

    rng = np.random.default_rng(1000 + seed)
    P = int(rng.choice(SIZES))
    N = int(rng.integers(1, 12))
    engine.set_layout([P])
    lo, hi = 0, P
    if P >= 256 and rng.random() < 0.5:  # a shard of a larger model, 64-aligned start
        lo = int(rng.integers(0, P // 64)) * 64
        hi = int(rng.integers(lo + 1, P + 1))
        engine.set_shard(lo, hi)
    pg = hi - lo
    engine.reserve(N)
    d = (rng.standard_normal((N, P)) * F(10.0 ** rng.uniform(-4, 1))).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.1, 3.0, N).astype(F)
    for k in rng.permutation(N):
        engine.ingest(int(k), d[k] if rng.random() < 0.5 else d[k, lo:hi])  # whole model or shard slice
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ck = torch.from_numpy(c[lo:hi].copy()).cuda()
    for step in range(3):
        mode = int(rng.integers(0, 3))
        engine.set_weights(w)
        want = coracle.fedavg(mode, np.ascontiguousarray(d[:, lo:hi]), c[lo:hi], w if mode == 2 else None)
        how = int(rng.integers(0, 3))
        if how == 0:
            got = engine.fedavg(mode, c[lo:hi])
        else:
            out = torch.full((pg,), float("nan"), device="cuda")
            torch.cuda.synchronize()
            if how == 1:
                engine.fedavg_device(mode, ck.data_ptr(), out.data_ptr(), s1.cuda_stream)
            else:  # param ranges alternating over two streams (the multi-GPU overlap)
                for i, (o, n) in enumerate(_ranges(pg, int(rng.integers(2, 9)))):
                    engine.fedavg_device_range(mode, o, n, ck.data_ptr(), out.data_ptr(),
                                               (s1 if i % 2 == 0 else s2).cuda_stream)
            # overwrite a client right away: the engine must order it after the folds in flight
            k = int(rng.integers(0, N))
            d[k] = (rng.standard_normal(P) * 1e-2).astype(F)
            engine.ingest(k, d[k])
            torch.cuda.synchronize()
            got = out.cpu().numpy()
        assert same(got, want), (seed, step, mode, how, P, N, lo, hi)


@pytest.mark.parametrize("seed", range(12))
def test_random_stream_sequences(engine, seed):
    rng = np.random.default_rng(2000 + seed)
    P = int(rng.choice(SIZES))
    N = int(rng.integers(1, 30))
    R = int(rng.integers(1, 9))
    batch = int(rng.integers(0, R + 1))
    mode = int(rng.integers(0, 3))
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.1, 3.0, N).astype(F)
    engine.set_layout([P])
    engine.reserve(R)
    engine.stream_begin(mode, batch)
    if mode == 2:
        engine.set_weights(w)
    b_eff = max(1, R // 2) if batch <= 0 else min(batch, R)
    window = R - b_eff + 1
    order, pending, nxt = [], [], 0  # an arrival order the ring admits
    while len(order) < N:
        while nxt < N and len(pending) < window and (not pending or nxt - min(pending) < window):
            pending.append(nxt)
            nxt += 1
        order.append(pending.pop(int(rng.integers(len(pending)))))
    for k in order:
        engine.ingest(k, d[k])
    got = engine.stream_finish(c)
    assert same(got, coracle.fedavg(mode, d, c, w if mode == 2 else None)), (seed, P, N, R, batch, mode)


@pytest.mark.parametrize("seed", range(8))
def test_random_secagg_sequences(engine, seed):
    import torch

    rng = np.random.default_rng(3000 + seed)
    P = int(rng.choice(SIZES))
    N, S = int(rng.integers(1, 9)), int(rng.integers(1, 4))
    sh = rng.integers(-2**63, 2**63 - 1, size=(N, S, P), dtype=np.int64, endpoint=True)
    engine.set_layout([P])
    engine.reserve(N, 1, S)
    for k in rng.permutation(N):
        engine.ingest(int(k), sh[k])
    want = O.secagg_sum(sh)
    if rng.random() < 0.5:
        s, dec = engine.secagg(10, 3)
    else:
        s_t = torch.empty(P, dtype=torch.int64, device="cuda")
        d_t = torch.empty(P, dtype=torch.float32, device="cuda")
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        torch.cuda.synchronize()
        for i, (o, n) in enumerate(_ranges(P, int(rng.integers(1, 6)))):
            engine.secagg_device_range(o, n, s_t.data_ptr(), d_t.data_ptr(), 10, 3, streams[i % 2].cuda_stream)
        torch.cuda.synchronize()
        s, dec = s_t.cpu().numpy(), d_t.cpu().numpy()
    assert np.array_equal(s, want), (seed, P, N, S)
    assert np.array_equal(bits(dec), bits(O.fix_prec_decode(want)))


def test_overwrite_waits_for_folds_on_both_streams(engine):
    """Range folds on two streams, then every slot overwritten from page-locked memory (DMA'd at
    once, no host staging): the copies must wait for the folds on BOTH streams."""
    import torch

    from pygrid_amd import PinnedBuffer

    rng = np.random.default_rng(77)
    P, N = 4_000_003, 1000  # 16 GB: the long fold runs ~2.4 ms; workgroups of its second wave read row 0
                            # ~1 ms in, long after the overwrite of slot 0 could have landed
    engine.set_layout([P])
    engine.reserve(N)
    engine.synth_fill(77, N)
    c = rng.standard_normal(P).astype(F)
    ck = torch.from_numpy(c).cuda()
    out = torch.empty_like(ck)
    zeros = PinnedBuffer((P,))
    zeros.array[:] = 0
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    try:
        cut = (P - 4096) // 4 * 4  # a long fold on s1, then a short one on s2: the LAST fold is the short one
        engine.fedavg_device_range(0, 0, cut, ck.data_ptr(), out.data_ptr(), s1.cuda_stream)
        engine.fedavg_device_range(0, cut, P - cut, ck.data_ptr(), out.data_ptr(), s2.cuda_stream)
        engine.ingest(0, zeros.array)  # overwrite slot 0 while the long fold still reads it
        torch.cuda.synchronize()
    finally:
        zeros.free()
    idx = np.unique(np.concatenate([rng.integers(0, P, 1000), [0, P - 1]])).astype(np.int64)
    d = np.stack([O.synth_diff(77, k, idx.astype(np.uint64)) for k in range(N)])
    assert same(out.cpu().numpy()[idx], coracle.fedavg(0, d, c[idx]))


@pytest.mark.parametrize("seed", range(40))
def test_random_report_cycles(engine, seed):
    """Report-time aggregation under random pressure: model sizes on and off the block grid, 1-40
    assigned workers with random non-reporters, random slot budgets (down to 2) and fold batches,
    shuffled arrival, three chained cycles on one engine (each cycle's output is the next one's
    checkpoint) -- every close bit-exact against the oracle's fold in WorkerCycle-id order."""
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(5000 + seed)
    P = int(rng.choice(SIZES))
    cut = sorted(int(x) for x in rng.choice(np.arange(1, P), size=min(2, P - 1), replace=False)) if P > 2 else []
    numel = [b - a for a, b in zip([0] + cut, cut + [P])]
    mode = int(rng.integers(0, 3))
    ckpt = [(rng.standard_normal(n) * 0.05).astype(F) for n in numel]
    for _ in range(3):
        n = int(rng.integers(1, 41))
        reporters = sorted(int(w) for w in rng.choice(n, size=int(rng.integers(1, n + 1)), replace=False))
        diffs = {w: [(rng.standard_normal(k) * 1e-2).astype(F) for k in numel] for w in reporters}
        weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n)}
        ck_pb = build_state_fast(ckpt)
        inc = IncrementalCycle(engine, numel, mode=mode, slots=int(rng.integers(2, n + 2)),
                               fold_batch=int(rng.integers(1, 9)), weights_by_worker=weights if mode == 2 else None,
                               checkpoint=ck_pb if rng.random() < 0.5 else None)
        for w in range(n):
            inc.assigned(w)
        for w in rng.permutation(reporters):
            inc.reported(int(w), build_state_fast(diffs[int(w)]))
        got = parse_state(inc.close(ck_pb))
        ref = [diffs[w] for w in reporters]
        want = (O.fedavg_mean(ckpt, ref) if mode == 0 else O.fedavg_iterative(ckpt, ref) if mode == 1 else
                O.fedavg_weighted(ckpt, ref, np.array([weights[w] for w in reporters], F)))
        for g, w in zip(got, want):
            assert same(g, w)
        ckpt = [np.asarray(g, F).reshape(-1) for g in got]


def test_many_closes_hold_device_and_host_memory_steady():
    """A node closes cycles for as long as it runs: 300 MNIST closes (bytes path) and 100
    report-time cycles on one engine must not grow device or host memory (no per-close leak of
    slabs, events, pinned pieces or fresh outputs)."""
    import ctypes as C
    import resource

    import torch

    from pygrid_amd import Engine
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast

    hip = C.CDLL("libamdhip64.so.7")

    def dev_free():
        free, total = C.c_size_t(0), C.c_size_t(0)
        assert hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
        return free.value

    torch.cuda.synchronize()
    rng = np.random.default_rng(77)
    shapes = [(392, 784), (392,), (10, 392), (10,)]
    numel = [int(np.prod(s)) for s in shapes]
    ck = build_state_fast([(rng.standard_normal(s) * 0.05).astype(F) for s in shapes])
    ds = [build_state_fast([(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes]) for _ in range(3)]
    with Engine(0) as eng:
        agg = CycleAggregator(eng)

        def round_of_closes(k):
            new = ck
            for _ in range(k):
                new = agg.average_plan_diffs({}, new, ds)
            for _ in range(k // 3):
                inc = IncrementalCycle(eng, numel, slots=3, fold_batch=1, checkpoint=new)
                for w in range(4):
                    inc.assigned(w)
                for w in (2, 1, 3):
                    inc.reported(w, ds[w - 1])
                new = inc.close(new)
            eng.sync()

        round_of_closes(30)  # warm: allocations that persist across cycles happen here
        free0, rss0 = dev_free(), resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
        round_of_closes(300)
        free1, rss1 = dev_free(), resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    assert free0 - free1 < (8 << 20), f"device memory fell by {(free0 - free1) >> 20} MiB over 400 closes"
    assert rss1 - rss0 < 64 * 1024, f"peak host RSS grew by {(rss1 - rss0) // 1024} MiB over 400 closes"
