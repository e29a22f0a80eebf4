"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bar: bit-exact for everything (fp32 FedAvg included: the kernels fold clients in the
reference's order with separately rounded IEEE ops).  NaN positions must match; NaN payload
bits are not compared.
"""
import hashlib
import json

import numpy as np
import pytest

from oracle import coracle
from oracle import oracle as O
from oracle.gen_golden import MNIST_SHAPES, mnist_inputs

pytestmark = pytest.mark.gpu
F = np.float32
MODES = {"mean": 0, "iter": 1, "weighted": 2}


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a)
    return a.shape == b.shape and np.array_equal(nan, np.isnan(b)) and np.array_equal(bits(a)[~nan], bits(b)[~nan])


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run_f32(engine, diffs, ckpt, mode, weights=None, numel=None):
    d = np.asarray(diffs, F)
    engine.set_layout(numel or [d.shape[1]])
    engine.reserve(d.shape[0])
    for c in range(d.shape[0]):
        engine.ingest(c, d[c])
    if weights is not None:
        engine.set_weights(weights)
    return engine.fedavg(mode, np.asarray(ckpt, F))


def test_engine_reports_device(engine):
    from pygrid_amd import device_count

    assert device_count() >= 1


@pytest.mark.parametrize("variant", list(range(-1, 24)))
def test_edge_fixtures_all_modes(engine, gold, variant):
    z = np.load(gold / "edge_f32.npz")
    engine.set_variant(variant)
    try:
        for name in z["names"]:
            d, c, w = z[f"{name}_diffs"], z[f"{name}_ckpt"], z[f"{name}_w"]
            for key, mode in MODES.items():
                got = run_f32(engine, d, c, mode, w if mode == 2 else None)
                assert same(got, z[f"{name}_{key}"]), (name, key, variant)
    finally:
        engine.set_variant(-1)


@pytest.mark.parametrize("variant", list(range(-1, 24)))
def test_variants_mid_size(engine, variant):
    """Full tiles and a partial last tile for every variant (W = 2 tiles are 512 columns)."""
    rng = np.random.default_rng(variant + 1)
    P, N = 100_003, 19
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.5, 2.0, N).astype(F)
    engine.set_variant(variant)
    try:
        for mode in (0, 1, 2):
            got = run_f32(engine, d, c, mode, w if mode == 2 else None)
            assert same(got, coracle.fedavg(mode, d, c, w if mode == 2 else None)), (variant, mode)
    finally:
        engine.set_variant(-1)


def test_kat_avg_plan(engine, gold):
    kat = json.loads((gold / "kat_avg_plan.json").read_text())
    numel = [int(np.prod(s)) for s in kat["shapes"]]
    P = sum(numel)
    diffs = np.stack([np.full(P, k, F) for k in kat["coeffs"]])
    out = run_f32(engine, diffs, np.zeros(P, F), 1, numel=numel)
    assert np.all(-out == F(kat["expected_avg"]))


def test_mnist_golden_host_ingest(engine, gold):
    g = json.loads((gold / "mnist_synth.json").read_text())
    diffs, ckpt = mnist_inputs(g["seed"], g["n_clients"])
    numel = [int(np.prod(s)) for s in MNIST_SHAPES]
    assert sha(run_f32(engine, diffs, ckpt, 0, numel=numel)) == g["sha256_mean"]
    assert sha(run_f32(engine, diffs, ckpt, 1, numel=numel)) == g["sha256_iter"]
    assert sha(run_f32(engine, diffs, ckpt, 2, np.asarray(g["weights"], F), numel=numel)) == g["sha256_weighted"]


def test_mnist_golden_device_generator(engine, gold):
    """The on-device synthetic generator reproduces the restated one bit for bit."""
    import torch

    g = json.loads((gold / "mnist_synth.json").read_text())
    numel = [int(np.prod(s)) for s in MNIST_SHAPES]
    engine.set_layout(numel)
    engine.reserve(g["n_clients"])
    engine.synth_fill(g["seed"], g["n_clients"])
    ck = torch.empty(sum(numel), dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    engine.synth_ckpt_device(g["seed"], ck.data_ptr())
    engine.fedavg_device(0, ck.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    assert sha(ck.cpu().numpy()) == g["sha256_ckpt"]
    assert sha(out.cpu().numpy()) == g["sha256_mean"]


def _slab_host(engine, rows, dtype):
    """The whole slab copied to the host (hipMemcpy through the HIP runtime the library links)."""
    import ctypes

    ptr, ld, bp = engine.slab()
    nb = 1 if bp == 0 else -(-engine.stats()["p_shard"] // ld)
    n = (nb - 1) * bp + rows * ld if bp else rows * ld
    host = np.empty(n, dtype)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipDeviceSynchronize()
    rc = hip.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(host.nbytes), 2)
    assert rc == 0
    return host, ld, bp


@pytest.mark.parametrize("P,N,parties", [(200_003, 3, 1), (311_650, 2, 1), (100_003, 2, 2), (1_000, 4, 1)])
def test_slab_layout(engine, P, N, parties):
    """Element (row r, param i) sits at (i // ld) * block_pitch + r * ld + i % ld (pgh_api.h)."""
    i = np.arange(P)
    if parties == 1:
        engine.set_layout([P])
        engine.reserve(N)
        for c in range(N):
            engine.ingest(c, (c * 1_000_000 + i).astype(F))  # exact in fp32 (< 2^24)
        host, ld, bp = _slab_host(engine, N, np.float32)
    else:
        engine.set_layout([P])
        engine.reserve(N, 1, parties)
        for c in range(N):
            engine.ingest(c, np.stack([(c * parties + s) * 10**9 + i for s in range(parties)]).astype(np.int64))
        host, ld, bp = _slab_host(engine, N * parties, np.int64)
    assert ld % 64 == 0 and (bp == 0 or (ld & (ld - 1)) == 0)
    if P > 70_000:
        assert bp > 0, "shards wider than one 256 KiB block must be column-blocked"
    for r in range(N * parties):
        got = host[(i // ld) * bp + r * ld + i % ld]
        want = (r * 1_000_000 + i) if parties == 1 else (r * 10**9 + i)
        assert np.array_equal(got, np.asarray(want, got.dtype)), r


def test_blocked_equals_row_major(gold):
    """PGH_BLOCK_BYTES=0 (one block: plain row-major rows) and the blocked default agree bit for
    bit, for every mode and a range-split fold."""
    import os

    import torch

    from pygrid_amd import Engine

    rng = np.random.default_rng(5)
    P, N = 300_001, 7
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.5, 2.0, N).astype(F)
    outs = []
    for bb in ("0", None):
        if bb is None:
            os.environ.pop("PGH_BLOCK_BYTES", None)
        else:
            os.environ["PGH_BLOCK_BYTES"] = bb
        try:
            with Engine(0) as eng:
                res = [run_f32(eng, d, c, m, w if m == 2 else None) for m in (0, 1, 2)]
                ck = torch.from_numpy(c).cuda()
                out = torch.empty_like(ck)
                for off in range(0, P, 65_536 + 4):  # ranges straddling block edges
                    eng.fedavg_device_range(0, off, min(65_540, P - off), ck.data_ptr(), out.data_ptr())
                torch.cuda.synchronize()
                res.append(out.cpu().numpy())
                outs.append((res, eng.slab()[2]))
        finally:
            os.environ.pop("PGH_BLOCK_BYTES", None)
    (rm, bp0), (bl, bp1) = outs
    assert bp0 == 0 and bp1 > 0
    for a, b in zip(rm, bl):
        assert same(a, b)
    assert same(bl[0], coracle.fedavg(0, d, c)) and same(bl[3], bl[0])


def test_smpc_vectors(engine, gold):
    from pygrid_amd.cycle import CycleAggregator

    z = np.load(gold / "smpc_vectors.npz")
    agg = CycleAggregator(engine)
    s, _ = agg.secure_aggregate(z["share_shares"])
    assert np.array_equal(s, z["share_x"])
    for op in ("add", "sub"):
        for k in range(3):
            s, d = agg.secure_aggregate(z[f"{op}{k}_shares"])
            assert np.array_equal(s, z[f"{op}{k}_sum"])
            assert np.array_equal(bits(d), bits(z[f"{op}{k}_dec"]))
            assert np.allclose(d, z[f"{op}{k}_ref"], atol=1e-3)  # the reference's own bar


def test_secagg_wrap(engine, gold):
    from pygrid_amd.cycle import CycleAggregator

    z = np.load(gold / "secagg_wrap.npz")
    agg = CycleAggregator(engine)
    s, d = agg.secure_aggregate(z["shares"])
    assert np.array_equal(s, z["sum"]) and np.array_equal(bits(d), bits(z["dec"]))
    s2, d2 = agg.secure_aggregate(z["shares"], base=2, precision_fractional=16)
    assert np.array_equal(s2, z["sum"]) and np.array_equal(bits(d2), bits(z["dec_base2_prec16"]))


@pytest.mark.parametrize("variant", [-1, 0, 3, 6, 7, 12, 14, 15, 17, 18])
def test_secagg_synthetic_sampled(engine, variant):
    """250 clients x 2 parties x 1M params generated on the GPU; bit-exact on a sampled subset."""
    import torch

    P, N, S = 1_000_003, 250, 2
    engine.set_layout([P])
    engine.reserve(N, 1, S)
    engine.synth_fill(99, N)
    engine.set_variant(variant)
    try:
        s = torch.empty(P, dtype=torch.int64, device="cuda")
        d = torch.empty(P, dtype=torch.float32, device="cuda")
        engine.secagg_device(s.data_ptr(), d.data_ptr())
        torch.cuda.synchronize()
    finally:
        engine.set_variant(-1)
    idx = np.unique(np.concatenate([np.arange(0, 64), np.random.default_rng(1).integers(0, P, 2000), [P - 1]]))
    want = np.zeros(idx.size, np.uint64)
    with np.errstate(over="ignore"):
        for c in range(N):
            want += O.secagg_sum(O.synth_shares(99, c, S, idx.astype(np.uint64))[None]).view(np.uint64)
    want = want.view(np.int64)
    got_s = s.cpu().numpy()[idx]
    got_d = d.cpu().numpy()[idx]
    assert np.array_equal(got_s, want)
    assert np.array_equal(bits(got_d), bits(O.fix_prec_decode(want)))


def test_secagg_config3_full_size_sampled(engine):
    """BASELINE config 3: ResNet-18 (P = 11,689,512) x 1,000 clients x 2 parties int64 resident
    (187.7 GB, 357 column blocks); sums and decodes bit-exact on sampled params incl. block edges."""
    import torch

    P, N, S, seed = 11_689_512, 1000, 2, 77
    engine.set_layout([P])
    engine.reserve(N, 1, S)
    engine.synth_fill(seed, N)
    s = torch.empty(P, dtype=torch.int64, device="cuda")
    d = torch.empty(P, dtype=torch.float32, device="cuda")
    engine.secagg_device(s.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    _, ld, bp = engine.slab()
    assert ld == 32768 and bp == N * S * ld
    edges = np.array([k * ld + e for k in (1, 2, 178, 356) for e in (-2, -1, 0, 1)])
    idx = np.unique(np.concatenate([np.arange(4), np.random.default_rng(3).integers(0, P, 1500), edges, [P - 1]]))
    want = np.zeros(idx.size, np.uint64)
    with np.errstate(over="ignore"):
        for c in range(N):
            want += O.secagg_sum(O.synth_shares(seed, c, S, idx.astype(np.uint64))[None]).view(np.uint64)
    want = want.view(np.int64)
    assert np.array_equal(s.cpu().numpy()[idx], want)
    assert np.array_equal(bits(d.cpu().numpy()[idx]), bits(O.fix_prec_decode(want)))
    engine.set_layout([1])  # release the 187 GB slab for the next test


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_resnet18_scale_sampled(engine, mode):
    """BASELINE config 2 shape (P = 11,689,512, N = 1,000) fully resident; bit-exact against the
    oracle on 4,096 sampled params x all 1,000 clients (diffs regenerated on the CPU)."""
    import torch

    P, N, seed = 11_689_512, 1000, 4321
    engine.set_layout([P])
    engine.reserve(N)
    engine.synth_fill(seed, N)
    w = (np.arange(N) % 7 + 1).astype(F) * F(0.5)
    if mode == 2:
        engine.set_weights(w)
    ck = torch.empty(P, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    engine.synth_ckpt_device(seed, ck.data_ptr())
    engine.fedavg_device(mode, ck.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    rng = np.random.default_rng(mode)
    edges = np.array([k * 65536 + e for k in (1, 2, 89, 178) for e in (-4, -1, 0, 3)])  # 256 KiB blocks
    idx = np.unique(np.concatenate([np.arange(8), rng.integers(0, P, 4072), edges, [P - 1]])).astype(np.int64)
    d = np.stack([O.synth_diff(seed, c, idx.astype(np.uint64)) for c in range(N)])
    c = O.synth_ckpt(seed, idx.astype(np.uint64))
    want = coracle.fedavg(mode, d, c, w if mode == 2 else None)
    assert same(out.cpu().numpy()[idx], want)


def test_shards_concatenate_bit_identically(engine):
    """Param-axis shards (what each rank of a multi-GPU run computes) equal the unsharded run."""
    from pygrid_amd import Engine
    from pygrid_amd.sharding import all_shard_bounds

    rng = np.random.default_rng(5)
    P, N = 100_003, 37
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    full = run_f32(engine, d, c, 0)
    parts = []
    with Engine(engine.device) as e2:
        e2.set_layout([P])
        for lo, hi in all_shard_bounds(P, 3):
            e2.set_shard(lo, hi)
            e2.reserve(N)
            for k in range(N):
                e2.ingest(k, d[k])
            parts.append(e2.fedavg(0, c[lo:hi]))
    assert same(np.concatenate(parts), full)


def test_state_bytes_roundtrip(engine):
    """Bytes in, bytes out: State diffs -> engine -> patched checkpoint, parsed back with
    google.protobuf (independent of the C++ walker)."""
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state, parse_state

    rng = np.random.default_rng(8)
    shapes = [(392, 784), (392,), (10, 392), (10,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(3)]
    agg = CycleAggregator(engine)
    ck_pb = build_state(ckpt, as_param=True)
    d_pb = [build_state(d, as_param=(i == 1)) for i, d in enumerate(diffs)]
    want = O.fedavg_mean(ckpt, diffs)
    # default: a fresh State like serialize_model_params (model_manager.py:82-90)
    new_pb = agg.average_plan_diffs({}, ck_pb, d_pb)
    for got, w in zip(parse_state(new_pb), want):
        assert same(got, w)
    # the old checkpoint's framing kept byte for byte, payloads replaced
    tpl_pb = agg.average_plan_diffs({}, ck_pb, d_pb, framing="template")
    assert len(tpl_pb) == len(ck_pb)
    for got, w in zip(parse_state(tpl_pb), want):
        assert same(got, w)


def test_new_checkpoint_is_framed_like_serialize_model_params(engine):
    """model_manager.py:82-90: State(state_placeholders=[PlaceHolder().instantiate(p) ...]) of the
    plain tensors model_param - diff_param: fresh ids (not the template's, different every close),
    torch_tensor entries (no inherited torch_param), no tags -- parsed with google.protobuf."""
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state, classes

    rng = np.random.default_rng(9)
    shapes = [(33, 17), (17,), (4, 33), (4,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(2)]
    ck_pb = build_state(ckpt, as_param=True)  # the template: Parameters with tags
    agg = CycleAggregator(engine)
    outs = [agg.average_plan_diffs({}, ck_pb, [build_state(d) for d in diffs]) for _ in range(2)]
    old = classes()["State"]()
    old.ParseFromString(ck_pb)
    old_ids = {ph.id.id_int for ph in old.placeholders}
    want = O.fedavg_mean(ckpt, diffs)
    seen = set()
    for pb in outs:
        st = classes()["State"]()
        st.ParseFromString(pb)
        assert len(st.placeholders) == len(st.tensors) == len(shapes)
        for ph, t, shape, w in zip(st.placeholders, st.tensors, shapes, want):
            assert list(ph.tags) == [] and not ph.description
            assert t.HasField("torch_tensor") and not t.HasField("torch_param")
            tt = t.torch_tensor
            assert list(tt.tags) == [] and tt.contents_data.dtype == "float32"
            assert tuple(tt.contents_data.shape.dims) == shape
            got = np.asarray(tt.contents_data.contents_float32, F).reshape(shape)
            assert same(got, w)
            for i in (ph.id.id_int, tt.id.id_int):
                assert 0 <= i < 10e10 and i not in old_ids and i not in seen
                seen.add(i)


def test_average_params_api(engine):
    from pygrid_amd.cycle import CycleAggregator

    rng = np.random.default_rng(9)
    shapes = [(3, 5), (7,), (1,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[rng.standard_normal(s).astype(F) for s in shapes] for _ in range(4)]
    agg = CycleAggregator(engine)
    for got, want in zip(agg.average_params({}, ckpt, diffs), O.fedavg_mean(ckpt, diffs)):
        assert same(got, want)
    w = [1.0, 2.0, 3.0, 4.0]
    for got, want in zip(agg.average_params({}, ckpt, diffs, weights=w), O.fedavg_weighted(ckpt, diffs, w)):
        assert same(got, want)


def test_errors_are_loud(engine):
    from pygrid_amd import AggregationError

    engine.set_layout([10])
    engine.reserve(3)
    with pytest.raises(AggregationError):
        engine.fedavg(0, np.zeros(10, F))  # nothing ingested
    engine.ingest(0, np.ones(10, F))
    engine.ingest(2, np.ones(10, F))
    with pytest.raises(AggregationError, match="missing"):
        engine.fedavg(0, np.zeros(10, F))
    with pytest.raises(AggregationError):
        engine.ingest(1, np.ones(11, F))
    with pytest.raises(AggregationError):
        engine.fedavg(7, np.zeros(10, F))
    with pytest.raises(AggregationError):
        engine.fedavg(2, np.zeros(10, F))  # weighted without weights


def test_fedavg_device_range_pieces_equal_whole(engine):
    """Folding the shard in param ranges (the multi-GPU overlap path) equals one fold."""
    import torch

    from pygrid_amd.sharding import OverlappedGather

    rng = np.random.default_rng(12)
    P, N = 200_003, 9
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    whole = run_f32(engine, d, c, 1)
    ck = torch.from_numpy(c).cuda()
    og = OverlappedGather(P, 1, 0, chunks=5)
    lp = og.local.data_ptr()
    og.run(lambda off, n, st: engine.fedavg_device_range(1, off, n, ck.data_ptr(), lp, st))
    assert same(og.assemble().cpu().numpy(), whole)
    from pygrid_amd import AggregationError
    with pytest.raises(AggregationError):
        engine.fedavg_device_range(1, 2, 10, ck.data_ptr(), lp)  # misaligned range


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 63, 64, 65])
@pytest.mark.parametrize("N", [1, 2, 9, 17])
def test_tiny_shapes(engine, P, N):
    rng = np.random.default_rng(P * 100 + N)
    d = rng.standard_normal((N, P)).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.5, 2, N).astype(F)
    for mode in (0, 1, 2):
        assert same(run_f32(engine, d, c, mode, w if mode == 2 else None),
                    coracle.fedavg(mode, d, c, w if mode == 2 else None)), (P, N, mode)


def test_state_ingest_into_shards(engine):
    """State bytes ingested by param-shard contexts: each takes its slice of the payload spans."""
    from pygrid_amd import Engine
    from pygrid_amd.sharding import all_shard_bounds
    from pygrid_amd.state_schema import build_state_fast

    rng = np.random.default_rng(21)
    shapes = [(13, 7), (5,), (300,), (64, 3), (1,)]
    numel = [int(np.prod(s)) for s in shapes]
    P = sum(numel)
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(6)]
    flat = np.stack([np.concatenate([t.reshape(-1) for t in d]) for d in diffs])
    c = rng.standard_normal(P).astype(F)
    want = coracle.fedavg(0, flat, c)
    parts = []
    with Engine(engine.device) as e2:
        e2.set_layout(numel)
        for lo, hi in all_shard_bounds(P, 3, align=4):
            e2.set_shard(lo, hi)
            e2.reserve(len(diffs))
            for k, d in enumerate(diffs):
                e2.ingest_state(k, build_state_fast(d))
            parts.append(e2.fedavg(0, c[lo:hi]))
    assert same(np.concatenate(parts), want)


def test_ingest_shard_sized_buffer(engine):
    rng = np.random.default_rng(22)
    P, N = 1000, 4
    d = rng.standard_normal((N, P)).astype(F)
    c = rng.standard_normal(P).astype(F)
    engine.set_layout([P])
    engine.set_shard(200, 700)
    engine.reserve(N)
    for k in range(N):
        engine.ingest(k, d[k] if k % 2 else d[k, 200:700].copy())  # whole model or shard slice
    assert same(engine.fedavg(0, c[200:700]), coracle.fedavg(0, d, c)[200:700])


def test_resident_checkpoint_chains_cycles(engine):
    """Three cycles back to back through State bytes: the new checkpoint stays in HBM and feeds
    the next cycle (no re-upload when the caller hands the returned bytes back)."""
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(31)
    shapes = [(64, 33), (33,), (7, 64), (7,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    agg = CycleAggregator(engine)
    pb = build_state_fast(ckpt)
    want = ckpt
    for cyc in range(3):
        diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(4 + cyc)]
        pb = agg.average_plan_diffs({}, pb, [build_state_fast(d) for d in diffs])
        want = O.fedavg_mean(want, diffs)
        for got, w in zip(parse_state(pb), want):
            assert same(got, w), cyc
    assert same(engine.ckpt_download(), np.concatenate([w.reshape(-1) for w in want]))


def test_resident_api_flat(engine):
    rng = np.random.default_rng(32)
    P, N = 5003, 6
    d = rng.standard_normal((N, P)).astype(F)
    c = rng.standard_normal(P).astype(F)
    engine.set_layout([P])
    engine.reserve(N)
    engine.ckpt_upload(c)
    for k in range(N):
        engine.ingest(k, d[k])
    engine.fedavg_resident(0)
    assert same(engine.ckpt_download(), coracle.fedavg(0, d, c))


def test_reingest_waits_for_inflight_fold(engine):
    """RESIDENT: overwriting a slot right after an async fold on the caller's stream must not
    change what that fold reads."""
    import torch

    rng = np.random.default_rng(41)
    P, N = 4_000_000, 40
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    new0 = (rng.standard_normal(P) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    engine.set_layout([P])
    engine.reserve(N)
    for k in range(N):
        engine.ingest(k, d[k])
    ck = torch.from_numpy(c).cuda()
    out1 = torch.empty_like(ck)
    out2 = torch.empty_like(ck)
    sp = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    engine.fedavg_device(0, ck.data_ptr(), out1.data_ptr(), sp)
    engine.ingest(0, new0)
    engine.fedavg_device(0, ck.data_ptr(), out2.data_ptr(), sp)
    torch.cuda.synchronize()
    idx = np.random.default_rng(0).integers(0, P, 3000)
    assert same(out1.cpu().numpy()[idx], coracle.fedavg(0, d[:, idx], c[idx]))
    d2 = d[:, idx].copy()
    d2[0] = new0[idx]
    assert same(out2.cpu().numpy()[idx], coracle.fedavg(0, d2, c[idx]))


def test_secagg_device_range_pieces_equal_whole(engine):
    """Share sums + decodes of param ranges (the multi-GPU secagg overlap) equal one launch."""
    import torch

    from pygrid_amd.sharding import OverlappedGather

    P, N, S = 300_007, 40, 2
    engine.set_layout([P])
    engine.reserve(N, 1, S)
    engine.synth_fill(5, N)
    s_whole = torch.empty(P, dtype=torch.int64, device="cuda")
    d_whole = torch.empty(P, dtype=torch.float32, device="cuda")
    engine.secagg_device(s_whole.data_ptr(), d_whole.data_ptr())
    s_part = torch.full((P,), -1, dtype=torch.int64, device="cuda")
    og = OverlappedGather(P, 1, 0, chunks=7)
    lp = og.local.data_ptr()
    og.run(lambda off, n, st: engine.secagg_device_range(off, n, s_part.data_ptr(), lp, 10, 3, st))
    d_part = og.assemble()
    torch.cuda.synchronize()
    assert torch.equal(s_part, s_whole)
    assert torch.equal(d_part.view(torch.int32), d_whole.view(torch.int32))
    from pygrid_amd import AggregationError
    with pytest.raises(AggregationError):
        engine.secagg_device_range(6, 10, s_part.data_ptr(), lp)  # misaligned range


def test_rccl_overlapped_gather_world1(engine):
    """The RCCL ("nccl" backend) all-gather path of OverlappedGather, forced at world size 1:
    async all_gather_into_tensor per fold range on the torch stream, wait, assemble."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from pygrid_amd.sharding import OverlappedGather

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(51)
        P, N = 1_000_003, 7
        d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
        c = rng.standard_normal(P).astype(F)
        engine.set_layout([P])
        engine.reserve(N)
        for k in range(N):
            engine.ingest(k, d[k])
        ck = torch.from_numpy(c).cuda()
        og = OverlappedGather(P, 1, 0, chunks=8)
        og.run(lambda off, n, st: engine.fedavg_device_range(0, off, n, ck.data_ptr(), og.local.data_ptr(), st),
               force_collective=True)
        full = og.assemble()
        torch.cuda.synchronize()
        idx = rng.integers(0, P, 2000)
        assert same(full.cpu().numpy()[idx], coracle.fedavg(0, d[:, idx], c[idx]))
    finally:
        dist.destroy_process_group()


def test_rccl_client_sharded_secagg_world1(engine):
    """Client-sharded secure aggregation through the RCCL path, forced at world size 1: share sums
    of param ranges (no decode), int64 reduce_scatter_tensor, decode kernel on the reduced slice,
    all_gather_into_tensor -- bit-identical to pgh_secagg's fused sum + decode."""
    import os
    import socket

    import torch
    import torch.distributed as dist

    from pygrid_amd.sharding import OverlappedReduceScatter

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        P, N, S = 1_000_003, 5, 2
        rng = np.random.default_rng(52)
        sh = rng.integers(-2**63, 2**63 - 1, size=(N, S, P), dtype=np.int64, endpoint=True)
        engine.set_layout([P])
        engine.reserve(N, 1, S)
        for k in range(N):
            engine.ingest(k, sh[k])
        want_s, want_d = engine.secagg()
        og = OverlappedReduceScatter(P, 1, 0, chunks=8)
        og.run(lambda a, n, st: engine.secagg_device_range(a, n, og.sums.data_ptr(), 0, 10, 3, st),
               lambda t, d, st: engine.secagg_decode_device(t.data_ptr(), t.numel(), d.data_ptr(), 10, 3, st),
               force_collective=True)
        got = og.assemble()
        torch.cuda.synchronize()
        assert np.array_equal(og.total[:P].cpu().numpy(), want_s)
        assert np.array_equal(bits(got.cpu().numpy()), bits(want_d))
        idx = rng.integers(0, P, 500)
        _, od = coracle.secagg(sh[:, :, idx], idx.size)
        assert np.array_equal(bits(got.cpu().numpy()[idx]), bits(od))
    finally:
        dist.destroy_process_group()


def test_stats_busy_time_is_union_of_launches(engine):
    """pgh_stats' kernel_busy_ms_total: the sum of the durations for launches on one stream (no
    overlap), never more than that sum for ranges alternating over two streams."""
    import torch

    P, N = 4_000_000, 16
    engine.set_layout([P])
    engine.reserve(N)
    engine.synth_fill(9, N)
    ck = torch.zeros(P, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    engine.reset_stats()
    for _ in range(4):
        engine.fedavg_device(0, ck.data_ptr(), out.data_ptr())
    st = engine.stats()
    assert st["kernel_launches"] == 4
    assert st["kernel_busy_ms_total"] == pytest.approx(st["kernel_ms_total"], rel=1e-3)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    engine.reset_stats()
    n = P // 8
    for i in range(8):
        s = torch.cuda.current_stream() if i % 2 == 0 else side
        engine.fedavg_device_range(0, i * n, n, ck.data_ptr(), out.data_ptr(), s.cuda_stream)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    st = engine.stats()
    assert st["kernel_launches"] == 8
    assert 0 < st["kernel_busy_ms_total"] <= st["kernel_ms_total"] * (1 + 1e-6)


def test_secagg_decode_device_edges(engine):
    """The stand-alone decode kernel on int64 extremes and float32 rounding boundaries equals the
    oracle's float32(int64) / 1000 bit for bit (and base 2 / prec 0 divisors)."""
    import torch

    from pygrid_amd import AggregationError

    v = np.array([0, 1, -1, 2**63 - 1, -2**63, 2**24 + 1, -(2**24 + 1), 2**53 + 1, 123456789, -999, 1000,
                  16_777_217_000], np.int64)
    v = np.concatenate([v, np.random.default_rng(3).integers(-2**63, 2**63 - 1, 10_001, dtype=np.int64)])
    t = torch.from_numpy(v).cuda()
    d = torch.empty(v.size, dtype=torch.float32, device="cuda")
    for base, prec in ((10, 3), (2, 5), (10, 0)):
        engine.secagg_decode_device(t.data_ptr(), v.size, d.data_ptr(), base, prec)
        torch.cuda.synchronize()
        assert np.array_equal(bits(d.cpu().numpy()), bits(O.fix_prec_decode(v, base, prec))), (base, prec)
    engine.secagg_decode_device(0, 0, 0)  # empty is fine
    with pytest.raises(AggregationError):
        engine.secagg_decode_device(t.data_ptr(), 4, d.data_ptr(), 1, 3)  # bad base


@pytest.mark.parametrize("variant", [-1, 0, 6, 11, 12, 13, 14, 15, 17, 18])
def test_iterative_division_shortcut_edges(engine, variant):
    """The iterative fold's reciprocal-multiply division (div shortcut in pgh_kernels.hip) around
    its fallback threshold |t| ~ 2^-125 * (k + 1), subnormals, zeros of both signs, overflow to
    inf and NaN -- lanes that need the real division sharing row batches with lanes that do not."""
    rng = np.random.default_rng(variant + 50)
    N, P = 70, 4103
    d = np.empty((N, P), F)
    kinds = rng.integers(0, 7, P)
    for c in range(N):
        y = F(c + 1)
        thr = F(2.0 ** -125) * y
        col = np.where(kinds == 0, thr * F(rng.uniform(0.5, 2.0)),                   # around the threshold
              np.where(kinds == 1, F(1e-41) * F(rng.uniform(-3, 3)),                  # subnormal
              np.where(kinds == 2, F(rng.choice([0.0, -0.0])),                        # signed zeros
              np.where(kinds == 3, F(3e38) * F(rng.choice([-1, 1])),                  # overflow: acc * k -> inf
              np.where(kinds == 4, F(2.0 ** -120) * F(rng.uniform(-1, 1)),            # small normal
                       rng.standard_normal(P).astype(F))))))
        d[c] = col.astype(F)
    d[5, ::97] = np.nan
    c = rng.standard_normal(P).astype(F)
    engine.set_variant(variant)
    try:
        got = run_f32(engine, d, c, 1)
    finally:
        engine.set_variant(-1)
    assert same(got, coracle.fedavg(1, d, c))


def test_iterative_division_exact_subnormal_midpoints(engine):
    """Quotients that are exact ties between two f32 subnormals, where the reciprocal multiply
    alone rounds the wrong way (e.g. 147 * 2^-149 / 98 = 1.5 * 2^-149 -> 2^-148 by ties-to-even;
    t * RN(1/98) lands just below the tie): the kernel's fallback to the real division keeps them
    bit-exact.  Clients 0..96 send zeros so the plan's running average is 0 when client 97's
    diff T * 2^-149 arrives (k = 97, y = 98)."""
    P, N = 2048, 98
    T = 49 * (2 * np.arange(P, dtype=np.uint32) + 1)  # odd multiples of y / 2: exact midpoints
    d = np.zeros((N, P), F)
    d[97] = T.view(F)
    c = np.zeros(P, F)
    for variant in (-1, 0, 13, 14, 17, 18):
        engine.set_variant(variant)
        try:
            got = run_f32(engine, d, c, 1)
        finally:
            engine.set_variant(-1)
        assert same(got, coracle.fedavg(1, d, c)), variant


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("P", [30_001, 40_000, 65_000, 100_003, 150_001, 250_000, 359_999, 400_003])
def test_auto_variant_mid_sizes(engine, P, mode):
    """The auto choice changes at 200 K and 360 K params (iterative v14 / v13 / v0, mean v11 / v13
    / v11): each side of both edges bit-exact against the scalar C oracle."""
    rng = np.random.default_rng(P % 1000 + mode)
    N = 12
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.5, 2.0, N).astype(F) if mode == 2 else None
    engine.set_variant(-1)
    assert same(run_f32(engine, d, c, mode, w), coracle.fedavg(mode, d, c, w))


def test_non_iterative_mean_plan_is_accelerated(engine):
    """cycle_manager.py:270-271 with a hosted plan that is the plain mean: the engine runs it (MEAN)
    and the new checkpoint equals what the node computes with the plan itself -- bit for bit; a
    plan that sums in another order is declined (the node keeps running it)."""
    import torch as th
    from functools import reduce

    from pygrid_amd import PlanNotAcceleratedError
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast, parse_state

    def plan(diffs):
        return [th.div(reduce(th.add, list(col)), len(diffs)) for col in zip(*diffs)]

    rng = np.random.default_rng(12)
    shapes = [(64, 50), (50,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(9)]
    with pytest.raises(PlanNotAcceleratedError):  # the default: a user plan runs in the node
        CycleAggregator(engine).average_plan_diffs({}, build_state_fast(ckpt), [build_state_fast(d) for d in diffs],
                                                   avg_plan=plan)
    agg = CycleAggregator(engine, mean_plans="probe")  # the operator's opt-in
    new = agg.average_plan_diffs({"iterative_plan": False}, build_state_fast(ckpt),
                                 [build_state_fast(d) for d in diffs], avg_plan=plan)
    avg = plan([[th.from_numpy(t) for t in d] for d in diffs])  # the node's own :270-271 + :293-296
    for got, c, a in zip(parse_state(new), ckpt, avg):
        assert same(got, (th.from_numpy(c) - a).numpy())
    with pytest.raises(PlanNotAcceleratedError):
        agg.average_plan_diffs({}, build_state_fast(ckpt), [build_state_fast(d) for d in diffs],
                               avg_plan=lambda ds: [th.stack(list(col)).mean(0) for col in zip(*ds)])


def test_float64_diff_declines_and_leaves_the_aggregator_usable(engine):
    """A diff holding a float64 tensor (well-formed: the reference would average it with torch's
    type promotion) is declined mid-ingest (ModelNotAcceleratedError: the node runs its own code
    for the cycle); the same aggregator then closes a float32 cycle bit-exactly, its resident
    checkpoint untouched by the declined one."""
    from pygrid_amd import ModelNotAcceleratedError
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast, classes, parse_state

    rng = np.random.default_rng(13)
    shapes = [(300, 7), (7,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for _ in range(4)]
    st = classes()["State"]()
    st.ParseFromString(build_state_fast(diffs[2]))
    td = st.tensors[1].torch_tensor.contents_data
    vals = list(td.contents_float32)
    td.ClearField("contents_float32")
    td.dtype = "float64"
    td.contents_float64.extend(vals)
    bad = st.SerializeToString()
    agg = CycleAggregator(engine)
    ck_pb = build_state_fast(ckpt)
    first = agg.average_plan_diffs({}, ck_pb, [build_state_fast(d) for d in diffs])  # resident now
    with pytest.raises(ModelNotAcceleratedError):
        agg.average_plan_diffs({}, first, [build_state_fast(diffs[0]), build_state_fast(diffs[1]), bad])
    new = agg.average_plan_diffs({}, first, [build_state_fast(d) for d in diffs])
    want = O.fedavg_mean(O.fedavg_mean(ckpt, diffs), diffs)
    for got, w in zip(parse_state(new), want):
        assert same(got, w)
