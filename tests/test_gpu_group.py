"""GPU: the multi-GPU group context (pgh_create_group) against the oracle and against one GPU.

On the one-GPU box a group's children share device 0 ("devices=[0, 0]"): every shard, fan-out
and peer-copy path of the group runs for real, and the RCCL path runs over a one-GPU group
(ncclCommInitAll over [0]; a communicator cannot hold one device twice).  The 8-GPU node is the
driver's.  Bar: bit-exact (fp32 folds included: every GPU folds every client of its shard in the
reference's order).
"""
import ctypes as C
import hashlib
import json
import subprocess

import numpy as np
import pytest

from conftest import GOLD, ROOT
from oracle import coracle
from oracle import oracle as O
from oracle.gen_golden import MNIST_SHAPES, mnist_inputs

pytestmark = pytest.mark.gpu
F = np.float32


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def group2():
    from pygrid_amd import Engine

    eng = Engine(devices=[0, 0])
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def group3():
    from pygrid_amd import Engine

    eng = Engine(devices=[0, 0, 0])
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def group8():
    """The driver's 8-GPU node layout (eight param shards, eight children), here all on GPU 0."""
    from pygrid_amd import Engine

    eng = Engine(devices=[0] * 8)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def group1():
    from pygrid_amd import Engine

    eng = Engine(devices=[0])
    yield eng
    eng.close()


def d2h(ptr: int, n: int, dtype=np.float32) -> np.ndarray:
    """Read n values from device memory (torch already loaded the HIP runtime)."""
    hip = C.CDLL("libamdhip64.so.7")
    out = np.empty(n, dtype=dtype)
    assert hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr), C.c_size_t(out.nbytes), 2) == 0
    return out


# ---- the plain-C binding, on the GPU --------------------------------------------------------------

@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_plain_c_consumer_closes_mnist_on_the_gpu(tmp_path, devices):
    """tests/c_abi_gpu_close.c: MNIST N=3 mean + iterative through the C ABI alone (single context
    and groups), against the golden SHA-256 (oracle/gen_golden.py)."""
    g = json.loads((GOLD / "mnist_synth.json").read_text())
    diffs, ckpt = mnist_inputs(g["seed"], g["n_clients"])
    numel = [int(np.prod(s)) for s in MNIST_SHAPES]
    inp, outp, exe = tmp_path / "in.bin", tmp_path / "out.bin", tmp_path / "close"
    with open(inp, "wb") as f:
        f.write(np.array([len(numel), diffs.shape[0]], np.int32).tobytes())
        f.write(np.array(numel, np.int64).tobytes())
        f.write(np.ascontiguousarray(diffs, F).tobytes())
        f.write(np.ascontiguousarray(ckpt, F).tobytes())
    lib_dir = ROOT / "pygrid_amd"
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "c_abi_gpu_close.c"), "-L", str(lib_dir), "-lpygrid_hip",
                    f"-Wl,-rpath,{lib_dir}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), str(inp), str(outp), str(len(devices)), *map(str, devices)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith(f"ok gpus={len(devices)}")
    out = np.fromfile(outp, dtype=F).reshape(2, -1)
    assert sha(out[0]) == g["sha256_mean"]
    assert sha(out[1]) == g["sha256_iter"]


# ---- param shards: bit-identical to one GPU ----------------------------------------------------------

def test_group_shape(group2, group3):
    assert group2.n_gpus == 2 and group3.n_gpus == 3
    with pytest.raises(Exception):
        group2.child(2)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("P", [1000, 4_000_003, 64 * 3 + 5])
def test_group_fedavg_matches_oracle(group3, mode, P):
    rng = np.random.default_rng(300 + mode)
    N = 7
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    w = rng.uniform(0.5, 2.0, N).astype(F)
    group3.set_layout([P])
    group3.reserve(N)
    for k in range(N):
        group3.ingest(k, d[k])
    if mode == 2:
        group3.set_weights(w)
    got = group3.fedavg(mode, c)
    assert np.array_equal(bits(got), bits(coracle.fedavg(mode, d, c, w if mode == 2 else None)))


def test_group_state_bytes_cycles_match_single_gpu(group2, engine):
    """CycleAggregator over a group: State bytes in, new checkpoint bytes out, three cycles chained
    through the resident checkpoint -- byte-identical to the single-GPU engine."""
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(311)
    shapes = [(96, 130), (130,), (7, 96), (7,)]
    ck = build_state_fast([rng.standard_normal(s).astype(F) for s in shapes])
    a1, a2 = CycleAggregator(engine), CycleAggregator(group2)
    p1 = p2 = ck
    for cyc in range(3):
        diffs = [build_state_fast([(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes]) for _ in range(5)]
        framing = "template" if cyc < 2 else "fresh"  # fresh ids differ per close: compare payloads
        p1 = a1.average_plan_diffs({}, p1, diffs, framing=framing)
        p2 = a2.average_plan_diffs({}, p2, diffs, framing=framing)
        if framing == "template":
            assert p1 == p2, cyc
        for x, y in zip(parse_state(p1), parse_state(p2)):
            assert np.array_equal(bits(x), bits(y)), cyc


def test_group_subrange_and_stream(group2):
    """set_shard on a group re-partitions the sub-range; STREAM folds through the ring per GPU."""
    rng = np.random.default_rng(312)
    P, N = 50_000, 9
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    group2.set_layout([P])
    group2.set_shard(1000, 40_000)
    group2.reserve(4)
    group2.stream_begin(0, 2)
    for k in range(N):
        group2.ingest(k, d[k])
    got = group2.stream_finish(c[1000:40_000])
    want = coracle.fedavg(0, d, c)[1000:40_000]
    assert np.array_equal(bits(got), bits(want))


def test_group_report_time_cycle(group2):
    """IncrementalCycle over a group: shuffled reports with dropouts, folded through the row table
    on every GPU."""
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(313)
    shapes = [(200, 41), (41,)]
    n = 40
    reporters = [w for w in range(n) if w != 0 and rng.random() >= 0.2]
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in reporters}
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck_pb = build_state_fast(ckpt)
    inc = IncrementalCycle(group2, [int(np.prod(s)) for s in shapes], slots=16, fold_batch=3, checkpoint=ck_pb)
    for w in range(n):
        inc.assigned(w)
    for w in rng.permutation(reporters):
        inc.reported(int(w), build_state_fast(diffs[int(w)]))
    new = inc.close(ck_pb)
    want = O.fedavg_mean(ckpt, [diffs[w] for w in sorted(reporters)])
    for got, w in zip(parse_state(new), want):
        assert np.array_equal(bits(got), bits(w))


def test_group_allgather_resident_peer_copies(group2):
    rng = np.random.default_rng(314)
    P, N = 10_007, 3
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    group2.set_layout([P])
    group2.reserve(N)
    group2.ckpt_upload(c)
    for k in range(N):
        group2.ingest(k, d[k])
    group2.fedavg_resident(0)
    ptrs = group2.allgather_resident()
    assert group2.group_backend() == 0  # two children on one device: peer copies
    want = coracle.fedavg(0, d, c)
    S = -(-(-(-P // 2)) // 64) * 64
    for p in ptrs:
        full = d2h(p, 2 * S)
        got = np.concatenate([full[:S], full[S:S + P - S]])
        assert np.array_equal(bits(got), bits(want))


def test_group1_allgather_over_rccl(group1):
    rng = np.random.default_rng(315)
    P, N = 4_099, 4
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    group1.set_layout([P])
    group1.reserve(N)
    group1.ckpt_upload(c)
    for k in range(N):
        group1.ingest(k, d[k])
    group1.fedavg_resident(1)
    (p,) = group1.allgather_resident()
    assert group1.group_backend() == 1  # ncclCommInitAll over [0]
    assert np.array_equal(bits(d2h(p, P)), bits(coracle.fedavg(1, d, c)))


# ---- secure aggregation: param shards and client shards ----------------------------------------------

def _shares(seed, N, S, P):
    idx = np.arange(P, dtype=np.uint64)
    return np.stack([O.synth_shares(seed, k, S, idx) for k in range(N)])


@pytest.mark.parametrize("client_shard", [False, True])
@pytest.mark.parametrize("N", [1, 2, 7])
def test_group_secagg(group3, client_shard, N):
    P, S = 3_001, 2
    sh = _shares(320 + N, N, S, P)
    sh[0, 0, :5] = [2**63 - 1, -2**63, -1, 1, 0]  # wrap-heavy
    group3.set_layout([P])
    group3.set_client_sharding(client_shard)
    group3.reserve(N, 1, S)
    for k in range(N):
        group3.ingest(k, sh[k])
    s, dec = group3.secagg(10, 3)
    ws = O.secagg_sum(sh)
    assert np.array_equal(s, ws)
    assert np.array_equal(bits(dec), bits(O.fix_prec_decode(ws)))
    group3.set_client_sharding(False)


def test_group_secagg_client_shard_from_share_state_bytes(group2):
    """Each client's share messages go only to the GPU that owns the client (its own PCIe link),
    decoded there; the reduce-scatter over peer copies makes the sums whole -- bit-exact."""
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.state_schema import build_state_i64_fast

    N, S = 5, 2
    numel = [700, 301]
    P = sum(numel)
    sh = _shares(330, N, S, P)
    msgs = [[build_state_i64_fast(np.split(sh[k, p], [numel[0]])) for p in range(S)] for k in range(N)]
    group2.set_client_sharding(True)
    try:
        s, dec = CycleAggregator(group2).secure_aggregate_states(numel, msgs)
    finally:
        group2.set_client_sharding(False)
    ws = O.secagg_sum(sh)
    assert np.array_equal(s, ws) and np.array_equal(bits(dec), bits(O.fix_prec_decode(ws)))


def test_group1_client_sharded_secagg_over_rccl(group1):
    N, S, P = 3, 2, 2_049
    sh = _shares(340, N, S, P)
    group1.set_layout([P])
    group1.set_client_sharding(True)
    try:
        group1.reserve(N, 1, S)
        group1.synth_fill(77, N)
        s, dec = group1.secagg(10, 3)
    finally:
        group1.set_client_sharding(False)
    idx = np.arange(P, dtype=np.uint64)
    ws = O.secagg_sum(np.stack([O.synth_shares(77, k, S, idx) for k in range(N)]))
    assert group1.group_backend() == 1
    assert np.array_equal(s, ws) and np.array_equal(bits(dec), bits(O.fix_prec_decode(ws)))


def test_group_client_sharded_synth_matches_oracle(group3):
    """Synthetic clients of a client-sharded group are generated under their GLOBAL index."""
    N, S, P = 8, 2, 1_500
    group3.set_layout([P])
    group3.set_client_sharding(True)
    try:
        group3.reserve(N, 1, S)
        group3.synth_fill(91, N)
        s, _ = group3.secagg(10, 3)
    finally:
        group3.set_client_sharding(False)
    idx = np.arange(P, dtype=np.uint64)
    assert np.array_equal(s, O.secagg_sum(np.stack([O.synth_shares(91, k, S, idx) for k in range(N)])))


def test_device_pointer_calls_refused_on_a_group(group2):
    from pygrid_amd.exceptions import AggregationError

    group2.set_layout([1000])
    group2.reserve(2)
    with pytest.raises(AggregationError, match="UNSUPPORTED"):
        group2.fedavg_device(0, 16, 16)
    with pytest.raises(AggregationError, match="UNSUPPORTED"):
        group2.slab()
    kid = group2.child(1)
    assert kid.slab()[0] != 0  # the child context owns a real slab


@pytest.mark.parametrize("seed", range(16))
def test_group_random_cycles(group2, group3, seed):
    """Randomized chained cycles on 2- and 3-child groups: model sizes from 1 param (one active
    child) to off-grid shards, close-time State closes and report-time cycles alternating, every
    mode, each cycle's output feeding the next -- bit-exact against the oracle."""
    _random_cycles(group2 if seed % 2 else group3, 7000 + seed)


@pytest.mark.parametrize("seed", range(6))
def test_group8_random_cycles(group8, seed):
    """The same randomized chained cycles on an eight-child group (the 8-GPU node's shard count):
    models smaller than eight params leave children without a shard."""
    _random_cycles(group8, 7100 + seed)


def _random_cycles(eng, seed):
    from pygrid_amd.cycle import CycleAggregator
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(seed)
    P = int(rng.choice([1, 5, 64, 65, 129, 191, 4_099, 70_001, 262_147]))
    cut = sorted(int(x) for x in rng.choice(np.arange(1, P), size=min(2, P - 1), replace=False)) if P > 2 else []
    numel = [b - a for a, b in zip([0] + cut, cut + [P])]
    ckpt = [(rng.standard_normal(k) * 0.05).astype(F) for k in numel]
    agg = CycleAggregator(eng)
    for step in range(3):
        n = int(rng.integers(1, 13))
        mode = int(rng.integers(0, 3))
        reporters = sorted(int(w) for w in rng.choice(n, size=int(rng.integers(1, n + 1)), replace=False))
        diffs = {w: [(rng.standard_normal(k) * 1e-2).astype(F) for k in numel] for w in reporters}
        weights = {w: float(rng.uniform(0.5, 3.0)) for w in range(n)}
        ref = [diffs[w] for w in reporters]
        wv = np.array([weights[w] for w in reporters], F)
        ck_pb = build_state_fast(ckpt)
        if step % 2 == 0:
            plan = None
            if mode == 1:
                def plan(avg, item, num):  # 01-Create-plan.ipynb:450-454
                    return [(a * num + i) / (num + 1) for a, i in zip(avg, item)]
            new = agg.average_plan_diffs({"iterative_plan": mode == 1}, ck_pb, [build_state_fast(diffs[w]) for w in reporters],
                                         plan, weights=wv if mode == 2 else None)
        else:
            inc = IncrementalCycle(eng, numel, mode=mode, slots=int(rng.integers(2, n + 2)),
                                   fold_batch=int(rng.integers(1, 5)), weights_by_worker=weights if mode == 2 else None,
                                   checkpoint=ck_pb)
            for w in range(n):
                inc.assigned(w)
            for w in rng.permutation(reporters):
                inc.reported(int(w), build_state_fast(diffs[int(w)]))
            new = inc.close(ck_pb)
        want = (O.fedavg_mean(ckpt, ref) if mode == 0 else O.fedavg_iterative(ckpt, ref) if mode == 1 else
                O.fedavg_weighted(ckpt, ref, wv))
        got = parse_state(new)
        for g, w in zip(got, want):
            assert np.array_equal(bits(g), bits(w))
        ckpt = [np.asarray(g, F).reshape(-1) for g in got]


# ---- eight children: the 8-GPU node's layout on one device -------------------------------------------

def test_group8_shape_and_peer_allgather(group8):
    assert group8.n_gpus == 8
    rng = np.random.default_rng(350)
    P, N = 100_003, 5
    d = (rng.standard_normal((N, P)) * 1e-2).astype(F)
    c = rng.standard_normal(P).astype(F)
    group8.set_layout([P])
    group8.reserve(N)
    group8.ckpt_upload(c)
    for k in range(N):
        group8.ingest(k, d[k])
    group8.fedavg_resident(0)
    ptrs = group8.allgather_resident()
    assert group8.group_backend() == 0 and len(ptrs) == 8
    want = coracle.fedavg(0, d, c)
    S = -(-(-(-P // 8)) // 64) * 64  # every shard padded to the same multiple of 64
    for p in ptrs:
        full = d2h(p, 8 * S)
        got = np.concatenate([full[k * S:k * S + min(S, P - k * S)] for k in range(8) if k * S < P])
        assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("client_shard", [False, True])
@pytest.mark.parametrize("N", [1, 7, 9])
def test_group8_secagg(group8, client_shard, N):
    """Param shards and client shards over eight children (fewer clients than children included)."""
    P, S = 5_003, 2
    sh = _shares(360 + N, N, S, P)
    sh[0, 0, :5] = [2**63 - 1, -2**63, -1, 1, 0]
    group8.set_layout([P])
    group8.set_client_sharding(client_shard)
    try:
        group8.reserve(N, 1, S)
        for k in range(N):
            group8.ingest(k, sh[k])
        s, dec = group8.secagg(10, 3)
    finally:
        group8.set_client_sharding(False)
    ws = O.secagg_sum(sh)
    assert np.array_equal(s, ws)
    assert np.array_equal(bits(dec), bits(O.fix_prec_decode(ws)))


def test_group8_report_time_cycle(group8):
    """Report-time folds fanned out to eight children: shuffled reports, dropouts, a re-report."""
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.state_schema import build_state_fast, parse_state

    rng = np.random.default_rng(370)
    shapes = [(300, 77), (77,), (5,)]
    n = 30
    reporters = [w for w in range(n) if w != 0 and rng.random() >= 0.2]
    diffs = {w: [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes] for w in reporters}
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    ck_pb = build_state_fast(ckpt)
    inc = IncrementalCycle(group8, [int(np.prod(s)) for s in shapes], slots=12, fold_batch=3, checkpoint=ck_pb)
    for w in range(n):
        inc.assigned(w)
    order = [int(w) for w in rng.permutation(reporters)]
    again = order[len(order) // 2]
    for w in order:
        inc.reported(w, build_state_fast(diffs[w]))
        if w == order[-3]:  # a re-report with a new diff, late in the cycle
            diffs[again] = [(rng.standard_normal(s) * 1e-2).astype(F) for s in shapes]
            inc.reported(again, build_state_fast(diffs[again]))
    new = inc.close(ck_pb)
    want = O.fedavg_mean(ckpt, [diffs[w] for w in sorted(reporters)])
    for got, w in zip(parse_state(new), want):
        assert np.array_equal(bits(got), bits(w))
