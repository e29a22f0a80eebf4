"""GPU: secure-aggregation shares ingested as State bytes (packed-varint contents_int64, decoded
on the GPU by k_varint_decode) -- bit-exact against google.protobuf's parse of the same bytes
and against the numpy oracle's Z_2^64 sum / fixed-point decode (PySyft 0.2.9 semantics,
test_basic_syft_operations.py:388-454; wire schema restated, parity unpinned)."""
import numpy as np
import pytest

from oracle import oracle as O
from pygrid_amd.exceptions import PyGridError
from pygrid_amd.state_schema import build_state_i64_fast, parse_state_i64, varint_encode, _field, _varint

pytestmark = pytest.mark.gpu

I64_MIN, I64_MAX = -2**63, 2**63 - 1


def split(flat, numel):
    out, o = [], 0
    for n in numel:
        out.append(flat[o:o + n])
        o += n
    return out


def every_length_values(n, rng):
    """Values whose varints take 1..10 bytes, interleaved at random, plus the int64 extremes."""
    bits = rng.integers(0, 64, n)
    v = (rng.integers(0, 2**62, n, dtype=np.int64).view(np.uint64) >> np.uint64(0)) & \
        ((np.uint64(1) << bits.astype(np.uint64)) - np.uint64(1))
    v = v.view(np.int64).copy()
    neg = rng.random(n) < 0.3
    v[neg] = -v[neg] - 1
    v[: min(n, 6)] = [0, 1, -1, I64_MIN, I64_MAX, 127][: min(n, 6)]
    return v


def shares_for(rng, n_clients, n_parties, P, kind="uniform"):
    if kind == "uniform":
        return rng.integers(I64_MIN, I64_MAX, (n_clients, n_parties, P), dtype=np.int64, endpoint=True)
    return np.stack([np.stack([every_length_values(P, rng) for _ in range(n_parties)]) for _ in range(n_clients)])


def ingest_all(engine, numel, sh):
    N, S, _ = sh.shape
    for c in range(N):
        engine.ingest_state_shares(c, [build_state_i64_fast(split(sh[c, s], numel)) for s in range(S)])


@pytest.mark.parametrize("numel,kind", [
    ([311_650], "uniform"),
    ([307_328, 392, 3_920, 10], "lengths"),            # MNIST 784-392-10 tensors
    ([5, 0, 70_000, 1, 0, 123_457], "lengths"),        # empty tensors, multi-chunk payloads
    ([9_000], "lengths"),                              # one chunk, a partial window
])
def test_share_state_ingest_matches_protobuf_and_oracle(engine, numel, kind):
    rng = np.random.default_rng(sum(numel) % 1000)
    P, N, S = sum(numel), 3, 2
    sh = shares_for(rng, N, S, P, kind)
    engine.set_layout(numel)
    engine.reserve(N, 1, S)
    ingest_all(engine, numel, sh)
    s, d = engine.secagg(10, 3)
    want = O.secagg_sum(sh)
    assert np.array_equal(s, want)
    assert np.array_equal(d.view(np.uint32), O.fix_prec_decode(want).view(np.uint32))


def test_share_state_rows_decode_exactly(engine):
    """One party, one client: the summed row IS the decoded payload; checked against
    google.protobuf's parse of the very bytes that were ingested."""
    rng = np.random.default_rng(5)
    numel = [70_001, 3, 200_000]
    vals = every_length_values(sum(numel), rng)
    pb = build_state_i64_fast(split(vals, numel))
    want = np.concatenate([a.reshape(-1) for a in parse_state_i64(pb)])
    assert np.array_equal(want, vals)
    engine.set_layout(numel)
    engine.reserve(1, 1, 1)
    engine.ingest_state_shares(0, [pb])
    s, _ = engine.secagg(10, 3)
    assert np.array_equal(s, want)


def test_share_state_varints_across_chunk_edges(engine):
    """A 10-byte varint straddling every 16 KiB chunk edge and 1 KiB window edge of the payload."""
    P = 40_000  # 10-byte varints: 400,000 payload bytes, 7 chunks
    vals = np.full(P, -5, dtype=np.int64)  # negative: 10 bytes each
    vals[::7] = 3                           # 1-byte varints shift the alignment
    pb = build_state_i64_fast([vals])
    payload = varint_encode(vals)
    ends = np.flatnonzero(np.frombuffer(payload, np.uint8) < 0x80)
    assert any(e % 16_384 < 9 for e in ends)  # some varint ends just past a chunk edge
    engine.set_layout([P])
    engine.reserve(1, 1, 1)
    engine.ingest_state_shares(0, [pb])
    s, _ = engine.secagg(10, 3)
    assert np.array_equal(s, vals)


def test_share_state_wave_edges(engine):
    """K4 (a wave per 16 KiB chunk, 1 KiB windows, lane t decoding the values that end in its 16
    bytes) on a payload built around its edges: 10-byte varints straddling chunk and window edges,
    16-byte lane regions holding 16 one-byte values beside regions holding one 10-byte value's
    tail, windows denser than its LDS stage (> 256 values), the int64 extremes, and a shard range
    cutting a window."""
    P = 120_000
    vals = np.full(P, -5, dtype=np.int64)                 # 10 bytes each
    vals[::7] = 3                                          # 1-byte values shift the alignment
    vals[50_000:53_000] = np.arange(3_000) % 128           # a run of 1-byte values (16 ends per lane)
    vals[60_000:60_050] = [0, -1, 2**63 - 1, -2**63, 127, 128, 2**56, 2**56 - 1, 2**63 - 2**56, -128] * 5
    payload = varint_encode(vals)
    ends = np.flatnonzero(np.frombuffer(payload, np.uint8) < 0x80)
    assert any(e % 16_384 < 9 for e in ends) and any(e % 1_024 < 9 for e in ends)
    numel = [70_001, P - 70_001]
    pb = build_state_i64_fast(split(vals, numel))
    engine.set_layout(numel)
    engine.reserve(1, 1, 1)
    engine.ingest_state_shares(0, [pb])
    s, _ = engine.secagg(10, 3)
    assert np.array_equal(s, vals)
    lo, hi = 50_688, 90_112  # a shard boundary inside a window
    engine.set_shard(lo, hi)
    try:
        engine.reserve(1, 1, 1)
        engine.ingest_state_shares(0, [pb])
        s, _ = engine.secagg(10, 3)
    finally:
        engine.set_layout(numel)
    assert np.array_equal(s, vals[lo:hi])


def test_share_state_sharded_context(engine):
    """A param shard decodes the whole payload and keeps its range (all ranks get every client's
    shares when clients are not sharded)."""
    rng = np.random.default_rng(11)
    numel = [100_000, 50_000]
    P, N, S = sum(numel), 2, 2
    sh = shares_for(rng, N, S, P, "lengths")
    lo, hi = 70_016, 130_048
    engine.set_layout(numel)
    engine.set_shard(lo, hi)
    try:
        engine.reserve(N, 1, S)
        ingest_all(engine, numel, sh)
        s, _ = engine.secagg(10, 3)
    finally:
        engine.set_layout(numel)
    assert np.array_equal(s, O.secagg_sum(sh)[lo:hi])


def test_share_state_stream_ring_equals_resident(engine):
    rng = np.random.default_rng(12)
    numel = [66_000, 17]
    P, N, S = sum(numel), 9, 2
    sh = shares_for(rng, N, S, P, "uniform")
    engine.set_layout(numel)
    engine.reserve(4, 1, S)
    engine.stream_begin(16, 2)  # PGH_STREAM_SECAGG, fold batch 2
    ingest_all(engine, numel, sh)
    s, d = engine.stream_finish_secagg(10, 3)
    assert np.array_equal(s, O.secagg_sum(sh))


def _bad_payload_message(payload: bytes, n_values: int) -> bytes:
    td = _field(1, 2, _field(1, 2, _varint(n_values))) + _field(2, 2, b"int64") + _field(10, 2, payload)
    tt = _field(2, 0, value=4) + _field(4, 2, td)
    return _field(2, 2, _field(1, 2, tt))


@pytest.mark.parametrize("case", ["overlong_at_chunk_edge", "overlong_inside", "cut_off", "count", "float32"])
def test_share_state_rejects_malformed_and_leaves_slab(engine, case):
    P = 40_000  # ~120 KB of payload: two chunks
    good = np.arange(P, dtype=np.int64) * 3 - 7
    payload = bytearray(varint_encode(good))
    n_values = P
    if case == "overlong_at_chunk_edge":   # 12 continuation bytes around byte 65,536 (a chunk edge)
        payload[65_530:65_542] = b"\xff" * 12
    elif case == "overlong_inside":
        payload[1_000:1_011] = b"\x81" * 11
    elif case == "cut_off":
        payload[-1] |= 0x80
    elif case == "count":
        n_values = P + 1
    msg = _bad_payload_message(bytes(payload), n_values)
    if case == "float32":
        from pygrid_amd.state_schema import build_state_fast
        msg = build_state_fast([np.zeros(P, np.float32)])
    engine.set_layout([P])
    engine.reserve(1, 1, 2)
    other = np.full(P, 5, dtype=np.int64)
    engine.ingest_state_shares(0, [build_state_i64_fast([good]), build_state_i64_fast([other])])
    with pytest.raises(PyGridError):  # party 0's message is fine, party 1's is not: neither row changes
        engine.ingest_state_shares(0, [build_state_i64_fast([np.zeros(P, np.int64)]), msg])
    s, _ = engine.secagg(10, 3)
    assert np.array_equal(s, good + other)


def test_share_state_resnet18_scale_sampled(engine):
    """ResNet-18 layout (62 tensors, P = 11,689,512) x 2 clients x 2 parties of uniform shares
    (~10 bytes per value on the wire): full sum compared with the oracle."""
    from pygrid_amd.workloads import RESNET18_SHAPES

    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    P, N, S = sum(numel), 2, 2
    rng = np.random.default_rng(13)
    sh = rng.integers(I64_MIN, I64_MAX, (N, S, P), dtype=np.int64, endpoint=True)
    engine.set_layout(numel)
    engine.reserve(N, 1, S)
    ingest_all(engine, numel, sh)
    s, d = engine.secagg(10, 3)
    want = O.secagg_sum(sh)
    assert np.array_equal(s, want)
    assert np.array_equal(d.view(np.uint32), O.fix_prec_decode(want).view(np.uint32))


def test_cycle_aggregator_secure_aggregate_states(engine):
    from pygrid_amd.cycle import CycleAggregator

    rng = np.random.default_rng(14)
    numel = [307_328, 392, 3_920, 10]
    P, N, S = sum(numel), 4, 3
    sh = shares_for(rng, N, S, P, "uniform")
    msgs = [[build_state_i64_fast(split(sh[c, s], numel)) for s in range(S)] for c in range(N)]
    s, d = CycleAggregator(engine).secure_aggregate_states(numel, msgs)
    want = O.secagg_sum(sh)
    assert np.array_equal(s, want)
    assert np.array_equal(d.view(np.uint32), O.fix_prec_decode(want).view(np.uint32))


@pytest.mark.parametrize("seed", range(12))
def test_share_state_random_value_mixes(engine, seed):
    """k_varint_decode under random mixes: windows of only 1-byte varints (1,024 values per 1 KiB
    window: 16 per lane, past the LDS stage), only 10-byte ones, runs of each, random tensor splits and party
    counts -- the decoded sum bit-exact against the oracle over google.protobuf-parsed shares."""
    rng = np.random.default_rng(900 + seed)
    P = int(rng.choice([1, 17, 4_096, 4_097, 65_536, 70_001, 150_000]))
    cut = sorted(int(x) for x in rng.choice(np.arange(1, P), size=min(3, P - 1), replace=False)) if P > 3 else []
    numel = [b - a for a, b in zip([0] + cut, cut + [P])]
    S, N = int(rng.integers(1, 4)), int(rng.integers(1, 4))

    def values():
        kind = rng.integers(0, 4)
        if kind == 0:
            return rng.integers(0, 128, P).astype(np.int64)             # 1-byte varints only
        if kind == 1:
            return -rng.integers(1, 2**62, P, dtype=np.int64)           # negative: 10 bytes each
        if kind == 2:                                                   # runs of short and long values
            v = rng.integers(0, 128, P).astype(np.int64)
            for a in rng.integers(0, P, 8):
                v[a:a + int(rng.integers(1, 5000))] = -7
            return v
        return every_length_values(P, rng)

    sh = np.stack([np.stack([values() for _ in range(S)]) for _ in range(N)])
    engine.set_layout(numel)
    engine.reserve(N, 1, S)
    ingest_all(engine, numel, sh)
    s, d = engine.secagg(10, 3)
    want = O.secagg_sum(sh)
    assert np.array_equal(s, want)
    assert np.array_equal(d.view(np.uint32), O.fix_prec_decode(want).view(np.uint32))


def test_share_state_decode_buffers_alternate_and_grow(engine):
    """The varint decodes run on their own stream with two alternating HBM byte buffers: messages of
    growing and shrinking wire size (1-byte to 10-byte varints, so each buffer grows while the other
    one's decode may be in flight), a client re-ingested right after its first decode, and a STREAM
    ring of two slots folded one client at a time (slots overwritten behind their folds) -- the sums
    bit-exact against the oracle."""
    rng = np.random.default_rng(15)
    numel = [90_001, 13]
    P, S, N = sum(numel), 2, 10
    sh = np.empty((N, S, P), np.int64)
    for c in range(N):  # alternate short and long varints, the long ones getting longer
        sh[c] = rng.integers(0, 128, (S, P)) if c % 2 == 0 else -rng.integers(1, 2**(20 + 4 * c), (S, P), dtype=np.int64)
    msgs = [[build_state_i64_fast(split(sh[c, s], numel)) for s in range(S)] for c in range(N)]
    engine.set_layout(numel)
    engine.reserve(N, 1, S)
    for c in range(N):
        engine.ingest_state_shares(c, msgs[c])
        if c == 3:  # overwrite client 1 (small messages) and client 3 (long ones) at once
            sh[1] = rng.integers(I64_MIN, I64_MAX, (S, P), dtype=np.int64, endpoint=True)
            engine.ingest_state_shares(1, [build_state_i64_fast(split(sh[1, s], numel)) for s in range(S)])
            engine.ingest_state_shares(3, msgs[3])
    s, d = engine.secagg(10, 3)
    want = O.secagg_sum(sh)
    assert np.array_equal(s, want)
    assert np.array_equal(d.view(np.uint32), O.fix_prec_decode(want).view(np.uint32))
    msgs[1] = [build_state_i64_fast(split(sh[1, s], numel)) for s in range(S)]
    engine.reserve(2, 1, S)
    engine.stream_begin(16, 1)  # PGH_STREAM_SECAGG, a fold per client through a ring of two slots
    for c in range(N):
        engine.ingest_state_shares(c, msgs[c])
    s2, _ = engine.stream_finish_secagg(10, 3)
    assert np.array_equal(s2, want)
