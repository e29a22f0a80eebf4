"""CPU: pin the oracle before trusting it.

* against the reference's literal torch expressions (cycle_manager.py:286-288, :293-296 and the
  avg_plan of 01-Create-plan.ipynb:450-454, called as at cycle_manager.py:269);
* against the reference's known-answer test (01-Create-plan.ipynb:486-501);
* against the SMPC tests' vectors and tolerances (test_basic_syft_operations.py:388-454);
* numpy restatement vs scalar C restatement, and both vs the committed golden fixtures.
"""
import hashlib
import json
from functools import reduce

import numpy as np
import pytest
import torch as th

from oracle import coracle
from oracle import oracle as O
from oracle.gen_golden import MNIST_SHAPES, mnist_inputs, split

F = np.float32


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    nan = np.isnan(a)
    return a.shape == b.shape and np.array_equal(nan, np.isnan(b)) and np.array_equal(bits(a)[~nan], bits(b)[~nan])


# ---- the reference's own code, evaluated in torch --------------------------------------------
def ref_hardcoded(model_params, diffs):
    """cycle_manager.py:276-296 verbatim (torch CPU)."""
    raw_diffs = [[diff[model_param] for diff in diffs] for model_param in range(len(model_params))]
    sums = [reduce(th.add, param) for param in raw_diffs]
    diff_avg = [th.div(param, len(diffs)) for param in sums]
    return [model_param - diff_param for model_param, diff_param in zip(model_params, diff_avg)]


def avg_plan(avg, item, num):
    """01-Create-plan.ipynb:450-454 verbatim."""
    new_avg = []
    for i, param in enumerate(avg):
        new_avg.append((avg[i] * num + item[i]) / (num + 1))
    return new_avg


def ref_iterative(model_params, diffs):
    """cycle_manager.py:266-269 + :293-296 verbatim."""
    diff_avg = diffs[0]
    for i, diff in enumerate(diffs[1:]):
        diff_avg = avg_plan(list(diff_avg), diff, th.tensor([i + 1]))
    return [model_param - diff_param for model_param, diff_param in zip(model_params, diff_avg)]


def _torchify(ckpt, diffs):
    return [th.from_numpy(np.array(p)) for p in ckpt], [[th.from_numpy(np.array(t)) for t in d] for d in diffs]


@pytest.mark.parametrize("n", [1, 2, 3, 7, 40])
def test_oracle_matches_reference_expressions(n):
    rng = np.random.default_rng(n)
    shapes = [(13, 7), (5,), (1,), (64,)]
    ckpt = [rng.standard_normal(s).astype(F) for s in shapes]
    diffs = [[(rng.standard_normal(s) * 10 ** rng.uniform(-6, 2)).astype(F) for s in shapes] for _ in range(n)]
    tc, td = _torchify(ckpt, diffs)
    for got, want in zip(O.fedavg_mean(ckpt, diffs), ref_hardcoded(tc, td)):
        assert same(got, want.numpy())
    for got, want in zip(O.fedavg_iterative(ckpt, diffs), ref_iterative(tc, td)):
        assert same(got, want.numpy())
    for got, want in zip(O.fedavg_mean_torch(tc, td), ref_hardcoded(tc, td)):  # the bench's CPU legs
        assert same(got.numpy(), want.numpy())
    for got, want in zip(O.fedavg_iterative_torch(tc, td), ref_iterative(tc, td)):
        assert same(got.numpy(), want.numpy())


def test_secagg_torch_restatement_matches_oracle():
    rng = np.random.default_rng(9)
    sh = rng.integers(-2**63, 2**63 - 1, size=(5, 2, 300), dtype=np.int64, endpoint=True)
    s, dec = O.secagg_sum_torch([[th.from_numpy(sh[c, p]) for p in range(2)] for c in range(5)])
    want = O.secagg_sum(sh)
    assert np.array_equal(s.numpy(), want)
    assert np.array_equal(dec.numpy().view(np.uint32), O.fix_prec_decode(want).view(np.uint32))


def test_oracle_matches_reference_on_edge_values():
    z = np.load("tests/golden/edge_f32.npz")
    for name in z["names"]:
        d, c = z[f"{name}_diffs"], z[f"{name}_ckpt"]
        tc, td = _torchify([c], [[row] for row in d])
        with np.errstate(all="ignore"):
            assert same(O.fedavg_mean([c], [[row] for row in d])[0], ref_hardcoded(tc, td)[0].numpy()), name
            assert same(O.fedavg_iterative([c], [[row] for row in d])[0], ref_iterative(tc, td)[0].numpy()), name


def test_kat_avg_plan(gold):
    """01-Create-plan.ipynb:486-501: avg of ones*[1, 5.5, 7, 55] == ones*17.125 exactly."""
    kat = json.loads((gold / "kat_avg_plan.json").read_text())
    shapes = [tuple(s) for s in kat["shapes"]]
    diffs = [[np.ones(s, F) * F(k) for s in shapes] for k in kat["coeffs"]]
    zero = [np.zeros(s, F) for s in shapes]
    out = O.fedavg_iterative(zero, diffs)
    for o in out:
        assert np.all(-o == F(kat["expected_avg"]))
    # and the same through the torch restatement of the notebook's own loop
    tz, td = _torchify(zero, diffs)
    for o in ref_iterative(tz, td):
        assert th.all(-o == kat["expected_avg"])


def test_weighted_reduces_to_mean_at_unit_weights():
    rng = np.random.default_rng(3)
    d = [[rng.standard_normal(33).astype(F)] for _ in range(9)]
    c = [rng.standard_normal(33).astype(F)]
    assert same(O.fedavg_weighted(c, d, np.ones(9, F))[0], O.fedavg_mean(c, d)[0])


def test_c_oracle_matches_numpy_oracle(gold):
    z = np.load(gold / "edge_f32.npz")
    for name in z["names"]:
        d, c, w = z[f"{name}_diffs"], z[f"{name}_ckpt"], z[f"{name}_w"]
        with np.errstate(all="ignore"):
            assert same(coracle.fedavg(0, d, c), z[f"{name}_mean"]), name
            assert same(coracle.fedavg(1, d, c), z[f"{name}_iter"]), name
            assert same(coracle.fedavg(2, d, c, w), z[f"{name}_weighted"]), name
            assert same(O.fedavg_mean([c], [[r] for r in d])[0], z[f"{name}_mean"]), name
            assert same(O.fedavg_iterative([c], [[r] for r in d])[0], z[f"{name}_iter"]), name
            assert same(O.fedavg_weighted([c], [[r] for r in d], w)[0], z[f"{name}_weighted"]), name


def test_c_oracle_padded_rows():
    rng = np.random.default_rng(11)
    d = rng.standard_normal((5, 64)).astype(F)
    c = rng.standard_normal(61).astype(F)
    want = O.fedavg_mean([c], [[r[:61]] for r in d])[0]
    assert same(coracle.fedavg(0, d, c), want)


def test_generator_c_matches_numpy():
    idx0, n = 1_000_003, 4099
    for stream, row, scale in ((O.STREAM_DIFF, 0, O.DIFF_SCALE), (O.STREAM_DIFF, 999, O.DIFF_SCALE),
                               (O.STREAM_CKPT, 0, O.CKPT_SCALE)):
        a = coracle.synth_f32(1234, stream, row, idx0, n, float(scale))
        b = O.bits_to_f32(O.synth_bits(1234, stream, row, np.arange(idx0, idx0 + n, dtype=np.uint64)), scale)
        assert same(a, b)
    u = coracle.synth_u64(77, O.STREAM_SHARE, 5, 10, 100)
    assert np.array_equal(u, O.synth_bits(77, O.STREAM_SHARE, 5, np.arange(10, 110, dtype=np.uint64)))


@pytest.mark.parametrize("idx0", [0, 64, 70_001])
def test_fast_generator_c_matches_numpy(idx0):
    n = 50_003
    a = coracle.synth_f32_fast(11, O.STREAM_DIFF, 5, idx0, n, float(O.DIFF_SCALE))
    b = O.synth_diff_fast(11, 5, np.arange(idx0, idx0 + n, dtype=np.uint64))
    assert np.array_equal(bits(a), bits(b))
    assert abs(float(b.mean())) < 2e-4 and 0.0095 < float(b.std()) < 0.0105


def test_generator_statistics():
    x = O.synth_diff(1234, 0, np.arange(200_000, dtype=np.uint64))
    assert abs(float(x.mean())) < 1e-4 and 0.0095 < float(x.std()) < 0.0105
    c = O.synth_ckpt(1234, np.arange(200_000, dtype=np.uint64))
    assert 0.047 < float(c.std()) < 0.053


def test_mnist_golden(gold):
    g = json.loads((gold / "mnist_synth.json").read_text())
    diffs, ckpt = mnist_inputs(g["seed"], g["n_clients"])
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert h(diffs) == g["sha256_diffs"] and h(ckpt) == g["sha256_ckpt"]
    ck = split(ckpt, MNIST_SHAPES)
    ds = [split(d, MNIST_SHAPES) for d in diffs]
    assert h(np.concatenate([a.reshape(-1) for a in O.fedavg_mean(ck, ds)])) == g["sha256_mean"]
    assert h(np.concatenate([a.reshape(-1) for a in O.fedavg_iterative(ck, ds)])) == g["sha256_iter"]
    w = np.asarray(g["weights"], F)
    assert h(np.concatenate([a.reshape(-1) for a in O.fedavg_weighted(ck, ds, w)])) == g["sha256_weighted"]
    # the C oracle on the flat layout agrees
    assert h(coracle.fedavg(0, diffs, ckpt)) == g["sha256_mean"]


def test_state_bytes_cycle_close_restatement(gold):
    """oracle.cycle_close_state_torch (bytes -> bytes, cycle_manager.py:240-303 over the restated
    State schema) decodes to the golden MNIST mean and keeps the checkpoint's framing."""
    from pygrid_amd.state_schema import build_state, parse_state

    g = json.loads((gold / "mnist_synth.json").read_text())
    diffs, ckpt = mnist_inputs(g["seed"], g["n_clients"])
    ck = split(ckpt, MNIST_SHAPES)
    ds = [split(d, MNIST_SHAPES) for d in diffs]
    ck_pb = build_state(ck, as_param=True)
    new = O.cycle_close_state_torch(ck_pb, [build_state(d) for d in ds])
    got = [a for a in parse_state(new)]
    assert [a.shape for a in got] == [tuple(s) for s in MNIST_SHAPES]
    flat = np.concatenate([a.reshape(-1) for a in got])
    assert hashlib.sha256(flat.tobytes()).hexdigest() == g["sha256_mean"]
    assert len(new) == len(ck_pb)  # same framing, payloads replaced


def test_secagg_state_restatement_matches_oracle():
    """oracle.secagg_close_state_torch (share State bytes -> torch int64 adds -> decode) equals the
    numpy share sum and decode, including int64 wrap."""
    from pygrid_amd.state_schema import build_state_i64_fast

    rng = np.random.default_rng(21)
    sh = rng.integers(-2**63, 2**63 - 1, (4, 2, 777), dtype=np.int64, endpoint=True)
    sh[0, 0, :3] = [2**63 - 1, -2**63, -1]
    msgs = [[build_state_i64_fast([sh[c, s][:500], sh[c, s][500:]]) for s in range(2)] for c in range(4)]
    s, d = O.secagg_close_state_torch(msgs)
    want = O.secagg_sum(sh)
    assert np.array_equal(s.numpy(), want)
    assert np.array_equal(bits(d.numpy()), bits(O.fix_prec_decode(want)))


# ---- secure aggregation ------------------------------------------------------------------------
def test_smpc_integer_share_reconstructs_exactly(gold):
    """test_basic_syft_operations.py:388-394."""
    z = np.load(gold / "smpc_vectors.npz")
    assert np.array_equal(O.secagg_sum(z["share_shares"]), z["share_x"])
    s, _ = coracle.secagg(z["share_shares"], z["share_x"].size)
    assert np.array_equal(s, z["share_x"])


@pytest.mark.parametrize("op", ["add", "sub"])
@pytest.mark.parametrize("k", [0, 1, 2])
def test_smpc_fixed_point_matches_reference_tolerance(gold, op, k):
    """test_basic_syft_operations.py:417-424 / :447-454: allclose(..., atol=1e-3)."""
    z = np.load(gold / "smpc_vectors.npz")
    sh = z[f"{op}{k}_shares"]
    tot = O.secagg_sum(sh)
    assert np.array_equal(tot, z[f"{op}{k}_sum"])
    dec = O.fix_prec_decode(tot)
    assert np.array_equal(bits(dec), bits(z[f"{op}{k}_dec"]))
    assert np.allclose(dec, z[f"{op}{k}_ref"], atol=1e-3)
    s, d = coracle.secagg(sh, sh.shape[-1])
    assert np.array_equal(s, tot) and np.array_equal(bits(d), bits(dec))


def test_secagg_wrap_and_rounding(gold):
    z = np.load(gold / "secagg_wrap.npz")
    assert np.array_equal(O.secagg_sum(z["shares"]), z["sum"])
    s, d = coracle.secagg(z["shares"], z["sum"].size)
    assert np.array_equal(s, z["sum"]) and np.array_equal(bits(d), bits(z["dec"]))
    # torch's own int64 wrap / float decode agree (the reference's arithmetic)
    t = th.from_numpy(z["shares"]).sum(dim=(0, 1))
    assert np.array_equal(t.numpy(), z["sum"])
    assert np.array_equal(bits((t.float() / 1000).numpy()), bits(z["dec"]))


def test_synth_shares_reconstruct():
    idx = np.arange(5000, 5100, dtype=np.uint64)
    for S in (2, 3):
        sh = O.synth_shares(42, 7, S, idx)
        x = O.bits_to_f32(O.synth_bits(42, O.STREAM_SECRET, 7, idx), O.DIFF_SCALE)
        assert np.array_equal(O.secagg_sum(sh[None]), O.fix_prec_encode(x))


def test_ready_to_average_oracle():
    """cycle_manager.py:196-210 truth table spot checks."""
    assert O.ready_to_average({}, 0)
    assert not O.ready_to_average({"min_diffs": 2}, 1)
    assert O.ready_to_average({"min_diffs": 2}, 2)
    assert O.ready_to_average({"max_diffs": 1}, 1)
    assert not O.ready_to_average({"max_diffs": 3}, 2)
    assert O.ready_to_average({"max_diffs": 3}, 2, cycle_end=5, now=6)
    assert not O.ready_to_average({"max_diffs": 3, "min_diffs": 3}, 2, cycle_end=5, now=6)
