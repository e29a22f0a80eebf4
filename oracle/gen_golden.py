"""Generate the committed golden fixtures under tests/golden/ -- TEST INFRASTRUCTURE ONLY.

    python -m oracle.gen_golden        (from the repo root)

Fixtures and what pins them:

* ``kat_avg_plan.json``       the reference's own known-answer test,
  ``examples/model-centric/01-Create-plan.ipynb:486-501`` (coefficients [1, 5.5, 7, 55] on the
  MNIST 784-392-10 parameter shapes iterate to exactly 17.125).
* ``smpc_vectors.npz``        the input vectors of ``tests/data_centric/test_basic_syft_operations.py``
  (:388-394 integer share/reconstruct; :398-424 fixed-point add; :427-454 fixed-point sub),
  split into 4 additive shares (the 4 nodes of ``tests/__init__.py:6-7``) with seeded words,
  plus the oracle's expected wrap-sums / decodes and the reference's float results (atol 1e-3).
* ``edge_f32.npz``            hand-built fp32 edge cases (N = 1, -0.0, subnormals, cancellation,
  inf/nan, ragged sizes) with oracle outputs for mean / iterative / weighted.
* ``secagg_wrap.npz``         int64 wrap-around and int64->float32 rounding boundaries.
* ``mnist_synth.json``        SHA-256 of the oracle's mean / iterative / weighted outputs on the
  synthetic MNIST N = 3 cycle (inputs regenerate from the seed via the restated generator).
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np

from . import oracle as O

ROOT = Path(__file__).resolve().parent.parent
GOLD = ROOT / "tests" / "golden"
MNIST_SHAPES = [(392, 784), (392,), (10, 392), (10,)]
MNIST_SEED = 1234


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def mnist_inputs(seed=MNIST_SEED, n=3):
    P = sum(int(np.prod(s)) for s in MNIST_SHAPES)
    idx = np.arange(P, dtype=np.uint64)
    diffs = np.stack([O.synth_diff(seed, c, idx) for c in range(n)])
    ckpt = O.synth_ckpt(seed, idx)
    return diffs, ckpt


def split(flat, shapes):
    out, off = [], 0
    for s in shapes:
        k = int(np.prod(s))
        out.append(flat[off:off + k].reshape(s))
        off += k
    return out


def flat_fedavg(fn, diffs2d, ckpt, *extra):
    return fn([ckpt], [[d] for d in diffs2d], *extra)[0]


def gen_kat():
    (GOLD / "kat_avg_plan.json").write_text(json.dumps({
        "source": "examples/model-centric/01-Create-plan.ipynb:486-501",
        "coeffs": [1, 5.5, 7, 55],
        "shapes": [list(s) for s in MNIST_SHAPES],
        "expected_avg": 17.125,
        "note": "avg_plan iterated over dummy diffs ones*coeff must eq ones*mean(coeffs) exactly",
    }, indent=1) + "\n")


SMPC_ADD = [  # test_basic_syft_operations.py:398-415 (also the sub cases :428-445)
    (np.array(1.0, np.float32), np.array(0.1, np.float32)),
    (np.array([[0.1, 1.2], [2.2, 3.1], [4.9, 5.2]], np.float32),
     np.array([[-3.2, 1.21], [-8.4, 34.9], [43.9, 50.2]], np.float32)),
    (np.array([[0.9039, 0.6291, 1.0795], [0.1586, 2.1939, -0.4900], [-0.1909, -0.7503, 1.9355]], np.float32),
     np.zeros(3, np.float32)),
]


def gen_smpc():
    rng = np.random.default_rng(20200909)
    arrays = {}
    S = 4  # Alice, Bob, Charlie, Dan
    # :388-394 share/reconstruct of th.tensor([1..6]) is integer exact
    x = np.arange(1, 7, dtype=np.int64)
    sh = O.make_shares(x, S, rng.integers(0, 2**63, size=(S - 1, 6), dtype=np.uint64) * np.uint64(2) + np.uint64(1))
    arrays["share_x"] = x
    arrays["share_shares"] = sh[None]
    arrays["share_sum"] = O.secagg_sum(sh[None])
    for k, (xa, ya) in enumerate(SMPC_ADD):
        xb, yb = np.broadcast_arrays(xa, ya)
        xb = xb.reshape(-1).astype(np.float32)
        yb = yb.reshape(-1).astype(np.float32)
        p = xb.size
        ex, ey = O.fix_prec_encode(xb), O.fix_prec_encode(yb)
        rx = rng.integers(0, 2**63, size=(S - 1, p), dtype=np.uint64) * np.uint64(2)
        ry = rng.integers(0, 2**63, size=(S - 1, p), dtype=np.uint64) * np.uint64(2)
        for op, sign in (("add", 1), ("sub", -1)):
            # client side: the second operand's shares negated for sub (x_s - y_s)
            shx = O.make_shares(ex, S, rx)
            shy = O.make_shares(ey, S, ry)
            if sign < 0:
                with np.errstate(over="ignore"):
                    shy = (np.zeros_like(shy.view(np.uint64)) - shy.view(np.uint64)).view(np.int64)
            shares = np.stack([shx, shy])  # [clients=2][S][p]
            tot = O.secagg_sum(shares)
            arrays[f"{op}{k}_shares"] = shares
            arrays[f"{op}{k}_sum"] = tot
            arrays[f"{op}{k}_dec"] = O.fix_prec_decode(tot)
            arrays[f"{op}{k}_ref"] = (xb + yb) if sign > 0 else (xb - yb)
    np.savez(GOLD / "smpc_vectors.npz", **arrays)


def gen_edge():
    f = np.float32
    tiny = np.float32(1.4e-45)  # smallest subnormal
    cases = {
        # name: (diffs [N][P], ckpt [P], weights [N])
        "n1": (np.array([[1.5, -0.0, 3e-39, -7.25, 0.1]], f), np.array([0.0, -0.0, 1.0, 2.0, 0.1], f), [2.0]),
        "negzero": (np.array([[-0.0, -0.0, 0.0], [-0.0, 0.0, -0.0]], f), np.array([-0.0, 0.0, -0.0], f), [1.0, 1.0]),
        "subnormal": (np.array([[tiny, 1e-38, -3e-39, 5e-39, 1.1754942e-38],
                                [tiny, -1e-38, 3e-39, 5e-39, 1e-45],
                                [tiny * 3, 2e-39, 1e-40, -5e-39, 0.0]], f),
                      np.array([0.0, 1e-38, 0.0, -1e-39, 1.2e-38], f), [1.0, 0.5, 3.0]),
        "cancel": (np.array([[1e30, 1.0, 3.4e38, -1e-8, 16777216.0, 0.1],
                             [-1e30, 1e-8, 3.4e38, 1e8, 1.0, 0.2],
                             [1.0, -1.0, -3.4e38, -1e8, 1.0, 0.3]], f),
                   np.array([0.0, 0.0, 0.0, 0.0, 0.0, 0.6], f), [1.0, 1.0, 1.0]),
        "nonfinite": (np.array([[np.inf, np.nan, 1.0, -np.inf], [1.0, 2.0, np.inf, np.inf]], f),
                      np.array([0.0, 1.0, np.inf, 0.0], f), [1.0, 2.0]),
        "ragged7": (np.linspace(-3, 3, 5 * 7, dtype=f).reshape(5, 7) * f(0.37), np.linspace(1, 2, 7, dtype=f),
                    [1.0, 2.0, 0.25, 4.0, 1.0]),
    }
    rng = np.random.default_rng(99)
    for n, p in ((17, 1), (9, 3), (4, 1023), (33, 130), (2, 4099)):
        cases[f"rand_n{n}_p{p}"] = (rng.standard_normal((n, p)).astype(f) * f(1e-2),
                                    rng.standard_normal(p).astype(f),
                                    list(rng.uniform(0.1, 10.0, n).astype(f)))
    arrays = {}
    for name, (d, c, w) in cases.items():
        arrays[f"{name}_diffs"] = d
        arrays[f"{name}_ckpt"] = c
        arrays[f"{name}_w"] = np.asarray(w, f)
        with np.errstate(all="ignore"):
            arrays[f"{name}_mean"] = flat_fedavg(O.fedavg_mean, d, c)
            arrays[f"{name}_iter"] = flat_fedavg(O.fedavg_iterative, d, c)
            arrays[f"{name}_weighted"] = flat_fedavg(O.fedavg_weighted, d, c, np.asarray(w, f))
    arrays["names"] = np.array(sorted(cases))
    np.savez(GOLD / "edge_f32.npz", **arrays)


def gen_wrap():
    i64 = np.int64
    M = np.iinfo(i64)
    vals = np.array([M.max, M.min, -1, 1, 2**24 + 1, 2**53 + 1, -(2**53) - 3, 2**62 + 2**38 + 1,
                     M.max - 2**38, 123456789012345, -987654321098765, 0, 2**31, -(2**31) - 1], dtype=i64)
    P = vals.size
    rng = np.random.default_rng(5)
    # 3 clients x 2 parties; client 0 carries vals, clients 1-2 push sums across the wrap
    with np.errstate(over="ignore"):
        c1 = np.full(P, M.max, i64)
        c2 = np.full(P, 2, i64)
        secrets = [vals, c1, c2]
        shares = np.stack([O.make_shares(s, 2, rng.integers(0, 2**63, size=(1, P), dtype=np.uint64) * np.uint64(2))
                           for s in secrets])
    tot = O.secagg_sum(shares)
    np.savez(GOLD / "secagg_wrap.npz", shares=shares, sum=tot, dec=O.fix_prec_decode(tot),
             dec_base2_prec16=(tot.astype(np.float32) / np.float32(2 ** 16)).astype(np.float32))


def gen_mnist():
    diffs, ckpt = mnist_inputs()
    w = np.array([1.0, 2.5, 0.75], np.float32)
    out = {
        "seed": MNIST_SEED, "n_clients": 3, "shapes": [list(s) for s in MNIST_SHAPES],
        "diff_scale": float(O.DIFF_SCALE), "ckpt_scale": float(O.CKPT_SCALE), "weights": w.tolist(),
        "sha256_diffs": sha(diffs), "sha256_ckpt": sha(ckpt),
        "sha256_mean": sha(flat_fedavg(O.fedavg_mean, diffs, ckpt)),
        "sha256_iter": sha(flat_fedavg(O.fedavg_iterative, diffs, ckpt)),
        "sha256_weighted": sha(flat_fedavg(O.fedavg_weighted, diffs, ckpt, w)),
        "head_mean": flat_fedavg(O.fedavg_mean, diffs[:, :8], ckpt[:8]).astype(float).tolist(),
        "first_diff_head": diffs[0, :8].astype(float).tolist(),
    }
    (GOLD / "mnist_synth.json").write_text(json.dumps(out, indent=1) + "\n")


def main():
    GOLD.mkdir(parents=True, exist_ok=True)
    gen_kat()
    gen_smpc()
    gen_edge()
    gen_wrap()
    gen_mnist()
    print("wrote", sorted(p.name for p in GOLD.iterdir()))


if __name__ == "__main__":
    main()
