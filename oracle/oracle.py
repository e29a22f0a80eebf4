"""CPU oracle for the PyGrid cycle-close aggregation path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product path (``pygrid_amd``) never
imports it and has no CPU fallback.

Every function below restates, in numpy with explicit float32/int64 arithmetic, one piece
of the reference's algorithm.  Citations are ``file:line`` under ``/root/reference``.

Parity pinning (see DESIGN.md "Oracle"):

* ``fedavg_iterative`` is pinned by the reference's own known-answer test
  (``examples/model-centric/01-Create-plan.ipynb:486-501``: coefficients [1, 5.5, 7, 55]
  iterate to exactly 17.125) and by a torch restatement of the plan expression evaluated
  in ``tests/test_oracle.py``.
* ``fedavg_mean`` is pinned by evaluating the reference's literal torch expressions
  (``reduce(th.add, ...)``, ``th.div(sum, N)``, ``model_param - diff_param``) in
  ``tests/test_oracle.py``; the reference has no test asserting averaged values, so this
  is the strongest pin available offline.
* ``secagg_*`` restates PySyft 0.2.9 FixedPrecisionTensor / AdditiveSharingTensor
  (external; not importable here).  Pinned by the reference's SMPC tests'
  own vectors and tolerances (``tests/data_centric/test_basic_syft_operations.py:388-454``:
  integer-exact share/reconstruct, fixed-point add/sub within atol=1e-3).
* ``fedavg_weighted`` has no reference counterpart (every reference branch is
  unweighted); it is pinned only by this oracle and reduces to ``fedavg_mean`` bit for
  bit at w == 1.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
U64 = np.uint64
I64 = np.int64

# ----------------------------------------------------------------------------------------
# (a5)+(a8) hard-coded mean:  cycle_manager.py:276-296
# ----------------------------------------------------------------------------------------


def fedavg_mean(model_params, diffs):
    """Restates ``CycleManager._average_plan_diffs`` hard-coded branch.

    ``cycle_manager.py:276-279`` transposes diffs to per-param lists,
    ``:286`` ``sums = [reduce(th.add, param) ...]`` is a LEFT fold
    ``((d0 + d1) + d2) + ...`` in float32 (the fold starts from d0, not from 0, which
    matters for -0.0), ``:288`` ``th.div(param, len(diffs))`` is IEEE float32 true division
    by float(N), and ``:293-296`` ``model_param - diff_param`` is a float32 subtract.

    model_params: list of T float32 arrays; diffs: list of N lists of T float32 arrays.
    Returns the list of T updated float32 arrays.
    """
    n = len(diffs)
    if n == 0:
        raise ValueError("no diffs to average")
    out = []
    for j, p in enumerate(model_params):
        acc = np.asarray(diffs[0][j], dtype=F32)
        for d in diffs[1:]:
            acc = (acc + np.asarray(d[j], dtype=F32)).astype(F32)
        avg = (acc / F32(n)).astype(F32)
        out.append((np.asarray(p, dtype=F32) - avg).astype(F32))
    return out


def fedavg_mean_torch(model_params, diffs):
    """The reference's hard-coded branch as it runs on the node: ``cycle_manager.py:276-296``
    evaluated in torch on CPU tensors (``reduce(th.add, ...)``, ``th.div(sum, len(diffs))``,
    ``model_param - diff_param``).  Bit-identical to ``fedavg_mean`` (``tests/test_oracle.py``);
    ``bench.py``'s ``cpu_baseline`` times it at the node's 1 thread and at all host cores."""
    from functools import reduce

    import torch as th

    raw = [[d[j] for d in diffs] for j in range(len(model_params))]
    sums = [reduce(th.add, param) for param in raw]
    avg = [th.div(param, len(diffs)) for param in sums]
    return [p - a for p, a in zip(model_params, avg)]


def _state_tensor(stt):
    return stt.torch_tensor if stt.HasField("torch_tensor") else stt.torch_param.tensor


def unserialize_state_torch(pb: bytes):
    """``ModelManager.unserialize_model_params`` (model_manager.py:94-103) restated with Google's
    protobuf runtime over the build's State schema restatement (``pygrid_amd.state_schema``;
    syft-proto 0.5.2 is absent): ``StatePB.ParseFromString`` (:98-99), then syft 0.2.9's protobuf
    tensor deserializer, i.e. ``torch.tensor(contents_<dtype>, dtype=...).reshape(shape)`` per
    tensor (``_unbufferize`` :101, ``state.tensors()`` :102).  Returns (tensors, parsed message)."""
    import torch as th

    from pygrid_amd.state_schema import classes

    st = classes()["State"]()
    st.ParseFromString(pb)
    ts = []
    for stt in st.tensors:
        tt = _state_tensor(stt)
        ts.append(th.tensor(tt.contents_data.contents_float32, dtype=th.float32)
                  .reshape(tuple(tt.contents_data.shape.dims)))
    return ts, st


def serialize_state_torch(st, params) -> bytes:
    """``ModelManager.serialize_model_params`` (model_manager.py:79-92) restated: every tensor's
    values written back into the State message as the repeated ``contents_float32`` field (syft's
    tensor serializer: ``.extend(tensor.flatten().tolist())``), then ``SerializeToString`` (:90).
    The parsed checkpoint message is reused as the frame (ids/tags kept), as in the engine."""
    for stt, t in zip(st.tensors, params):
        tt = _state_tensor(stt)
        del tt.contents_data.contents_float32[:]
        tt.contents_data.contents_float32.extend(t.reshape(-1).tolist())
    return st.SerializeToString()


def cycle_close_state_torch(ckpt_pb: bytes, diff_pbs):
    """The node's hard-coded cycle close on bytes, ``cycle_manager.py:240-303``: unserialize the
    checkpoint (:240) and every reported diff (:247-250), mean (:276-288), apply (:293-296),
    serialize the new checkpoint (:303).  ``bench.py``'s cpu_baseline leg times it (the whole
    bytes -> bytes close the engine replaces); ``tests/test_oracle.py`` checks its values against
    ``fedavg_mean``."""
    params, st = unserialize_state_torch(ckpt_pb)
    diffs = [unserialize_state_torch(pb)[0] for pb in diff_pbs]
    return serialize_state_torch(st, fedavg_mean_torch(params, diffs))


# ----------------------------------------------------------------------------------------
# (a6)+(a8) hosted iterative avg plan: cycle_manager.py:266-269 + 01-Create-plan.ipynb:450-454
# ----------------------------------------------------------------------------------------


def fedavg_iterative(model_params, diffs):
    """Restates the iterative hosted-plan branch.

    ``cycle_manager.py:267-269``: ``diff_avg = diffs[0]``; for i, diff in
    enumerate(diffs[1:]): ``diff_avg = avg_plan(list(diff_avg), diff, th.tensor([i + 1]))``.
    The plan (``01-Create-plan.ipynb:450-454``) computes ``(avg[i] * num + item[i]) /
    (num + 1)``; ``num`` is an int64 tensor, promoted to float32 (exact for k < 2**24),
    and each of mul, add, div is rounded separately (no fused multiply-add).
    Then ``:293-296`` subtracts from the checkpoint.
    """
    n = len(diffs)
    if n == 0:
        raise ValueError("no diffs to average")
    out = []
    for j, p in enumerate(model_params):
        a = np.asarray(diffs[0][j], dtype=F32)
        for k in range(1, n):
            prod = (a * F32(k)).astype(F32)
            s = (prod + np.asarray(diffs[k][j], dtype=F32)).astype(F32)
            a = (s / F32(k + 1)).astype(F32)
        out.append((np.asarray(p, dtype=F32) - a).astype(F32))
    return out


def fedavg_iterative_torch(model_params, diffs):
    """The iterative branch as the node runs it, in torch on CPU tensors:
    ``cycle_manager.py:266-269`` calling the plan of ``01-Create-plan.ipynb:450-454`` with
    ``th.tensor([i + 1])`` (the plan's ops executed directly instead of through syft's Plan
    interpreter, so this is a lower bound on the reference's time).  Bit-identical to
    ``fedavg_iterative`` (``tests/test_oracle.py``)."""
    import torch as th

    def avg_plan(avg, item, num):
        return [(a * num + i) / (num + 1) for a, i in zip(avg, item)]

    diff_avg = diffs[0]
    for i, diff in enumerate(diffs[1:]):
        diff_avg = avg_plan(list(diff_avg), diff, th.tensor([i + 1]))
    return [p - a for p, a in zip(model_params, diff_avg)]


# ----------------------------------------------------------------------------------------
# weighted FedAvg (north_star; no reference counterpart -- build-owned definition)
# ----------------------------------------------------------------------------------------


def weight_total(weights):
    """Left fold of the client weights in float32 (the divisor of ``fedavg_weighted``)."""
    w = np.asarray(weights, dtype=F32)
    tot = w[0]
    for x in w[1:]:
        tot = F32(tot + x)
    return F32(tot)


def fedavg_weighted(model_params, diffs, weights):
    """``ckpt - (sum_c w_c * d_c) / (sum_c w_c)``, all float32, clients folded in index
    order, each product rounded before its add (no FMA).  With w == 1 every product is
    exact, the divisor is float(N), and the result equals ``fedavg_mean`` bit for bit.
    """
    n = len(diffs)
    if n == 0:
        raise ValueError("no diffs to average")
    w = np.asarray(weights, dtype=F32)
    if w.shape != (n,):
        raise ValueError("need one weight per diff")
    wt = weight_total(w)
    out = []
    for j, p in enumerate(model_params):
        acc = (np.asarray(diffs[0][j], dtype=F32) * w[0]).astype(F32)
        for c in range(1, n):
            acc = (acc + (np.asarray(diffs[c][j], dtype=F32) * w[c]).astype(F32)).astype(F32)
        avg = (acc / wt).astype(F32)
        out.append((np.asarray(p, dtype=F32) - avg).astype(F32))
    return out


# ----------------------------------------------------------------------------------------
# (a3) readiness predicate: cycle_manager.py:196-210
# ----------------------------------------------------------------------------------------


def ready_to_average(server_config, received_diffs, cycle_end=None, now=None):
    """Restates ``complete_cycle``'s readiness test, ``cycle_manager.py:196-210``."""
    min_diffs = server_config.get("min_diffs", None)
    max_diffs = server_config.get("max_diffs", None)
    hit_diffs_limit = received_diffs >= max_diffs if max_diffs is not None else False
    hit_time_limit = (now >= cycle_end) if cycle_end is not None else False
    no_limits = max_diffs is None and cycle_end is None
    has_enough = received_diffs >= min_diffs if min_diffs is not None else True
    return bool(has_enough and (no_limits or hit_diffs_limit or hit_time_limit))


# ----------------------------------------------------------------------------------------
# (a10) secure aggregation: PySyft 0.2.9 FixedPrecisionTensor + AdditiveSharingTensor
# exercised at tests/data_centric/test_basic_syft_operations.py:388-454
# ----------------------------------------------------------------------------------------


def secagg_sum_torch(shares):
    """The server-side share aggregation as torch runs it (syft's AdditiveSharingTensor ``add``
    is a torch int64 add per share, wrapping): ``shares`` a list over clients of lists over
    parties of int64 tensors; returns the int64 sum and its fixed-point decode
    (``.float() / 10**3``).  Equal to ``secagg_sum`` / ``fix_prec_decode``."""
    from functools import reduce

    import torch as th

    s = reduce(th.add, [sh for client in shares for sh in client])
    return s, s.float() / 1000


def secagg_close_state_torch(share_msgs, base=10, precision_fractional=3):
    """Secure aggregation from share State bytes on the host, the way the syft path would: every
    party message parsed (``StatePB.ParseFromString`` + ``torch.tensor(contents_int64)`` per
    tensor, as ``unserialize_state_torch`` does for float32), the shares added as torch int64
    (wrapping), the sum decoded ``.float() / base**prec``.  ``share_msgs[c][s]`` = bytes.
    ``bench.py``'s cpu_baseline leg for ``resnet18-secagg-state``; ``tests/test_oracle.py`` checks
    it against ``secagg_sum`` / ``fix_prec_decode``."""
    import torch as th

    from pygrid_amd.state_schema import classes

    State = classes()["State"]
    acc = None
    for client in share_msgs:
        for pb in client:
            st = State()
            st.ParseFromString(pb)
            flat = th.cat([th.tensor(_state_tensor(stt).contents_data.contents_int64, dtype=th.int64).reshape(-1)
                           for stt in st.tensors])
            acc = flat if acc is None else acc + flat
    return acc, acc.float() / float(base ** precision_fractional)


def fix_prec_encode(x, base=10, precision_fractional=3):
    """``x.fix_prec()``: float32 ``x * base**prec`` (one rounding), truncated toward zero
    to int64 (syft 0.2.9 ``.long()``)."""
    scale = F32(base ** precision_fractional)
    y = (np.asarray(x, dtype=F32) * scale).astype(F32)
    return np.trunc(y).astype(I64)


def secagg_sum(shares):
    """Sum ``shares[N][S][P]`` int64 over clients and parties, wrapping mod 2**64
    (Z_2^64 addition is associative and commutative, so order is irrelevant)."""
    s = np.asarray(shares, dtype=I64).view(U64)
    acc = np.zeros(s.shape[-1], dtype=U64)
    with np.errstate(over="ignore"):
        for c in range(s.shape[0]):
            for p in range(s.shape[1]):
                acc += s[c, p]
    return acc.view(I64)


def fix_prec_decode(v, base=10, precision_fractional=3):
    """``.float_prec()``: float32(int64) rounded to nearest even, then IEEE float32
    division by float(base**prec)."""
    return (np.asarray(v, dtype=I64).astype(F32) / F32(base ** precision_fractional)).astype(F32)


def make_shares(enc, n_parties, rng_u64):
    """Split int64 ``enc[P]`` into ``n_parties`` additive shares over Z_2^64.  The first
    S-1 shares are the given uniform u64 words; the last one makes the wrap-sum exact."""
    enc = np.asarray(enc, dtype=I64).view(U64)
    sh = np.empty((n_parties, enc.shape[0]), dtype=U64)
    with np.errstate(over="ignore"):
        acc = np.zeros_like(enc)
        for p in range(n_parties - 1):
            sh[p] = rng_u64[p]
            acc += sh[p]
        sh[n_parties - 1] = enc - acc
    return sh.view(I64)


# ----------------------------------------------------------------------------------------
# Deterministic synthetic inputs, restated bit for bit from the
# on-device generator in pygrid_amd/csrc/pgh_kernels.hip.  Integer-only hashing plus one
# exact int->float conversion and one correctly rounded multiply, so CPU and GPU agree.
# ----------------------------------------------------------------------------------------

_M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
STREAM_DIFF, STREAM_CKPT, STREAM_SECRET, STREAM_SHARE = 0, 1, 2, 3
DIFF_SCALE = F32(2.6429e-7)    # sigma ~ 1e-2 for an Irwin-Hall(4 x u16) variate
CKPT_SCALE = F32(1.32145e-6)   # sigma ~ 5e-2


def splitmix64_scalar(x):
    z = (x + GOLDEN) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def splitmix64(x):
    """Vectorised splitmix64 finaliser over a uint64 array."""
    x = np.asarray(x, dtype=U64)
    with np.errstate(over="ignore"):
        z = x + U64(GOLDEN)
        z = (z ^ (z >> U64(30))) * U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> U64(27))) * U64(0x94D049BB133111EB)
        return z ^ (z >> U64(31))


def row_key(seed, stream, row):
    """Per-(stream, row) base counter; row = client index (or client*S + party)."""
    k = splitmix64_scalar((seed ^ (stream << 48)) & _M64)
    return splitmix64_scalar(k ^ ((row * 0xD1B54A32D192ED03) & _M64))


def synth_bits(seed, stream, row, idx):
    """u64 words for global param indices ``idx`` of one row."""
    base = U64(row_key(seed, stream, row))
    with np.errstate(over="ignore"):
        return splitmix64(base + np.asarray(idx, dtype=U64))


def bits_to_f32(bits, scale):
    """Irwin-Hall(4 x u16) - mean, exact int->float, times ``scale`` (one rounding)."""
    b = np.asarray(bits, dtype=U64)
    s = ((b & U64(0xFFFF)) + ((b >> U64(16)) & U64(0xFFFF))
         + ((b >> U64(32)) & U64(0xFFFF)) + ((b >> U64(48)) & U64(0xFFFF)))
    v = s.astype(I64) - I64(131070)
    return (v.astype(F32) * F32(scale)).astype(F32)


def synth_diff(seed, client, idx):
    return bits_to_f32(synth_bits(seed, STREAM_DIFF, client, idx), DIFF_SCALE)


def synth_diff_fast(seed, client, idx):
    """Generator kind 1 (``pgh_set_synth_kind(ctx, 1)``, config 4's data source): param g takes
    u16 number g & 3 of splitmix64(row_key + (g >> 2)), centred, times 2 * DIFF_SCALE."""
    g = np.asarray(idx, dtype=U64)
    base = U64(row_key(seed, STREAM_DIFF, client))
    with np.errstate(over="ignore"):
        h = splitmix64(base + (g >> U64(2)))
    u = (h >> (U64(16) * (g & U64(3)))) & U64(0xFFFF)
    return ((u.astype(I64) - I64(32768)).astype(F32) * (F32(2) * DIFF_SCALE)).astype(F32)


def synth_ckpt(seed, idx):
    return bits_to_f32(synth_bits(seed, STREAM_CKPT, 0, idx), CKPT_SCALE)


def synth_shares(seed, client, n_parties, idx, base=10, precision_fractional=3):
    """Shares ``[S][len(idx)]`` of client ``client``'s secret diff at params ``idx``."""
    x = bits_to_f32(synth_bits(seed, STREAM_SECRET, client, idx), DIFF_SCALE)
    enc = fix_prec_encode(x, base, precision_fractional)
    rnd = [synth_bits(seed, STREAM_SHARE, client * n_parties + p, idx) for p in range(n_parties - 1)]
    return make_shares(enc, n_parties, rnd)
