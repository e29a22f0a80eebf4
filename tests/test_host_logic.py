"""CPU: host-side logic of the drop-in -- readiness predicate, plan dispatch, the
_average_plan_diffs wiring, and the State codec (host-only C++ in libpygrid_hip)."""
import itertools
from functools import reduce
import types

import numpy as np
import pytest
import torch as th

from oracle import oracle as O
from pygrid_amd import ITERATIVE_MEAN, MEAN, WEIGHTED_MEAN, AggregationError, PlanNotAcceleratedError, StateParseError
from pygrid_amd import cycle, state
from pygrid_amd.state_schema import build_state, classes, parse_state, varint_encode

F = np.float32


# ---- readiness (cycle_manager.py:196-210) ------------------------------------------------------
def test_ready_to_average_matches_oracle_exhaustively():
    opts = [None, 0, 1, 3]
    for mn, mx, recv, end, now in itertools.product(opts, opts, [0, 1, 2, 3, 4], [None, 5], [4, 5, 6]):
        cfg = {}
        if mn is not None:
            cfg["min_diffs"] = mn
        if mx is not None:
            cfg["max_diffs"] = mx
        assert cycle.ready_to_average(cfg, recv, end, now) == O.ready_to_average(cfg, recv, end, now)


# ---- plan dispatch (SURVEY 8(b) dispatch rule) ---------------------------------------------------
def canonical_plan(avg, item, num):  # 01-Create-plan.ipynb:450-454
    new_avg = []
    for i, param in enumerate(avg):
        new_avg.append((avg[i] * num + item[i]) / (num + 1))
    return new_avg


def reassociated_plan(avg, item, num):  # mathematically equal, rounds differently
    return [avg[i] * (num / (num + 1)) + item[i] / (num + 1) for i in range(len(avg))]


def mean_plan(diffs):  # a hosted non-iterative plan that is the hard-coded mean, cycle_manager.py:284-288
    import torch as th
    from functools import reduce

    return [th.div(reduce(th.add, list(col)), len(diffs)) for col in zip(*diffs)]


def loop_mean_plan(diffs):  # the same arithmetic written as a loop: also accepted
    out = [d.clone() for d in diffs[0]]
    for d in diffs[1:]:
        out = [a + b for a, b in zip(out, d)]
    return [a / len(diffs) for a in out]


def stack_mean_plan(diffs):  # th.stack(...).mean(0): another summation order -- declined
    import torch as th

    return [th.stack(list(col)).mean(0) for col in zip(*diffs)]


def zero_start_plan(diffs):  # python sum() starts at int 0: 0 + (-0.0) = +0.0 -- declined
    return [sum(col) / len(diffs) for col in zip(*diffs)]


def reversed_plan(diffs):  # folds the clients last to first -- declined
    return mean_plan(diffs[::-1])


def test_non_iterative_plan_dispatch():
    """cycle_manager.py:270-271: a non-iterative hosted plan is accelerated only when it is the
    hard-coded mean bit for bit on the probes; every other plan stays with the node."""
    assert cycle.is_mean_plan(mean_plan) and cycle.is_mean_plan(loop_mean_plan)
    assert cycle.select_mode({"iterative_plan": False}, mean_plan) == MEAN
    for plan in (stack_mean_plan, zero_start_plan, reversed_plan, canonical_plan, lambda d: None):
        assert not cycle.is_mean_plan(plan), plan
        with pytest.raises(PlanNotAcceleratedError):
            cycle.select_mode({}, plan)


def test_select_mode_dispatch():
    assert cycle.select_mode({}, None) == MEAN
    assert cycle.select_mode({"iterative_plan": True}, None) == MEAN
    assert cycle.select_mode({"iterative_plan": True}, canonical_plan) == ITERATIVE_MEAN
    assert cycle.select_mode({}, None, weights=[1, 2]) == WEIGHTED_MEAN
    with pytest.raises(PlanNotAcceleratedError):
        cycle.select_mode({"iterative_plan": False}, canonical_plan)  # :270-271 user-defined plan
    with pytest.raises(PlanNotAcceleratedError):
        cycle.select_mode({"iterative_plan": True}, reassociated_plan)
    with pytest.raises(PlanNotAcceleratedError):
        cycle.select_mode({"iterative_plan": True}, lambda a, b, n: [x * 2 for x in a])
    with pytest.raises(PlanNotAcceleratedError):
        cycle.select_mode({"iterative_plan": True}, lambda a, b, n: 1 / 0)


def test_canonical_probe_uses_reference_calling_convention():
    seen = []

    def plan(avg, item, num):
        seen.append((type(avg), num.dtype, tuple(num.shape)))
        return canonical_plan(avg, item, num)

    assert cycle.is_canonical_iterative_plan(plan)
    assert seen[0] == (list, th.int64, (1,))  # avg_plan(list(diff_avg), diff, th.tensor([i + 1]))


# ---- _average_plan_diffs wiring (cycle_manager.py:234-245, :304-323) -----------------------------
class FakeWarehouse:
    def __init__(self, rows=None):
        self.rows = rows or []
        self.updates = 0

    def query(self, **kw):
        return [r for r in self.rows if all(getattr(r, k) == v for k, v in kw.items())]

    def count(self, **kw):
        return len(self.query(**kw))

    def update(self):
        self.updates += 1


def _fake_node(avg_plan_value=None, num_cycles=0):
    ns = types.SimpleNamespace
    model = ns(id=7)
    ckpt = ns(value=b"CKPT")
    saved = []
    model_manager = ns(get=lambda **kw: model, load=lambda **kw: ckpt, save=lambda mid, data: saved.append((mid, data)))
    plan_rec = ns(value=avg_plan_value) if avg_plan_value else None
    process_manager = ns(get_plan=lambda **kw: plan_rec)
    plan_manager = ns(deserialize_plan=lambda b: canonical_plan if b == b"CANON" else reassociated_plan)
    reports = [ns(cycle_id=3, is_completed=True, diff=b"D%d" % k) for k in range(3)]
    cyc = ns(id=3, fl_process_id=11, version="1.0", is_completed=False)
    created = []
    self_ = ns(_worker_cycles=FakeWarehouse(reports), _cycles=FakeWarehouse([cyc]),
               create=lambda pid, ver, length: created.append((pid, ver, length)))
    return model_manager, process_manager, plan_manager, self_, cyc, saved, created


class FakeAggregator:
    def __init__(self):
        self.calls = []

    def average_plan_diffs(self, server_config, checkpoint, diffs, avg_plan=None, weights=None, framing="fresh",
                           plan_key=None):  # CycleAggregator.average_plan_diffs's signature
        cycle.select_mode(server_config, avg_plan, plan_key=plan_key)  # same dispatch as the real one
        self.calls.append((checkpoint, list(diffs), avg_plan))
        self.framing = framing
        return b"NEW"


@pytest.fixture(autouse=True)
def _fresh_plan_cache(monkeypatch):
    """The tests below exercise the opt-in probe of non-iterative plans (PGH_MEAN_PLANS=probe);
    test_non_iterative_plans_are_declined_by_default covers the default."""
    monkeypatch.setenv("PGH_MEAN_PLANS", "probe")
    cycle._MODE_CACHE.clear()
    yield
    cycle._MODE_CACHE.clear()


def test_non_iterative_plans_are_declined_by_default(monkeypatch):
    """a probe cannot prove a user plan is the mean, so by default a non-iterative
    hosted plan runs in the node (cycle_manager.py:270-271) -- even one that IS the mean."""
    monkeypatch.delenv("PGH_MEAN_PLANS", raising=False)
    with pytest.raises(PlanNotAcceleratedError, match="opt in"):
        cycle.select_mode({}, mean_plan, plan_key=b"P0")
    assert cycle.select_mode({}, mean_plan, plan_key=b"P0", mean_plans="probe") == MEAN  # a separate verdict
    with pytest.raises(PlanNotAcceleratedError):
        cycle.cached_mode({}, b"P0")  # the default policy's verdict is cached too
    assert cycle.select_mode({"iterative_plan": True}, canonical_plan) == ITERATIVE_MEAN  # unaffected
    with pytest.raises(AggregationError):
        cycle.mean_plan_policy("always")


def conv_special_plan(diffs):
    """The mean, except that 4-D (conv) tensors are halved: passes 1-D probes only."""
    out = mean_plan(diffs)
    return [o / 2 if o.dim() == 4 else o for o in out]


def count_special_plan(diffs):
    """The mean, except above 50 clients (where it trims the first one)."""
    return mean_plan(diffs[1:] if len(diffs) > 50 else diffs)


def test_probe_uses_the_models_ranks_and_the_cycles_client_count():
    assert cycle.is_mean_plan(conv_special_plan)  # what the 1-D probes alone would accept
    assert not cycle.is_mean_plan(conv_special_plan, shapes=[(64, 3, 7, 7), (64,)], n_clients=4)
    assert cycle.is_mean_plan(count_special_plan, shapes=[(64, 3, 7, 7), (64,)], n_clients=10)
    assert not cycle.is_mean_plan(count_special_plan, shapes=[(64, 3, 7, 7), (64,)], n_clients=100)
    assert cycle.is_mean_plan(mean_plan, shapes=[(64, 3, 7, 7), (64,), (10, 512)], n_clients=100)


def test_plan_verdict_is_cached_by_plan_bytes():
    """A node's avg plan is fixed for its FL process: probe it once per plan (its bytes), not once
    per cycle; a declined plan stays declined; another plan (or the other iterative flag) is probed."""
    calls = []

    def mean_plan(diffs):
        calls.append(1)
        return [th.div(reduce(th.add, [d[j] for d in diffs]), len(diffs)) for j in range(len(diffs[0]))]

    assert cycle.select_mode({}, mean_plan, plan_key=b"P1") == cycle.MEAN
    n = len(calls)
    assert n > 0
    assert cycle.select_mode({}, mean_plan, plan_key=b"P1") == cycle.MEAN and len(calls) == n
    assert cycle.cached_mode({}, b"P1") == cycle.MEAN and cycle.cached_mode({}, b"P2") is None
    with pytest.raises(PlanNotAcceleratedError):
        cycle.select_mode({"iterative_plan": True}, mean_plan, plan_key=b"P1")  # not the iterative form
    with pytest.raises(PlanNotAcceleratedError):
        cycle.cached_mode({"iterative_plan": True}, b"P1")
    assert cycle.select_mode({}, mean_plan) == cycle.MEAN and len(calls) > n  # no key: probed


def test_wiring_skips_deserializing_a_probed_plan():
    mm, pm, plm, self_, cyc, saved, created = _fake_node(avg_plan_value=b"CANON")
    loads = []
    deser = plm.deserialize_plan
    plm.deserialize_plan = lambda b: loads.append(b) or deser(b)
    agg = FakeAggregator()
    fn = cycle.make_average_plan_diffs(agg, mm, pm, plm, original=None)
    fn(self_, {"iterative_plan": True}, cyc)
    fn(self_, {"iterative_plan": True}, cyc)
    assert loads == [b"CANON"] and len(agg.calls) == 2 and len(saved) == 2


def test_wiring_hardcoded_path():
    mm, pm, plm, self_, cyc, saved, created = _fake_node()
    agg = FakeAggregator()
    fn = cycle.make_average_plan_diffs(agg, mm, pm, plm, original=None)
    fn(self_, {"cycle_length": 60}, cyc)
    assert agg.calls == [(b"CKPT", [b"D0", b"D1", b"D2"], None)]
    assert saved == [(7, b"NEW")]
    assert cyc.is_completed and self_._cycles.updates == 1
    assert created == [(11, "1.0", 60)]  # num_cycles 0 -> next cycle created (:315-320)


def test_wiring_declines_to_reference_for_unknown_plans():
    mm, pm, plm, self_, cyc, saved, created = _fake_node(avg_plan_value=b"OTHER")
    ran = []
    fn = cycle.make_average_plan_diffs(FakeAggregator(), mm, pm, plm,
                                       original=lambda s, cfg, c: ran.append((cfg, c)))
    fn(self_, {"iterative_plan": True}, cyc)
    assert ran and saved == []


def test_wiring_iterative_plan_accelerated_and_fl_done():
    mm, pm, plm, self_, cyc, saved, created = _fake_node(avg_plan_value=b"CANON")
    self_._cycles.rows[0].is_completed = True  # count(is_completed=True) -> 1 == num_cycles
    agg = FakeAggregator()
    fn = cycle.make_average_plan_diffs(agg, mm, pm, plm, original=None)
    fn(self_, {"iterative_plan": True, "num_cycles": 1}, cyc)
    assert agg.calls[0][2] is canonical_plan and saved == [(7, b"NEW")] and created == []


def _state_with(kinds):
    """State bytes via google.protobuf with one tensor per entry of ``kinds``: "f32", "f64", "i64",
    "bin" (TorchTensor.contents_bin), "f32-as-param"."""
    st = classes()["State"]()
    for k, kind in enumerate(kinds):
        st.placeholders.add().id.id_int = 10 + k
        stt = st.tensors.add()
        tt = stt.torch_param.tensor if kind == "f32-as-param" else stt.torch_tensor
        tt.id.id_int = 10 + k
        tt.serializer = 4
        if kind == "bin":
            tt.contents_bin = b"\x80\x02torch-blob"
            continue
        tt.contents_data.shape.dims.extend([3])
        if kind in ("f32", "f32-as-param"):
            tt.contents_data.dtype = "float32"
            tt.contents_data.contents_float32.extend([1.0, -2.0, 0.5])
        elif kind == "f64":
            tt.contents_data.dtype = "float64"
            tt.contents_data.contents_float64.extend([1.0, -2.0, 0.5])
        else:
            tt.contents_data.dtype = "int64"
            tt.contents_data.contents_int64.extend([1, -2, 5])
    return st.SerializeToString()


@pytest.mark.parametrize("kinds,bad", [(["f32", "f32-as-param"], []), (["f32", "f64"], [1]), (["i64", "f32"], [0]),
                                       (["bin"], [0]), (["f64", "i64", "bin"], [0, 1, 2])])
def test_non_float32_tensors_found_from_framing(kinds, bad):
    from pygrid_amd import state_schema

    pb = _state_with(kinds)
    assert state_schema.non_float32_tensors(pb) == bad
    if bad:  # the walker the engine uses refuses them
        with pytest.raises(StateParseError):
            state.scan(pb)
    with pytest.raises(ValueError):
        state_schema.non_float32_tensors(pb[:-2])  # cut-off bytes are malformed, not "another dtype"


class _NoEngine:
    """Engine stand-in for dispatch tests that must decline before any engine call."""
    ckpt_owner = None

    def __getattr__(self, name):
        raise AssertionError(f"engine.{name} touched")


def test_non_float32_checkpoint_declined_before_the_engine():
    from pygrid_amd import ModelNotAcceleratedError

    agg = cycle.CycleAggregator(engine=_NoEngine())
    with pytest.raises(ModelNotAcceleratedError):
        agg.average_plan_diffs({}, _state_with(["f32", "f64"]), [_state_with(["f32", "f32"])])
    with pytest.raises(StateParseError):  # malformed bytes still raise the parse error
        agg.average_plan_diffs({}, _state_with(["f32", "f32"])[:-3], [_state_with(["f32", "f32"])])


def test_wiring_declines_non_float32_models_to_the_reference():
    from pygrid_amd import ModelNotAcceleratedError

    class Refusing(FakeAggregator):
        def average_plan_diffs(self, *a, **k):
            raise ModelNotAcceleratedError("float64 model")

    mm, pm, plm, self_, cyc, saved, created = _fake_node()
    ran = []
    fn = cycle.make_average_plan_diffs(Refusing(), mm, pm, plm, original=lambda s, cfg, c: ran.append(c))
    fn(self_, {}, cyc)
    assert ran == [cyc] and saved == [] and not cyc.is_completed


# ---- State codec (host-only C++) -----------------------------------------------------------------
SHAPES = [(392, 784), (392,), (10, 392), (10,)]


def _tensors(seed=0):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(s).astype(F) for s in SHAPES]


@pytest.mark.parametrize("as_param", [False, True])
def test_state_scan_and_unserialize(as_param):
    ts = _tensors()
    pb = build_state(ts, as_param=as_param)
    spans = state.scan(pb)
    assert [c for _, c in spans] == [t.size for t in ts]
    for got, want in zip(state.unserialize_model_params(pb, SHAPES), ts):
        assert np.array_equal(got, want)


def test_state_patch_roundtrips_through_google_protobuf():
    ts = _tensors(1)
    pb = build_state(ts, ids=[11, 22, 33, 44])
    new = np.arange(sum(t.size for t in ts), dtype=F) * F(0.5)
    out = state.serialize_model_params(pb, new)
    assert len(out) == len(pb)
    parsed = parse_state(out)
    off = 0
    for t, p in zip(ts, parsed):
        assert p.shape == t.shape
        assert np.array_equal(p.reshape(-1), new[off:off + t.size])
        off += t.size
    st = classes()["State"]()
    st.ParseFromString(out)  # ids / tags / shapes untouched
    assert [ph.id.id_int for ph in st.placeholders] == [11, 22, 33, 44]


def test_state_scan_skips_unknown_fields_and_zero_size():
    cls = classes()
    st = cls["State"]()
    st.ParseFromString(build_state([np.zeros((0,), F), np.ones(3, F)]))
    t = st.tensors[1].torch_tensor
    t.description = "x" * 300  # a long unknown-to-the-walker string field
    t.tags.extend(["a", "b"])
    pb = st.SerializeToString()
    assert [c for _, c in state.scan(pb)] == [0, 3]
    assert np.array_equal(state.flat_params(pb), np.ones(3, F))


@pytest.mark.parametrize("mutate", ["truncate", "dtype", "shape"])
def test_state_errors(mutate):
    cls = classes()
    pb = build_state([np.ones((2, 3), F)])
    if mutate == "truncate":
        pb = pb[:-3]
    else:
        st = cls["State"]()
        st.ParseFromString(pb)
        td = st.tensors[0].torch_tensor.contents_data
        if mutate == "dtype":
            td.dtype = "float64"
        else:
            del td.shape.dims[:]
            td.shape.dims.extend([4, 2])
        pb = st.SerializeToString()
    with pytest.raises(StateParseError):
        state.scan(pb)


def test_state_patch_rejects_wrong_value_count():
    pb = build_state([np.ones(5, F)])
    with pytest.raises(StateParseError):
        state.serialize_model_params(pb, np.zeros(4, F))


def test_build_state_fast_is_byte_identical():
    from pygrid_amd.state_schema import build_state_fast

    for ts in (_tensors(3), [np.zeros((0,), F), np.ones((2, 3), F), np.array([1.5], F)]):
        assert build_state_fast(ts) == build_state(ts)
        assert build_state_fast(ts, ids=[7, 0, 99, 5][:len(ts)]) == build_state(ts, ids=[7, 0, 99, 5][:len(ts)])


# ---- secure-aggregation shares as State bytes (packed-varint int64, host-side checks) -----------
def _every_length(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    sh = rng.integers(0, 64, n).astype(np.uint64)
    v = (v.view(np.uint64) >> sh).view(np.int64)  # 1..10-byte varints
    v[: min(n, 4)] = [0, -1, -2**63, 2**63 - 1][: min(n, 4)]
    return v


def test_share_state_builders_agree_with_google_protobuf():
    from pygrid_amd.state_schema import build_state_i64, build_state_i64_fast, parse_state_i64

    ts = [_every_length(n, n).reshape(s) for n, s in ((12, (3, 4)), (0, (0,)), (1000, (10, 100)), (1, (1,)))]
    fast = build_state_i64_fast(ts)
    assert fast == build_state_i64(ts)
    for got, want in zip(parse_state_i64(fast), ts):
        assert np.array_equal(got, want)
    spans = state.scan_shares(fast)
    assert [c for _, _, c in spans] == [t.size for t in ts]
    assert all(nb == len(varint_encode(t)) for (_, nb, _), t in zip(spans, ts))


def test_varint_encode_matches_protobuf_varints():
    from pygrid_amd.state_schema import _varint

    v = _every_length(3000, 7)
    assert varint_encode(v) == b"".join(_varint(int(x) & (2**64 - 1)) for x in v)


@pytest.mark.parametrize("n", [1, 9, 63, 64, 65, 127, 640, 4097])
def test_share_scan_counts_and_overlong_fuzz(n):
    """The walker's per-payload varint count and 10-byte limit against a byte-by-byte Python
    reference, on random payload bytes around every 64-byte block edge."""
    from pygrid_amd.state_schema import _field, _varint

    rng = np.random.default_rng(n)
    for trial in range(40):
        p = rng.integers(0, 256, n, dtype=np.uint8)
        cont_rate = rng.choice([0.3, 0.7, 0.9, 0.97])
        p = np.where(rng.random(n) < cont_rate, p | 0x80, p & 0x7F).astype(np.uint8)
        p[-1] &= 0x7F if trial % 3 else 0xFF
        payload = p.tobytes()
        run, ok, count = 0, True, 0
        for b in payload:
            if b & 0x80:
                run += 1
                ok = ok and run <= 9
            else:
                count += 1
                run = 0
        ok = ok and run == 0
        td = _field(2, 2, b"int64") + _field(10, 2, payload)
        msg = _field(2, 2, _field(1, 2, _field(4, 2, td)))
        if ok:
            assert state.scan_shares(msg) == [(len(msg) - n, n, count)]
        else:
            with pytest.raises(StateParseError):
                state.scan_shares(msg)


def test_share_scan_rejects_float_payload_and_f32_scan_rejects_shares():
    from pygrid_amd.state_schema import build_state_i64_fast

    with pytest.raises(StateParseError):
        state.scan_shares(build_state([np.ones(3, F)]))
    with pytest.raises(StateParseError):
        state.scan(build_state_i64_fast([np.arange(3, dtype=np.int64)]))


# ---- Engine plumbing: a failing call's message survives another thread's call ---------------------
def test_serialized_keeps_error_message_per_thread():
    import ctypes as C
    import threading

    from pygrid_amd.engine import _Serialized

    class FakeLib:
        """Stands in for libpygrid_hip: one error string per context, as pgh_last_error has."""
        err = b""

        def pgh_fail(self, ctx, tag):
            FakeLib.err = tag
            return -3

        def pgh_ok(self, ctx):
            return 0

        def pgh_last_error(self, ctx):
            return FakeLib.err

    lib = _Serialized(FakeLib(), threading.RLock())
    h = C.c_void_p(1)
    assert lib.pgh_fail(h, b"first") == -3
    t = threading.Thread(target=lambda: lib.pgh_fail(h, b"other thread"))
    t.start()
    t.join()
    assert lib.pgh_ok(h) == 0
    assert lib.errors.msg == "first"
