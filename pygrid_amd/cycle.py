"""Host-side mirror of PyGrid Node's cycle-close path, with the arithmetic on the GPU.

Reference: ``CycleManager.complete_cycle`` / ``_average_plan_diffs``,
``apps/node/src/app/main/model_centric/cycles/cycle_manager.py:180-323``.

* ``ready_to_average`` restates the readiness predicate (``:196-210``).
* ``select_mode`` is the dispatch rule: no hosted plan -> hard-coded mean
  (``:273-288``); hosted plan + ``iterative_plan`` whose behaviour is the canonical
  ``(avg * num + item) / (num + 1)`` (``01-Create-plan.ipynb:450-454``) -> iterative mean
  (``:266-269``); a hosted non-iterative plan (``:270-271``) is user code the node runs itself
  unless the operator opts in (``mean_plans="probe"`` / ``PGH_MEAN_PLANS=probe``): then a plan
  whose output is bit-identical to ``reduce(th.add) / N`` on probe inputs -- including tensors of
  the real model's ranks and layer count and the cycle's client count -- runs as the hard-coded
  mean.  A probe cannot PROVE that a plan is the mean (a plan may special-case shapes or counts
  the probe did not try), which is why it is opt-in.  Anything else raises
  ``PlanNotAcceleratedError`` so the node keeps running the reference code for it.
* ``CycleAggregator.average_plan_diffs`` replaces the slice ``:240-303``: checkpoint bytes +
  diff bytes in, new checkpoint bytes out.  DB reads/writes and cycle bookkeeping stay with
  the caller (``make_average_plan_diffs`` shows the wiring).
"""
from __future__ import annotations

import contextlib
import logging
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import state as state_codec
from .engine import ITERATIVE_MEAN, MEAN, WEIGHTED_MEAN, F32, I64, Engine
from .exceptions import AggregationError, ModelNotAcceleratedError, PlanNotAcceleratedError, StateParseError


def ready_to_average(server_config: dict, received_diffs: int, cycle_end=None, now=None) -> bool:
    """``cycle_manager.py:196-210``."""
    min_diffs = server_config.get("min_diffs", None)
    max_diffs = server_config.get("max_diffs", None)
    hit_diffs_limit = received_diffs >= max_diffs if max_diffs is not None else False
    hit_time_limit = now >= cycle_end if cycle_end is not None else False
    no_limits = max_diffs is None and cycle_end is None
    has_enough_diffs = received_diffs >= min_diffs if min_diffs is not None else True
    return bool(has_enough_diffs and (no_limits or hit_diffs_limit or hit_time_limit))


def _canonical_step(avg, item, k):
    f = np.float32
    return ((avg.astype(f) * f(k)).astype(f) + item.astype(f)).astype(f) / f(k + 1)


def is_canonical_iterative_plan(avg_plan: Callable) -> bool:
    """Run the hosted plan once on small probe tensors (the way ``cycle_manager.py:269`` calls
    it: ``avg_plan(list(avg), diff, th.tensor([k]))``) and compare bit for bit with the
    canonical step.  Probes cover several k, signs, magnitudes and a subnormal."""
    import torch as th

    rng = np.random.default_rng(7)
    probe_avg = [rng.standard_normal(17).astype(np.float32) * 1e-2,
                 np.array([1.0, -2.5, 3.0e-39, 7.0], np.float32)]
    probe_item = [rng.standard_normal(17).astype(np.float32),
                  np.array([55.0, 0.125, -1.0e-38, 3.3], np.float32)]
    for k in (1, 2, 7, 1000):
        try:
            res = avg_plan([th.from_numpy(a.copy()) for a in probe_avg],
                           [th.from_numpy(b.copy()) for b in probe_item], th.tensor([k]))
        except Exception as e:  # noqa: BLE001 -- any failure means "not the canonical plan"
            logging.info("avg plan probe failed: %s", e)
            return False
        res = list(res)
        if len(res) != len(probe_avg):
            return False
        for got, a, b in zip(res, probe_avg, probe_item):
            got = np.asarray(got.detach().cpu().numpy() if hasattr(got, "detach") else got, dtype=np.float32)
            want = _canonical_step(a, b, k)
            if got.shape != want.shape or not np.array_equal(got.view(np.uint32), want.view(np.uint32)):
                return False
    return True


def _mean_probes(shapes=None, n_clients=None):
    """Probe inputs for a non-iterative plan: several client counts, values of mixed magnitude (so a
    re-associated or pairwise sum rounds differently), exact cancellations, signed zeros,
    subnormals and an overflow to inf.  With the real model's ``shapes``: also diffs of that many
    tensors of the same ranks (every dimension clipped to 3, so the probe stays small), at 1, 2 and
    3 clients and at the cycle's own client count ``n_clients``."""
    rng = np.random.default_rng(11)
    probes = []
    for n in (1, 2, 3, 7, 33):
        diffs = []
        for c in range(n):
            mixed = (rng.standard_normal(97) * 10.0 ** rng.integers(-4, 5, 97)).astype(np.float32)
            special = np.array([-0.0, 3.0e-39 * (c + 1), 1e8 if c % 2 else -1e8, 1.0, 3.0e38, -1e-45],
                               np.float32)
            diffs.append([mixed, special])
        probes.append(diffs)
    if shapes:
        small = [tuple(min(int(d), 3) for d in s) for s in shapes]
        counts = sorted({1, 2, 3} | ({int(n_clients)} if n_clients and n_clients <= 4096 else set()))
        for n in counts:
            probes.append([[(rng.standard_normal(s) * 10.0 ** rng.integers(-4, 5, s)).astype(np.float32)
                            for s in small] for _ in range(n)])
    return probes


def _reference_mean(diffs):
    """cycle_manager.py:276-288 on the probe: left fold with th.add, then th.div by the python int N."""
    import torch as th
    from functools import reduce

    cols = [[th.from_numpy(d[j].copy()) for d in diffs] for j in range(len(diffs[0]))]
    return [th.div(reduce(th.add, col), len(diffs)).numpy() for col in cols]


def is_mean_plan(avg_plan: Callable, shapes=None, n_clients=None) -> bool:
    """A hosted NON-iterative avg plan (called as ``avg_plan(diffs)``, cycle_manager.py:270-271) is
    user code; it maps to the hard-coded mean only if, on every probe, its output equals
    ``reduce(th.add) / N`` (:286-288) bit for bit (NaN-free probes; signed zeros, subnormals and
    infinities compared exactly).  Anything else -- another order of summation, a mean through a
    pairwise reduction, a weighting, an exception -- leaves the plan to the node.  Passing the
    model's ``shapes`` and the cycle's ``n_clients`` adds probes of that layer count, those ranks
    and that client count."""
    import torch as th

    for diffs in _mean_probes(shapes, n_clients):
        try:
            res = avg_plan([[th.from_numpy(t.copy()) for t in d] for d in diffs])
            res = list(res)
        except Exception as e:  # noqa: BLE001 -- any failure means "not the plain mean"
            logging.info("avg plan probe failed: %s", e)
            return False
        want = _reference_mean(diffs)
        if len(res) != len(want):
            return False
        for got, w in zip(res, want):
            if not hasattr(got, "detach") or got.dtype != th.float32:
                return False
            got = got.detach().cpu().numpy()
            if got.shape != w.shape or not np.array_equal(got.view(np.uint32), w.view(np.uint32)):
                return False
    return True


_MODE_CACHE: dict = {}  # (sha256 of the plan's bytes, iterative flag, mean-plan policy) -> mode, or the decline message
_MODE_CACHE_MAX = 256


def mean_plan_policy(mean_plans: Optional[str] = None) -> str:
    """"decline" (default: a non-iterative hosted plan runs in the node, as in the reference) or
    "probe" (opt-in: a plan that probes bit-identical to the hard-coded mean runs as MEAN)."""
    import os

    got = mean_plans or os.environ.get("PGH_MEAN_PLANS", "decline")
    if got not in ("decline", "probe"):
        raise AggregationError(f"mean_plans must be 'decline' or 'probe', not {got!r}")
    return got


def _plan_cache_key(server_config: dict, plan_key, mean_plans: Optional[str] = None) -> Optional[tuple]:
    if plan_key is None:
        return None
    import hashlib

    raw = plan_key if isinstance(plan_key, (bytes, bytearray, memoryview)) else str(plan_key).encode()
    iterative = bool(server_config.get("iterative_plan", False))
    return hashlib.sha256(raw).digest(), iterative, None if iterative else mean_plan_policy(mean_plans)


def cached_mode(server_config: dict, plan_key, mean_plans: Optional[str] = None) -> Optional[int]:
    """The dispatch decision already made for this hosted plan (its serialized bytes), or None.
    Raises PlanNotAcceleratedError again for a plan that was declined."""
    key = _plan_cache_key(server_config, plan_key, mean_plans)
    if key is None or key not in _MODE_CACHE:
        return None
    got = _MODE_CACHE[key]
    if isinstance(got, str):
        raise PlanNotAcceleratedError(got)
    return got


def select_mode(server_config: dict, avg_plan: Optional[Callable] = None, weights=None, plan_key=None,
                mean_plans: Optional[str] = None, shapes=None, n_clients=None) -> int:
    """Dispatch rule (module docstring).  ``plan_key`` -- the hosted plan's serialized bytes
    (``avg_plan_rec.value``, cycle_manager.py:256) -- caches the probe's verdict: a node's avg plan
    is fixed for its FL process, and probing a non-iterative plan costs ~2.6 ms of torch calls,
    five times an MNIST close.  ``mean_plans`` (or ``PGH_MEAN_PLANS``): see ``mean_plan_policy``;
    ``shapes`` / ``n_clients``: the model's tensor shapes and the cycle's client count, probed too
    (the verdict is cached for the plan's bytes, i.e. from the first cycle's shapes and count)."""
    if weights is not None:
        return WEIGHTED_MEAN
    if avg_plan is None:
        return MEAN  # "Fallback to simple hardcoded avg plan", cycle_manager.py:274
    key = _plan_cache_key(server_config, plan_key, mean_plans)
    if key is not None:
        got = cached_mode(server_config, plan_key, mean_plans)
        if got is not None:
            return got
        try:
            mode = _probe_mode(server_config, avg_plan, mean_plans, shapes, n_clients)
        except PlanNotAcceleratedError as e:
            _remember(key, str(e))
            raise
        _remember(key, mode)
        return mode
    return _probe_mode(server_config, avg_plan, mean_plans, shapes, n_clients)


def _remember(key, verdict):
    if len(_MODE_CACHE) >= _MODE_CACHE_MAX:
        _MODE_CACHE.pop(next(iter(_MODE_CACHE)))
    _MODE_CACHE[key] = verdict


def _probe_mode(server_config: dict, avg_plan: Callable, mean_plans=None, shapes=None, n_clients=None) -> int:
    if not server_config.get("iterative_plan", False):
        if mean_plan_policy(mean_plans) != "probe":
            raise PlanNotAcceleratedError("non-iterative hosted avg plan: user code, run by the node "
                                          "(cycle_manager.py:270-271; opt in with mean_plans='probe')")
        if callable(shapes):
            shapes = shapes()
        if is_mean_plan(avg_plan, shapes, n_clients):  # :270-271 with a plan that IS the hard-coded mean
            return MEAN
        raise PlanNotAcceleratedError("non-iterative hosted avg plan is not reduce(th.add) / N (cycle_manager.py:270-271)")
    if not is_canonical_iterative_plan(avg_plan):
        raise PlanNotAcceleratedError("iterative avg plan is not (avg * num + item) / (num + 1)")
    return ITERATIVE_MEAN


def _decline_non_float32(pb: bytes, what: str):
    """After the State walker refused ``pb``: well-formed bytes holding non-float32 tensors are a
    model the engine does not implement (``ModelNotAcceleratedError``: the node averages it with
    its own code, cycle_manager.py:240-303, torch type promotion included); anything else is
    malformed and the caller re-raises the parse error."""
    from . import state_schema

    try:
        bad = state_schema.non_float32_tensors(pb)
    except ValueError:
        return
    if bad:
        raise ModelNotAcceleratedError(f"{what} holds non-float32 tensors {bad[:8]} (the engine is fp32-only)")


def _shapes_or_none(pb: bytes):
    from . import state_schema

    try:
        return state_schema.tensor_shapes(pb)
    except Exception:  # noqa: BLE001 -- malformed bytes: the engine's own parse reports them
        return None


class CycleAggregator:
    """Owns one Engine across cycles; the slab is re-used while it fits.  ``devices=[0, ..., 7]``
    gives the node's single process every GPU of the node (``pgh_create_group``: parameter shards,
    each GPU's slice of every diff over its own PCIe link, bit-identical results)."""

    def __init__(self, engine: Optional[Engine] = None, device: int = 0, devices: Optional[Sequence[int]] = None,
                 mean_plans: Optional[str] = None):
        if engine is None:
            engine = Engine(devices=devices) if devices is not None else Engine(device)
        self.engine = engine
        self.mean_plans = mean_plan_policy(mean_plans)  # non-iterative hosted plans: "decline" | "probe"
        self._numel: tuple = ()
        self._cap = 0
        self._dtype = None
        self._parties = 0
        self._resident = None  # the checkpoint bytes object whose params are resident in HBM

    def _prepare(self, numel: Sequence[int], n: int, dtype: int = F32, parties: int = 1):
        # the engine's own state is the truth: another user of the same engine may have changed it
        eng = self.engine
        numel = tuple(int(x) for x in numel)
        if numel != tuple(eng.numel) or numel != self._numel:  # (a new aggregator always lays out)
            eng.set_layout(numel)
            self._resident = None
        if n > eng.max_clients or dtype != eng.dtype or (dtype != F32 and parties != eng.parties):
            eng.reserve(max(n, 1), dtype, parties)
            self._resident = None
        else:
            eng.reset()
        if hasattr(eng, "set_ingest_ranges"):
            eng.set_ingest_ranges(False)  # every diff at once: whole-message copies keep the PCIe rate
        self._numel, self._cap, self._dtype, self._parties = numel, eng.max_clients, dtype, parties

    # ---- bytes in / bytes out: the replaceable slice cycle_manager.py:240-303 -------------------
    def average_plan_diffs(self, server_config: dict, checkpoint: bytes, diffs: Sequence[bytes],
                           avg_plan: Optional[Callable] = None, weights=None, framing: str = "fresh",
                           plan_key=None) -> bytes:
        """New checkpoint bytes.  ``framing="fresh"`` (default) frames them like the reference's
        ``serialize_model_params`` (model_manager.py:82-90: new placeholder / tensor ids, plain
        torch_tensor entries, no tags); ``"template"`` keeps the old checkpoint's framing byte for
        byte and only replaces the payloads (ids and tags survive).  ``plan_key``: the hosted
        plan's serialized bytes, to probe it once per plan instead of once per cycle."""
        if framing not in ("fresh", "template"):
            raise AggregationError(f"unknown checkpoint framing {framing!r}")
        if len(diffs) == 0:
            raise AggregationError("no diffs to average")
        mode = select_mode(server_config, avg_plan, weights, plan_key=plan_key, mean_plans=self.mean_plans,
                           shapes=lambda: _shapes_or_none(checkpoint), n_clients=len(diffs))
        try:
            numel = state_codec.tensor_numels(checkpoint)  # :240
        except StateParseError:
            _decline_non_float32(checkpoint, "the checkpoint")
            raise
        self._prepare(numel, len(diffs))
        if checkpoint is not self._resident or self.engine.ckpt_owner is not self:
            self.engine.ckpt_upload_state(checkpoint)  # else: the last cycle's output is still in HBM
        for i, d in enumerate(diffs):  # :247-250
            try:
                self.engine.ingest_state(i, d)
            except StateParseError:
                _decline_non_float32(d, f"diff {i}")
                raise
        if mode == WEIGHTED_MEAN:
            self.engine.set_weights(weights)
        # From the fold on, HBM holds the NEW checkpoint: until its bytes exist, nobody may take the
        # resident copy for `checkpoint` (a retry after a failed patch would fold twice).
        self.engine.ckpt_owner = None
        self._resident = None
        self.engine.fedavg_resident(mode)  # :252-296
        new = (state_codec.fresh_checkpoint(self.engine, checkpoint) if framing == "fresh"  # :303
               else self.engine.ckpt_patch_state(checkpoint))
        self.engine.ckpt_owner = self
        self.engine.ckpt_bytes = new  # the bytes whose params are resident (IncrementalCycle reuses them)
        self._resident = new
        return new

    # ---- tensor lists in / out (what the reference holds after unserialize) ---------------------
    def average_params(self, server_config: dict, model_params: Sequence[np.ndarray],
                       diffs: Sequence[Sequence[np.ndarray]], avg_plan: Optional[Callable] = None,
                       weights=None) -> List[np.ndarray]:
        if len(diffs) == 0:
            raise AggregationError("no diffs to average")
        shapes = [np.shape(p) for p in model_params]
        mode = select_mode(server_config, avg_plan, weights, mean_plans=self.mean_plans, shapes=shapes,
                           n_clients=len(diffs))
        numel = [int(np.prod(s)) for s in shapes]
        self._prepare(numel, len(diffs))
        for i, d in enumerate(diffs):
            if len(d) != len(numel):
                raise AggregationError(f"diff {i} has {len(d)} tensors, model has {len(numel)}")
            self.engine.ingest(i, np.concatenate([np.asarray(t, np.float32).reshape(-1) for t in d]))
        if mode == WEIGHTED_MEAN:
            self.engine.set_weights(weights)
        flat = np.concatenate([np.asarray(p, np.float32).reshape(-1) for p in model_params])
        self._resident = None  # the host-buffer fold overwrites the resident checkpoint
        out = self.engine.fedavg(mode, flat)
        res, off = [], 0
        for s, n in zip(shapes, numel):
            res.append(out[off:off + n].reshape(s))
            off += n
        return res

    # ---- secure aggregation (PySyft share add + get + float_prec) ------------------------------
    def secure_aggregate(self, shares: np.ndarray, base: int = 10, precision_fractional: int = 3):
        """shares: int64 [clients][parties][P].  Returns (int64 wrap-sum [P], float32 decoded [P])."""
        sh = np.ascontiguousarray(shares, dtype=np.int64)
        if sh.ndim != 3:
            raise AggregationError("shares must be [clients][parties][P]")
        n, s, p = sh.shape
        self._prepare([p], n, I64, s)
        self._resident = None
        for c in range(n):
            self.engine.ingest(c, sh[c])
        return self.engine.secagg(base, precision_fractional)


    def secure_aggregate_states(self, numel: Sequence[int], share_msgs: Sequence[Sequence[bytes]],
                                base: int = 10, precision_fractional: int = 3):
        """Secure aggregation from the wire: ``share_msgs[client][party]`` = State bytes of that
        party's int64 shares (packed-varint ``contents_int64``, tensors in ``numel`` order).  The
        payloads are decoded on the GPU; returns (int64 wrap-sum [P], float32 decoded [P])."""
        if len(share_msgs) == 0:
            raise AggregationError("no shares to aggregate")
        parties = len(share_msgs[0])
        self._prepare(numel, len(share_msgs), I64, parties)
        self._resident = None
        for c, msgs in enumerate(share_msgs):
            if len(msgs) != parties:
                raise AggregationError(f"client {c} sent {len(msgs)} share messages, client 0 sent {parties}")
            self.engine.ingest_state_shares(c, msgs)
        return self.engine.secagg(base, precision_fractional)


def _probed_plan(*_a, **_k):  # stands in for a hosted plan whose verdict is cached (never called)
    raise AssertionError("a cached plan verdict was not used")


def make_average_plan_diffs(aggregator: CycleAggregator, model_manager, process_manager, plan_manager,
                            original: Callable, gate: Optional[Callable] = None, framing: str = "fresh") -> Callable:
    """Build a drop-in ``CycleManager._average_plan_diffs(self, server_config, cycle)``.

    DB I/O mirrors ``cycle_manager.py:234-245`` and ``:304-323``; the arithmetic slice
    ``:240-303`` goes to the engine.  A user-defined (non-iterative) avg plan, which the engine
    does not implement, runs the reference's ``original`` method unchanged.
    Engine errors are NOT retried on the CPU: they raise ``PyGridError`` subclasses, which
    ``tasks.complete_cycle`` logs (``tasks/cycle.py:28-37``), like any failed cycle close.
    ``gate()``: a context manager held while the completed rows and their diffs are read (the
    node's report gate: a re-report's DB write lands wholly before or after that read).
    ``framing``: the new checkpoint's framing (``CycleAggregator.average_plan_diffs``).
    """

    def _average_plan_diffs(self, server_config: dict, cycle):
        _model = model_manager.get(fl_process_id=cycle.fl_process_id)
        _checkpoint = model_manager.load(model_id=_model.id)
        with gate() if gate is not None else contextlib.nullcontext():
            reports = self._worker_cycles.query(cycle_id=cycle.id, is_completed=True)
            diffs = [r.diff for r in reports]  # what :247-250 reads, at the query
        try:
            avg_plan, plan_key = hosted_plan(server_config, cycle, process_manager, plan_manager,
                                             getattr(aggregator, "mean_plans", None))
            new_ckpt = aggregator.average_plan_diffs(server_config, _checkpoint.value, diffs, avg_plan,
                                                     plan_key=plan_key, framing=framing)
        except PlanNotAcceleratedError as e:
            logging.info("engine declined (%s): running the reference averaging", e)
            return original(self, server_config, cycle)
        finish_cycle(self, server_config, cycle, model_manager, _model.id, new_ckpt)

    return _average_plan_diffs


def hosted_plan(server_config: dict, cycle, process_manager, plan_manager, mean_plans=None):
    """(avg_plan, plan_key) as ``cycle_manager.py:252-258`` looks them up; a plan whose verdict is
    cached needs no deserializing (only its verdict is used)."""
    avg_plan_rec = process_manager.get_plan(fl_process_id=cycle.fl_process_id, is_avg_plan=True)
    if not (avg_plan_rec and avg_plan_rec.value):
        return None, None
    plan_key = avg_plan_rec.value
    if cached_mode(server_config, plan_key, mean_plans) is None:
        return plan_manager.deserialize_plan(avg_plan_rec.value), plan_key
    return _probed_plan, plan_key


def finish_cycle(cm, server_config: dict, cycle, model_manager, model_id, new_ckpt: bytes):
    """``cycle_manager.py:303-323``: save the new checkpoint, complete the cycle, open the next."""
    model_manager.save(model_id, new_ckpt)
    cycle.is_completed = True
    cm._cycles.update()
    completed = cm._cycles.count(fl_process_id=cycle.fl_process_id, is_completed=True)
    max_cycles = server_config.get("num_cycles", 0)
    if completed < max_cycles or max_cycles == 0:
        cm.create(cycle.fl_process_id, cycle.version, server_config.get("cycle_length"))
    else:
        logging.info("FL is done!")
