"""CPU, world_size 2 (gloo): the multi-GPU path's host logic.

Each rank owns the parameter shard ``shard_bounds(P, world, rank)`` for every client, folds it
(here the oracle stands in for the rank's GPU: it is the checker, the sharding and the
collective are the code under test), and ``gather_flat`` assembles the new checkpoint with one
all-gather.  The result must equal the unsharded fold bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pygrid_amd.sharding import (OverlappedGather, OverlappedReduceScatter, all_shard_bounds, client_bounds,
                                 gather_flat, shard_bounds)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, P, N, mode, q):
    from oracle import coracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(1234)  # every rank sees the same clients
        d = (rng.standard_normal((N, P)) * 1e-2).astype(np.float32)
        c = rng.standard_normal(P).astype(np.float32)
        lo, hi = shard_bounds(P, world, rank)
        if hi > lo:
            w = np.linspace(0.5, 2.0, N).astype(np.float32)
            part = coracle.fedavg(mode, np.ascontiguousarray(d[:, lo:hi]), c[lo:hi], w if mode == 2 else None)
        else:
            part = np.empty(0, np.float32)
        full = gather_flat(torch.from_numpy(part), P, world, rank)
        # chunked fold + overlapped all-gather (what bench.py runs at N > 1)
        og = OverlappedGather(P, world, rank, chunks=3, device="cpu", tail=2)

        def fold_range(off, n, stream):
            w = np.linspace(0.5, 2.0, N).astype(np.float32)
            og.local[off:off + n] = torch.from_numpy(coracle.fedavg(
                mode, np.ascontiguousarray(d[:, lo + off:lo + off + n]), c[lo + off:lo + off + n],
                w if mode == 2 else None))
        og.run(fold_range)
        full2 = og.assemble()
        assert torch.equal(full2.view(torch.int32), full.view(torch.int32))
        # timing contract of bench.py: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, full.numpy().tobytes(), float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,N,mode,world", [(10_007, 5, 0, 2), (130, 3, 1, 2), (64, 4, 2, 2), (1, 2, 0, 2),
                                             (10_007, 5, 1, 4), (1_000, 3, 2, 8), (200, 2, 0, 8)])
def test_sharded_fold_and_gather_is_bit_identical(P, N, mode, world):
    """World 2 and -- rehearsing the driver's 4- and 8-GPU runs on the CPU -- worlds 4 and 8,
    including shards of fewer than 64 params and ranks holding nothing."""
    from oracle import coracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, N, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(1234)
    d = (rng.standard_normal((N, P)) * 1e-2).astype(np.float32)
    c = rng.standard_normal(P).astype(np.float32)
    w = np.linspace(0.5, 2.0, N).astype(np.float32)
    want = coracle.fedavg(mode, d, c, w if mode == 2 else None)
    for rank, blob, tmax in res:
        got = np.frombuffer(blob, dtype=np.float32)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), rank
        assert tmax == float(world)


@pytest.mark.parametrize("P", [1, 63, 64, 65, 10_000, 11_689_512, 100_000_000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_bounds_partition(P, world):
    b = all_shard_bounds(P, world)
    assert b[0][0] == 0 and b[-1][1] == P
    for (lo, hi), (lo2, _) in zip(b, b[1:]):
        assert hi == lo2 and lo <= hi
    for lo, hi in b:
        assert lo % 64 == 0 or lo == P
    sizes = [hi - lo for lo, hi in b]
    assert max(sizes) - min(x for x in sizes if x > 0 or P < world * 64) <= max(sizes)


def test_weak_scaling_shards_equal():
    """bench.py's weak scaling: P = world x P_g, every rank's shard within one alignment unit of P_g."""
    Pg = 11_689_512
    for world in (1, 2, 4, 8):
        for lo, hi in all_shard_bounds(world * Pg, world):
            assert abs((hi - lo) - Pg) < 64 * world


def _shares(P, N, S):
    rng = np.random.default_rng(99)
    sh = rng.integers(-2**63, 2**63 - 1, size=(N, S, P), dtype=np.int64, endpoint=True)
    sh[:, :, :3] = np.iinfo(np.int64).max  # wrap many times over
    return sh


def _cs_worker(rank, world, port, P, N, S, chunks, q):
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = _shares(P, N, S)
        c0, c1 = client_bounds(N, world, rank)  # this rank ingests only its own clients
        og = OverlappedReduceScatter(P, world, rank, chunks=chunks, device="cpu", tail=2)

        def sum_range(a, n, stream):
            if c1 > c0:
                og.sums[a:a + n] = torch.from_numpy(O.secagg_sum(sh[c0:c1, :, a:a + n]))
            else:
                og.sums[a:a + n] = 0

        def decode(total, dec, stream):
            dec.copy_(torch.from_numpy(O.fix_prec_decode(total.numpy())))
        og.run(sum_range, decode)
        q.put((rank, og.assemble().numpy().tobytes(), og.total.numpy().tobytes(), og.L))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,N,S,chunks,world", [(10_007, 5, 2, 3, 2), (130, 3, 3, 8, 2), (1, 1, 2, 1, 2),
                                                  (300, 7, 2, 2, 2), (10_007, 9, 2, 3, 4), (500, 5, 2, 2, 8)])
def test_client_sharded_secagg_reduce_scatter_is_bit_identical(P, N, S, chunks, world):
    """Secure aggregation with the CLIENTS sharded (north_star: reduce-scatter when clients are
    sharded): per-rank Z_2^64 sums reduce-scattered, decoded per slice, all-gathered -- equal bit
    for bit to one rank summing every client, and the reduced slices are the full sum's."""
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cs_worker, args=(r, world, port, P, N, S, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sh = _shares(P, N, S)
    want_sum = O.secagg_sum(sh)
    want = O.fix_prec_decode(want_sum)
    for rank, blob, tot, L in res:
        got = np.frombuffer(blob, dtype=np.float32)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), rank
        full = np.zeros(L, np.int64)
        full[:P] = want_sum
        m = L // world
        og_ranges = OverlappedReduceScatter(P, world, rank, chunks=chunks, device="cpu", tail=2).ranges
        mine = np.concatenate([full[a + rank * (b - a) // world: a + (rank + 1) * (b - a) // world]
                               for a, b in og_ranges])
        assert mine.size == m and np.array_equal(np.frombuffer(tot, dtype=np.int64), mine)


@pytest.mark.parametrize("N", [0, 1, 7, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_client_bounds_partition(N, world):
    b = [client_bounds(N, world, r) for r in range(world)]
    assert b[0][0] == 0 and b[-1][1] == N
    assert all(hi == lo2 for (_, hi), (lo2, _) in zip(b, b[1:]))
    assert max(hi - lo for lo, hi in b) - min(hi - lo for lo, hi in b) <= 1


@pytest.mark.parametrize("length,chunks,unit,tail", [(11_689_536, 8, 64, 3), (100, 8, 64, 3), (64, 1, 64, 3),
                                                     (1, 8, 64, 2), (93_516_288, 8, 512, 3), (640, 3, 64, 9),
                                                     (0, 4, 64, 1)])
def test_plan_ranges_partition(length, chunks, unit, tail):
    from pygrid_amd.sharding import plan_ranges

    r = plan_ranges(length, chunks, unit, tail)
    if length == 0:
        assert r == []
        return
    assert r[0][0] == 0 and r[-1][1] == length
    assert all(b > a and a % unit == 0 for a, b in r)
    assert all(b == a2 for (_, b), (a2, _) in zip(r, r[1:]))
    assert len(r) <= chunks + tail


def _check_worker(rank, world, port, P, corrupt, q):
    """bench.check_sampled at world > 1: every rank samples its shard and computes the expected
    values from its own 'inputs'; rank 0 compares the all-gathered vector."""
    import sys
    import types

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    sys.argv = ["bench.py"]
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(P, world, rank)
        part = (torch.arange(lo, hi, dtype=torch.float32) * 0.25)
        if corrupt and rank == world - 1 and hi > lo:
            part[-1] = torch.nextafter(part[-1], torch.tensor(1e9))  # one ulp off at the last shard's edge
        full = gather_flat(part, P, world, rank)
        ctx = types.SimpleNamespace(torch=torch, world=world, rank=rank, dist=dist)
        got = bench.check_sampled(ctx, types.SimpleNamespace(seed=5), full, lo, hi,
                                  lambda idx: idx.astype(np.float32) * np.float32(0.25))
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_bench_check_leg_over_two_ranks(corrupt):
    P, world = 10_001, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, P, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert res[1] is None  # only rank 0 reports
    r0 = res[0]
    assert r0["ranks"] == 2 and r0["params_checked"] >= 4096
    assert r0["bit_exact"] is (not corrupt) and r0["mismatches"] == int(corrupt)
