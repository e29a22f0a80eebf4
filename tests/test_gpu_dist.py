"""GPU, two processes: the one-process-per-GPU path of bench.py at N = 2, with the real HIP folds.

Both ranks run on GPU 0 over gloo (RCCL needs one GPU per rank; the 8-GPU node is the driver's):
``OverlappedGather`` folds each rank's param shard range by range with ``pgh_fedavg_device_range``
and all-gathers the ranges, ``OverlappedReduceScatter`` sums each rank's own clients' shares with
``pgh_secagg_device_range``, reduce-scatters the Z_2^64 sums and decodes with
``pgh_secagg_decode_device``.  Checked bit for bit against the oracle.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from oracle import coracle
    from oracle import oracle as O
    from pygrid_amd import Engine
    from pygrid_amd.sharding import OverlappedGather, OverlappedReduceScatter, client_bounds, shard_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        eng = Engine(0)
        # fp32: param shards, every client on every rank, ranges folded beside the gather
        P, N = 300_007, 6
        rng = np.random.default_rng(55)
        d = (rng.standard_normal((N, P)) * 1e-2).astype(np.float32)
        c = rng.standard_normal(P).astype(np.float32)
        for mode in (0, 1, 2):
            lo, hi = shard_bounds(P, world, rank)
            eng.set_layout([P])
            eng.set_shard(lo, hi)
            eng.reserve(N)
            for k in range(N):
                eng.ingest(k, d[k])
            w = np.linspace(0.5, 2.0, N).astype(np.float32)
            if mode == 2:
                eng.set_weights(w)
            ck = torch.from_numpy(c[lo:hi].copy()).cuda()
            og = OverlappedGather(P, world, rank, chunks=4, tail=2)
            lp = og.local.data_ptr()
            og.run(lambda off, n, st: eng.fedavg_device_range(mode, off, n, ck.data_ptr(), lp, st))
            got = og.assemble().cpu().numpy()
            want = coracle.fedavg(mode, d, c, w if mode == 2 else None)
            out[f"fedavg{mode}"] = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        # int64 shares: clients sharded, reduce-scatter of the sums, per-rank decode, all-gather
        P2, N2, S = 100_003, 5, 2
        idx = np.arange(P2, dtype=np.uint64)
        shares = np.stack([O.synth_shares(66, k, S, idx) for k in range(N2)])
        shares[0, 0, :3] = [2**63 - 1, -2**63, -1]
        a, b = client_bounds(N2, world, rank)
        eng.set_layout([P2])
        eng.reserve(max(b - a, 1), 1, S)
        for k in range(a, b):
            eng.ingest(k - a, shares[k])
        rs = OverlappedReduceScatter(P2, world, rank, chunks=3, tail=1)
        sp = rs.sums.data_ptr()
        rs.run(lambda off, n, st: eng.secagg_device_range(off, n, sp, 0, 10, 3, st),
               lambda t, dd, st: eng.secagg_decode_device(t.data_ptr(), t.numel(), dd.data_ptr(), 10, 3, st))
        dec = rs.assemble().cpu().numpy()
        ws = O.secagg_sum(shares)
        out["secagg"] = bool(np.array_equal(dec.view(np.uint32), O.fix_prec_decode(ws).view(np.uint32)))
        eng.close()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        out["error"] = repr(e)
    finally:
        dist.destroy_process_group()
    q.put((rank, out))


def test_two_ranks_on_one_gpu_fold_and_exchange_bit_exact():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert "error" not in res[r], res[r]
        assert all(res[r].values()), res[r]
