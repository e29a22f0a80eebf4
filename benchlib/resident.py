"""The HBM-resident and streamed workloads (BASELINE configs 2-5), per rank and on a one-process
group: one step = one fold of every client diff of the shard (plus the exchange at N > 1)."""
from __future__ import annotations

from benchlib.roofline import roofline_of
from benchlib.world import check_resident, check_sampled, record, timed


def run_resident(ctx, args, eng, mode, dtype, N, parties, pg, P, lo, hi):
    torch = ctx.torch

    eng.reserve(N, dtype, parties)
    eng.synth_fill(args.seed, N)
    sp = torch.cuda.current_stream().cuda_stream
    if dtype == 0:
        ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
        out = torch.empty_like(ckpt)
        eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
        if mode == 2:
            eng.set_weights([(c % 7 + 1) * 0.5 for c in range(N)])
        if ctx.world > 1:
            # fold the shard in 8 param ranges; RCCL all-gathers range i beside the fold of i + 1
            from pygrid_amd.sharding import OverlappedGather
            og = OverlappedGather(P, ctx.world, ctx.rank, chunks=args.gather_chunks, tail=args.gather_tail)
            lp = og.local.data_ptr()

            def step():
                og.run(lambda off, n, st: eng.fedavg_device_range(mode, off, n, ckpt.data_ptr(), lp, st))
                og.assemble()
        else:
            def step():
                eng.fedavg_device(mode, ckpt.data_ptr(), out.data_ptr(), sp)
        diff_bytes, dt, kernel = 4 * N * pg, "f32", "k_fedavg"
    else:
        s_out = torch.empty(pg, dtype=torch.int64, device="cuda")
        d_out = torch.empty(pg, dtype=torch.float32, device="cuda")
        if ctx.world > 1:
            # decoded shard gathered range by range beside the share sum of the next range
            from pygrid_amd.sharding import OverlappedGather
            og = OverlappedGather(P, ctx.world, ctx.rank, chunks=args.gather_chunks, tail=args.gather_tail)
            lp = og.local.data_ptr()

            def step():
                og.run(lambda off, n, st: eng.secagg_device_range(off, n, s_out.data_ptr(), lp, 10, 3, st))
                og.assemble()
        else:
            def step():
                eng.secagg_device(s_out.data_ptr(), d_out.data_ptr(), 10, 3, sp)
        diff_bytes, dt, kernel = 8 * parties * N * pg, "int64", "k_secagg"
    torch.cuda.synchronize()
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    checked = None
    if args.check:
        full = og.assemble() if ctx.world > 1 else (out if dtype == 0 else d_out)
        checked = check_resident(ctx, args, full, mode, dtype, N, parties, lo, hi, s_out if dtype == 1 else None)
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    cfg = {"workload": f"{args.workload}: P_shard={pg} params/GPU x {N} clients"
                       + (f" x {parties} parties int64" if dtype == 1 else " fp32") + ", resident in HBM",
           "clients": N, "params_per_gpu": pg, "params_total": P,
           "parallelism": f"param-shard{ctx.world}" + (
               f" + {ctx.coll} all-gather ({args.gather_chunks} ranges, last halved {args.gather_tail}x, overlapped with the fold)" if ctx.world > 1 else ""),
           "kernel_variant": eng.effective_variant(mode if dtype == 0 else 16)}
    rec = record(ctx, args, args.workload, value, el, dt, cfg,
                 roofline_of(st, args.workload, cfg["kernel_variant"], kernel),
                 {"check": checked} if args.check else None)
    return rec  # cpu_baseline: measured before the world formed (baseline.pre_world_cpu_baseline)


def run_secagg_clients(ctx, args, eng, N, S, P):
    """Config 3 with client sharding (north_star: reduce-scatter when clients are sharded): rank r
    holds the 2-party int64 shares of its own N clients for all P params (a different client set
    per rank: seed + rank), sums them range by range, and OverlappedReduceScatter reduce-scatters
    the Z_2^64 sums, decodes each rank's slice and all-gathers the decoded vector."""
    torch = ctx.torch
    from pygrid_amd.sharding import OverlappedReduceScatter

    eng.reserve(N, 1, S)
    eng.synth_fill(args.seed + ctx.rank, N)
    og = OverlappedReduceScatter(P, ctx.world, ctx.rank, chunks=args.gather_chunks, tail=args.gather_tail)
    sp = og.sums.data_ptr()

    def step():
        og.run(lambda a, n, st: eng.secagg_device_range(a, n, sp, 0, 10, 3, st),
               lambda t, d, st: eng.secagg_decode_device(t.data_ptr(), t.numel(), d.data_ptr(), 10, 3, st))
        og.assemble()
    torch.cuda.synchronize()
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    diff_bytes = 8 * S * N * P
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    cfg = {"workload": f"secagg-clients: {N} clients/GPU x {S} parties int64 x P={P} (ResNet-18) on every rank, "
                       "clients sharded, resident in HBM",
           "clients": N * ctx.world, "clients_per_gpu": N, "params_per_gpu": P, "params_total": P,
           "parallelism": f"client-shard{ctx.world} + {ctx.coll or 'no'} int64 reduce-scatter / decode / all-gather "
                          f"({args.gather_chunks} ranges, last halved {args.gather_tail}x, overlapped with the share sum)",
           "kernel_variant": eng.effective_variant(16)}
    # roofline: the share-sum launches (k_secagg); the decode kernel (12 B/param) is not in the stats
    rec = record(ctx, args, "secagg-clients", value, el, "int64", cfg,
                 roofline_of(st, "secagg-clients", cfg["kernel_variant"], "k_secagg"))
    return rec


def run_c4(ctx, args, eng, N, pg, P):
    """Config 4 shard: N clients streamed through an R-slot ring; each chunk generated on the GPU
    (stand-in for arriving data) and folded in client order, generator and fold alternating on one
    stream (r02p: 12-14 % faster than beside it)."""
    torch = ctx.torch
    from pygrid_amd.sharding import gather_flat

    R = args.ring or min(1000, N)  # a cycle of fewer clients than the ring (a rehearsal) needs no more slots
    chunk = max(1, R // 2)
    eng.reserve(R)
    eng.set_synth_kind(1 if args.synth == "fast" else 0)
    ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ckpt)
    sp = torch.cuda.current_stream().cuda_stream
    eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
    torch.cuda.synchronize()

    full = [out]

    def step():
        eng.stream_begin(0, chunk)
        for c0 in range(0, N, chunk):
            eng.synth_ingest(args.seed, c0, min(chunk, N - c0))
        eng.stream_finish_device(ckpt.data_ptr(), out.data_ptr(), sp)
        if ctx.world > 1:
            full[0] = gather_flat(out, P, ctx.world, ctx.rank)
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    checked = None
    if args.check:
        def expected(idx):
            import numpy as np

            from oracle import coracle
            from oracle import oracle as O

            u = idx.astype(np.uint64)
            gen = O.synth_diff_fast if args.synth == "fast" else O.synth_diff
            return coracle.fedavg(0, np.stack([gen(args.seed, k, u) for k in range(N)]), O.synth_ckpt(args.seed, u))
        checked = check_sampled(ctx, args, full[0], eng.lo, eng.hi, expected)
    diff_bytes = 4 * N * pg
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    kern_gbs = ctx.sum_over_ranks(4 * N * pg * args.steps / (st["kernel_ms_total"] / 1e3) / 1e9)
    cfg = {"workload": f"c4-stream: P_shard={pg} params/GPU x {N} clients fp32 (SURVEY 8(d) config 4 shard), "
                       f"{R}-slot HBM ring, {chunk}-client chunks generated on-device ({args.synth} generator)",
           "clients": N, "params_per_gpu": pg, "params_total": P, "ring_slots": R, "fold_batch": chunk, "generator": args.synth,
           "parallelism": f"param-shard{ctx.world}" + (f" + {ctx.coll} all-gather" if ctx.world > 1 else ""),
           "kernel_variant": eng.effective_variant()}
    extra = {"fold_kernel_client_diff_GBps_aggregated": round(kern_gbs, 1),
             "note": "value includes on-device generation of every chunk (writes 4 B/param/client, "
                     "alternating with the fold); the fold kernels alone are fold_kernel_*"}
    if args.check:
        extra["check"] = checked
    rec = record(ctx, args, "c4-stream", value, el, "f32", cfg,
                 roofline_of(st, "c4-stream", cfg["kernel_variant"], "k_fedavg"), extra)
    return rec


def run_c5(ctx, args, eng, N, pg, P):
    """Config 5 shard: iterative plan over N clients whose diffs arrive from page-locked host
    memory; every H2D copy overlaps the fold of the previously copied clients."""
    torch = ctx.torch
    import numpy as np

    from pygrid_amd import PinnedBuffer
    from pygrid_amd.sharding import gather_flat

    R = args.ring or 8
    batch = max(1, R // 2)  # fold half the ring at a time: the other half takes the next H2D copies
    n_host = 4  # distinct host buffers, re-sent as different clients
    bufs = [PinnedBuffer((pg,)) for _ in range(n_host)]  # shard-sized host diffs
    rng = np.random.default_rng(args.seed + ctx.rank)
    for b in bufs:
        b.array[:] = rng.standard_normal(pg, dtype=np.float32) * np.float32(1e-2)
    eng.reserve(R)
    ckpt = torch.empty(pg, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ckpt)
    sp = torch.cuda.current_stream().cuda_stream
    eng.synth_ckpt_device(args.seed, ckpt.data_ptr(), sp)
    torch.cuda.synchronize()

    full = [out]

    def step():
        eng.stream_begin(1, batch)
        for k in range(N):
            eng.ingest(k, bufs[k % n_host].array)
        eng.stream_finish_device(ckpt.data_ptr(), out.data_ptr(), sp)
        if ctx.world > 1:
            full[0] = gather_flat(out, P, ctx.world, ctx.rank)
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    checked = None
    if args.check:
        lo = eng.lo

        def expected(idx):
            from oracle import coracle
            from oracle import oracle as O

            d = np.stack([bufs[k % n_host].array[idx - lo] for k in range(N)])
            return coracle.fedavg(1, d, O.synth_ckpt(args.seed, idx.astype(np.uint64)))
        checked = check_sampled(ctx, args, full[0], eng.lo, eng.hi, expected)
    diff_bytes = 4 * N * pg
    value = diff_bytes * ctx.world * args.steps / el / 1e9
    kern_gbs = 4 * N * pg * args.steps / (st["kernel_ms_total"] / 1e3) / 1e9
    ingest_gbs = st["h2d_bytes_total"] / (st["h2d_ms_total"] / 1e3) / 1e9 if st["h2d_ms_total"] else None
    cfg = {"workload": f"c5-ingest: P_shard={pg} params/GPU x {N} clients fp32 iterative plan (SURVEY 8(d) "
                       f"config 5 shard), pinned host -> HBM over PCIe, {R}-slot ring, fold batch {batch}",
           "clients": N, "params_per_gpu": pg, "params_total": P, "ring_slots": R, "fold_batch": batch,
           "parallelism": f"param-shard{ctx.world}" + (f" + {ctx.coll} all-gather" if ctx.world > 1 else ""),
           "kernel_variant": eng.effective_variant(1)}
    extra = {"bound_by": "PCIe host->device (Gen5 x16, 63 GB/s spec per GPU)",
             "ingest_GBps_per_gpu": round(ingest_gbs, 2) if ingest_gbs else None,
             "fold_kernel_client_diff_GBps_per_gpu": round(kern_gbs, 1)}
    if args.check:
        extra["check"] = checked
    rec = record(ctx, args, "c5-ingest", value, el, "f32", cfg,
                 roofline_of(st, "c5-ingest", cfg["kernel_variant"], "k_fedavg"), extra)
    for b in bufs:
        b.free()
    return rec


def group_exchange(eng) -> str:
    """How a group's collective ran: RCCL (distinct devices) or the library's peer copies (repeated
    devices, PGH_RCCL=0, or a group of one before its first collective)."""
    return {1: "RCCL (ncclAllGather / ncclReduceScatter)", 0: "peer-copy"}.get(eng.group_backend(), "no collective")


def run_group_resident(ctx, args, eng, mode, dtype, N, parties, Pg):
    """The resident configs on a one-process group: GPU g folds its Pg-param shard of a
    (G x Pg)-param model over all N clients (weak scaling like the per-rank runs), then the new
    checkpoint is all-gathered into a full copy on every GPU (ncclAllGather); secagg writes the
    decoded sum into a page-locked host array slice by slice."""
    import numpy as np

    from pygrid_amd import PinnedBuffer

    G = ctx.n_gpus
    P = Pg * G
    eng.set_layout([P])
    eng.reserve(N, dtype, parties)
    eng.synth_fill(args.seed, N)
    bufs = []
    if dtype == 0:
        eng.ckpt_upload(np.full(P, 0.01, np.float32))
        if mode == 2:
            eng.set_weights([(c % 7 + 1) * 0.5 for c in range(N)])

        def step():
            eng.fedavg_resident(mode)
            eng.allgather_resident()
        diff_bytes, dt, kernel = 4 * N * P, "f32", "k_fedavg"
    else:
        bufs = [PinnedBuffer((P,), np.int64), PinnedBuffer((P,), np.float32)]

        def step():
            eng.secagg(10, 3, out_sum=bufs[0].array, out_dec=bufs[1].array)
        diff_bytes, dt, kernel = 8 * parties * N * P, "int64", "k_secagg"
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    value = diff_bytes * args.steps / el / 1e9
    cfg = {"workload": f"{args.workload}: P_shard={Pg} params/GPU x {N} clients"
                       + (f" x {parties} parties int64" if dtype == 1 else " fp32") + ", resident in HBM",
           "clients": N, "params_per_gpu": Pg, "params_total": P,
           "parallelism": f"param-shard{G} in one process (pgh_create_group, one host thread per GPU)" + (
               f" + {group_exchange(eng)} all-gather of the new checkpoint" if dtype == 0 else " + host slices"),
           "rccl": eng.group_backend() == 1, "exchange": group_exchange(eng), "devices": ctx.devices,
           "kernel_variant": eng.effective_variant(mode if dtype == 0 else 16)}
    rec = record(ctx, args, args.workload, value, el, dt, cfg,
                 roofline_of(st, args.workload, cfg["kernel_variant"], kernel, G))
    for b in bufs:
        b.free()
    return rec


def run_group_secagg_clients(ctx, args, eng, N, S, P):
    """Config 3 client-sharded on a one-process group: GPU g holds its own N clients x S parties
    over the whole model, the Z_2^64 sums are reduce-scattered (ncclReduceScatter, uint64 SUM), GPU
    g decodes its slice and writes it into the page-locked host outputs."""
    import numpy as np

    from pygrid_amd import PinnedBuffer

    G = ctx.n_gpus
    eng.set_layout([P])
    eng.set_client_sharding(True)
    eng.reserve(N * G, 1, S)
    eng.synth_fill(args.seed, N * G)
    bufs = [PinnedBuffer((P,), np.int64), PinnedBuffer((P,), np.float32)]

    def step():
        eng.secagg(10, 3, out_sum=bufs[0].array, out_dec=bufs[1].array)
    el, st = timed(ctx, step, args.steps, args.warmup, eng)
    value = 8 * S * N * G * P * args.steps / el / 1e9
    cfg = {"workload": f"secagg-clients: {N} clients/GPU x {S} parties int64 x P={P} (ResNet-18), clients sharded "
                       "over the GPUs of one process, resident in HBM",
           "clients": N * G, "clients_per_gpu": N, "params_per_gpu": P, "params_total": P,
           "parallelism": f"client-shard{G} in one process (pgh_create_group) + {group_exchange(eng)} reduce-scatter of "
                          "the Z_2^64 sums + per-GPU decode + host slices",
           "rccl": eng.group_backend() == 1, "exchange": group_exchange(eng), "devices": ctx.devices,
           "kernel_variant": eng.effective_variant(16)}
    rec = record(ctx, args, "secagg-clients", value, el, "int64", cfg,
                 roofline_of(st, "secagg-clients", cfg["kernel_variant"], "k_secagg", G))
    for b in bufs:
        b.free()
    return rec
