"""Parameter-axis sharding across the GPUs of one node.

One process per GPU.  Rank r owns the contiguous flat range ``shard_bounds(P, world, r)``
of the concatenated parameter vector, for EVERY client, so each rank folds its params over
all clients in client order: the fp32 result is bit-identical to one GPU.  Clients are never
split across ranks on the fp32 path (that would reorder the sum).

The only collective is the all-gather of the new checkpoint's shards (the node serializes one
checkpoint; ``cycle_manager.py:303-304``): one ``all_gather`` of equal padded shards over
RCCL/xGMI (``torch.distributed`` backend "nccl"), or gloo on CPU in tests.

Secure aggregation may instead shard the CLIENTS (``client_bounds``): each rank sums the shares
of its own clients over the whole parameter vector, the int64 sums are reduce-scattered (SUM,
wrap-around: addition mod 2^64 is associative and commutative, so any client split is exact),
each rank decodes its part and the decoded vector is all-gathered (``OverlappedReduceScatter``).
That is the layout when each GPU ingests a different subset of clients over its own PCIe link.
"""
from __future__ import annotations

from typing import List, Tuple

ALIGN = 64  # elements: shard starts stay 256-byte aligned in the flat fp32 vector


def shard_size(P: int, world: int, align: int = ALIGN) -> int:
    per = -(-P // world)
    return -(-per // align) * align


def shard_bounds(P: int, world: int, rank: int, align: int = ALIGN) -> Tuple[int, int]:
    if not (0 <= rank < world) or P <= 0:
        raise ValueError(f"bad shard request P={P} world={world} rank={rank}")
    s = shard_size(P, world, align)
    lo = min(rank * s, P)
    hi = min(lo + s, P)
    return lo, hi


def all_shard_bounds(P: int, world: int, align: int = ALIGN) -> List[Tuple[int, int]]:
    return [shard_bounds(P, world, r, align) for r in range(world)]


def plan_ranges(length: int, chunks: int, unit: int = ALIGN, tail: int = 0) -> List[Tuple[int, int]]:
    """Cut ``[0, length)`` into ``chunks`` equal ranges (multiples of ``unit``), then split the
    last one in halves ``tail`` times (c/2, c/4, ..., c/2^tail, c/2^tail): the collective of the
    last range is the only one not hidden behind a later fold, so a short last range shortens
    the exposed tail of the step without cutting every range small."""
    if length <= 0:
        return []
    c = -(-length // max(1, chunks))
    c = -(-c // unit) * unit
    cuts = list(range(0, length, c))[1:]
    last = cuts[-1] if cuts else 0
    for _ in range(max(0, tail)):
        half = -(-((length - last) // 2) // unit) * unit
        if half <= 0 or last + half >= length:
            break
        last += half
        cuts.append(last)
    edges = [0] + cuts + [length]
    return [(a, b) for a, b in zip(edges, edges[1:]) if b > a]


def gather_flat(shard, P: int, world: int, rank: int, align: int = ALIGN, group=None):
    """All-gather every rank's output shard into the full flat vector (torch tensors).

    ``shard`` holds this rank's ``hi - lo`` values (any device the backend supports); it is
    padded to the common shard size, gathered, and the padding dropped.
    """
    import torch
    import torch.distributed as dist

    s = shard_size(P, world, align)
    lo, hi = shard_bounds(P, world, rank, align)
    if shard.numel() != hi - lo:
        raise ValueError(f"rank {rank} shard has {shard.numel()} values, expected {hi - lo}")
    if shard.numel() == s:
        send = shard.contiguous()
    else:
        send = torch.zeros(s, dtype=shard.dtype, device=shard.device)
        send[: hi - lo].copy_(shard)
    recv = torch.empty(world * s, dtype=shard.dtype, device=shard.device)
    if send.device.type != "cpu" and dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(recv, send, group=group)
    else:
        dist.all_gather(list(recv.chunk(world)), send, group=group)
    if world * s == P:
        return recv
    parts = [recv[r * s: r * s + (b - a)] for r, (a, b) in enumerate(all_shard_bounds(P, world, align))]
    return torch.cat(parts)


class OverlappedGather:
    """All-gather the new checkpoint chunk by chunk while later chunks are still being folded.

    The shard is split into ``chunks`` aligned param ranges.  For each range the caller's
    ``fold_range(off, n, stream)`` enqueues the fold of shard-relative ``[off, off + n)`` into
    ``self.local`` on ``stream`` (a HIP stream handle, or None on CPU), then an async
    ``all_gather_into_tensor`` of that range is issued from the same stream: RCCL waits for that
    fold only, so gather i runs beside fold i + 1 and only the last range's gather is exposed.
    On the GPU the ranges alternate over two streams, so fold i + 1 starts while fold i drains
    its last workgroups (one stream: +3.3 % for 8 ranges; two: none, ``tools/ab_ranges.py``).
    Each gathered range is copied into its place in the flat vector on its own stream right after
    its gather, so ``assemble()`` costs nothing; it returns the flat P-vector, valid until the
    next ``run()``.
    """

    def __init__(self, P: int, world: int, rank: int, chunks: int = 4, device="cuda", dtype=None, group=None,
                 align: int = ALIGN, streams: int = 2, tail: int = 0):
        import torch

        dtype = dtype or torch.float32
        self.P, self.world, self.rank, self.group = P, world, rank, group
        self.s = shard_size(P, world, align)
        self.lo, self.hi = shard_bounds(P, world, rank, align)
        self.pg = self.hi - self.lo
        self.ranges = plan_ranges(self.s, chunks, align, tail)
        self.local = torch.zeros(self.s, dtype=dtype, device=device)
        self.recv = [torch.empty(world * (b - a), dtype=dtype, device=device) for a, b in self.ranges]
        self.out = torch.empty(world * self.s, dtype=dtype, device=device)
        self.cuda = self.local.device.type == "cuda"
        self.side = [torch.cuda.Stream(device=self.local.device) for _ in range(max(0, streams - 1))] if self.cuda \
            else []

    def run(self, fold_range, force_collective: bool = False):
        """``force_collective`` issues the all-gathers even at world size 1 (tests the RCCL path
        on a one-GPU box)."""
        import contextlib

        import torch
        import torch.distributed as dist

        main = torch.cuda.current_stream(self.local.device) if self.cuda else None
        streams = [main] + self.side
        for st in self.side:
            st.wait_stream(main)  # every range after the caller's earlier work (previous gathers included)
        grid = self.out.view(self.world, self.s)
        for i, ((a, b), r) in enumerate(zip(self.ranges, self.recv)):
            st = streams[i % len(streams)]
            with torch.cuda.stream(st) if st is not None else contextlib.nullcontext():
                n = min(b, self.pg) - a
                if n > 0:
                    fold_range(a, n, st.cuda_stream if st is not None else None)
                if self.world > 1 or force_collective:
                    if self.cuda and dist.get_backend(self.group) == "nccl":
                        w = dist.all_gather_into_tensor(r, self.local[a:b], group=self.group, async_op=True)
                    else:
                        w = dist.all_gather(list(r.chunk(self.world)), self.local[a:b], group=self.group,
                                            async_op=True)
                    w.wait()  # this range's stream waits for its gather (the other stream folds on)
                    grid[:, a:b].copy_(r.view(self.world, b - a))
                else:
                    grid[:, a:b].copy_(self.local[a:b].view(1, b - a))
        for st in self.side:
            main.wait_stream(st)

    def assemble(self):
        return self.out[: self.P]


def client_bounds(N: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous client range of ``rank`` when clients are sharded (secure aggregation only)."""
    if not (0 <= rank < world) or N < 0:
        raise ValueError(f"bad client shard request N={N} world={world} rank={rank}")
    q, r = divmod(N, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


class OverlappedReduceScatter:
    """Client-sharded secure aggregation across ranks, pipelined over param ranges.

    Every rank holds the shares of its own clients for the whole parameter vector (length P).
    The vector is cut into ranges whose length is a multiple of ``world * align``; for range
    ``[a, b)``, on alternating streams:

    1. ``sum_range(a, n, stream)`` writes the rank's Z_2^64 share sum of ``[a, a + n)`` into
       ``self.sums[a:a + n]`` (the engine's ``secagg_device_range`` with no decode; ``stream`` is
       a HIP stream handle, or None on CPU);
    2. ``reduce_scatter_tensor`` (int64 SUM, wraps mod 2^64) leaves rank r the total of the
       r-th ``(b - a) / world`` slice of the range;
    3. ``decode(total, dec, stream)`` decodes that slice (int64 tensor -> float32 tensor of the
       same length; ``secagg_decode_device``);
    4. ``all_gather_into_tensor`` puts the decoded slices of every rank back in range order,
       straight into ``self.out[a:b]``.

    Range i's collectives run beside the share sum of range i + 1.  ``self.out[:P]`` is the
    decoded vector (bit-identical to one GPU summing every client), ``self.total`` holds this
    rank's reduced int64 slices (range by range).  ``sums`` tail past P stays zero.
    """

    def __init__(self, P: int, world: int, rank: int, chunks: int = 8, device="cuda", group=None,
                 align: int = ALIGN, streams: int = 2, tail: int = 0):
        import torch

        self.P, self.world, self.rank, self.group = P, world, rank, group
        unit = world * align
        self.L = -(-P // unit) * unit
        self.ranges = plan_ranges(self.L, chunks, unit, tail)
        self.sums = torch.zeros(self.L, dtype=torch.int64, device=device)
        self.total = torch.empty(self.L // world, dtype=torch.int64, device=device)
        self.dec = torch.empty(self.L // world, dtype=torch.float32, device=device)
        self.out = torch.empty(self.L, dtype=torch.float32, device=device)
        self.cuda = self.sums.device.type == "cuda"
        self.side = [torch.cuda.Stream(device=self.sums.device) for _ in range(max(0, streams - 1))] \
            if self.cuda else []

    def run(self, sum_range, decode, force_collective: bool = False):
        import contextlib

        import torch
        import torch.distributed as dist

        collective = self.world > 1 or force_collective
        main = torch.cuda.current_stream(self.sums.device) if self.cuda else None
        streams = [main] + self.side
        for st in self.side:
            st.wait_stream(main)
        nccl = collective and self.cuda and dist.get_backend(self.group) == "nccl"
        for i, (a, b) in enumerate(self.ranges):
            st = streams[i % len(streams)]
            h = st.cuda_stream if st is not None else None
            m = (b - a) // self.world
            t, d = self.total[a // self.world: a // self.world + m], self.dec[a // self.world: a // self.world + m]
            with torch.cuda.stream(st) if st is not None else contextlib.nullcontext():
                n = min(b, self.P) - a
                if n > 0:
                    sum_range(a, n, h)
                if collective:
                    if nccl:
                        dist.reduce_scatter_tensor(t, self.sums[a:b], group=self.group, async_op=True).wait()
                    else:
                        dist.reduce_scatter(t, list(self.sums[a:b].chunk(self.world)), group=self.group,
                                            async_op=True).wait()
                else:
                    t.copy_(self.sums[a:b])
                decode(t, d, h)
                if collective:
                    if nccl:
                        dist.all_gather_into_tensor(self.out[a:b], d, group=self.group, async_op=True).wait()
                    else:
                        dist.all_gather(list(self.out[a:b].chunk(self.world)), d, group=self.group,
                                        async_op=True).wait()
                else:
                    self.out[a:b].copy_(d)
        for st in self.side:
            main.wait_stream(st)

    def assemble(self):
        return self.out[: self.P]
