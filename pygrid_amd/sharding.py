"""Parameter-axis sharding across the GPUs of one node.

One process per GPU.  Rank r owns the contiguous flat range ``shard_bounds(P, world, r)``
of the concatenated parameter vector, for EVERY client, so each rank folds its params over
all clients in client order: the fp32 result is bit-identical to one GPU.  Clients are never
split across ranks on the fp32 path (that would reorder the sum).

The only collective is the all-gather of the new checkpoint's shards (the node serializes one
checkpoint; ``cycle_manager.py:303-304``): one ``all_gather`` of equal padded shards over
RCCL/xGMI (``torch.distributed`` backend "nccl"), or gloo on CPU in tests.
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
                 align: int = ALIGN, streams: int = 2):
        import torch

        dtype = dtype or torch.float32
        self.P, self.world, self.rank, self.group = P, world, rank, group
        self.s = shard_size(P, world, align)
        self.lo, self.hi = shard_bounds(P, world, rank, align)
        self.pg = self.hi - self.lo
        c = -(-self.s // max(1, chunks))
        c = -(-c // align) * align
        self.ranges = [(a, min(a + c, self.s)) for a in range(0, self.s, c)]
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
