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
    if hasattr(dist, "all_gather_into_tensor") and send.device.type != "cpu":
        dist.all_gather_into_tensor(recv, send, group=group)
    else:
        dist.all_gather(list(recv.chunk(world)), send, group=group)
    if world * s == P:
        return recv
    parts = [recv[r * s: r * s + (b - a)] for r, (a, b) in enumerate(all_shard_bounds(P, world, align))]
    return torch.cat(parts)
