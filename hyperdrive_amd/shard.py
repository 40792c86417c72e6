"""Multi-GPU sharding of a batch.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, "gloo"
in the CPU tests).  Verification is embarrassingly parallel per message, so
rank k verifies the contiguous index range ``shard_range(n, k, world)`` of a
batch whose metadata is replicated on every rank; the only exchange is an
all-gather of the per-rank valid bitmaps (n/32 words in total, latency-bound
over xGMI).  The tally then needs the global first-wins order, so every rank
tallies the whole batch from the gathered bitmap (hd_tally_device_bitmap).
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n: int, rank: int, world: int, align: int = 32) -> Tuple[int, int]:
    """[lo, hi) of rank's shard: contiguous, bitmap-word aligned (every shard
    but the last is a multiple of ``align`` messages), covering [0, n)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    per = (n + world - 1) // world
    per = (per + align - 1) // align * align
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return lo, hi


def gather_bitmaps(local_bits, n: int, world: int, group=None):
    """All-gather per-rank valid bitmaps (int32 tensors of shard_len/32 words,
    shard-aligned) into one bitmap of ceil(n/32) words, in rank order.

    Every shard except the last is a whole number of words (shard_range's
    alignment), so the concatenation is exactly the global bitmap."""
    import torch
    import torch.distributed as dist
    per_words = [(shard_range(n, r, world)[1] - shard_range(n, r, world)[0] + 31) // 32 for r in range(world)]
    if len(set(per_words)) == 1:
        out = torch.empty(per_words[0] * world, dtype=local_bits.dtype, device=local_bits.device)
        dist.all_gather_into_tensor(out, local_bits.contiguous(), group=group)
        return out[: (n + 31) // 32]
    # ragged last shard: pad to the largest shard, gather, then trim
    width = max(per_words)
    padded = torch.zeros(width, dtype=local_bits.dtype, device=local_bits.device)
    padded[: local_bits.numel()] = local_bits
    out = torch.empty(width * world, dtype=local_bits.dtype, device=local_bits.device)
    dist.all_gather_into_tensor(out, padded, group=group)
    parts = [out[r * width: r * width + per_words[r]] for r in range(world)]
    return torch.cat(parts)[: (n + 31) // 32]
