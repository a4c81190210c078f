"""Multi-GPU driver: one process per GPU, signature-index sharding, optional
verdict-bitmap all-gather (collective C1).

Signatures are independent units, so a batch is split into contiguous index
ranges, one per rank, with no data-path collective; each rank stages and
verifies only its shard on its own device (``Context(LOCAL_RANK)``).  Shard
boundaries are aligned to 32 so every rank's accept bitmap covers whole 32-bit
words and the global bitmap is the plain concatenation of the per-rank words —
that is the one collective, an all-gather over RCCL (``torch.distributed``
backend "nccl") of ``ceil(n_rank / 32)`` words per rank (12.5 MB for 100M
signatures).  The same code runs over gloo on CPU tensors (tests).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .crypto import PackedBatch, PreparedBatch


def shard_bounds(n: int, world: int, align: int = 32) -> list[int]:
    """Boundaries b_0 = 0 <= b_1 <= ... <= b_world = n of contiguous shards; every
    interior boundary is a multiple of `align`."""
    if world < 1:
        raise ValueError("world must be >= 1")
    b = [min(n, (r * n // world) // align * align) for r in range(world)]
    b.append(n)
    b[0] = 0
    return b


def slice_batch(b: PackedBatch, lo: int, hi: int) -> PackedBatch:
    """Shard [lo, hi) of a packed batch, with its own compacted message arena."""
    if hi <= lo:
        return PackedBatch(0, b.scheme[:0], b.pk[:0], b.pk_stride, b.sig[:0], b.sig_stride, b.sig_len[:0],
                           np.zeros(1, np.uint8), b.msg_off[:0], b.msg_len[:0])
    off = b.msg_off[lo:hi].astype(np.uint64)
    ln = b.msg_len[lo:hi]
    start = int(off.min())
    end = int((off + ln).max())
    arena = b.msg[start:max(end, start + 1)].copy()
    return PackedBatch(hi - lo, b.scheme[lo:hi].copy(), b.pk[lo:hi].copy(), b.pk_stride, b.sig[lo:hi].copy(),
                       b.sig_stride, b.sig_len[lo:hi].copy(), arena, off - np.uint64(start), ln.copy())


def pack_bits(accept: np.ndarray) -> np.ndarray:
    """Accept mask -> little-endian uint32 words (bit i%32 of word i/32)."""
    bits = np.packbits(accept.astype(np.uint8), bitorder="little")
    pad = (-len(bits)) % 4
    return np.concatenate([bits, np.zeros(pad, np.uint8)]).view(np.uint32)


def allgather_bitmap(local_words, bounds: list[int], rank: int, group=None):
    """All-gathers per-rank accept-bitmap words (torch tensor, int32, on the
    rank's device for RCCL or on CPU for gloo) into the global bitmap."""
    import torch
    import torch.distributed as dist
    world = len(bounds) - 1
    words = [(bounds[r + 1] - bounds[r] + 31) // 32 for r in range(world)]
    mx = max(words) if words else 0
    buf = torch.zeros(mx, dtype=torch.int32, device=local_words.device)
    buf[:local_words.numel()] = local_words
    out = [torch.zeros(mx, dtype=torch.int32, device=local_words.device) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return torch.cat([out[r][:words[r]] for r in range(world)])


def verify_sharded(ctx: _lib.Context, batch: PackedBatch, rank: int, world: int, mode: int = _lib.MODE_IS_VALID,
                   group=None):
    """Each rank verifies its shard of `batch` on its device and all ranks
    receive the global accept bitmap.  Returns (local verdicts, global bitmap
    as a torch tensor on the rank's device, bounds)."""
    import torch
    bounds = shard_bounds(batch.n, world)
    lo, hi = bounds[rank], bounds[rank + 1]
    shard = slice_batch(batch, lo, hi)
    nwords = (shard.n + 31) // 32
    local = torch.zeros(max(nwords, 1), dtype=torch.int32, device=f"cuda:{ctx.device}")
    verdicts = np.zeros(0, np.uint8)
    if shard.n:
        pb = PreparedBatch(ctx, shard)
        verdicts = pb.verify(mode, want_verdicts=True, device_bitmap_ptr=local.data_ptr())
        pb.close()
    glob = allgather_bitmap(local[:nwords], bounds, rank, group)
    return verdicts, glob, bounds
