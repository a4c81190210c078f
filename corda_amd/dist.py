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


# Relative device cost of one verification per scheme id (measured kernel time per
# signature on MI355X, 1 KB messages: Ed25519 hash+points+msm 12.4 ms / 1M; secp256k1
# prep+msm 14.0 ms / 1M; P-256 20.2 ms / 1M — profiles/r01q_bench_*.json; the op model
# of SURVEY 8(e) gives the same ordering, 1.18 M vs 1.56 / 1.69 M ops).
SCHEME_COST = {4: 1.0, 2: 1.13, 3: 1.63}


def shard_bounds_weighted(scheme: np.ndarray, world: int, align: int = 32, cost: dict | None = None) -> list[int]:
    """Contiguous 32-aligned index shards of a mixed-scheme batch with equal device
    COST per rank (Ed25519 and ECDSA differ by ~1.4x), so the slowest rank
    — the one the max-over-ranks timing waits for — does not carry all the ECDSA work.
    Elements of other schemes cost nothing on the device (they are rejected up front)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    cost = cost or SCHEME_COST
    n = len(scheme)
    w = np.zeros(n, dtype=np.float64)
    for sid, c in cost.items():
        w[scheme[:n] == sid] = c
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    b = [0]
    for r in range(1, world):
        i = int(np.searchsorted(cum, total * r / world, side="left"))
        b.append(max(b[-1], min(n, i // align * align)))
    b.append(n)
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


def check_bounds(bounds: list[int], world: int, n_local: int | None = None, rank: int = 0) -> None:
    """Shard boundaries as ``gather_ordered`` needs them: ``world + 1`` entries from 0,
    non-decreasing, interior ones multiples of 32; with ``n_local``, the rank's own
    element count must be its shard's (a mismatch would misplace its words silently)."""
    if len(bounds) != world + 1:
        raise ValueError(f"{len(bounds)} shard boundaries for {world} ranks")
    if bounds[0] != 0 or any(bounds[r + 1] < bounds[r] for r in range(world)):
        raise ValueError("shard boundaries must start at 0 and be non-decreasing")
    if any(x % 32 for x in bounds[1:-1]):
        raise ValueError("shard boundaries must be multiples of 32")
    if n_local is not None and n_local != bounds[rank + 1] - bounds[rank]:
        raise ValueError(f"rank {rank} holds {n_local} elements, its shard [{bounds[rank]}, {bounds[rank + 1]}) "
                         f"has {bounds[rank + 1] - bounds[rank]}")


def gather_ordered(local_words, bounds: list[int], out=None, ordered=None, group=None, n_local: int | None = None):
    """C1 for shards of any sizes in ONE collective: every rank contributes
    ``words_max`` = the largest shard's word count (its own words zero-padded, as
    ``all_gather_into_tensor`` needs equal pieces), then rank r's
    ``ceil((b[r+1] - b[r]) / 32)`` words move to word ``b[r] / 32`` of the index-ordered
    global bitmap (shards are 32-aligned, so words never straddle ranks).  When every
    shard has ``words_max`` words the gathered buffer is already in index order and no
    copy runs.  ``local_words``: int32 tensor of at least ``words_max`` words (the tail
    past the rank's own words must be zero); ``out`` / ``ordered``: optional preallocated
    buffers of ``world * words_max`` / ``ceil(n / 32)`` words; ``n_local``: the rank's
    element count, checked against its shard.  Returns the global bitmap."""
    import torch
    import torch.distributed as dist
    world = len(bounds) - 1
    check_bounds(bounds, dist.get_world_size(group), n_local, dist.get_rank(group) if n_local is not None else 0)
    words = [(bounds[r + 1] - bounds[r] + 31) // 32 for r in range(world)]
    wmax = max(max(words), 1)
    if local_words.numel() < wmax:
        raise ValueError(f"local bitmap has {local_words.numel()} words, the largest shard needs {wmax}")
    if out is None:
        out = torch.empty(world * wmax, dtype=torch.int32, device=local_words.device)
    dist.all_gather_into_tensor(out, local_words[:wmax].contiguous(), group=group)
    total = (bounds[-1] + 31) // 32
    if all(w == wmax for w in words[:-1]):
        return out[:total]  # rank r's words already sit at r * wmax = b[r] / 32
    if ordered is None:
        ordered = torch.empty(total, dtype=torch.int32, device=local_words.device)
    for r in range(world):
        ordered[bounds[r] // 32:bounds[r] // 32 + words[r]] = out[r * wmax:r * wmax + words[r]]
    return ordered


def verify_sharded(ctx: _lib.Context, batch: PackedBatch, rank: int, world: int, mode: int = _lib.MODE_IS_VALID,
                   group=None):
    """Each rank verifies its shard of `batch` on its device and all ranks
    receive the global accept bitmap.  Returns (local verdicts, global bitmap
    as a torch tensor on the rank's device, bounds)."""
    import torch
    mixed = batch.n and len(np.unique(batch.scheme[:batch.n])) > 1
    bounds = shard_bounds_weighted(batch.scheme, world) if mixed else shard_bounds(batch.n, world)
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


class ShardBacklog:
    """Config 5 on one rank: the rank's index shard of a notary backlog, staged in
    HBM as a sequence of PreparedBatch chunks (each a multiple of 32 elements but
    the last, so chunk c's accept words land at word offset sum(len_j / 32, j < c) of
    ONE device bitmap), verified chunk after chunk into that bitmap, then the C1
    all-gather over RCCL.  Chunks bound the library's scratch (SURVEY 8d config 5:
    streamed in 2^24 pieces); the bitmap never leaves the device."""

    def __init__(self, ctx: _lib.Context, chunks, words: int | None = None, bounds: list[int] | None = None):
        """``bounds``: the global 32-aligned shard boundaries (``shard_bounds``), so that
        allgather returns the index-ordered global bitmap for any world size; ``words``
        (default: the largest shard's word count from ``bounds``) sizes the local bitmap."""
        import torch
        self.ctx, self.bounds = ctx, bounds
        if bounds is not None:
            words = max(words or 0, max((bounds[r + 1] - bounds[r] + 31) // 32 for r in range(len(bounds) - 1)))
        self.batches, self.sizes = [], []
        for b in chunks:
            if self.sizes and self.sizes[-1] % 32:
                raise ValueError("only the last chunk may have a length that is not a multiple of 32")
            self.batches.append(PreparedBatch(ctx, b))
            self.sizes.append(b.n)
        self.n = sum(self.sizes)
        need = (self.n + 31) // 32
        self.words = max(need, words or 0, 1)
        self.bitmap = torch.zeros(self.words, dtype=torch.int32, device=f"cuda:{ctx.device}")

    def verify(self, mode: int = _lib.MODE_IS_VALID):
        """Every chunk verified into its slice of the device bitmap (no host copy)."""
        off = 0
        for pb, m in zip(self.batches, self.sizes):
            pb.verify(mode, want_verdicts=False, device_bitmap_ptr=self.bitmap.data_ptr() + 4 * off)
            off += (m + 31) // 32
        return self.bitmap

    def allgather(self, out=None, ordered=None, group=None):
        """C1: the global accept bitmap in index order (``gather_ordered`` over the
        backlog's ``bounds``; without bounds, equal shards of ``words`` words each are
        assumed and the gathered words are returned as they are)."""
        import torch
        import torch.distributed as dist
        if self.bounds is not None:
            return gather_ordered(self.bitmap, self.bounds, out, ordered, group, n_local=self.n)
        world = dist.get_world_size(group)
        if out is None:
            out = torch.zeros(self.words * world, dtype=torch.int32, device=self.bitmap.device)
        dist.all_gather_into_tensor(out, self.bitmap, group=group)
        return out

    def close(self):
        for pb in self.batches:
            pb.close()
        self.batches = []


# status word of a rank whose verify raised something other than CordaGpuError
STATUS_EXCEPTION = -1000


class ShardFailure(RuntimeError):
    """No rank could verify some index range (every rank failed, or a rank failed again
    on the range redistributed to it)."""


def redistribute(bounds: list[int], failed: list[int], survivors: list[int]) -> dict[int, list[tuple[int, int]]]:
    """Each failed rank's index range [b_f, b_f+1) re-split over the surviving ranks with
    ``shard_bounds`` (32-aligned inside the range, so every piece owns whole bitmap words):
    {survivor: [(lo, hi), ...]} in failed-rank order."""
    plan: dict[int, list[tuple[int, int]]] = {s: [] for s in survivors}
    for f in failed:
        lo, hi = bounds[f], bounds[f + 1]
        sub = shard_bounds(hi - lo, len(survivors))
        for j, s in enumerate(survivors):
            if sub[j + 1] > sub[j]:
                plan[s].append((lo + sub[j], lo + sub[j + 1]))
    return plan


def _gather_status(code: int, world: int, device, group=None) -> list[int]:
    import torch
    import torch.distributed as dist
    out = torch.zeros(world, dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(out, torch.tensor([code], dtype=torch.int32, device=device), group=group)
    return [int(x) for x in out.cpu()]


def verify_sharded_resilient(n: int, verify, group=None, device="cpu", bounds: list[int] | None = None):
    """Sharded verification that survives a failing rank (SURVEY §5 "per-GPU error →
    re-run that shard on the remaining GPUs"; the reference's analogue is the verifier
    redistribution of VerifierTests.kt:74-100).

    ``verify(lo, hi)`` verifies elements [lo, hi) on this rank's device and returns their
    accept words (``pack_bits``, uint32); it raises ``_lib.CordaGpuError`` when the library
    returns a status < 0 (device or allocation failure).  Steps:

    1. every rank verifies its shard ``bounds[r]..bounds[r+1]`` (default ``shard_bounds``);
    2. the ranks exchange one status word each (a world-sized all-gather);
    3. each failed rank's range is re-split over the survivors (``redistribute``) and
       verified there — a failed rank takes no further work, but stays in the collectives
       so no rank blocks, and the caller exits it non-zero (nothing re-execs);
    4. ONE bitmap all-gather of every rank's pieces (equal padded pieces, as
       ``gather_ordered``), placed at word lo/32 of the index-ordered global bitmap.

    Without failures this is ``gather_ordered`` plus the status word.  A second failure
    during redistribution raises ``ShardFailure`` on every rank (they agree through a
    second status exchange).  Any other exception ``verify`` raises on a rank (a wrong word
    count, ``MemoryError``, a torch / HIP ``RuntimeError``) fails that rank the same way —
    status ``STATUS_EXCEPTION``, its range redistributed — and is re-raised on that rank
    only after the last collective, so no rank is left waiting in one.  Returns (global
    bitmap as an int32 tensor on ``device``, the failed ranks)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    bounds = bounds if bounds is not None else shard_bounds(n, world)
    check_bounds(bounds, world)
    pieces: list[tuple[int, int, np.ndarray]] = []
    kept: list[BaseException] = []

    def attempt(lo, hi) -> int:
        if hi == lo:
            pieces.append((lo, hi, np.zeros(0, np.uint32)))
            return 0
        try:
            w = np.asarray(verify(lo, hi), dtype=np.uint32)
            if len(w) != (hi - lo + 31) // 32:
                raise ValueError(f"verify({lo}, {hi}) returned {len(w)} words")
        except _lib.CordaGpuError as e:
            return e.status if e.status != 0 else -1
        except Exception as e:  # noqa: BLE001 — kept, re-raised after the collectives
            kept.append(e)
            return STATUS_EXCEPTION
        pieces.append((lo, hi, w))
        return 0

    def reraise_kept(exc: BaseException | None = None):
        if kept:
            raise kept[0] from exc
        if exc is not None:
            raise exc

    status = _gather_status(attempt(bounds[rank], bounds[rank + 1]), world, device, group)
    failed = [r for r in range(world) if status[r] != 0]
    survivors = [r for r in range(world) if status[r] == 0]
    plan: dict[int, list[tuple[int, int]]] = {}
    if failed:
        if not survivors:
            reraise_kept(ShardFailure(f"every rank failed (status {status})"))
        plan = redistribute(bounds, failed, survivors)
        code = 0
        for lo, hi in plan.get(rank, []) if rank in survivors else []:
            code = code or attempt(lo, hi)
        again = _gather_status(code, world, device, group)
        if any(again):
            reraise_kept(ShardFailure(f"redistributed ranges failed again (status {again})"))
    layout = {r: ([(bounds[r], bounds[r + 1])] if status[r] == 0 else []) + plan.get(r, []) for r in range(world)}
    nwords = {r: sum((hi - lo + 31) // 32 for lo, hi in layout[r]) for r in range(world)}
    wmax = max(max(nwords.values()), 1)
    local = torch.zeros(wmax, dtype=torch.int32, device=device)
    pos = 0
    for lo, hi, w in pieces:  # (appended in layout order: the own shard, then the plan's pieces)
        local[pos:pos + len(w)] = torch.from_numpy(w.view(np.int32).copy()).to(device)
        pos += len(w)
    out = torch.empty(world * wmax, dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(out, local, group=group)
    ordered = torch.zeros((bounds[-1] + 31) // 32, dtype=torch.int32, device=device)
    for r in range(world):
        at = r * wmax
        for lo, hi in layout[r]:
            k = (hi - lo + 31) // 32
            ordered[lo // 32:lo // 32 + k] = out[at:at + k]
            at += k
    reraise_kept()  # this rank's own exception, now that every collective is done
    return ordered, failed


def gpu_shard_verifier(ctx: _lib.Context, batch: PackedBatch, mode: int = _lib.MODE_IS_VALID):
    """``verify(lo, hi)`` for ``verify_sharded_resilient`` on this rank's context: stages
    elements [lo, hi) of ``batch`` (``slice_batch``) and verifies them through the C ABI."""
    def verify(lo: int, hi: int) -> np.ndarray:
        pb = PreparedBatch(ctx, slice_batch(batch, lo, hi))
        try:
            return pack_bits(pb.verify(mode) == _lib.ACCEPT)[:(hi - lo + 31) // 32]
        finally:
            pb.close()
    return verify
