"""Multi-GPU path on CPU: world-size-2 gloo processes exercise the shard
boundaries and the verdict-bitmap all-gather (C1) that bench.py / dist.py run
over RCCL on MI355X.  Verdicts come from the C oracle here (no GPU), so the test
also proves the sharded verdict set equals the single-process one."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import ctypes

    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))
    from corda_amd import dist as D
    from corda_amd.crypto import PackedBatch
    import datagen
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=40, seed=3, threads=2), 0.2, seed=4)
        full = PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                           w.msg_len)
        bounds = D.shard_bounds(n, world)
        shard = D.slice_batch(full, bounds[rank], bounds[rank + 1])
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.oracle_verify_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, vp]
        v = np.zeros(max(shard.n, 1), np.uint8)
        P = lambda a: a.ctypes.data  # noqa: E731
        lib.oracle_verify_batch(P(shard.scheme), P(shard.pk), shard.pk_stride, P(shard.sig), shard.sig_stride,
                                P(shard.sig_len), P(shard.msg), P(shard.msg_off), P(shard.msg_len), shard.n, 0, 1,
                                P(v))
        words = torch.from_numpy(D.pack_bits(v[:shard.n] == 0).view(np.int32).copy())
        glob = D.allgather_bitmap(words, bounds, rank)
        if rank == 0:
            allv = np.zeros(n, np.uint8)
            lib.oracle_verify_batch(P(full.scheme), P(full.pk), full.pk_stride, P(full.sig), full.sig_stride,
                                    P(full.sig_len), P(full.msg), P(full.msg_off), P(full.msg_len), n, 0, 2, P(allv))
            exp = D.pack_bits(allv == 0).view(np.int32)
            q.put(bool(np.array_equal(glob.numpy(), exp)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 4096 + 17])
def test_two_rank_sharded_bitmap_allgather(n):
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_shard_bounds():
    from corda_amd.dist import shard_bounds
    for n in (0, 1, 31, 32, 1000, 10**6 + 7):
        for world in (1, 2, 3, 8):
            b = shard_bounds(n, world)
            assert b[0] == 0 and b[-1] == n and len(b) == world + 1
            assert all(b[i] <= b[i + 1] for i in range(world))
            assert all(x % 32 == 0 for x in b[1:-1])


def test_check_bounds_rejects_mismatched_shards():
    """gather_ordered's validation (a bad bounds list would misplace words silently)."""
    from corda_amd.dist import check_bounds, shard_bounds
    b = shard_bounds(1000, 3)
    check_bounds(b, 3)
    check_bounds(b, 3, n_local=b[2] - b[1], rank=1)
    for bad, world, kw in ((b, 2, {}), ([32] + b[1:], 3, {}), ([0, 64, 32, 1000], 3, {}), ([0, 33, 64, 1000], 3, {}),
                           (b, 3, {"n_local": b[1] + 1, "rank": 0})):
        with pytest.raises(ValueError):
            check_bounds(bad, world, **kw)


def test_pack_bits_matches_device_layout():
    from corda_amd.dist import pack_bits
    m = np.zeros(70, bool)
    m[[0, 5, 31, 32, 69]] = True
    w = pack_bits(m)
    assert w.dtype == np.uint32 and len(w) == 3
    assert w[0] == (1 | 1 << 5 | 1 << 31) and w[1] == 1 and w[2] == 1 << 5


def test_cost_weighted_shards_balance_mixed_batches():
    """Mixed Ed25519 / ECDSA batches split by device cost, not count: the
    per-rank cost differs by at most one aligned block from the ideal share, every
    interior boundary is a multiple of 32, and a uniform batch splits like shard_bounds."""
    from corda_amd import dist as D
    rng = np.random.default_rng(3)
    # ECDSA clustered at the end (config 3 / 4 layouts put curves in runs)
    scheme = np.concatenate([np.full(60_000, 4), rng.choice([2, 3], 40_000)]).astype(np.uint8)
    for world in (2, 3, 8):
        b = D.shard_bounds_weighted(scheme, world)
        assert b[0] == 0 and b[-1] == len(scheme) and all(x % 32 == 0 for x in b[1:-1])
        costs = [sum(D.SCHEME_COST[int(s)] for s in scheme[b[r]:b[r + 1]]) for r in range(world)]
        ideal = sum(costs) / world
        assert max(costs) - ideal <= 32 * max(D.SCHEME_COST.values()) + 1e-6
        counts = np.diff(b)
        assert counts[-1] < counts[0]  # the ECDSA-heavy tail gets fewer elements
    same = np.full(10_000, 4, np.uint8)
    assert D.shard_bounds_weighted(same, 4) == D.shard_bounds(10_000, 4)


def _gather_worker(rank, world, port, total, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from corda_amd import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        accept = rng.random(total) < 0.9  # the same global verdicts on every rank
        bounds = D.shard_bounds(total, world)
        lo, hi = bounds[rank], bounds[rank + 1]
        wmax = max((bounds[r + 1] - bounds[r] + 31) // 32 for r in range(world))
        local = torch.zeros(wmax + 3, dtype=torch.int32)  # longer than needed, like a padded device bitmap
        mine = D.pack_bits(accept[lo:hi]).view(np.int32)
        local[:len(mine)] = torch.from_numpy(mine.copy())
        glob = D.gather_ordered(local, bounds)
        q.put((rank, bool(np.array_equal(glob.numpy(), D.pack_bits(accept).view(np.int32)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(3, 100_003), (3, 96), (2, 33), (8, 100_003), (8, 1000), (8, 100)])
def test_gather_ordered_uneven_shards(world, total):
    """ShardBacklog.allgather's collective (dist.gather_ordered) at world 3 with uneven
    32-aligned shards: one all_gather_into_tensor of equal padded pieces, then every rank's
    words moved to word bounds[r]/32 — the global bitmap equals pack_bits of the global
    verdicts on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    res = sorted(q.get(timeout=5) for _ in range(world))
    assert res == [(r, True) for r in range(world)]


def _resilient_worker(rank, world, port, n, fail_ranks, fail_again, q, fail_kind="gpu"):
    """One rank of verify_sharded_resilient over gloo; verify() is the C oracle on the
    rank's slice, and ranks in fail_ranks raise the error a failing cg_batch_verify
    raises (CordaGpuError, status < 0).  fail_again: a survivor that also fails on its
    redistributed piece.  Exit code 3 for a failed rank (the caller's contract)."""
    import ctypes
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))
    from corda_amd import _lib
    from corda_amd import dist as D
    from corda_amd.crypto import PackedBatch
    import datagen
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    code = 0
    try:
        w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=40, seed=5, threads=2), 0.2, seed=6)
        full = PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                           w.msg_len)
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.oracle_verify_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, vp]
        P = lambda a: a.ctypes.data  # noqa: E731
        calls = []

        def verify(lo, hi):
            calls.append((lo, hi))
            if rank in fail_ranks or (rank == fail_again and len(calls) > 1):
                if fail_kind == "runtime":
                    raise RuntimeError("HIP error: injected")
                if fail_kind != "words":
                    raise _lib.CordaGpuError(-3, "injected allocation failure (CG_DEBUG_FAIL_ALLOC)")
            s = D.slice_batch(full, lo, hi)
            v = np.zeros(max(s.n, 1), np.uint8)
            lib.oracle_verify_batch(P(s.scheme), P(s.pk), s.pk_stride, P(s.sig), s.sig_stride, P(s.sig_len),
                                    P(s.msg), P(s.msg_off), P(s.msg_len), s.n, 0, 1, P(v))
            words = D.pack_bits(v[:s.n] == 0)
            return words[:-1] if fail_kind == "words" and rank in fail_ranks else words

        try:
            glob, failed = D.verify_sharded_resilient(n, verify)
        except D.ShardFailure:
            q.put((rank, "ShardFailure", calls))
            return
        except (RuntimeError, ValueError) as e:  # the rank's own verify exception, after the collectives
            q.put((rank, type(e).__name__, calls))
            q.close()
            q.join_thread()  # flushed before the hard exit
            dist.destroy_process_group()
            os._exit(3)
        allv = np.zeros(n, np.uint8)
        lib.oracle_verify_batch(P(full.scheme), P(full.pk), full.pk_stride, P(full.sig), full.sig_stride,
                                P(full.sig_len), P(full.msg), P(full.msg_off), P(full.msg_len), n, 0, 2, P(allv))
        ok = bool(np.array_equal(glob.numpy(), D.pack_bits(allv == 0).view(np.int32)))
        q.put((rank, ok, failed, calls))
        code = 3 if rank in failed else 0
    finally:
        dist.destroy_process_group()
    if code:
        os._exit(code)


def _run_resilient(world, n, fail_ranks, fail_again=-1, fail_kind="gpu"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resilient_worker, args=(r, world, port, n, fail_ranks, fail_again, q, fail_kind))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = sorted((q.get(timeout=5) for _ in range(world)), key=lambda t: t[0])
    return [p.exitcode for p in procs], res


@pytest.mark.parametrize("world,n,fail", [(3, 3000, (1,)), (3, 2017, (2,)), (3, 4096 + 33, (0, 2)), (2, 777, ()),
                                         (8, 20_000 + 17, (3, 6))])
def test_shard_failure_redistributes_to_survivors(world, n, fail):
    """verify_sharded_resilient at world 3 (and 2, and the driver's 8) over gloo with one or two ranks whose
    verify fails (the CordaGpuError a cg_batch_verify returning < 0 raises, as
    CG_DEBUG_FAIL_ALLOC injects on the GPU): each failed range is re-split over the
    survivors, the gathered bitmap equals the oracle's for the whole batch on EVERY rank,
    survivors verified their own shard plus their piece of each failed range (32-aligned),
    and the failed ranks exit non-zero while the survivors exit 0."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built")
    codes, res = _run_resilient(world, n, set(fail))
    assert [r[1] for r in res] == [True] * world, res
    assert all(r[2] == list(fail) for r in res)
    assert codes == [3 if r in fail else 0 for r in range(world)]
    from corda_amd import dist as D
    b = D.shard_bounds(n, world)
    survivors = [r for r in range(world) if r not in fail]
    plan = D.redistribute(b, list(fail), survivors)
    covered = []
    for r, _, _, calls in res:
        if r in fail:
            assert calls == [(b[r], b[r + 1])]
        else:
            assert calls == [(b[r], b[r + 1])] + plan[r]
            covered += calls
    covered.sort()
    assert covered[0][0] == 0 and covered[-1][1] == n and all(x[1] == y[0] for x, y in zip(covered, covered[1:]))
    assert all(lo % 32 == 0 for lo, _ in covered)


def test_shard_failure_twice_raises_everywhere():
    """A survivor that also fails on its redistributed piece: every rank raises
    ShardFailure (they agree through the second status exchange; none blocks)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built")
    codes, res = _run_resilient(3, 3000, {1}, fail_again=2)
    assert [r[1] for r in res] == ["ShardFailure"] * 3 and codes == [0, 0, 0]


@pytest.mark.parametrize("kind,exc", [("runtime", "RuntimeError"), ("words", "ValueError")])
def test_shard_failure_other_exceptions_do_not_block(kind, exc):
    """A rank whose verify raises something other than CordaGpuError — a torch / HIP
    RuntimeError, or a wrong accept-word count (ValueError) — fails like a device
    failure: its range goes to the survivors, who get the oracle's bitmap, and the
    rank re-raises its own exception only after the last collective (no rank blocks)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built")
    codes, res = _run_resilient(3, 3000, {1}, fail_kind=kind)
    assert res[0][1] is True and res[2][1] is True and res[0][2] == [1] and res[2][2] == [1], res
    assert res[1][1] == exc, res
    assert codes == [0, 3, 0]
