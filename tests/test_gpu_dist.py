"""Sharded verification on the GPU through torch.distributed over RCCL
("nccl" backend), world size 1 on the test box (the 8-GPU run is the driver's):
the device accept bitmap produced by cg_batch_verify feeds the all-gather
directly and equals the verdicts."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))

pytestmark = pytest.mark.gpu


def test_verify_sharded_rccl_world1(gpu_ctx):
    import torch
    import torch.distributed as dist
    import datagen
    from corda_amd import dist as D
    from corda_amd.crypto import PackedBatch
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(gpu_ctx.device)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        w = datagen.add_ed25519_adversarial(datagen.make_batch(5000 + 13, msg_bytes=64, seed=6), 0.1, seed=6)
        b = PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                        w.msg_len)
        v, glob, bounds = D.verify_sharded(gpu_ctx, b, 0, 1)
        assert bounds == [0, w.n]
        exp = D.pack_bits(v == 0).view(np.int32)
        assert np.array_equal(glob.cpu().numpy(), exp)
    finally:
        dist.destroy_process_group()


def test_backlog_chunks_into_one_device_bitmap_world1(gpu_ctx, oracle):
    """Config 5's chunked path (corda_amd.dist.ShardBacklog, what bench.py
    --workload backlog runs): several PreparedBatch chunks verified into consecutive
    word slices of ONE device bitmap, then the RCCL all-gather; compared bit for bit
    with the oracle's verdicts of the whole shard (32-aligned chunks + a ragged last)."""
    import torch
    import torch.distributed as dist
    import datagen
    from corda_amd import dist as D
    from corda_amd.crypto import PackedBatch
    from test_gpu_ed25519 import oracle_verdicts
    n = 50_013
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=32, seed=17, key_base=31337), 0.05, seed=8)
    full = PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                       w.msg_len)
    with pytest.raises(ValueError):
        D.ShardBacklog(gpu_ctx, [D.slice_batch(full, 0, 100), D.slice_batch(full, 100, 200)])
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(gpu_ctx.device)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        chunk = 8192
        bl = D.ShardBacklog(gpu_ctx, (D.slice_batch(full, c, min(n, c + chunk)) for c in range(0, n, chunk)))
        assert bl.sizes[:-1] == [chunk] * (len(bl.sizes) - 1) and bl.n == n
        bl.verify()
        glob = bl.allgather()
        exp = D.pack_bits(oracle_verdicts(oracle, w, 0) == 0).view(np.int32)
        assert np.array_equal(glob.cpu().numpy()[:len(exp)], exp)
        bl.close()
    finally:
        dist.destroy_process_group()


def test_wrong_length_keys_stay_key_invalid_on_every_path(gpu_ctx, oracle):
    """Keys of the wrong length (31 / 33 bytes) cannot be PublicKey objects: pack() flags
    them in the scheme id (CG_SCHEME_FLAG_KEY_INVALID) and the library reports KEY_INVALID
    for them on every path — verify_packed and its bitmap, a PreparedBatch (host verdicts
    and the device bitmap), and verify_sharded over RCCL — with several of them in one
    32-element bitmap word, and never verifies them against a zero key."""
    import torch
    import torch.distributed as dist
    import datagen
    from corda_amd import crypto
    from corda_amd import dist as D
    from corda_amd._lib import KEY_INVALID, MODE_DO_VERIFY, MODE_IS_VALID
    from test_gpu_ed25519 import oracle_verdicts
    w = datagen.add_ed25519_adversarial(datagen.make_batch(300, msg_bytes=50, seed=91, key_base=9100), 0.1, seed=3)
    keys = [bytes(w.pk[i, :32]) for i in range(w.n)]
    bad = [0, 1, 3, 31, 40, 299]
    for j, i in enumerate(bad):
        keys[i] = keys[i][:31] if j % 2 == 0 else keys[i] + b"\0"
    sigs = [bytes(w.sig[i, :w.sig_len[i]]) for i in range(w.n)]
    msgs = [bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]]) for i in range(w.n)]
    b = crypto.pack(crypto.EDDSA_ED25519_SHA512, keys, sigs, msgs)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        exp[bad] = KEY_INVALID
        v, bm = crypto.verify_packed(gpu_ctx, b, mode, bitmap=True)
        assert np.array_equal(v, exp)
        assert np.array_equal(bm.view(np.int32), D.pack_bits(exp == 0).view(np.int32))
        pb = crypto.PreparedBatch(gpu_ctx, b)
        dev = torch.zeros((w.n + 31) // 32, dtype=torch.int32, device=f"cuda:{gpu_ctx.device}")
        assert np.array_equal(pb.verify(mode, device_bitmap_ptr=dev.data_ptr()), exp)
        assert np.array_equal(dev.cpu().numpy(), D.pack_bits(exp == 0).view(np.int32))
        pb.close()
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(gpu_ctx.device)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
        exp[bad] = KEY_INVALID
        v, glob, _ = D.verify_sharded(gpu_ctx, b, 0, 1)
        assert np.array_equal(v, exp)
        assert np.array_equal(glob.cpu().numpy(), D.pack_bits(exp == 0).view(np.int32))
    finally:
        dist.destroy_process_group()


def _gpu_resilient_worker(rank, world, port, n, fail_rank, q):
    """One rank on the test box's single GPU (its own cg context on device 0; the
    collectives over gloo, since RCCL needs one GPU per rank): verify_sharded_resilient
    with the GPU verifier; fail_rank's context injects an allocation failure
    (CG_DEBUG_FAIL_ALLOC), so its cg_batch_create returns CG_E_OUT_OF_MEMORY."""
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import datagen
    from corda_amd import Context
    from corda_amd import dist as D
    from corda_amd._lib import DEBUG_FAIL_ALLOC
    from corda_amd.crypto import PackedBatch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    code = 0
    try:
        w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=64, seed=19, key_base=77_000), 0.1, seed=9)
        b = PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                        w.msg_len)
        with Context(0) as ctx:
            if rank == fail_rank:
                ctx.set_debug(DEBUG_FAIL_ALLOC, 1)
            glob, failed = D.verify_sharded_resilient(n, D.gpu_shard_verifier(ctx, b))
        q.put((rank, glob.numpy().tobytes(), failed))
        code = 3 if rank in failed else 0
    finally:
        dist.destroy_process_group()
    if code:
        os._exit(code)


def test_shard_failure_redistribution_on_gpu(oracle):
    """SURVEY §5 per-GPU failure handling on the device: three ranks share the box's GPU,
    rank 1's library fails its allocation (CG_DEBUG_FAIL_ALLOC); its index range is
    re-verified by ranks 0 and 2 through cg_batch_create / cg_batch_verify, every rank's
    gathered bitmap equals the oracle's for the whole batch, and rank 1 exits non-zero."""
    import multiprocessing as mp
    from corda_amd import dist as D
    from test_gpu_ed25519 import oracle_verdicts
    import datagen
    n = 20_000 + 21
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=64, seed=19, key_base=77_000), 0.1, seed=9)
    exp = D.pack_bits(oracle_verdicts(oracle, w, 0) == 0).view(np.int32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    procs = [ctx.Process(target=_gpu_resilient_worker, args=(r, 3, port, n, 1, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(3)), key=lambda t: t[0])
    for p in procs:
        p.join(60)
    assert [p.exitcode for p in procs] == [0, 3, 0]
    for rank, glob, failed in res:
        assert failed == [1]
        assert np.array_equal(np.frombuffer(glob, np.int32), exp), rank


def test_resilient_world1_rccl(gpu_ctx, oracle):
    """verify_sharded_resilient over RCCL at world 1 (status word and bitmap all-gathers
    on the device): equals the oracle; with the rank's allocation failing there is no
    survivor and it raises ShardFailure."""
    import torch
    import torch.distributed as dist
    import datagen
    from corda_amd import dist as D
    from corda_amd._lib import DEBUG_FAIL_ALLOC
    from corda_amd.crypto import PackedBatch
    from test_gpu_ed25519 import oracle_verdicts
    w = datagen.add_ed25519_adversarial(datagen.make_batch(3000 + 5, msg_bytes=50, seed=23, key_base=88_000), 0.1,
                                        seed=3)
    b = PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off, w.msg_len)
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(gpu_ctx.device)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        dev = f"cuda:{gpu_ctx.device}"
        glob, failed = D.verify_sharded_resilient(w.n, D.gpu_shard_verifier(gpu_ctx, b), device=dev)
        assert failed == [] and glob.device.type == "cuda"
        assert np.array_equal(glob.cpu().numpy(), D.pack_bits(oracle_verdicts(oracle, w, 0) == 0).view(np.int32))
        gpu_ctx.set_debug(DEBUG_FAIL_ALLOC, 1)
        with pytest.raises(D.ShardFailure):
            D.verify_sharded_resilient(w.n, D.gpu_shard_verifier(gpu_ctx, b), device=dev)
    finally:
        gpu_ctx.set_debug(DEBUG_FAIL_ALLOC, 0)
        dist.destroy_process_group()
