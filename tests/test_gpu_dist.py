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
