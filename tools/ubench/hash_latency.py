"""Latency of the Ed25519 hash kernel at a serving-size call (4,096 signatures, one wave
per SIMD), by message size, with and without the half-size reduction (the
cg_set_debug hook forcing (c0, c1) = (h, 1) on every lane skips it): what part of the
kernel's chain is SHA-512 and what part the scalar work.  Library HIP events; JSON."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))


def main():
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import DEBUG_FORCE_FULL_LENGTH, MODE_IS_VALID
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    out = {"n": n}
    with Context(0) as ctx:
        for mb in (32, 1024):
            w = datagen.make_batch(n, msg_bytes=mb, seed=5, key_base=0)
            b = crypto.PackedBatch(w.n, None, np.ascontiguousarray(w.pk[:, :32]), 32,
                                   np.ascontiguousarray(w.sig[:, :64]), 64, None, w.msg, w.msg_off, w.msg_len)
            for full in (0, 1):
                ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, full)
                for _ in range(3):
                    crypto.verify_packed(ctx, b, MODE_IS_VALID)
                ctx.set_profiling(True)
                ctx.reset_stats()
                for _ in range(20):
                    crypto.verify_packed(ctx, b, MODE_IS_VALID)
                ms, launches, _ = ctx.kernel_stats("ed25519_hash")
                ctx.set_profiling(False)
                out[f"hash_ms_{mb}B_{'full' if full else 'half'}"] = round(ms / max(launches, 1), 4)
            ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
