"""Where the time of one host-buffer verify call goes, on the GPU box:

    python tools/e2e_timeline.py [--sizes 4096,65536,262144] [--out gpurun_out/e2e_timeline.txt]

Runs cg_verify_batch on config-2 elements (Ed25519, 1 KB messages, the compact
Ed25519-only layout) with the library's per-span HIP events on and
CORDA_AMD_TIMELINE naming the output file, so every copy / staging / kernel span of
the call is written with its start and end (ms from the call's first span); the
summary (tools/timeline.py) of the last call of each size follows on stdout, with
the call's host wall time.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,65536,262144")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "e2e_timeline.txt"))
    ap.add_argument("--pinned", action="store_true")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    os.environ["CORDA_AMD_TIMELINE"] = a.out  # read once by the library, before the first call
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import MODE_IS_VALID
    sizes = [int(x) for x in a.sizes.split(",")]
    w = datagen.make_batch(max(sizes), msg_bytes=1024, seed=42, key_base=0, ref_seed_stride=4096)
    with Context(0) as ctx:
        for n in sizes:
            s = w.subset(np.arange(n))
            b = crypto.PackedBatch(s.n, None, np.ascontiguousarray(s.pk[:, :32]), 32,
                                   np.ascontiguousarray(s.sig[:, :64]), 64, None, s.msg, s.msg_off, s.msg_len)
            if a.pinned:
                ctx.register_host(b.pk, b.sig, b.msg, b.msg_off, b.msg_len)
            for _ in range(3):
                crypto.verify_packed(ctx, b, MODE_IS_VALID)
            if os.path.exists(a.out):
                os.remove(a.out)
            ctx.set_profiling(True)
            t0 = time.perf_counter()
            crypto.verify_packed(ctx, b, MODE_IS_VALID)
            wall = (time.perf_counter() - t0) * 1e3
            ctx.set_profiling(False)
            if a.pinned:
                ctx.unregister_host(b.pk, b.sig, b.msg, b.msg_off, b.msg_len)
            print(f"== n={n} pinned={a.pinned} wall {wall:.3f} ms (profiling on)", flush=True)
            if os.path.exists(a.out):
                subprocess.run([sys.executable, os.path.join(ROOT, "tools", "timeline.py"), a.out], check=False)


if __name__ == "__main__":
    main()
