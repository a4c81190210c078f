"""Why does the bench's back-to-back p50 loop of host-buffer calls measure slower than its
host_share loop over the same batch?  Runs the 32 B bench layout (bench.e2e_record_32b's
rows) under several call patterns, interleaved, and prints the medians.

    python tools/e2e_pattern.py [--sizes 65536,262144] [--runs 21] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))
import bench  # noqa: E402


def rows_32b(w, m):
    from corda_amd import crypto
    sub = w.subset(np.arange(m))
    sl = sub.sig_len[:m].astype(np.uint32)
    ragged = bool((sl != 64).any())
    ss = max(64, (int(sl.max()) + 3) // 4 * 4) if ragged else 64
    sg = np.zeros((m, ss), dtype=np.uint8)
    sg[:, :min(ss, sub.sig_stride)] = sub.sig[:m, :min(ss, sub.sig_stride)]
    return crypto.PackedBatch(m, None, np.ascontiguousarray(sub.pk[:, :32]), 32, sg, ss,
                              np.ascontiguousarray(sl) if ragged else None, sub.msg, sub.msg_off, sub.msg_len)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,262144")
    ap.add_argument("--runs", type=int, default=21)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import MODE_IS_VALID
    sizes = [int(s) for s in a.sizes.split(",")]
    w = datagen.make_batch(max(sizes), msg_bytes=32, seed=4242, key_base=1 << 36, threads=bench.cpu_threads(),
                           ref_seed_stride=4096)
    w = datagen.add_ed25519_adversarial(w, frac=0.01, seed=77)
    res = {}
    with Context(0) as ctx:
        for m in sizes:
            sb = rows_32b(w, m)
            call = lambda: crypto.verify_packed(ctx, sb, MODE_IS_VALID)  # noqa: E731
            for _ in range(3):
                call()

            def loop(pre=None, post=None):
                ts = []
                for _ in range(a.runs):
                    if pre:
                        pre()
                    t0 = time.perf_counter()
                    call()
                    ts.append((time.perf_counter() - t0) * 1e3)
                    if post:
                        post()
                return round(statistics.median(ts), 3)

            def prof_loop(level, stats):
                ctx.set_profiling(level)
                try:
                    return loop(ctx.reset_stats if stats else None,
                                (lambda: ctx.kernel_stats("call")) if stats else None)
                finally:
                    ctx.set_profiling(False)

            pats = {
                "back_to_back": lambda: loop(),
                "sleep_1ms_between": lambda: loop(post=lambda: time.sleep(1e-3)),
                "profiling2_with_stats": lambda: prof_loop(2, True),
                "profiling2_no_stats": lambda: prof_loop(2, False),
                "reset_stats_only": lambda: loop(ctx.reset_stats, lambda: ctx.kernel_stats("call")),
            }
            got = {k: [] for k in pats}
            for _ in range(a.rounds):
                for k, f in pats.items():
                    got[k].append(f())
            res[m] = got
            print(m, json.dumps(got), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
