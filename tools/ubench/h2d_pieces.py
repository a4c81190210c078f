"""What does the copy pipeline of a 262,144 x 1 KB host verify pay per DMA?  Times pageable
host->device copies of the same bytes cut the ways cg_verify_batch could cut them:

    one      the whole arena + rows as one copy each (the floor)
    chunked  the pipeline's pattern: 8 chunks (head / tail 0.25), each its arena piece then five row arrays
    upfront  the five row arrays for the whole call first, then the 8 arena pieces
    arena8   the 8 arena pieces alone

    python tools/ubench/h2d_pieces.py [--n 262144] [--msg 1024] [--reps 7] [--out f.json]

Copies go through the HIP runtime torch has loaded (hipMemcpyAsync on one stream, wall time
to hipStreamSynchronize), from pageable numpy buffers like the bench's.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import time

import numpy as np
import torch


def hip_lib():
    torch.cuda.init()
    with open("/proc/self/maps") as f:
        paths = {l.split()[-1] for l in f if "libamdhip64" in l}
    return ctypes.CDLL(sorted(paths)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--msg", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    hip = hip_lib()
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    n, m = a.n, a.msg
    arena = np.random.default_rng(1).integers(0, 256, n * m, dtype=np.uint8)
    rows = {"off": np.arange(n, dtype=np.uint64) * m, "len": np.full(n, m, np.uint32),
            "pk": np.zeros((n, 32), np.uint8), "sig": np.zeros((n, 68), np.uint8), "sl": np.full(n, 64, np.uint32)}
    per = {k: v.nbytes // n for k, v in rows.items()}
    total = arena.nbytes + sum(v.nbytes for v in rows.values())
    dev = torch.empty(total + 4096, dtype=torch.uint8, device="cuda")
    base = dev.data_ptr()
    stream = torch.cuda.current_stream().cuda_stream
    K, head = 8, 0.25
    reg = n / (K - 2 + 2 * head)
    cuts = [0]
    for k in range(K):
        cuts.append(min(n, int(round(cuts[-1] + (head if k in (0, K - 1) else 1.0) * reg))))
    cuts[-1] = n

    def cp(dst_off, host, lo_b, nb):
        if nb:
            assert hip.hipMemcpyAsync(base + dst_off, host.ctypes.data + lo_b, nb, 1, stream) == 0

    roff = {}
    o = arena.nbytes
    for k, v in rows.items():
        roff[k] = o
        o += v.nbytes

    def rows_range(lo, hi):
        for k, v in rows.items():
            cp(roff[k] + lo * per[k], v, lo * per[k], (hi - lo) * per[k])

    pats = {
        "one": lambda: (cp(0, arena, 0, arena.nbytes), rows_range(0, n)),
        "chunked": lambda: [(cp(cuts[k] * m, arena, cuts[k] * m, (cuts[k + 1] - cuts[k]) * m),
                             rows_range(cuts[k], cuts[k + 1])) for k in range(K)],
        "upfront": lambda: (rows_range(0, n), [cp(cuts[k] * m, arena, cuts[k] * m, (cuts[k + 1] - cuts[k]) * m)
                                               for k in range(K)]),
        "arena8": lambda: [cp(cuts[k] * m, arena, cuts[k] * m, (cuts[k + 1] - cuts[k]) * m) for k in range(K)],
    }
    res = {}
    for _ in range(2):
        for name, f in pats.items():
            f()
            hip.hipStreamSynchronize(stream)
    for name, f in pats.items():
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            f()
            hip.hipStreamSynchronize(stream)
            ts.append((time.perf_counter() - t0) * 1e3)
        nb = arena.nbytes if name == "arena8" else total
        res[name] = {"p50_ms": round(statistics.median(ts), 3), "min_ms": round(min(ts), 3),
                     "GBps_p50": round(nb / statistics.median(ts) / 1e6, 1), "bytes": nb}
        print(name, res[name], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"n": n, "msg": m, "chunks": cuts, "patterns": res}, f, indent=1)


if __name__ == "__main__":
    main()
