"""End-to-end (host buffers in, verdicts out) latency of cg_verify_batch over its
pipeline settings, on the GPU box:

    python tools/e2e_sweep.py [--out gpurun_out/e2e_sweep.json]

For each batch size (config-2 elements: Ed25519, 1 KB messages, distinct keys) and
each setting of CORDA_AMD_VERIFY_CHUNKS / _MIN_CHUNK / _HEAD / _TAIL / _RING (set on the
context with cg_set_option), the p50 of 15 calls after 3 warm-ups; also the same with the
input buffers page-locked (cg_register_host) and the raw pageable / pinned H2D rates,
so every p50 can be put against the PCIe bound of its bytes.
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

SETTINGS = [
    {"CORDA_AMD_VERIFY_CHUNKS": "1"},
    {},  # library defaults
    {"CORDA_AMD_VERIFY_RING": "0"},
] + [dict({"CORDA_AMD_VERIFY_CHUNKS": str(k), "CORDA_AMD_VERIFY_MIN_CHUNK": "1024", "CORDA_AMD_VERIFY_HEAD": str(h),
           "CORDA_AMD_VERIFY_TAIL": str(t)}, **extra)
     for k, h, t in ((2, 0.5, 0.5), (3, 0.5, 0.5), (4, 0.5, 0.5), (4, 1, 0.5), (6, 0.5, 0.5), (6, 1, 0.5),
                     (8, 0.5, 0.5))
     for extra in ({}, {"CORDA_AMD_VERIFY_RING": "0"})]
KEYS = ("CORDA_AMD_VERIFY_CHUNKS", "CORDA_AMD_VERIFY_MIN_CHUNK", "CORDA_AMD_VERIFY_HEAD", "CORDA_AMD_VERIFY_TAIL",
        "CORDA_AMD_VERIFY_SERIAL", "CORDA_AMD_VERIFY_RING", "CORDA_AMD_ED_PAIR_MAX", "CORDA_AMD_ED_QUAD_MAX", "CORDA_AMD_ED_OCT_MAX", "CORDA_AMD_VERIFY_ONE_DMA",
        "CORDA_AMD_VERIFY_LANES", "CORDA_AMD_VERIFY_POLICY", "CORDA_AMD_COPY_THREADS", "CORDA_AMD_ARENA_BESIDE")


def h2d_rates(mb=256):
    import torch
    src = np.random.default_rng(1).integers(0, 255, mb << 20, dtype=np.uint8)
    dst = torch.empty(mb << 20, dtype=torch.uint8, device="cuda")
    out = {}
    for name, t in (("pageable", torch.from_numpy(src)), ("pinned", torch.from_numpy(src).pin_memory())):
        dst.copy_(t)
        torch.cuda.synchronize()
        best = 0.0
        for _ in range(5):
            t0 = time.perf_counter()
            dst.copy_(t)
            torch.cuda.synchronize()
            best = max(best, (mb << 20) / (time.perf_counter() - t0) / 1e9)
        out[name] = round(best, 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "e2e_sweep.json"))
    ap.add_argument("--sizes", default="4096,16384,65536,262144")
    ap.add_argument("--runs", type=int, default=15)
    ap.add_argument("--grid", default=None,
                    help="settings to try instead of the built-in list: ';'-separated, each ','-separated "
                         "VAR=value pairs ('' = library defaults), e.g. 'CORDA_AMD_VERIFY_HEAD=0.25;'")
    ap.add_argument("--pageable-only", action="store_true")
    ap.add_argument("--msg-bytes", type=int, default=1024, help="message length (32: the production tx-id shape)")
    ap.add_argument("--spans", action="store_true", help="also one profiled call per row: bench.e2e_spans")
    ap.add_argument("--timeline", action="store_true", help="with --spans: every span of that call, in start order")
    ap.add_argument("--bench-layout", action="store_true",
                    help="the driver bench line's layout: 1 %% adversarial (E1-E12), ragged E12 rows with sig_len, "
                         "signature stride 68 (bench.py e2e_record_32b / latency)")
    ap.add_argument("--adversarial", type=float, default=None, help="with --bench-layout: this fraction instead of 1 %%")
    ap.add_argument("--adv-classes", default=None, help="with --bench-layout: keep only these classes mutated "
                                                        "(comma-separated, e.g. E12); the other mutated rows are re-signed valid")
    ap.add_argument("--force-ragged", action="store_true", help="sig_len array and stride 68 even if every row is 64 B")
    a = ap.parse_args()
    if a.spans:
        import tempfile
        os.environ.setdefault("CORDA_AMD_TIMELINE", os.path.join(tempfile.gettempdir(), f"e2e_sweep_{os.getpid()}.txt"))
    settings = SETTINGS if a.grid is None else [
        dict(kv.split("=", 1) for kv in g.split(",") if kv) for g in a.grid.split(";")]
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import ACCEPT, MODE_IS_VALID
    sizes = [int(x) for x in a.sizes.split(",")]
    w = datagen.make_batch(max(sizes), msg_bytes=a.msg_bytes, seed=42, key_base=0, ref_seed_stride=4096)
    if a.bench_layout:
        clean = datagen.make_batch(max(sizes), msg_bytes=a.msg_bytes, seed=42, key_base=0, ref_seed_stride=4096) \
            if a.adv_classes else None
        w = datagen.add_ed25519_adversarial(w, frac=0.01 if a.adversarial is None else a.adversarial, seed=77)
        if a.adv_classes:  # restore every mutated row outside the kept classes
            keep = set(a.adv_classes.split(","))
            for i, c in enumerate(w.classes):
                if c != "valid" and c not in keep:
                    w.pk[i], w.sig[i], w.sig_len[i] = clean.pk[i], clean.sig[i], clean.sig_len[i]
                    o = int(w.msg_off[i])
                    w.msg[o:o + a.msg_bytes] = clean.msg[o:o + a.msg_bytes]
                    w.msg_len[i] = a.msg_bytes
                    w.classes[i] = "valid"
    res = {"h2d_GBps": h2d_rates(), "runs": a.runs, "rows": []}
    with Context(0) as ctx:
        for n in sizes:
            s = w.subset(np.arange(n))
            sl = s.sig_len[:n].astype(np.uint32)
            ragged = (a.bench_layout and bool((sl != 64).any())) or a.force_ragged
            ss = max(64, (int(sl.max()) + 3) // 4 * 4) if ragged else 64
            if a.force_ragged:
                ss = max(ss, 68)
            sg = np.zeros((n, ss), dtype=np.uint8)
            sg[:, :min(ss, s.sig_stride)] = s.sig[:n, :min(ss, s.sig_stride)]
            b = crypto.PackedBatch(s.n, None, np.ascontiguousarray(s.pk[:, :32]), 32, sg, ss,
                                   np.ascontiguousarray(sl) if ragged else None, s.msg, s.msg_off, s.msg_len)
            nbytes = sum(x.nbytes for x in (b.pk, b.sig, b.msg, b.msg_off, b.msg_len)) + (sl.nbytes if ragged else 0)
            for pinned in ((False,) if a.pageable_only else (False, True)):
                if pinned:
                    ctx.register_host(b.pk, b.sig, b.msg, b.msg_off, b.msg_len)
                for st in settings:
                    for k in set(KEYS).union(*settings):  # (cg_set_option: the context's knobs)
                        ctx.set_option(k, None)
                    for k, v in st.items():
                        ctx.set_option(k, v)
                    for _ in range(3):
                        v = crypto.verify_packed(ctx, b, MODE_IS_VALID)
                    ok = bool((v == ACCEPT).all()) if not a.bench_layout else \
                        bool((v[np.array([c == "valid" for c in s.classes[:n]])] == ACCEPT).all())
                    ts = []
                    for _ in range(a.runs):
                        t0 = time.perf_counter()
                        crypto.verify_packed(ctx, b, MODE_IS_VALID)
                        ts.append(time.perf_counter() - t0)
                    p50 = statistics.median(ts) * 1e3
                    row = {"n": n, "msg_bytes": a.msg_bytes, "pinned": pinned, "setting": st, "p50_ms": round(p50, 3),
                           "min_ms": round(min(ts) * 1e3, 3), "bytes": nbytes, "all_accept": ok,
                           "GBps": round(nbytes / (p50 / 1e3) / 1e9, 2)}
                    if a.spans:
                        import bench
                        sp = bench.e2e_spans(ctx, lambda: crypto.verify_packed(ctx, b, MODE_IS_VALID),
                                             os.environ["CORDA_AMD_TIMELINE"], timeline=a.timeline)
                        row["spans"] = {k: v for k, v in (sp or {}).items() if k not in ("spans", "timeline")}
                        if a.timeline:
                            row["timeline"] = (sp or {}).get("timeline")
                        row["kernels"] = {k: (v["count"], v["first_start_ms"], v["last_end_ms"], v["sum_ms"])
                                          for k, v in (sp or {}).get("spans", {}).items()}
                    res["rows"].append(row)
                    print(json.dumps(row), flush=True)
                if pinned:
                    ctx.unregister_host(b.pk, b.sig, b.msg, b.msg_off, b.msg_len)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["h2d_GBps"]))


if __name__ == "__main__":
    main()
