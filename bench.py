#!/usr/bin/env python3
"""Benchmark of the hot path: batch Ed25519 verification on MI355X.

Metric (BASELINE.json): Ed25519 verifies/s at 1/2/4/8 MI355X + % of INT32 VALU
peak; p50 batch latency.  Workload at N=1 = BASELINE config 2: 1,048,576
EDDSA_ED25519_SHA512 signatures, distinct keys, 1 KB messages, 1 % adversarial
(classes E1–E12).  A step = one cg_batch_verify over the batch, inputs resident
in HBM (staged once by cg_batch_create) — prep + MSM kernels, verdicts, accept
bitmap; for N > 1 the step also all-gathers the per-rank accept bitmaps over RCCL
(C1).  Scaling is weak: every rank verifies its own 1M-signature index shard
(distinct keys per shard), so per-GPU work is fixed as N grows.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line on rank 0.  See DESIGN.md "Measurement" for the op model
behind `roofline` and the CPU baseline.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))

# SURVEY.md §8(d) fixed algorithmic op model (INT32 ops per 1 KB-message Ed25519
# verify), split between the two kernels (bench/roofline_model.json).
with open(os.path.join(ROOT, "bench", "roofline_model.json")) as _f:
    OP_MODEL = json.load(_f)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=1 << 20, help="signatures per GPU")
    p.add_argument("--msg-bytes", type=int, default=1024)
    p.add_argument("--adversarial", type=float, default=0.01)
    p.add_argument("--latency-runs", type=int, default=21)
    p.add_argument("--cpu-sample", type=int, default=131072, help="signatures in the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def host_cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cpu_threads():
    # the GPU box grants this process a 16-CPU share even though nproc shows the machine
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() else (os.cpu_count() or 1)
    return max(1, min(n, 16))


def cpu_baseline(w, threads):
    """The C oracle (i2p-exact restatement, oracle/liboracle.so) timed on host
    cores over a bounded sample of the same workload.  Kind "port": the JVM
    reference cannot run on the box (no JVM / jars)."""
    import subprocess
    lib_path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib_path):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")], stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(lib_path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.oracle_verify_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, vp]
    out = np.empty(w.n, dtype=np.uint8)
    P = lambda a: a.ctypes.data  # noqa: E731
    t0 = time.perf_counter()
    lib.oracle_verify_batch(P(w.scheme), P(w.pk), w.pk_stride, P(w.sig), w.sig_stride, P(w.sig_len), P(w.msg),
                            P(w.msg_off), P(w.msg_len), w.n, 0, threads, P(out))
    dt = time.perf_counter() - t0
    return w.n / dt, dt, out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import ACCEPT, MODE_IS_VALID

    n = args.batch
    t_gen = time.perf_counter()
    w = datagen.make_batch(n, msg_bytes=args.msg_bytes, seed=42 + rank, key_base=rank * n,
                           threads=cpu_threads())
    if args.adversarial > 0:
        w = datagen.add_ed25519_adversarial(w, frac=args.adversarial, seed=1 + rank)
    t_gen = time.perf_counter() - t_gen

    ctx = Context(local_rank)
    pb = crypto.PreparedBatch(ctx, crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride,
                                                      w.sig_len, w.msg, w.msg_off, w.msg_len))
    nwords = (n + 31) // 32
    bitmap_dev = gathered = None
    if dist is not None:
        import torch
        bitmap_dev = torch.zeros(nwords, dtype=torch.int32, device="cuda")
        gathered = torch.zeros(nwords * world, dtype=torch.int32, device="cuda")

    def step():
        pb.verify(MODE_IS_VALID, want_verdicts=False,
                  device_bitmap_ptr=None if bitmap_dev is None else bitmap_dev.data_ptr())
        if dist is not None:
            dist.all_gather_into_tensor(gathered, bitmap_dev)  # C1: verdict-bitmap all-gather over RCCL

    def sync():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    ctx.set_profiling(True)
    ctx.reset_stats()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    msm_ms, msm_launches, msm_items = ctx.kernel_stats("ed25519_msm")
    prep_ms, prep_launches, prep_items = ctx.kernel_stats("ed25519_prep")
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # verdict sanity (outside the timed region)
    verdict = pb.verify(MODE_IS_VALID)
    adv = np.array([c != "valid" for c in w.classes])
    untouched_ok = bool((verdict[~adv] == ACCEPT).all())
    accepts = int((verdict == ACCEPT).sum())

    # p50 batch latency: device-only (resident batch) and end-to-end (H2D + kernels + D2H)
    lat_dev, lat_e2e = [], []
    if rank == 0:
        runs = args.latency_runs
        for _ in range(runs):
            t1 = time.perf_counter(); pb.verify(MODE_IS_VALID, want_verdicts=False); lat_dev.append(time.perf_counter() - t1)
        e2e_n = min(n, 1 << 18)
        sub = w.subset(np.arange(e2e_n))
        sb = crypto.PackedBatch(sub.n, sub.scheme, sub.pk, sub.pk_stride, sub.sig, sub.sig_stride, sub.sig_len,
                                sub.msg, sub.msg_off, sub.msg_len)
        crypto.verify_packed(ctx, sb, MODE_IS_VALID)
        for _ in range(runs):
            t1 = time.perf_counter(); crypto.verify_packed(ctx, sb, MODE_IS_VALID); lat_e2e.append(time.perf_counter() - t1)

    total = n * world * args.steps
    value = total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    per_launch = msm_items / max(msm_launches, 1)
    avg_msm_s = msm_ms / max(msm_launches, 1) / 1e3
    avg_prep_s = prep_ms / max(prep_launches, 1) / 1e3
    peak = OP_MODEL["peak_int32_tops"]
    ops_msm = OP_MODEL["ed25519_1kb"]["msm"]
    ops_prep = OP_MODEL["ed25519_1kb"]["prep"]
    achieved = ops_msm * per_launch / avg_msm_s / 1e12 if avg_msm_s > 0 else 0.0
    achieved_prep = ops_prep * per_launch / avg_prep_s / 1e12 if avg_prep_s > 0 else 0.0
    path_ops = OP_MODEL["ed25519_1kb"]["total"]
    traffic, pmc = None, {}
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):  # measured in separate rocprofv3 --pmc passes (tools/pmc_*.sh)
        with open(tpath) as f:
            pmc = json.load(f)
        traffic = pmc.get("ed25519_msm_bytes_per_launch")
    hw = None
    if pmc.get("ed25519_msm_valu_instr_per_verify") and avg_msm_s > 0:
        # hardware view: VALU lane-instructions actually issued per second (instruction count
        # per verify from SQ_INSTS_VALU, time from this run's HIP events)
        lane_ops = pmc["ed25519_msm_valu_instr_per_verify"] * per_launch / avg_msm_s
        clk = pmc.get("ed25519_msm_effective_clock_GHz")
        hw = {"valu_instr_per_verify": pmc["ed25519_msm_valu_instr_per_verify"],
              "valu_lane_ops_T": round(lane_ops / 1e12, 2), "frac_of_peak": round(lane_ops / 1e12 / peak, 3),
              "pmc_clock_GHz": clk,
              "frac_of_peak_at_pmc_clock": round(lane_ops / (256 * 64 * clk * 1e9), 3) if clk else None,
              "source": pmc.get("source")}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = cpu_threads()
        sample = w.subset(np.arange(min(args.cpu_sample, n)))
        rate, dt, cv = cpu_baseline(sample, threads)
        cpu = {"value": round(rate, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
               "sample": f"first {sample.n} signatures of the same workload (1 KB msgs, incl. its adversarial "
                         f"elements), C i2p-exact restatement (oracle/liboracle.so) on {threads} threads of "
                         f"'{host_cpu_model()}', {dt:.1f} s wall",
               "verdicts_match_gpu": bool(np.array_equal(cv, verdict[:sample.n]))}

    if rank == 0:
        line = {
            "metric": "Ed25519 verifies/sec",
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": "BASELINE config 2: EDDSA_ED25519_SHA512 batch verify, distinct keys, "
                                   f"{args.msg_bytes} B messages, {args.adversarial:.0%} adversarial (E1-E12)",
                       "batch_per_gpu": n, "global_batch": n * world, "msg_bytes": args.msg_bytes,
                       "parallelism": f"dp{world} (signature-index shards" +
                                      (", RCCL all-gather of accept bitmaps)" if world > 1 else ")")},
            "roofline": {"bound": "valu_int32", "kernel": "ed25519_msm", "achieved": round(achieved, 3),
                         "peak": peak, "unit": "TOPS", "frac": round(achieved / peak, 4), "traffic": traffic,
                         "ops_per_unit": ops_msm, "units_per_launch": per_launch,
                         "avg_launch_ms": round(avg_msm_s * 1e3, 3), "hw_valu": hw},
            "path_frac_of_int32_peak": round(value / world * path_ops / 1e12 / peak, 4),
            "prep_kernel": {"achieved": round(achieved_prep, 3), "avg_launch_ms": round(avg_prep_s * 1e3, 3)},
            "latency": {"p50_device_ms": round(statistics.median(lat_dev) * 1e3, 3) if lat_dev else None,
                        "p50_e2e_ms": round(statistics.median(lat_e2e) * 1e3, 3) if lat_e2e else None,
                        "e2e_batch": min(n, 1 << 18), "runs": args.latency_runs},
            "cpu_baseline": cpu,
            "checks": {"accepts": accepts, "untouched_all_accept": untouched_ok, "datagen_s": round(t_gen, 1)},
        }
        print(json.dumps(line), flush=True)
    pb.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
