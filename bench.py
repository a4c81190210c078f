#!/usr/bin/env python3
"""Benchmark of the hot path: batch signature verification on MI355X.

Metric (BASELINE.json): Ed25519 verifies/s at 1/2/4/8 MI355X + % of INT32 VALU
peak; p50 batch latency.  The default workload (the driver's bench line) is
BASELINE config 2: 1,048,576 EDDSA_ED25519_SHA512 signatures per GPU, distinct
keys, 1 KB messages, 1 % adversarial (classes E1–E12).  A step = one
cg_batch_verify over the batch, inputs resident in HBM (staged once by
cg_batch_create) — hash + points + MSM kernels, verdicts, accept bitmap; for N > 1 the
step also all-gathers the per-rank accept bitmaps over RCCL (C1).  Scaling is
weak: every rank verifies its own 1M-signature index shard (distinct keys per
shard), so per-GPU work is fixed as N grows.

The other BASELINE configs are reachable with ``--workload`` (each prints its
own JSON line; they are evidence for DESIGN.md, not the driver's line):

    ecdsa    config 3: 1M ECDSA_SECP256R1_SHA256 + 1M ECDSA_SECP256K1_SHA256, 1 KB
             messages, 1 % adversarial (D1–D8)
    tx       config 4: 1M SignedTransactions (trader-demo / loadtest shapes):
             Merkle tx-id recompute + every signature over the id + first
             failing signature per tx, host buffers in and out (cg_tx_verify_batch)
    backlog  config 5: 100M Ed25519 signatures over 32 B tx ids, split by index
             over the ranks (strong scaling), staged in 2^24 chunks, verdict-
             bitmap all-gather over RCCL
    ftx      SURVEY 8(f) row 1: 1M FilteredTransaction.verify (non-validating
             notary: filtered-leaf hashes + partial Merkle tree + multiset check)

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ed25519|ecdsa|tx|backlog|ftx]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Multi-GPU: under torchrun (WORLD_SIZE set) every process is one rank and
WORLD_SIZE must equal --gpus (else exit 2).  Without WORLD_SIZE and --gpus N > 1
this process is only a launcher: it starts N rank processes of itself (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their env)
before anything touches the GPU, waits for them, and exits with the first
failing rank's code; rank 0 prints the line.  ``--dry-run`` runs the same
launcher / barrier / max-over-ranks / all-gather logic over gloo on CPU tensors
with a synthetic step (no GPU; tests/test_bench_launcher.py).

Prints ONE JSON line on rank 0.  See DESIGN.md "Measurement" for the roofline
(issued VALU lane-ops of the dominant kernel against the 78.6 T lane-op/s
INT32 VALU peak, instruction counts from the committed rocprofv3 PMC pass of the
same kernel sources) and the CPU baseline.
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import platform
import socket
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))

# SURVEY.md §8(d) fixed algorithmic op model (INT32 ops per verify), committed
# once in bench/roofline_model.json, and the INT32 VALU peak: 256 CUs x 4 SIMD-32
# x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s (MI355X_MICROARCH.md: "4 SIMD-32 vector
# units" per CU, a wave64 VALU instruction in 2 cycles).
with open(os.path.join(ROOT, "bench", "roofline_model.json")) as _f:
    OP_MODEL = json.load(_f)
PEAK = OP_MODEL["peak_int32_tops"]
SIMDS = 1024  # 256 CUs x 4 SIMDs (MI355X); a wave64 VALU instruction holds one SIMD 2 or 4 cycles


def kernel_src_hash() -> str:
    """Hash of the device sources (*.hip, *.h) + build file; the PMC summaries carry
    the same hash, so a bench line can say whether its instruction counts belong to
    the kernels it ran (tools/pmc_report.py writes it; host-side cordagpu.cpp does
    not change a kernel's instruction stream and is left out)."""
    d = os.path.join(ROOT, "corda_amd", "csrc")
    h = hashlib.sha256()
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".h")) or name == "Makefile":
            with open(os.path.join(d, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=["ed25519", "ecdsa", "tx", "backlog", "ftx"], default="ed25519")
    p.add_argument("--batch", type=int, default=None,
                   help="per-GPU units (default: 1M signatures / 1M per curve / 1M txs; backlog: 100M total)")
    p.add_argument("--pool", type=int, default=None,
                   help="distinct signed tuples generated and tiled to --batch (default: ecdsa all distinct, "
                        "tx 131072, backlog 1M per rank)")
    p.add_argument("--msg-bytes", type=int, default=None)
    p.add_argument("--adversarial", type=float, default=0.01)
    p.add_argument("--latency-runs", type=int, default=21)
    p.add_argument("--cpu-sample", type=int, default=None, help="units in the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--key-reuse", type=int, default=0,
                   help="ed25519/backlog/tx: draw signer keys from this many distinct keys (0 = all distinct)")
    p.add_argument("--no-extra", action="store_true",
                   help="ed25519 (N=1): skip the 32 B tx-id end-to-end record and the config-3 / config-4 sub-records")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher / barrier / all-gather logic over gloo on CPU, synthetic step (tests)")
    a = p.parse_args()
    a.pool_set = a.pool is not None
    if a.pool is None:
        a.pool = 131072
    return a


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int | None:
    """Returns None when this process is a rank (torchrun, or --gpus 1), else
    starts --gpus rank processes of this script and returns the exit code to use.
    Runs before anything touches the GPU: the children are fresh processes (no
    exec from a process with an initialised device)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}; refusing to report a mislabelled line",
                  file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    alive = list(procs)
    stop_at = None
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                stop_at = time.monotonic() + 30
                for q in alive:  # a dead rank leaves the others waiting in a collective
                    q.terminate()
        if stop_at is not None and time.monotonic() > stop_at:
            for q in alive:  # one that ignored SIGTERM (e.g. inside a GPU call)
                q.kill()
            stop_at = None
        time.sleep(0.2)
    return rc


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
    """Host threads for this rank's datagen / CPU baseline: the box's CPU share (it grants
    a 16-CPU share even though nproc shows the machine; OMP_NUM_THREADS says so) divided
    over the ranks on this node, so 8 ranks do not oversubscribe it 8x."""
    env = os.environ.get("OMP_NUM_THREADS")
    share = max(1, min(int(env) if env and env.isdigit() else (os.cpu_count() or 1), 16))
    local = os.environ.get("LOCAL_WORLD_SIZE") or os.environ.get("WORLD_SIZE") or "1"
    return max(1, share // max(1, int(local) if local.isdigit() else 1))


def dist_timeout_s() -> float:
    """Bound on every collective (and the process-group rendezvous): a rank that hangs
    makes the others fail with an error instead of waiting forever, so the launcher
    sees a non-zero exit and stops the rest.  Datagen happens before the first barrier
    and takes well under a minute per rank; CORDA_AMD_DIST_TIMEOUT_S overrides."""
    return float(os.environ.get("CORDA_AMD_DIST_TIMEOUT_S", "600"))


def oracle_lib():
    """The C oracle (i2p/BC-exact restatement, test infrastructure): used only for
    the cpu_baseline leg, never on the measured path."""
    import subprocess
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")], stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.oracle_verify_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, vp]
    lib.oracle_txid_batch.argtypes = [vp, vp, vp, vp, vp, sz, vp]
    return lib


def oracle_verify(w, threads, mode=0):
    lib = oracle_lib()
    out = np.empty(max(w.n, 1), dtype=np.uint8)
    P = lambda a: a.ctypes.data  # noqa: E731
    t0 = time.perf_counter()
    lib.oracle_verify_batch(P(w.scheme), P(w.pk), w.pk_stride, P(w.sig), w.sig_stride, P(w.sig_len), P(w.msg),
                            P(w.msg_off), P(w.msg_len), w.n, mode, threads, P(out))
    return out[:w.n], time.perf_counter() - t0


class Dist:
    """One rank per GPU: torch.distributed over RCCL ("nccl") when WORLD_SIZE > 1
    (launched by torchrun or by launch_ranks); gloo on CPU tensors for --dry-run."""

    def __init__(self, cpu: bool = False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.cpu = cpu
        self.device = "cpu" if cpu else "cuda"
        self.d = None
        if self.world > 1:
            import datetime

            import torch
            import torch.distributed as dist
            timeout = datetime.timedelta(seconds=dist_timeout_s())
            if cpu:
                dist.init_process_group("gloo", timeout=timeout)
            else:
                torch.cuda.set_device(self.local_rank)
                # RCCL: the watchdog aborts a collective past `timeout` and fails the process
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank), timeout=timeout)
            self.d = dist

    def sync(self):
        if self.d is not None:
            self.d.barrier()
        if not self.cpu:
            import torch
            torch.cuda.synchronize()

    def max(self, x: float) -> float:
        if self.d is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self.d.all_reduce(t, op=self.d.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.d is not None:
            self.d.destroy_process_group()


def timed(dist, ctx, step, steps, warmup):
    """W untimed steps, then exactly K timed steps between barrier+sync pairs;
    returns the max over ranks of the elapsed seconds (kernel stats reset at the
    start of the timed region, HIP events on the library stream)."""
    for _ in range(warmup):
        step()
    ctx.set_profiling(True)
    ctx.reset_stats()
    dist.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dist.sync()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    return dist.max(elapsed)


ED_PREP_KERNELS = ("ed25519_hash", "ed25519_points")
ED_KERNELS = [*ED_PREP_KERNELS, "ed25519_msm"]
ED_REUSE_KERNELS = ["ed25519_keyprep"]  # the key-reuse path only (distinct keys decoded once per verify)
ED_AUX_KERNELS = ["ed25519_bucket"]  # the grouped MSM's two lane-classing kernels (one span)


def timeline_path(rank):
    """The library's span log (CORDA_AMD_TIMELINE, read once by libcordagpu at its first
    timed call): set before the first Context so the e2e span breakdown can be read."""
    path = os.path.join(tempfile.gettempdir(), f"corda_amd_timeline_{os.getpid()}_{rank}.txt")
    os.environ.setdefault("CORDA_AMD_TIMELINE", path)
    return os.environ["CORDA_AMD_TIMELINE"]


def e2e_spans(ctx, call, path, timeline=False):
    """Where one host-buffer call's time goes: the call runs once with the library's
    HIP-event spans on, and its timeline group (times relative to the 'call' span's
    begin, recorded at the library's entry on idle streams) is summarised: the call's
    GPU span, host pre-work before the first H2D copy, the copies, each kernel's first
    start / last end / summed duration, and what the host wall adds after the last
    device event (the final sync's wake-up, the Python wrapper)."""
    with open(path, "w"):
        pass
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    call()
    wall = (time.perf_counter() - t0) * 1e3
    ctx.set_profiling(False)
    try:
        groups = [g for g in open(path).read().split("# call\n") if g.strip()]
    except OSError:
        return None
    if not groups:
        return None
    rows = [(n, float(a), float(b)) for n, a, b in (ln.split() for ln in groups[-1].splitlines())]
    spans = {}
    for n, a, b in rows:
        e = spans.setdefault(n, {"count": 0, "first_start_ms": a, "last_end_ms": b, "sum_ms": 0.0})
        e["count"] += 1
        e["first_start_ms"] = min(e["first_start_ms"], a)
        e["last_end_ms"] = max(e["last_end_ms"], b)
        e["sum_ms"] += b - a
    for e in spans.values():
        for k in ("first_start_ms", "last_end_ms", "sum_ms"):
            e[k] = round(e[k], 3)
    call_ms = spans.get("call", {}).get("last_end_ms")
    h2d = [v for k, v in spans.items() if k.startswith("h2d")]
    kern = [v for k, v in spans.items() if k.startswith("ed25519") or k == "stage"]
    out = {"wall_ms": round(wall, 3), "call_gpu_ms": call_ms, "spans": spans}
    if timeline:  # every span, in start order
        out["timeline"] = [(n, round(a, 3), round(b, 3)) for n, a, b in sorted(rows, key=lambda r: r[1])]
    if h2d:
        out["host_pre_ms"] = round(min(v["first_start_ms"] for v in h2d), 3)
        out["h2d_end_ms"] = round(max(v["last_end_ms"] for v in h2d), 3)
    if kern:
        out["kernels_end_ms"] = round(max(v["last_end_ms"] for v in kern), 3)
        if h2d:
            out["kernels_after_last_h2d_ms"] = round(out["kernels_end_ms"] - out["h2d_end_ms"], 3)
    if call_ms is not None:
        out["host_after_gpu_ms"] = round(wall - call_ms, 3)
    return out


def host_share(ctx, call, runs):
    """The host's share of a host-buffer call, without per-kernel profiling: each call
    runs with only its "call" span on (cg_set_profiling 2: two HIP events, from the
    library's entry on idle streams to the verdict download), so wall - GPU span is
    the host work before the first GPU command and after the last one (staging copies,
    the final sync's wake-up, frees, the Python wrapper).  Medians over `runs` calls."""
    walls, gpus = [], []
    ctx.set_profiling(2)
    try:
        for _ in range(runs):
            ctx.reset_stats()
            t0 = time.perf_counter()
            call()
            walls.append((time.perf_counter() - t0) * 1e3)
            ms, launches, _ = ctx.kernel_stats("call")
            if launches == 1:
                gpus.append(ms)
    finally:
        ctx.set_profiling(False)
    if not gpus:
        return None
    return {"wall_ms_p50": round(statistics.median(walls), 3), "gpu_call_ms_p50": round(statistics.median(gpus), 3),
            "host_ms_p50": round(statistics.median([w - g for w, g in zip(walls, gpus)]), 3), "runs": len(gpus)}


def kstats(ctx, names):
    out = {}
    for k in names:
        ms, launches, items = ctx.kernel_stats(k)
        if launches:
            out[k] = {"avg_launch_ms": round(ms / launches, 4), "launches": launches,
                      "units_per_launch": items / launches}
    return out


def pmc_view(name="pmc_traffic.json"):
    tpath = os.path.join(ROOT, "profiles", name)
    if os.path.exists(tpath):  # measured in separate rocprofv3 --pmc passes (tools/profile_gpu.sh)
        with open(tpath) as f:
            return json.load(f)
    return {}


def valu_roofline(pmc, kernel, units_per_launch, avg_launch_s, model_ops=None):
    """Roofline of one kernel against the INT32 VALU peak.

    achieved = VALU lane-instructions the kernel issues per unit (SQ_INSTS_VALU /
    SQ_WAVES of the committed rocprofv3 PMC pass, profiles/<tag>_pmc_summary.json)
    x units per launch / the launch's average duration (HIP events on the stream
    the kernel runs on, this run).  `pmc_src_hash_matches` says whether the PMC
    pass profiled the very kernel sources this run built (tools/pmc_report.py
    stamps the hash).  model_* = SURVEY 8(d)'s fixed op model of the reference
    algorithm over the same time (it prices 253 doublings + an inversion; the
    kernels do ~130 doublings and no inversion, so model_frac is not a roofline
    fraction and can exceed 1)."""
    e = pmc.get("kernels", {}).get(kernel, {})
    instr = e.get("valu_instr_per_unit")
    out = {"bound": "valu_int32", "kernel": kernel, "unit": "T lane-ops/s", "peak": PEAK,
           "units_per_launch": units_per_launch, "avg_launch_ms": round(avg_launch_s * 1e3, 4),
           "valu_instr_per_unit": instr, "achieved": None, "frac": None,
           "traffic": e.get("hbm_bytes_per_unit") and round(e["hbm_bytes_per_unit"] * units_per_launch),
           "traffic_note": "HBM bytes per launch from the PMC pass: (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB, "
                           "FETCH doubled for the 16-B-per-lane table loads (MI355X_MICROARCH.md HBM section)",
           "pmc_source": pmc.get("source"), "pmc_commit": pmc.get("commit"),
           "pmc_src_hash_matches": pmc.get("src_hash") == kernel_src_hash() if pmc else False,
           "pmc_clock_GHz": e.get("effective_clock_GHz"), "occupancy": e.get("occupancy")}
    if instr and avg_launch_s > 0:
        ach = instr * units_per_launch / avg_launch_s / 1e12
        out["achieved"] = round(ach, 3)
        out["frac"] = round(ach / PEAK, 4)
        # issue utilisation: a 64-bit VALU op (v_mad_i64_i32, 64-bit shifts: SQ_INSTS_VALU_INT64) holds the
        # SIMD for 4 cycles, a 32-bit one for 2 (profiles/r02a_isa_rates.json; 32-bit multiplies, v_lshlrev
        # and a few more take 4 too, so this is a lower bound); cycles the mix needs / cycles available at 2.4
        # GHz and at the PMC pass's measured clock
        i64 = e.get("int64_instr_per_unit")
        if i64 is not None:
            need = (2.0 * (instr - i64) + 4.0 * i64) * units_per_launch / (SIMDS * 64)  # cycles per SIMD
            out["issue_util"] = round(need / (avg_launch_s * 2.4e9), 4)
            clk = e.get("effective_clock_GHz")
            if clk:
                out["issue_util_at_pmc_clock"] = round(need / (avg_launch_s * clk * 1e9), 4)
    if model_ops and avg_launch_s > 0:
        m = model_ops * units_per_launch / avg_launch_s / 1e12
        out["model_ops_per_unit"] = model_ops
        out["model_achieved"] = round(m, 3)
        out["model_frac"] = round(m / PEAK, 4)
    return out


def base_line(args, dist, metric, unit, value, ms_per_step, config, scaling="weak"):
    return {"metric": metric, "value": round(value, 1), "unit": unit, "n_gpus": dist.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "int32", "data": "synthetic", "config": config}


def pcie_h2d_peak_GBps(device=0, mb=512, reps=5):
    """Measured host-to-device rate from page-locked memory on this box (the
    roofline of the paths that start from host buffers)."""
    import torch
    src = torch.empty(mb << 20, dtype=torch.uint8).pin_memory()
    dst = torch.empty(mb << 20, dtype=torch.uint8, device=f"cuda:{device}")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        dst.copy_(src, non_blocking=True)
        b.record()
        b.synchronize()
        best = max(best, (mb << 20) / (a.elapsed_time(b) / 1e3) / 1e9)
    del src, dst
    return round(best, 2)


# ------------------------------------------------------------------ --dry-run
def _dry_words(lo: int, hi: int) -> np.ndarray:
    """Accept-bitmap words of the synthetic dry-run verdicts (element i accepts iff
    i % 7 != 3) for indices [lo, hi), lo a multiple of 32; built in 2^22 pieces."""
    from corda_amd import dist as D
    step = 1 << 22
    parts = [D.pack_bits((np.arange(a, min(hi, a + step), dtype=np.int64) % 7) != 3) for a in range(lo, hi, step)]
    return np.concatenate(parts).view(np.int32) if parts else np.zeros(0, np.int32)


def run_dry(args, dist):
    """The multi-rank plumbing without a GPU: every rank owns a synthetic index
    shard, a step packs a verdict bitmap and all-gathers it (gloo), timing is the
    max over ranks between barriers — what the real workloads do over RCCL.
    ``--workload backlog`` uses config 5's shapes: ``--batch`` (default 100 M) is the
    TOTAL, split by ``shard_bounds`` (uneven for world 3, 6, 7 ...), gathered with
    ``gather_ordered`` as ShardBacklog.allgather does; otherwise ``--batch`` per rank."""
    import torch
    from corda_amd import dist as D
    if os.environ.get("CORDA_AMD_DRY_FAIL_RANK") == str(dist.rank):
        sys.exit(3)  # tests: a failing rank must fail the launcher
    if os.environ.get("CORDA_AMD_DRY_HANG_RANK") == str(dist.rank):
        time.sleep(3600)  # tests: a hung rank — the others' collectives time out, the launcher fails
    backlog = args.workload == "backlog"
    total = (args.batch or 100_000_000) if backlog else (args.batch or 4096) * dist.world
    bounds = D.shard_bounds(total, dist.world)
    lo, hi = bounds[dist.rank], bounds[dist.rank + 1]
    wmax = max((bounds[r + 1] - bounds[r] + 31) // 32 for r in range(dist.world))
    words = torch.zeros(max(wmax, 1), dtype=torch.int32)
    mine = _dry_words(lo, hi)
    words[:len(mine)] = torch.from_numpy(mine.copy())
    got = [None]

    def step():
        if dist.d is None:
            got[0] = words[:len(mine)]
        elif backlog:
            got[0] = D.gather_ordered(words, bounds)
        else:
            got[0] = D.allgather_bitmap(words[:len(mine)], bounds, dist.rank)

    for _ in range(args.warmup):
        step()
    dist.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dist.sync()
    elapsed = dist.max(time.perf_counter() - t0)
    ok = bool(np.array_equal(got[0].numpy(), _dry_words(0, total))) if dist.rank == 0 else None
    line = base_line(args, dist, "dry-run bitmap all-gathers/sec", "steps/s", args.steps / max(elapsed, 1e-9),
                     elapsed * 1e3 / args.steps, {"workload": "dry run (gloo, CPU)" + (", config-5 shards" if backlog
                                                                                        else ""),
                                                  "batch_per_gpu": hi - lo, "global_batch": total,
                                                  "shard_elements": [bounds[r + 1] - bounds[r]
                                                                     for r in range(dist.world)],
                                                  "parallelism": f"dp{dist.world}"})
    line["checks"] = {"bitmap_matches": ok, "rank_pid_world": dist.world}
    line["dry_run"] = True
    return line


# ------------------------------------------------------------------ config 2
def run_ed25519(args, dist):
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import ACCEPT, MODE_IS_VALID

    n = args.batch or (1 << 20)
    msg_bytes = args.msg_bytes or 1024
    rank, world = dist.rank, dist.world
    t_gen = time.perf_counter()
    # distinct keys, every 4,096th one a reference test key (seeds 20..110)
    w = datagen.make_batch(n, msg_bytes=msg_bytes, seed=42 + rank, key_base=rank * n, threads=cpu_threads(),
                           key_reuse=args.key_reuse, ref_seed_stride=4096)
    if args.adversarial > 0:
        w = datagen.add_ed25519_adversarial(w, frac=args.adversarial, seed=1 + rank)
    t_gen = time.perf_counter() - t_gen

    tl_path = timeline_path(rank)
    ctx = Context(dist.local_rank)
    pb = crypto.PreparedBatch(ctx, crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride,
                                                      w.sig_len, w.msg, w.msg_off, w.msg_len))
    nwords = (n + 31) // 32
    bitmap_dev = gathered = None
    if dist.d is not None:
        import torch
        bitmap_dev = torch.zeros(nwords, dtype=torch.int32, device="cuda")
        gathered = torch.zeros(nwords * world, dtype=torch.int32, device="cuda")

    def step():
        pb.verify(MODE_IS_VALID, want_verdicts=False,
                  device_bitmap_ptr=None if bitmap_dev is None else bitmap_dev.data_ptr())
        if dist.d is not None:
            dist.d.all_gather_into_tensor(gathered, bitmap_dev)  # C1: verdict-bitmap all-gather over RCCL

    elapsed = timed(dist, ctx, step, args.steps, args.warmup)
    ks = kstats(ctx, ED_KERNELS + ED_REUSE_KERNELS + ED_AUX_KERNELS)
    # In the timed step the points kernel runs beside the hash kernel (CORDA_AMD_ED_OVERLAP) and a
    # split batch runs as pieces on two streams, so those HIP-event spans overlap: the per-kernel
    # times and the roofline come from 3 extra steps with both off (each kernel alone over the
    # whole batch); the timed step's own spans are kept as kernels_in_step.
    ks_step = ks
    with ctx.options(ED_SPLIT=1, ED_OVERLAP=0):  # (cg_set_option: this context only)
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(3):
            step()
        ks = kstats(ctx, ED_KERNELS + ED_REUSE_KERNELS + ED_AUX_KERNELS)
        ctx.set_profiling(False)
    split_note = ("kernels / roofline: 3 extra steps with the options CORDA_AMD_ED_SPLIT=1 CORDA_AMD_ED_OVERLAP=0 (each kernel "
                  "alone over the whole batch); kernels_in_step: the timed steps' own spans (a resident batch runs the points kernel after the hash kernel)")

    # verdict check (outside the timed region): untouched elements must accept
    verdict = pb.verify(MODE_IS_VALID)
    adv = np.array([c != "valid" for c in w.classes])
    untouched_ok = bool((verdict[~adv] == ACCEPT).all())
    accepts = int((verdict == ACCEPT).sum())

    # p50 batch latency: device-only (resident batch) and end-to-end (H2D + kernels + D2H)
    lat_dev, lat_e2e, lat_small, lat_small_off, spans = [], [], {}, {}, {}
    host_e2e = None
    e2e_bytes, e2e_ok, h2d_peak = 0, None, None
    e2e_n = min(n, 1 << 18)
    if rank == 0:
        for _ in range(args.latency_runs):
            t1 = time.perf_counter(); pb.verify(MODE_IS_VALID, want_verdicts=False); lat_dev.append(time.perf_counter() - t1)
        # end to end from pageable host buffers in the layout an Ed25519-only caller packs
        # (32-byte keys, 64-byte R||S rows, no scheme / sig_len arrays)
        sub = w.subset(np.arange(e2e_n))
        # signature lengths travel only when some row is not 64 bytes (the E12 class: 0 / 63 / 65)
        sl = sub.sig_len[:sub.n].astype(np.uint32)
        ragged = bool((sl != 64).any())
        ss = max(64, (int(sl.max()) + 3) // 4 * 4) if ragged else 64
        sg = np.zeros((sub.n, ss), dtype=np.uint8)
        sg[:, :min(ss, sub.sig_stride)] = sub.sig[:sub.n, :min(ss, sub.sig_stride)]
        sb = crypto.PackedBatch(sub.n, None, np.ascontiguousarray(sub.pk[:, :32]), 32, sg, ss,
                                np.ascontiguousarray(sl) if ragged else None, sub.msg, sub.msg_off, sub.msg_len)
        e2e_bytes = sum(x.nbytes for x in (sb.pk, sb.sig, sb.msg_off, sb.msg_len)) + int(sb.msg_len.sum())
        if ragged:
            e2e_bytes += sl.nbytes
        e2e_ok = bool(np.array_equal(crypto.verify_packed(ctx, sb, MODE_IS_VALID), verdict[:e2e_n]))
        for _ in range(args.latency_runs):
            t1 = time.perf_counter(); crypto.verify_packed(ctx, sb, MODE_IS_VALID); lat_e2e.append(time.perf_counter() - t1)
        spans[e2e_n] = e2e_spans(ctx, lambda: crypto.verify_packed(ctx, sb, MODE_IS_VALID), tl_path)
        host_e2e = host_share(ctx, lambda: crypto.verify_packed(ctx, sb, MODE_IS_VALID), args.latency_runs)
        h2d_peak = pcie_h2d_peak_GBps(dist.local_rank)
        # serving-size batches (a notary's request queue): end-to-end p50 from host buffers,
        # with the latency mode (two lanes per signature for pieces <= CORDA_AMD_ED_PAIR_MAX)
        # as the library chooses it and, beside it, forced off
        for bn in (4096, 16384, 65536):
            if bn > n:
                continue
            s2 = w.subset(np.arange(bn))
            b2 = crypto.PackedBatch(s2.n, s2.scheme, s2.pk, s2.pk_stride, s2.sig, s2.sig_stride, s2.sig_len,
                                    s2.msg, s2.msg_off, s2.msg_len)
            for dest, env in ((lat_small, None), (lat_small_off, "0")):
                if env is not None:
                    ctx.set_option("CORDA_AMD_ED_PAIR_MAX", env)
                try:
                    got2 = crypto.verify_packed(ctx, b2, MODE_IS_VALID)
                    ts = []
                    for _ in range(args.latency_runs):
                        t1 = time.perf_counter(); crypto.verify_packed(ctx, b2, MODE_IS_VALID); ts.append(time.perf_counter() - t1)
                    dest[bn] = {"p50_ms": round(statistics.median(ts) * 1e3, 3),
                                "verdicts_match": bool(np.array_equal(got2, verdict[:bn]))}
                    if env is None:
                        spans[bn] = e2e_spans(ctx, lambda: crypto.verify_packed(ctx, b2, MODE_IS_VALID), tl_path)
                        dest[bn]["host_share"] = host_share(ctx, lambda: crypto.verify_packed(ctx, b2, MODE_IS_VALID),
                                                            args.latency_runs)
                finally:
                    if env is not None:
                        ctx.set_option("CORDA_AMD_ED_PAIR_MAX", None)

    value = n * world * args.steps / elapsed
    model = OP_MODEL["ed25519_1kb" if msg_bytes > 32 else "ed25519_32b"]
    # the key-reuse path runs other kernels under the same timing names (points_r, msm_r),
    # profiled in their own PMC pass (profiles/pmc_ed25519_reuse.json)
    reuse = args.key_reuse > 0
    pmc = pmc_view("pmc_ed25519_reuse.json" if reuse else "pmc_ed25519.json")
    kname = {k: f"cg_{k}_r" if reuse and k != "ed25519_hash" else f"cg_{k}" for k in ED_KERNELS}
    msm = ks.get("ed25519_msm", {})
    roof = valu_roofline(pmc, kname["ed25519_msm"], msm.get("units_per_launch", 0),
                         msm.get("avg_launch_ms", 0) / 1e3, model["msm"])
    prep = {k: valu_roofline(pmc, kname[k], ks.get(k, {}).get("units_per_launch", 0),
                             ks.get(k, {}).get("avg_launch_ms", 0) / 1e3) for k in ED_PREP_KERNELS}
    # whole path: VALU lane-instructions of the three kernels per verify x verifies/s
    path_instr = sum((pmc.get("kernels", {}).get(kname[k], {}).get("valu_instr_per_unit") or 0) for k in ED_KERNELS)
    path = {"valu_instr_per_verify": path_instr or None,
            "achieved": round(path_instr * value / world / 1e12, 3) if path_instr else None,
            "frac": round(path_instr * value / world / 1e12 / PEAK, 4) if path_instr else None,
            "model_frac": round(value / world * model["total"] / 1e12 / PEAK, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = cpu_threads()
        sample = w.subset(np.arange(min(args.cpu_sample or 524288, n)))
        cv, dt = oracle_verify(sample, threads)
        cpu = {"value": round(sample.n / dt, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
               "sample": f"first {sample.n} signatures of the same workload ({msg_bytes} B msgs, incl. its "
                         f"adversarial elements), C i2p-exact restatement (oracle/liboracle.so) on {threads} "
                         f"threads of '{host_cpu_model()}', {dt:.1f} s wall",
               "verdicts_match_gpu": bool(np.array_equal(cv, verdict[:sample.n]))}
        # SURVEY 8(d) also asks for a single-thread run: 1/16 of the same sample on one core
        one = w.subset(np.arange(max(1, sample.n // 16)))
        cv1, dt1 = oracle_verify(one, 1)
        cpu["single_thread"] = {"value": round(one.n / dt1, 1), "cores": 1, "sample": f"first {one.n} signatures",
                                "verdicts_match_gpu": bool(np.array_equal(cv1, verdict[:one.n]))}

    line = base_line(args, dist, "Ed25519 verifies/sec", "verifies/s", value, elapsed * 1e3 / args.steps, {
        "workload": "BASELINE config 2: EDDSA_ED25519_SHA512 batch verify, "
                    + (f"keys drawn from {args.key_reuse} signers" if args.key_reuse else
                       "distinct keys (every 4096th a reference test key, seeds 20..110)")
                    + f", {msg_bytes} B messages, {args.adversarial:.0%} adversarial (E1-E12)",
        "batch_per_gpu": n, "global_batch": n * world, "msg_bytes": msg_bytes,
        "parallelism": f"dp{world} (signature-index shards" + (", RCCL all-gather of accept bitmaps)" if world > 1 else ")")})
    line.update({
        "roofline": roof,
        "path_roofline": path,
        "prep_kernels": {k: {"achieved": v["achieved"], "frac": v["frac"], "avg_launch_ms": v["avg_launch_ms"],
                             "valu_instr_per_unit": v["valu_instr_per_unit"]} for k, v in prep.items()},
        "kernels": ks,
        "kernels_in_step": ks_step, "kernel_timing_note": split_note,
        "latency": {"p50_device_ms": round(statistics.median(lat_dev) * 1e3, 3) if lat_dev else None,
                    "p50_e2e_ms": round(statistics.median(lat_e2e) * 1e3, 3) if lat_e2e else None,
                    "e2e_batch": e2e_n, "runs": args.latency_runs,
                    "e2e_bytes": e2e_bytes if lat_e2e else None,
                    "e2e_layout": (f"Ed25519-only host rows: pk_stride 32, sig_stride {sb.sig_stride}, scheme_id NULL, "
                                   f"sig_len {'given (ragged E12 rows)' if sb.sig_len is not None else 'NULL'}; "
                                   "pageable numpy buffers") if lat_e2e else None,
                    "e2e_verdicts_match": e2e_ok if lat_e2e else None,
                    "e2e_host_share": host_e2e,
                    "h2d_peak_GBps": h2d_peak if lat_e2e else None,
                    "e2e_pcie_frac": round(e2e_bytes / statistics.median(lat_e2e) / 1e9 / h2d_peak, 4)
                    if lat_e2e else None,
                    "p50_e2e_ms_by_batch": lat_small,
                    "p50_e2e_ms_by_batch_latency_mode_off": lat_small_off,
                    "e2e_spans": spans,
                    "e2e_spans_note": "one profiled call per size (HIP events on, so slightly slower than the p50 "
                                      "runs); times in ms from the library's entry ('call' span begin)"},
        "cpu_baseline": cpu,
        "checks": {"accepts": accepts, "untouched_all_accept": untouched_ok, "datagen_s": round(t_gen, 1)},
    })
    pb.close()
    ctx.close()
    return line


def e2e_record_32b(args, dist, sizes=(4096, 65536, 262144)):
    """End to end at the production message shape: 32-byte tx ids (WireTransaction.id,
    WireTransaction.kt:39, signed over by TransactionWithSignatures.kt:58-62), host
    buffers in the Ed25519-only caller layout (32-byte keys, 64-byte R||S rows, sig_len
    only for ragged rows), pageable; p50 of --latency-runs calls and one profiled call's
    spans per size; verdicts checked against the same batch staged in HBM."""
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import MODE_IS_VALID
    n = max(sizes)
    w = datagen.make_batch(n, msg_bytes=32, seed=4242, key_base=1 << 36, threads=cpu_threads(), ref_seed_stride=4096)
    if args.adversarial > 0:
        w = datagen.add_ed25519_adversarial(w, frac=args.adversarial, seed=77)
    tl_path = timeline_path(dist.rank)
    out = {"msg_bytes": 32, "runs": args.latency_runs, "by_batch": {}, "spans": {},
           "layout": "Ed25519-only host rows: pk_stride 32, sig_stride 64 (68 + sig_len for ragged E12 rows), "
                     "scheme_id NULL; pageable numpy buffers; 1 % adversarial (E1-E12)"}
    with Context(dist.local_rank) as ctx:
        pb = crypto.PreparedBatch(ctx, crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride,
                                                          w.sig_len, w.msg, w.msg_off, w.msg_len))
        ref = pb.verify(MODE_IS_VALID)
        for m in sizes:
            sub = w.subset(np.arange(m))
            sl = sub.sig_len[:m].astype(np.uint32)
            ragged = bool((sl != 64).any())
            ss = max(64, (int(sl.max()) + 3) // 4 * 4) if ragged else 64
            sg = np.zeros((m, ss), dtype=np.uint8)
            sg[:, :min(ss, sub.sig_stride)] = sub.sig[:m, :min(ss, sub.sig_stride)]
            sb = crypto.PackedBatch(m, None, np.ascontiguousarray(sub.pk[:, :32]), 32, sg, ss,
                                    np.ascontiguousarray(sl) if ragged else None, sub.msg, sub.msg_off, sub.msg_len)
            nbytes = sum(x.nbytes for x in (sb.pk, sb.sig, sb.msg_off, sb.msg_len)) + int(sb.msg_len.sum()) + \
                (sl.nbytes if ragged else 0)
            ok = bool(np.array_equal(crypto.verify_packed(ctx, sb, MODE_IS_VALID), ref[:m]))
            ts = []
            for _ in range(args.latency_runs):
                t1 = time.perf_counter(); crypto.verify_packed(ctx, sb, MODE_IS_VALID); ts.append(time.perf_counter() - t1)
            sp = statistics.median(ts)
            out["by_batch"][m] = {"p50_ms": round(sp * 1e3, 3), "verifies_per_s": round(m / sp, 1), "bytes": nbytes,
                                  "verdicts_match": ok}
            sps = e2e_spans(ctx, lambda: crypto.verify_packed(ctx, sb, MODE_IS_VALID), tl_path)
            out["spans"][m] = {k: v for k, v in (sps or {}).items() if k != "spans"}
            out["by_batch"][m]["host_share"] = host_share(ctx, lambda: crypto.verify_packed(ctx, sb, MODE_IS_VALID),
                                                          args.latency_runs)
        dev = []
        for _ in range(max(3, args.latency_runs // 3)):
            t1 = time.perf_counter(); pb.verify(MODE_IS_VALID, want_verdicts=False); dev.append(time.perf_counter() - t1)
        out["p50_device_ms"] = {n: round(statistics.median(dev) * 1e3, 3)}
        pb.close()
    return out


def _subrecord(line, sub):
    """A workload's own JSON line, carried inside the driver's N = 1 line (its timing
    settings stated beside it)."""
    keep = ("metric", "value", "unit", "ms_per_step", "config", "roofline", "path_roofline", "kernels",
            "signatures_per_s", "merkle_kernels", "cpu_baseline", "checks", "latency")
    out = {k: line[k] for k in keep if k in line}
    out.update({"steps": sub.steps, "warmup": sub.warmup})
    return out


def config3_subrecord(args, dist, per_curve=1 << 20):
    """BASELINE config 3 at its stated size — 1,048,576 ECDSA_SECP256K1_SHA256 +
    1,048,576 ECDSA_SECP256R1_SHA256, distinct keys, 1 KB messages, 1 % adversarial
    (D1-D8) — timed exactly as --workload ecdsa times it, with its own VALU roofline
    (the slower curve's MSM against profiles/pmc_ecdsa.json) and CPU baseline (the C
    BC-exact port on a 65,536-signature sample, verdicts compared)."""
    sub = argparse.Namespace(**vars(args))
    sub.batch, sub.msg_bytes, sub.pool_set = per_curve, 1024, False
    sub.steps, sub.warmup, sub.latency_runs = 5, 2, 3
    sub.no_cpu_baseline, sub.cpu_sample = args.no_cpu_baseline, 65536
    return _subrecord(run_ecdsa(sub, dist), sub)


def config4_subrecord(args, dist, n_tx=1 << 20):
    """BASELINE config 4 at its stated size — 1,048,576 SignedTransactions (trader-demo /
    loadtest shapes, 70/15/15 % Ed25519/R1/K1 signatures over the recomputed 32 B ids, 1 %
    tampered), host buffers in, per-tx first failing signature out — timed exactly as
    --workload tx times it, with its PCIe roofline (host-to-device bytes per step against
    the box's measured pinned copy rate) and CPU baseline (the C port's tx ids + per-
    signature verify on a 98,304-tx sample — ~20 s of CPU work on 16 threads — ids and
    first-bad indices compared)."""
    sub = argparse.Namespace(**vars(args))
    sub.batch, sub.pool, sub.pool_set, sub.msg_bytes, sub.key_reuse = n_tx, 131072, False, None, 0
    sub.steps, sub.warmup = 5, 2
    sub.no_cpu_baseline, sub.cpu_sample = args.no_cpu_baseline, 98304
    return _subrecord(run_tx(sub, dist), sub)


# ------------------------------------------------------------------ config 3
def run_ecdsa(args, dist):
    import datagen
    from corda_amd import Context, crypto
    from corda_amd import dist as D
    from corda_amd._lib import ACCEPT, MODE_IS_VALID

    n = args.batch or (1 << 20)  # per curve
    msg_bytes = args.msg_bytes or 1024
    pool = min(args.pool, n) if args.pool_set else n  # distinct keys unless --pool caps them
    rank, world = dist.rank, dist.world
    t_gen = time.perf_counter()
    # K1 elements first, then R1; distinct keys per curve (or a pool tiled to size)
    p = datagen.make_batch(2 * pool, msg_bytes=msg_bytes, scheme=np.repeat(np.array([2, 3], np.uint8), pool),
                           seed=42 + rank, key_base=(1 << 32) + rank * 2 * pool, threads=cpu_threads())
    if pool == n:
        w = p
    else:
        k1 = p.subset(np.arange(pool)).tiled(n)
        r1 = p.subset(np.arange(pool, 2 * pool)).tiled(n)
        w = datagen.Workload(2 * n, np.concatenate([k1.scheme, r1.scheme]), np.concatenate([k1.pk, r1.pk]), 64,
                             np.concatenate([k1.sig, r1.sig]), k1.sig_stride, np.concatenate([k1.sig_len, r1.sig_len]),
                             np.concatenate([k1.msg[:-16], r1.msg]),
                             np.concatenate([k1.msg_off, r1.msg_off + np.uint64(len(k1.msg) - 16)]),
                             np.concatenate([k1.msg_len, r1.msg_len]), ["valid"] * (2 * n))
        del k1, r1
    del p
    if args.adversarial > 0:
        w = datagen.add_ecdsa_adversarial(w, frac=args.adversarial, seed=1 + rank)
    t_gen = time.perf_counter() - t_gen

    ctx = Context(dist.local_rank)
    packed = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                                w.msg_len)
    pb = crypto.PreparedBatch(ctx, packed)
    bitmap_dev = gathered = None
    if dist.d is not None:
        import torch
        nwords = (w.n + 31) // 32
        bitmap_dev = torch.zeros(nwords, dtype=torch.int32, device="cuda")
        gathered = torch.zeros(nwords * world, dtype=torch.int32, device="cuda")

    def step():
        pb.verify(MODE_IS_VALID, want_verdicts=False,
                  device_bitmap_ptr=None if bitmap_dev is None else bitmap_dev.data_ptr())
        if dist.d is not None:
            dist.d.all_gather_into_tensor(gathered, bitmap_dev)

    elapsed = timed(dist, ctx, step, args.steps, args.warmup)
    names = ["ecdsa_k1_der", "ecdsa_k1_prep", "ecdsa_k1_msm", "ecdsa_r1_der", "ecdsa_r1_prep", "ecdsa_r1_msm"]
    ks_mixed = kstats(ctx, names)
    verdict = pb.verify(MODE_IS_VALID)
    adv = np.array([c != "valid" for c in w.classes])
    untouched_ok = bool((verdict[~adv] == ACCEPT).all())
    lat_dev = []
    if rank == 0:
        for _ in range(args.latency_runs):
            t1 = time.perf_counter(); pb.verify(MODE_IS_VALID, want_verdicts=False); lat_dev.append(time.perf_counter() - t1)
    pb.close()

    # Kernel calibration outside the timed region: each curve's half verified alone,
    # so its kernels' HIP-event times are not stretched by the other curve's stream
    # (the mixed step runs both curves concurrently).
    ks = {}
    for lo, hi in ((0, n), (n, 2 * n)):
        cb = crypto.PreparedBatch(ctx, D.slice_batch(packed, lo, hi))
        cb.verify(MODE_IS_VALID, want_verdicts=False)
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(max(2, min(args.steps, 5))):
            cb.verify(MODE_IS_VALID, want_verdicts=False)
        ctx.set_profiling(False)
        ks.update(kstats(ctx, names))
        cb.close()

    value = w.n * world * args.steps / elapsed
    key = "1kb" if msg_bytes > 32 else "32b"
    ops = {"k1": OP_MODEL["ecdsa_secp256k1"][key], "r1": OP_MODEL["ecdsa_p256"][key]}
    pmc = pmc_view("pmc_ecdsa.json")
    per_curve = {}
    for c in ("k1", "r1"):
        ms = ks.get(f"ecdsa_{c}_msm", {})
        per_curve[c] = valu_roofline(pmc, f"cg_ecdsa_msm_{c}", ms.get("units_per_launch", 0),
                                     ms.get("avg_launch_ms", 0) / 1e3)
        per_curve[c]["curve_kernel_ms"] = round(sum(ks.get(f"ecdsa_{c}_{k}", {}).get("avg_launch_ms", 0)
                                                    for k in ("prep", "msm")), 3)
    dom = max(per_curve, key=lambda c: per_curve[c]["avg_launch_ms"])  # the dominant kernel: the slower msm
    roof = dict(per_curve[dom])
    roof["other_curve"] = per_curve["k1" if dom == "r1" else "r1"]
    kinstr = {c: sum((pmc.get("kernels", {}).get(f"cg_{k}_{c}", {}).get("valu_instr_per_unit") or 0)
                     for k in ("ecdsa_prep_a", "ecdsa_prep_b", "ecdsa_msm")) for c in ("k1", "r1")}
    path_instr = (kinstr["k1"] + kinstr["r1"]) / 2
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = cpu_threads()
        m = min(args.cpu_sample or 131072, n)
        idx = np.concatenate([np.arange(m // 2), n + np.arange(m // 2)])
        sample = w.subset(idx)
        cv, dt = oracle_verify(sample, threads)
        cpu = {"value": round(sample.n / dt, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
               "sample": f"{sample.n} signatures (half K1, half R1) of the same workload, C BC-1.57-exact "
                         f"restatement (oracle/liboracle.so, generic 4x64 Montgomery) on {threads} threads of "
                         f"'{host_cpu_model()}', {dt:.1f} s wall",
               "verdicts_match_gpu": bool(np.array_equal(cv, verdict[idx]))}
    line = base_line(args, dist, "ECDSA verifies/sec", "verifies/s", value, elapsed * 1e3 / args.steps, {
        "workload": f"BASELINE config 3: {n} ECDSA_SECP256K1_SHA256 + {n} ECDSA_SECP256R1_SHA256 per GPU, "
                    f"{msg_bytes} B messages, {args.adversarial:.0%} adversarial (D1-D8); "
                    + ("distinct keys" if pool == n else f"{pool} distinct signed tuples per curve tiled to size")
                    + "; every step re-parses the DER signatures (K4) from the device-resident raw rows",
        "batch_per_gpu": w.n, "global_batch": w.n * world, "msg_bytes": msg_bytes,
        "parallelism": f"dp{world} (signature-index shards)"})
    line.update({
        "roofline": roof,
        "path_roofline": {"valu_instr_per_verify": round(path_instr) or None,
                          "frac": round(path_instr * value / world / 1e12 / PEAK, 4) if path_instr else None,
                          "model_frac": round(value / world * (ops["k1"] + ops["r1"]) / 2 / 1e12 / PEAK, 4)},
        "kernels": ks, "kernels_mixed_step_overlapping": ks_mixed,
        "latency": {"p50_device_ms": round(statistics.median(lat_dev) * 1e3, 3) if lat_dev else None,
                    "runs": args.latency_runs},
        "cpu_baseline": cpu,
        "checks": {"untouched_all_accept": untouched_ok, "accepts": int((verdict == ACCEPT).sum()),
                   "datagen_s": round(t_gen, 1)},
    })
    ctx.close()
    return line


# ------------------------------------------------------------------ config 4
def merkle_ops(w):
    """§8(d) Merkle op model for a tx batch: SHA-256 blocks x 2300."""
    k = np.diff(w.comp_start).astype(np.int64)
    kp = 2 ** np.ceil(np.log2(np.maximum(k, 1))).astype(np.int64)
    is_salt = np.zeros(len(w.comp_len), dtype=bool)
    is_salt[w.comp_start[1:] - 1] = True
    blocks = np.where(is_salt, (w.comp_len.astype(np.int64) + 9 + 63) // 64,
                      (w.comp_len.astype(np.int64) + 32 + 9 + 63) // 64).sum()
    blocks += (k - 1).sum() + ((kp - 1) * 2).sum()
    return int(blocks) * OP_MODEL["primitives"]["sha256_block"]


def run_tx(args, dist):
    import datagen
    from corda_amd import Context
    from corda_amd._lib import ACCEPT, MODE_DO_VERIFY, ptr

    n_tx = args.batch or (1 << 20)
    pool = min(args.pool, n_tx)
    rank, world = dist.rank, dist.world
    t_gen = time.perf_counter()
    p = datagen.make_tx_batch(pool, seed=4 + rank, key_base=9_000_000 + rank * 4 * pool, threads=cpu_threads(),
                              tamper_frac=0.0, key_reuse=args.key_reuse)
    w = datagen.tile_tx_batch(p, n_tx, tamper_frac=args.adversarial, seed=5 + rank)
    t_gen = time.perf_counter() - t_gen
    n_sig = int(w.sig_start[-1])
    ctx = Context(dist.local_rank)
    first_bad = np.zeros(n_tx, dtype=np.int32)
    verdict = np.zeros(n_sig, dtype=np.uint8)
    ids = np.zeros(32 * n_tx, dtype=np.uint8)

    # a notary-side JVM verifier reuses its direct ByteBuffers: page-lock them once
    host_bufs = (w.arena, w.comp_off, w.comp_len, w.comp_start, w.salts, w.sig_start, w.scheme, w.pk, w.sig,
                 w.sig_len, first_bad, verdict, ids)
    ctx.register_host(*host_bufs)

    def step():
        ctx.check(ctx.lib.cg_tx_verify_batch(ctx.h, MODE_DO_VERIFY, n_tx, ptr(w.arena), len(w.arena), ptr(w.comp_off),
                                             ptr(w.comp_len), ptr(w.comp_start), ptr(w.salts), ptr(w.sig_start),
                                             ptr(w.scheme), ptr(w.pk), 64, ptr(w.sig), 72, ptr(w.sig_len),
                                             ptr(first_bad), ptr(verdict), ptr(ids)))

    elapsed = timed(dist, ctx, step, args.steps, args.warmup)
    ctx.unregister_host(*host_bufs)
    names = ["merkle_leaf", "merkle_tree", *ED_KERNELS, "ecdsa_k1_prep", "ecdsa_k1_msm",
             "ecdsa_r1_prep", "ecdsa_r1_msm"]
    ks = kstats(ctx, names)
    ids_ok = bool(np.array_equal(ids.reshape(-1, 32)[~w.tampered], w.ids.reshape(-1, 32)[~w.tampered]))
    checks = {"untampered_ids_match_signed_ids": ids_ok,
              "tampered_first_bad_is_0": bool((first_bad[w.tampered] == 0).all()),
              "untampered_all_valid": bool((first_bad[~w.tampered] == -1).all()),
              "signatures": n_sig, "datagen_s": round(t_gen, 1)}
    value = n_tx * world * args.steps / elapsed
    # Merkle kernels: the whole batch's SHA-256 op model over the summed launch time of
    # one step (the batch is hashed in several tx-range chunks, one launch pair each)
    merkle_ms = sum(ks.get(k, {}).get("avg_launch_ms", 0) * ks.get(k, {}).get("launches", 0)
                    for k in ("merkle_leaf", "merkle_tree")) / args.steps
    mops = merkle_ops(w)
    # what binds this path: the host->device upload of the caller's buffers
    h2d = (len(w.arena) + w.comp_off.nbytes + w.comp_len.nbytes + w.comp_start.nbytes + w.salts.nbytes +
           w.sig_start.nbytes + w.scheme.nbytes + w.pk.nbytes + w.sig.nbytes + w.sig_len.nbytes)
    d2h = first_bad.nbytes + verdict.nbytes + ids.nbytes
    pcie = pcie_h2d_peak_GBps(dist.local_rank)
    step_s = elapsed / args.steps
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from concurrent.futures import ThreadPoolExecutor
        threads = cpu_threads()
        m = min(args.cpu_sample or 65536, n_tx)
        lib = oracle_lib()
        t0 = time.perf_counter()
        cids = np.zeros(32 * m, dtype=np.uint8)

        def txid_slice(lo, hi):  # ctypes releases the GIL: one oracle call per thread
            cs = w.comp_start[lo:hi + 1]
            lib.oracle_txid_batch(ptr(w.arena), ptr(w.comp_off), ptr(w.comp_len), cs.ctypes.data,
                                  w.salts[32 * lo:].ctypes.data, hi - lo, cids[32 * lo:].ctypes.data)

        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda t: txid_slice(m * t // threads, m * (t + 1) // threads), range(threads)))
        ns = int(w.sig_start[m])
        msg_off = np.repeat(np.arange(m, dtype=np.uint64) * 32, np.diff(w.sig_start[:m + 1]))
        sw = datagen.Workload(ns, w.scheme[:ns], w.pk[:ns], 64, w.sig[:ns], 72, w.sig_len[:ns], cids, msg_off,
                              np.full(ns, 32, np.uint32))
        cv, _ = oracle_verify(sw, threads, mode=MODE_DO_VERIFY)
        dt = time.perf_counter() - t0
        cfb = np.full(m, -1, dtype=np.int32)
        for t in np.flatnonzero([(cv[w.sig_start[t]:w.sig_start[t + 1]] != ACCEPT).any() for t in range(m)]):
            cfb[t] = int(np.flatnonzero(cv[w.sig_start[t]:w.sig_start[t + 1]] != ACCEPT)[0])
        cpu = {"value": round(m / dt, 1), "unit": "tx/s", "cores": threads, "kind": "port",
               "sample": f"first {m} txs ({ns} signatures) of the same workload: C restatement tx ids + "
                         f"per-signature verify (oracle/liboracle.so) on {threads} threads of "
                         f"'{host_cpu_model()}', {dt:.1f} s wall",
               "ids_match_gpu": bool(np.array_equal(cids, ids[:32 * m])),
               "first_bad_match_gpu": bool(np.array_equal(cfb, first_bad[:m]))}
    line = base_line(args, dist, "SignedTransaction verifies/sec", "tx/s", value, elapsed * 1e3 / args.steps, {
        "workload": f"BASELINE config 4: {n_tx} SignedTransactions per GPU (trader-demo/loadtest shapes, "
                    f"{n_sig} signatures, 70/15/15 % Ed25519/R1/K1 over the 32 B id, {args.adversarial:.0%} "
                    f"tampered); {pool} distinct txs tiled to size; "
                    + (f"signers drawn from {args.key_reuse} keys per scheme mix; " if args.key_reuse else "")
                    + "host buffers (page-locked once via cg_register_host) in, per-tx first-bad out",
        "batch_per_gpu": n_tx, "global_batch": n_tx * world, "parallelism": f"dp{world} (tx-index shards)"})
    line.update({
        "signatures_per_s": round(n_sig * world * args.steps / elapsed, 1),
        "roofline": {"bound": "pcie", "kernel": "whole step (host buffers in, results out)",
                     "achieved": round(h2d / step_s / 1e9, 2), "peak": pcie, "unit": "GB/s",
                     "frac": round(h2d / step_s / 1e9 / pcie, 4), "traffic": h2d + d2h,
                     "h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
                     "peak_note": "measured pinned host-to-device copy rate on this box (512 MB, best of 5)"},
        "merkle_kernels": {"ms_per_step": round(merkle_ms, 3), "model_ops_per_step": mops,
                           "model_achieved_T": round(mops / (merkle_ms / 1e3) / 1e12, 3) if merkle_ms else None},
        "kernels": ks,
        "kernels_note": "HIP-event spans per kernel; the ECDSA curves run on their own streams beside the Ed25519 "
                        "kernels, so spans overlap and do not add up to the step",
        "cpu_baseline": cpu, "checks": checks})
    ctx.close()
    return line


# ------------------------------------------------------------------ §8(f) row 1
def run_ftx(args, dist):
    """Non-validating notary: FilteredTransaction.verify over a batch (SURVEY §8f
    rank 1; NonValidatingNotaryFlow.kt:25-27 -> MerkleTransaction.kt:173-178 ->
    PartialMerkleTree.kt:130-155)."""
    import datagen
    from corda_amd import Context
    from corda_amd._lib import ptr

    n = args.batch or (1 << 20)
    rank, world = dist.rank, dist.world
    t_gen = time.perf_counter()
    pool = datagen.make_ftx_batch(min(args.pool, n), seed=11 + rank)
    w = datagen.tile_ftx_batch(pool, n, adversarial=args.adversarial, seed=12 + rank)
    t_gen = time.perf_counter() - t_gen
    ctx = Context(dist.local_rank)
    out = np.zeros(n, dtype=np.uint8)
    arrs = (w.arena, w.comp_off, w.comp_len, w.comp_start, w.nonces, w.node_start, w.node_kind, w.node_hash, w.roots)
    ctx.register_host(*arrs, out)

    def step():
        ctx.check(ctx.lib.cg_ftx_verify_batch(ctx.h, n, ptr(w.arena), len(w.arena), *(ptr(x) for x in arrs[1:]),
                                              ptr(out)))

    elapsed = timed(dist, ctx, step, args.steps, args.warmup)
    ctx.unregister_host(*arrs, out)
    ks = kstats(ctx, ["merkle_leaf", "pmt_eval"])
    blocks = int(((w.comp_len.astype(np.int64) + 32 + 9 + 63) // 64).sum() + 2 * int((w.node_kind == 2).sum()))
    ops = blocks * OP_MODEL["primitives"]["sha256_block"]
    kms = sum(ks.get(k, {}).get("avg_launch_ms", 0) for k in ("merkle_leaf", "pmt_eval"))
    value = n * world * args.steps / elapsed
    h2d = len(w.arena) + sum(x.nbytes for x in arrs[1:])
    pcie = pcie_h2d_peak_GBps(dist.local_rank)
    step_s = elapsed / args.steps
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        m = min(args.cpu_sample or 2097152, n)
        lib = oracle_lib()
        lib.oracle_ftx_verify_batch.argtypes = [ctypes.c_void_p] * 9 + [ctypes.c_size_t, ctypes.c_void_p]
        cres = np.zeros(m, dtype=np.uint8)
        t0 = time.perf_counter()
        lib.oracle_ftx_verify_batch(*(x.ctypes.data for x in arrs), m, cres.ctypes.data)
        dt = time.perf_counter() - t0
        cpu = {"value": round(m / dt, 1), "unit": "ftx/s", "cores": 1, "kind": "port",
               "sample": f"first {m} filtered txs of the same workload, C restatement (oracle/liboracle.so "
                         f"oracle_ftx_verify_batch, single thread of '{host_cpu_model()}'), {dt:.1f} s wall",
               "results_match_gpu": bool(np.array_equal(cres, out[:m]))}
    line = base_line(args, dist, "FilteredTransaction verifies/sec", "ftx/s", value, elapsed * 1e3 / args.steps, {
        "workload": f"SURVEY 8(f) row 1 (non-validating notary): {n} FilteredTransactions per GPU = config-4 "
                    "transactions filtered to inputs + time window (NotaryFlow.kt:72), partial Merkle tree over "
                    f"the full tx, {args.adversarial:.0%} adversarial (component / root / tree-hash byte flips); "
                    "host buffers (page-locked once) in, results out",
        "batch_per_gpu": n, "global_batch": n * world, "parallelism": f"dp{world} (ftx-index shards)"})
    line.update({
        "roofline": {"bound": "pcie", "kernel": "whole step (host buffers in, results out)",
                     "achieved": round(h2d / step_s / 1e9, 2), "peak": pcie, "unit": "GB/s",
                     "frac": round(h2d / step_s / 1e9 / pcie, 4), "traffic": h2d + out.nbytes,
                     "h2d_bytes_per_step": h2d,
                     "peak_note": "measured pinned host-to-device copy rate on this box (512 MB, best of 5)"},
        "sha256_kernels": {"ms_per_step": round(kms, 3), "model_ops_per_step": ops, "sha256_blocks": blocks,
                           "model_achieved_T": round(ops / (kms / 1e3) / 1e12, 3) if kms else None},
        "kernels": ks, "cpu_baseline": cpu,
        "checks": {"results_match_generator": bool(np.array_equal(out, w.expected)), "false": int(out.sum()),
                   "components": int(w.comp_start[-1]), "nodes": int(w.node_start[-1]), "datagen_s": round(t_gen, 1)}})
    ctx.close()
    return line


# ------------------------------------------------------------------ config 5
def run_backlog(args, dist):
    import datagen
    from corda_amd import Context, crypto
    from corda_amd._lib import ACCEPT, MODE_IS_VALID

    from corda_amd import dist as D
    total = args.batch or 100_000_000
    rank, world = dist.rank, dist.world
    bounds = D.shard_bounds(total, world)  # 32-aligned index shards: bitmap words concatenate
    lo, hi = bounds[rank], bounds[rank + 1]
    n = hi - lo
    chunk = 1 << 24
    # distinct signed tuples per rank, tiled to the shard: 2^23 by default — about the
    # most the box's 16 host threads sign (keygen + sign, OpenSSL) in a minute
    pool = min(args.pool if args.pool_set else 1 << 23, n)
    msg_bytes = args.msg_bytes or 32
    t_gen = time.perf_counter()
    p = datagen.make_batch(pool, msg_bytes=msg_bytes, seed=42 + rank, key_base=(2 << 32) + rank * pool,
                           threads=cpu_threads(), key_reuse=args.key_reuse)
    t_gen = time.perf_counter() - t_gen
    ctx = Context(dist.local_rank)
    if not args.key_reuse:  # config 5 has distinct keys: the tiling's repeats must not reach the key-reuse path
        ctx.set_option("CORDA_AMD_KEY_REUSE", 0)
    adv_ok = [True]
    first = {}
    t_stage = time.perf_counter()

    def chunks():
        for c0 in range(0, n, chunk):
            m = min(chunk, n - c0)
            w = p.tiled(m)
            if args.adversarial > 0:
                w = datagen.add_ed25519_adversarial(w, frac=args.adversarial, seed=1000 * rank + c0 // chunk)
            pb = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg,
                                    w.msg_off, w.msg_len)
            if c0 == 0:  # verdict spot check on the first chunk; its head is the CPU-baseline sample
                v = crypto.verify_packed(ctx, pb, MODE_IS_VALID)
                adv = np.array([c != "valid" for c in w.classes])
                adv_ok[0] = bool((v[~adv] == ACCEPT).all())
                if rank == 0 and world == 1 and not args.no_cpu_baseline:
                    k = min(args.cpu_sample or 1 << 19, m)
                    first["sample"], first["verdicts"] = w.subset(np.arange(k)), v[:k].copy()
            yield pb

    # the rank's shard staged as 2^24-element chunks verified into one device bitmap (C1 input)
    backlog = D.ShardBacklog(ctx, chunks(), bounds=bounds)
    t_stage = time.perf_counter() - t_stage
    sizes = backlog.sizes
    gathered = None
    if dist.d is not None:
        import torch
        gathered = torch.zeros(backlog.words * world, dtype=torch.int32, device="cuda")
        ordered = torch.zeros((total + 31) // 32, dtype=torch.int32, device="cuda")

    def step():
        backlog.verify(MODE_IS_VALID)
        if dist.d is not None:
            backlog.allgather(gathered, ordered)  # C1: the index-ordered global bitmap

    elapsed = timed(dist, ctx, step, args.steps, args.warmup)
    ks = kstats(ctx, ED_KERNELS + ED_REUSE_KERNELS)
    value = total * args.steps / elapsed
    model = OP_MODEL["ed25519_32b" if msg_bytes <= 32 else "ed25519_1kb"]
    msm = ks.get("ed25519_msm", {})
    reuse = args.key_reuse > 0
    roof = valu_roofline(pmc_view("pmc_ed25519_reuse.json" if reuse else "pmc_ed25519.json"),
                         "cg_ed25519_msm_r" if reuse else "cg_ed25519_msm", msm.get("units_per_launch", 0),
                         msm.get("avg_launch_ms", 0) / 1e3, model["msm"])
    roof["pmc_note"] = "instruction counts from the config-2 (1 KB message) PMC pass; the msm kernel does not " \
                       "read messages, so its count per verify is the same for 32 B ids"
    cpu = None
    if first:
        threads = cpu_threads()
        sample = first["sample"]
        cv, dt = oracle_verify(sample, threads)
        cpu = {"value": round(sample.n / dt, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
               "sample": f"first {sample.n} signatures of rank 0's first chunk ({msg_bytes} B ids, incl. its "
                         f"adversarial elements), C i2p-exact restatement (oracle/liboracle.so) on {threads} threads "
                         f"of '{host_cpu_model()}', {dt:.1f} s wall",
               "verdicts_match_gpu": bool(np.array_equal(cv, first["verdicts"]))}
    line = base_line(args, dist, "Ed25519 verifies/sec (100M notary backlog)", "verifies/s", value,
                     elapsed * 1e3 / args.steps, {
                         "workload": f"BASELINE config 5: {total} EDDSA_ED25519_SHA512 signatures over {msg_bytes} B "
                                     f"tx ids split by index over {world} GPU(s), staged in 2^24 chunks, "
                                     f"{args.adversarial:.0%} adversarial; {pool} distinct signed tuples per rank "
                                     "tiled to size" + ("" if args.key_reuse else
                                                        " (balanced per-signature path forced, "
                                                        "CORDA_AMD_KEY_REUSE=0: no key dedupe of the tiling)"),
                         "batch_per_gpu": n, "global_batch": total,
                         "parallelism": f"dp{world} (index shards" + (", RCCL all-gather)" if world > 1 else ")")},
                     scaling="strong")
    line.update({
        "roofline": roof,
        "kernels": ks, "cpu_baseline": cpu,
        "checks": {"first_chunk_untouched_all_accept": adv_ok[0], "datagen_s": round(t_gen, 1),
                   "distinct_tuples_per_rank": pool,
                   "stage_s": round(t_stage, 1), "chunks": len(sizes)}})
    backlog.close()
    ctx.close()
    return line


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        return rc
    dist = Dist(cpu=args.dry_run)
    run = run_dry if args.dry_run else {"ed25519": run_ed25519, "ecdsa": run_ecdsa, "tx": run_tx,
                                        "backlog": run_backlog, "ftx": run_ftx}[args.workload]
    line = run(args, dist)
    if (args.workload == "ed25519" and not args.dry_run and dist.world == 1 and not args.no_extra
            and not args.key_reuse and not args.batch and not args.msg_bytes):
        # the driver's N = 1 line also carries the production tx-id shape end to end and
        # driver-observed configs 3 and 4 at their BASELINE sizes (each from its own
        # context, after the config-2 timing)
        line["latency_32b"] = e2e_record_32b(args, dist)
        line["config3"] = config3_subrecord(args, dist)
        line["config4"] = config4_subrecord(args, dist)
    if dist.rank == 0:
        line["kernel_src_hash"] = kernel_src_hash()
        print(json.dumps(line), flush=True)
    dist.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
