"""bench.py's multi-GPU plumbing on CPU (no GPU): the --gpus N launcher starts N
rank processes itself (so the driver's `python bench.py --gpus N` really runs N
ranks), a WORLD_SIZE that disagrees with --gpus is refused, a failing rank fails
the launcher, and the roofline helper reports fractions of the 78.6 T peak."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def _run(args, env, timeout=180):
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True,
                          timeout=timeout, cwd="/tmp")


@pytest.mark.parametrize("n", [2, 3, 8])
def test_launcher_spawns_n_gloo_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "1000"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == n and line["steps"] == 3 and line["warmup"] == 1
    assert line["config"]["global_batch"] == 1000 * n
    assert line["checks"]["bitmap_matches"] is True


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--dry-run"], _env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_failing_rank_fails_the_launcher():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "2"], _env(CORDA_AMD_DRY_FAIL_RANK="1"), timeout=240)
    assert r.returncode != 0


def test_hung_rank_times_out_at_world_8():
    """One of 8 ranks hangs before its first collective: the others' collectives hit the
    process-group timeout (CORDA_AMD_DIST_TIMEOUT_S, the same bound bench.py puts on RCCL)
    and fail, the launcher stops the hung rank and exits non-zero — no stall."""
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "8", "--dry-run", "--steps", "2"],
             _env(CORDA_AMD_DRY_HANG_RANK="5", CORDA_AMD_DIST_TIMEOUT_S="8"), timeout=240)
    assert r.returncode != 0
    assert time.monotonic() - t0 < 120
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_cpu_thread_budget_per_rank(monkeypatch):
    """Datagen / CPU-baseline threads: the 16-CPU share split over the node's ranks."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    for world, want in ((None, 16), ("1", 16), ("2", 8), ("8", 2), ("32", 1)):
        monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
        monkeypatch.delenv("WORLD_SIZE", raising=False)
        if world:
            monkeypatch.setenv("LOCAL_WORLD_SIZE", world)
        assert bench.cpu_threads() == want


def test_single_rank_dry_run_without_launcher():
    r = _run(["--dry-run", "--steps", "2"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_valu_roofline_fraction_of_peak():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.PEAK == pytest.approx(78.6)
    pmc = {"source": "x", "src_hash": bench.kernel_src_hash(),
           "kernels": {"cg_ed25519_msm": {"valu_instr_per_unit": 200000, "hbm_bytes_per_unit": 1000.0}}}
    r = bench.valu_roofline(pmc, "cg_ed25519_msm", 1 << 20, 7.5e-3, model_ops=987510)
    ach = 200000 * (1 << 20) / 7.5e-3 / 1e12
    assert r["achieved"] == pytest.approx(ach, rel=1e-3)
    assert r["frac"] == pytest.approx(ach / 78.6, rel=1e-3) and r["frac"] <= 1
    assert r["pmc_src_hash_matches"] is True
    assert r["traffic"] == 1000 * (1 << 20)
    assert r["model_frac"] > 1  # the op model is not a roofline (see valu_roofline's docstring)
    stale = dict(pmc, src_hash="0" * 16)
    assert bench.valu_roofline(stale, "cg_ed25519_msm", 1, 1.0)["pmc_src_hash_matches"] is False


def test_pmc_report_hash_matches_bench_hash():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    sys.path.insert(0, ROOT)
    import bench
    import pmc_report
    assert pmc_report.src_identity()[1] == bench.kernel_src_hash()


@pytest.mark.parametrize("n,batch", [(8, None), (3, 1000003), (7, None)])
def test_backlog_dry_run_config5_shards(n, batch):
    """Config 5's C1 at the driver's rank counts: 100 M signatures (default) split into
    32-aligned shards — even at 8 ranks, uneven at 3 and 7 — each rank's bitmap gathered
    with corda_amd.dist.gather_ordered (ShardBacklog.allgather's collective) over gloo; rank
    0 checks the global bitmap is in index order, bit for bit."""
    args = ["--gpus", str(n), "--dry-run", "--workload", "backlog", "--steps", "2", "--warmup", "1"]
    if batch:
        args += ["--batch", str(batch)]
    r = _run(args, _env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert line["n_gpus"] == n and line["config"]["global_batch"] == (batch or 100_000_000)
    assert sum(line["config"]["shard_elements"]) == (batch or 100_000_000)
    if n != 8:
        assert len(set(line["config"]["shard_elements"])) > 1  # really uneven
    assert line["checks"]["bitmap_matches"] is True
