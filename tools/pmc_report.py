#!/usr/bin/env python3
"""Reduce a tools/profile_gpu.sh run into the committed profile summaries.

    python tools/pmc_report.py gpurun_out/prof_r01b r01b [--grid 1048576]

Writes profiles/<tag>_rocprof_kernel_stats.csv (rocprofv3 --stats output),
profiles/<tag>_rocprof_trace_summary.json, profiles/<tag>_pmc/ (raw counter CSVs),
profiles/<tag>_pmc_summary.json and refreshes profiles/pmc_traffic.json, which
bench.py reads for the `traffic` field and the hardware-VALU view.

Conventions (MI355X_MICROARCH.md, HBM / rocprofv3 section):
  * SQ_INSTS_VALU counts wave instructions; per-lane (= per-verify) count is
    SQ_INSTS_VALU / SQ_WAVES.
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration.
  * FETCH_SIZE / WRITE_SIZE are KiB; HBM bytes = (c * FETCH_SIZE + WRITE_SIZE) * 1024
    with c = 2 for kernels whose dominant loads are 16 B per lane (the guide's gfx950
    rule: FETCH_SIZE reports half of those bytes) and c = 1 otherwise.
  * peak = 256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from prof_summary import short, trace  # noqa: E402

PEAK_LANE_OPS_PER_CLK = 256 * 4 * 32  # CUs x SIMD-32 units x lanes (MI355X_MICROARCH.md)
PEAK_T = 78.6  # at 2.4 GHz
SIMDS = 256 * 4


def isa_regs():
    path = os.path.join(ROOT, "profiles", "isa_registers.json")
    return json.load(open(path))["kernels"] if os.path.exists(path) else {}


def occupancy(e, c, regs):
    """Register pressure (code object, tools/isa_regs.py) and the measured mean
    residency: SQ_WAVE_CYCLES counts quad-cycles summed over waves, GRBM_GUI_ACTIVE
    cycles summed over the 8 XCDs (MI355X_MICROARCH.md, PMC units)."""
    k = e.get("kernel_short", "")
    r = regs.get(k) or next((v for n, v in regs.items() if n.startswith(k + "<")), {})
    m = re.match(r"(.*?)(?:_([np]))?_([kr]1)$", k)  # prof_summary.short() names of the curve templates
    if not r and m:
        base, inv, curve = m.group(1), m.group(2), m.group(3).upper()
        r = regs.get(f"{base}<Inv{inv.upper()}<{curve}> >" if inv else f"{base}<{curve}>", {})
    for key in ("vgpr", "agpr", "sgpr", "vgpr_spill", "scratch_bytes", "lds_bytes", "waves_per_simd_limit"):
        if key in r:
            e[key] = r[key]
    if c.get("SQ_WAVE_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
        e["mean_waves_per_simd"] = round(4 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS), 3)


def load_counters(paths, grid):
    agg = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if int(r.get("Grid_Size", 0) or 0) != grid:
                continue
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[(k, r["Counter_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
    return agg, dur


def occupancy_fields(kernels):
    out = {}
    for k in ("hash", "points", "msm"):
        e = kernels.get(f"cg_ed25519_{k}", {})
        out[f"ed25519_{k}_occupancy"] = {key: e.get(key) for key in
                                         ("vgpr", "vgpr_spill", "waves_per_simd_limit", "mean_waves_per_simd")}
    return out


def augment(tag):
    """Adds register pressure and mean residency to an existing summary (from its
    stored counters): python tools/pmc_report.py --augment r01p"""
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.json")
    summary = json.load(open(path))
    regs = isa_regs()
    for k, e in summary["kernels"].items():
        e["kernel_short"] = k
        occupancy(e, e.get("counters", {}), regs)
        e.pop("kernel_short")
        e["counters"] = e.pop("counters", {})
    with open(path, "w") as f:
        json.dump(summary, f, indent=1)
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath))
        if traffic.get("source") == f"profiles/{tag}_pmc_summary.json":
            traffic.update(occupancy_fields(summary["kernels"]))
            with open(tpath, "w") as f:
                json.dump(traffic, f, indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "counters"} for k, v in summary["kernels"].items()},
                     indent=1))


def src_identity():
    """(git commit, kernel source hash) of the tree being profiled; bench.py
    recomputes the hash to tell whether a summary matches its kernels."""
    import hashlib
    src_hash = None
    try:
        d = os.path.join(ROOT, "corda_amd", "csrc")
        h = hashlib.sha256()
        for name in sorted(os.listdir(d)):
            if name.endswith((".hip", ".h")) or name == "Makefile":
                with open(os.path.join(d, name), "rb") as f:
                    h.update(name.encode() + b"\0" + f.read())
        src_hash = h.hexdigest()[:16]
    except OSError:
        pass
    commit = os.environ.get("PROFILE_COMMIT")
    if not commit:
        try:
            import subprocess
            commit = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"],
                                             stderr=subprocess.DEVNULL).decode().strip()
        except Exception:  # noqa: BLE001 (no git on the box: the caller passes PROFILE_COMMIT)
            commit = None
    return commit, src_hash


# kernels whose dominant loads are 16-B-per-lane (global_load_dwordx4): FETCH_SIZE
# counts half of those bytes on gfx950 (MI355X_MICROARCH.md, HBM / rocprofv3)
WIDE_LOAD_KERNELS = ("cg_ed25519_msm", "cg_ecdsa_msm_k1", "cg_ecdsa_msm_r1", "cg_merkle_leaf", "cg_ecdsa_prep_a_k1",
                     "cg_ecdsa_prep_a_r1")


def main():
    if sys.argv[1] == "--augment":
        return augment(sys.argv[2])
    src, tag = sys.argv[1], sys.argv[2]
    grid = int(sys.argv[sys.argv.index("--grid") + 1]) if "--grid" in sys.argv else 1 << 20
    out_name = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "pmc_ed25519.json"
    prof = os.path.join(ROOT, "profiles")
    tr = glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)
    st = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        shutil.copy(st[0], os.path.join(prof, f"{tag}_rocprof_kernel_stats.csv"))
    trace_rows = trace(tr[0]) if tr else []
    with open(os.path.join(prof, f"{tag}_rocprof_trace_summary.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --kernel-trace --stats over bench.py (tools/profile_gpu.sh {tag})",
                   "kernels": trace_rows}, f, indent=1)
    pmc_csv = sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True))
    raw_dir = os.path.join(prof, f"{tag}_pmc")
    os.makedirs(raw_dir, exist_ok=True)
    for p in pmc_csv:
        shutil.copy(p, os.path.join(raw_dir, os.path.basename(p)))
    agg, dur = load_counters(pmc_csv, grid)
    regs = isa_regs()
    kernels = {}
    for k, cs in agg.items():
        c = {n: statistics.median(v) for n, v in cs.items()}
        d = {n: statistics.median(dur[(k, n)]) for n in cs}
        t_ms = [r["avg_ms"] for r in trace_rows if r["kernel"] == k and r["grid_threads"] == grid]
        avg_s = t_ms[0] / 1e3 if t_ms else d.get("SQ_INSTS_VALU", 0.0)
        e = {"grid_threads": grid, "avg_ms_trace": round(avg_s * 1e3, 4)}
        waves = c.get("SQ_WAVES") or grid / 64
        if "SQ_INSTS_VALU" in c:
            per_lane = c["SQ_INSTS_VALU"] / waves
            lane_ops = per_lane * grid / avg_s
            e["valu_instr_per_unit"] = round(per_lane)
            e["valu_lane_ops_per_s_T"] = round(lane_ops / 1e12, 2)
            e["frac_of_78.6T_peak"] = round(lane_ops / (PEAK_T * 1e12), 4)
            if "SQ_INSTS_VALU_INT64" in c:
                e["int64_instr_per_unit"] = round(c["SQ_INSTS_VALU_INT64"] / waves)
            if "GRBM_GUI_ACTIVE" in c and d.get("GRBM_GUI_ACTIVE"):
                clk = c["GRBM_GUI_ACTIVE"] / 8 / d["GRBM_GUI_ACTIVE"]
                e["effective_clock_GHz"] = round(clk / 1e9, 3)
                e["frac_of_peak_at_measured_clock"] = round(
                    c["SQ_INSTS_VALU"] * 64 / d["SQ_INSTS_VALU"] / (PEAK_LANE_OPS_PER_CLK * clk), 4)
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_BUSY_CYCLES" in c:
            e["active_valu_per_busy_cycle"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_BUSY_CYCLES"], 3)
        if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
            e["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
            e["wait_inst_any_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            fetch = c["FETCH_SIZE"] * (2 if k in WIDE_LOAD_KERNELS else 1)
            b = (fetch + c["WRITE_SIZE"]) * 1024
            e["fetch_correction"] = 2 if k in WIDE_LOAD_KERNELS else 1
            e["hbm_bytes_per_launch"] = round(b)
            e["hbm_bytes_per_unit"] = round(b / grid, 1)
            e["hbm_GBps"] = round(b / avg_s / 1e9, 1)
        if "TCC_HIT_sum" in c:
            e["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1), 4)
        e["kernel_short"] = k
        occupancy(e, c, regs)
        e.pop("kernel_short")
        e["counters"] = c
        kernels[k] = e
    commit, src_hash = src_identity()
    summary = {"source": f"rocprofv3 --pmc passes over `python3 bench.py --steps 3` (tools/profile_gpu.sh {tag}); "
                         f"raw CSVs in profiles/{tag}_pmc/",
               "commit": commit, "src_hash": src_hash,
               "notes": __doc__.split("Conventions")[1].strip().splitlines(),
               "kernels": kernels}
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # the per-kernel view bench.py joins with its own HIP-event times
    view = {"source": f"profiles/{tag}_pmc_summary.json", "commit": commit, "src_hash": src_hash,
            "peak_T": PEAK_T, "kernels": {}}
    for k, e in kernels.items():
        if e.get("valu_instr_per_unit", 0) < 500:
            continue  # staging / bitmap helpers
        view["kernels"][k] = {key: e.get(key) for key in ("valu_instr_per_unit", "int64_instr_per_unit",
                                                            "hbm_bytes_per_unit", "effective_clock_GHz",
                                                            "frac_of_peak_at_measured_clock", "l2_hit_rate")}
        view["kernels"][k]["occupancy"] = {key: e.get(key) for key in
                                           ("vgpr", "vgpr_spill", "waves_per_simd_limit", "mean_waves_per_simd")}
    with open(os.path.join(prof, out_name), "w") as f:
        json.dump(view, f, indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "counters"} for k, v in kernels.items()},
                     indent=1))


if __name__ == "__main__":
    main()
