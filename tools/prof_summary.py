#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace CSV per (kernel, grid size), and join
--pmc counter CSVs per kernel.  Used to produce the committed profiles/*.json.

    python tools/prof_summary.py trace gpurun_out/prof/x_kernel_trace.csv
    python tools/prof_summary.py pmc gpurun_out/pmc/x_counter_collection.csv [more.csv]
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    """Kernel name without the signature; template instances of the two ECDSA
    curves (and the two batched-inversion moduli) get a suffix."""
    m = re.search(r"(cg_[a-z0-9_]+|k_[a-z0-9_]+|__amd_rocclr_[A-Za-z]+)", name)
    base = m.group(1) if m else name[:60]
    for tag, suf in (("InvN", "_n"), ("InvP", "_p")):
        if tag in name:
            base += suf
    for tag, suf in (("CurveK1", "_k1"), ("CurveR1", "_r1")):
        if tag in name:
            base += suf
    return base


def trace(path):
    rows = list(csv.DictReader(open(path)))
    groups = defaultdict(list)
    meta = {}
    for r in rows:
        k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]))
        groups[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        meta[k] = {"vgpr": int(r.get("VGPR_Count", 0) or 0), "agpr": int(r.get("Accum_VGPR_Count", 0) or 0),
                   "sgpr": int(r.get("SGPR_Count", 0) or 0), "lds": int(r.get("LDS_Block_Size", 0) or 0),
                   "wg": int(r["Workgroup_Size_X"])}
    out = []
    for (k, g), ds in sorted(groups.items(), key=lambda x: -sum(x[1])):
        out.append({"kernel": k, "grid_threads": g, "calls": len(ds), "avg_ms": round(statistics.mean(ds), 4),
                    "median_ms": round(statistics.median(ds), 4), "min_ms": round(min(ds), 4),
                    "total_ms": round(sum(ds), 3), **meta[(k, g)]})
    return out


def pmc(paths):
    agg = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = (short(r["Kernel_Name"]), int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for (k, g), cs in agg.items():
        out.append({"kernel": k, "grid_threads": g,
                    "counters_per_dispatch": {c: statistics.median(v) for c, v in cs.items()}})
    return out


if __name__ == "__main__":
    mode = sys.argv[1]
    res = trace(sys.argv[2]) if mode == "trace" else pmc(sys.argv[2:])
    print(json.dumps(res, indent=1))
