"""Per-opcode census of the P-256 (or secp256k1) MSM's dynamic VALU instruction stream
(cg_ecdsa_msm<C> in ecdsa_kernels.hip, ecdsa_joint / ecdsa_joint_glv in cg_ecdsa.h),
weighted by gfx950's measured issue rates — the ECDSA counterpart of tools/isa_census.py.

    make -C corda_amd/csrc isa
    python tools/ecdsa_census.py [--curve R1] [--pmc profiles/pmc_ecdsa.json] [--frac 0.477]
        [--out profiles/r06_ecdsa_census.json]

The listing is cut into straight-line segments at every label and branch.  P-256's joint
loop runs 65 windows (i = 64..0): the doubling loop (the segment that branches to itself)
4 x 64 times; the Q mixed addition (the first segment of >= 1,300 instructions after it) 65
times, the G mixed addition (the next such segment but the exceptional ones) 17 times (16-bit
windows, i % 4 == 0); each addition's exceptional arm (P == +-Q: an inline doubling,
crafted keys only) 0 times; the other segments of the loop body 65 times (the G arm's 17);
the prologue (prep_b folded in: scalars, digits, the k Q table to affine; its one inner
loop 7 times, k = 2..8) and the x check once.  The modelled total is printed against the
PMC pass's SQ_INSTS_VALU / SQ_WAVES.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_census as C  # noqa: E402

MANGLED = {"R1": "_ZN12_GLOBAL__N_112cg_ecdsa_msmIN2cg7CurveR1", "K1": "_ZN12_GLOBAL__N_112cg_ecdsa_msmIN2cg7CurveK1"}


def segments(asm: str, prefix: str):
    lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    segs, cur, ops = [], "entry", []
    for i in range(start + 1, end):
        t = lines[i].strip()
        m = re.match(r"^(\.LBB\d+_\d+):", t)
        if m:
            segs.append({"label": cur, "ops": ops, "br": None})
            cur, ops = m.group(1), []
            continue
        if t.startswith("v_"):
            ops.append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm")):
            segs.append({"label": cur, "ops": ops, "br": t.split(";")[0].strip()})
            cur, ops = cur + "'", []
    segs.append({"label": cur, "ops": ops, "br": None})
    return segs


def r1_multiplicities(segs, windows=65, g_adds=17):
    idx = {s["label"]: k for k, s in enumerate(segs)}
    dbl = next(k for k, s in enumerate(segs) if s["br"] and s["br"].split()[-1] == s["label"])
    latch = max(k for k, s in enumerate(segs) if s["br"] and s["br"].startswith("s_branch")
                and idx.get(s["br"].split()[-1], 1 << 30) < k)
    header = idx[segs[latch]["br"].split()[-1]]
    big = [k for k in range(dbl + 1, latch) if len(segs[k]["ops"]) >= 1300]
    q_main, q_exc, g_main, g_exc = big[:4]
    mult = [1.0] * len(segs)
    inner = [k for k in range(header) if segs[k]["br"] and segs[k]["br"].startswith("s_branch")
             and idx.get(segs[k]["br"].split()[-1], 1 << 30) <= k]
    for k in range(len(segs)):
        if header <= k <= latch:
            mult[k] = windows
        if k == dbl:
            mult[k] = 4 * (windows - 1)
        elif k in (q_exc, g_exc):
            mult[k] = 0
        elif g_main <= k < latch - 1:
            mult[k] = g_adds
    for k in inner:  # the prologue's inner loop (k Q table to affine): the loop body segment
        mult[k] = 7
    return mult, {"doubling": segs[dbl]["label"], "q_add": segs[q_main]["label"], "g_add": segs[g_main]["label"],
                  "window_header": segs[header]["label"], "latch": segs[latch]["label"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=os.path.join(ROOT, "corda_amd", "csrc", "build", "ecdsa_kernels.s"))
    ap.add_argument("--curve", default="R1", choices=["R1"])
    ap.add_argument("--rates", default=os.path.join(ROOT, "profiles", "r02a_isa_rates.json"))
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_ecdsa.json"))
    ap.add_argument("--frac", type=float, default=None, help="measured fraction of the 78.6 T peak (bench roofline)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rates = C.load_rates(a.rates)
    segs = segments(a.asm, MANGLED[a.curve])
    mult, regions = r1_multiplicities(segs)
    cnt, cyc = collections.Counter(), collections.Counter()
    per_region = collections.Counter()
    for s, m in zip(segs, mult):
        for t in s["ops"]:
            k = C.op_key(t)
            cnt[k] += m
            cyc[k] += m * C.cycles_of(k, rates)
        lab = s["label"]
        tag = "doubling" if lab == regions["doubling"] else "q_add" if lab == regions["q_add"] else \
            "g_add" if lab == regions["g_add"] else "other"
        per_region[tag] += m * len(s["ops"])
    n, c = sum(cnt.values()), sum(cyc.values())
    pmc = json.load(open(a.pmc))
    kname = f"cg_ecdsa_msm_{a.curve.lower()}"
    target = (pmc.get("kernels", {}).get(kname) or {}).get("valu_instr_per_unit")
    four = sum(v for k, v in cnt.items() if C.cycles_of(k, rates) > 3.0)
    ceiling = 2.0 * n / c
    # the same mix with the VCC-mask v_cndmask_b32 at an SGPR mask's 4 cycles (r06g A/B:
    # replacing the MSM's VCC selects by bit selects measured no faster)
    c_vcc4 = c - cyc["v_cndmask_b32 (vcc)"] + 4.17 * cnt["v_cndmask_b32 (vcc)"]
    out = {"kernel": kname, "asm": os.path.relpath(a.asm, ROOT), "rates": os.path.relpath(a.rates, ROOT),
           "pmc_valu_per_verify": target, "model_valu_per_verify": round(n),
           "model_vs_pmc": round(n / target, 4) if target else None,
           "regions": regions, "valu_per_verify_by_region": {k: round(v) for k, v in per_region.items()},
           "instr_per_doubling": len(segs[[s["label"] for s in segs].index(regions["doubling"])]["ops"]),
           "instr_per_q_add": len(segs[[s["label"] for s in segs].index(regions["q_add"])]["ops"]),
           "issue_cycles_per_verify": round(c), "avg_cycles_per_instr": round(c / n, 3),
           "four_cycle_share": round(four / n, 3), "issue_ceiling_frac": round(ceiling, 4),
           "issue_ceiling_frac_vcc_cndmask_at_4_cycles": round(2.0 * n / c_vcc4, 4),
           "opcodes": [{"op": k, "per_verify": round(v), "share": round(v / n, 4),
                        "cycles_each": round(C.cycles_of(k, rates), 2), "cycle_share": round(cyc[k] / c, 4)}
                       for k, v in cnt.most_common()]}
    if a.frac is not None:
        out["measured_frac"] = a.frac
        out["issue_util"] = round(a.frac / ceiling, 4)
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "opcodes"}, indent=1))
    for o in out["opcodes"][:14]:
        print(f"  {o['op']:26s} {o['per_verify']:8d}  {o['share']:.3f}  x{o['cycles_each']:.2f}  cyc {o['cycle_share']:.3f}")


if __name__ == "__main__":
    main()
