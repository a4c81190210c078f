"""Per-opcode census of a kernel's DYNAMIC VALU instruction stream, weighted by the
measured issue rates of gfx950 (profiles/r02a_isa_rates.json, tools/ubench/isa_rates.hip):
what the instruction mix alone allows (the issue ceiling) and how close the measured
kernel gets to it.

    python tools/isa_census.py [--asm corda_amd/csrc/build/ed25519_kernels.s]
        [--pmc profiles/pmc_ed25519.json] [--frac 0.447] [--out profiles/r05_msm_census.json]

`make -C corda_amd/csrc isa` writes the listing.  The dynamic multiplicity of each
static instruction of cg_ed25519_msm comes from its control flow (ed25519_msm in
cg_ed25519.h): the window loop (header = the target of the loop's closing s_branch)
runs W times; inside it the doubling loop (the s_cbranch_scc0 back edge) runs 3 times per
window after the first, the rest of the "j != nwin - 1" arm W - 1 times, the else arm
(the first window: the add into the identity, after s_andn2_saveexec) once, the common
R-addition part W times, and the B-window arm (the last block before the closing
s_branch) 128 / 16 = 8 times.  W (the wave's digit count, ~34) is solved so the model's
VALU total equals the PMC pass's SQ_INSTS_VALU / SQ_WAVES per verify.

Cycles per wave64 instruction = 2 * 78.64 / R, R = the opcode's measured lane-op rate in
T/s (78.64 T = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz); an opcode the table lacks counts
4 cycles (every VALU op outside the short 2-cycle list is 4-cycle on gfx950).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 78.64  # T lane-ops/s at 2.4 GHz

# ISA mnemonic (without the _e32/_e64 encoding suffix) -> key in r02a_isa_rates.json
RATE_KEY = {
    "v_mad_i64_i32": "mad_i64_i32", "v_mad_u64_u32": "mad_u64_u32", "v_mul_lo_u32": "mul_lo_u32",
    "v_mul_hi_u32": "mul_hi_u32", "v_mad_i32_i24": "mad_i32_i24", "v_mad_u32_u24": "mad_u32_u24",
    "v_mul_u32_u24": "mul_u32_u24", "v_mul_i32_i24": "mul_i32_i24",
    "v_lshlrev_b32": "lshlrev_b32", "v_lshrrev_b32": "lshrrev_b32", "v_ashrrev_i32": "ashrrev_i32",
    "v_ashrrev_i64": "ashr_i64", "v_lshlrev_b64": "lshlrev_b64", "v_lshrrev_b64": "lshrrev_b64",
    "v_lshl_add_u64": "lshl_add_u64", "v_lshl_add_u32": "lshl_add", "v_lshl_or_b32": "lshl_or",
    "v_and_b32": "and_b32", "v_or_b32": "or_b32", "v_xor_b32": "xor_b32", "v_not_b32": "not_b32",
    "v_and_or_b32": "and_or", "v_or3_b32": "or3_b32", "v_bitop3_b32": "bitop3", "v_xad_u32": "xad",
    "v_add_u32": "add_const", "v_sub_u32": "sub_u32", "v_subrev_u32": "subrev_u32", "v_add3_u32": "add3_u32",
    "v_add_co_u32": "add_co_u32", "v_addc_co_u32": "addc_co_u32", "v_sub_co_u32": "sub_co_u32",
    "v_subb_co_u32": "addc_co_u32", "v_subrev_co_u32": "sub_co_u32",
    "v_mov_b32": "mov_b32", "v_mov_b64": "mov_b64", "v_alignbit_b32": "alignbit", "v_bfe_u32": "bfe_u32",
    "v_bfe_i32": "bfe_i32", "v_bfi_b32": "bfi_b32", "v_perm_b32": "perm_b32", "v_max_i32": "max_i32",
    "v_min_u32": "min_u32", "v_bcnt_u32_b32": "bcnt", "v_add_f32": "add_f32", "v_mul_f32": "mul_f32",
    "v_fma_f32": "fma_f32", "v_fma_f64": "fma_f64", "v_mul_f64": "mul_f64", "v_add_f64": "add_f64",
}


def load_rates(path):
    with open(path) as f:
        return {k: v["Tops"] for k, v in json.load(f)["rates"].items()}


def op_key(text: str) -> str:
    op = text.split()[0]
    base = re.sub(r"_e(32|64)$", "", op)
    if base == "v_cndmask_b32":  # the lane mask in VCC issues ~5x slower than in an SGPR pair
        return "v_cndmask_b32 (vcc)" if "vcc" in text.split(",")[-1] or op.endswith("_e32") else "v_cndmask_b32 (sgpr)"
    return base


def cycles_of(key: str, rates: dict) -> float:
    if key == "v_cndmask_b32 (vcc)":
        return 2 * PEAK / rates["cndmask"]
    if key == "v_cndmask_b32 (sgpr)":
        return 2 * PEAK / rates["cndmask_s"]
    r = rates.get(RATE_KEY.get(key, ""), 0.0)
    return 2 * PEAK / r if r else 4.0


def kernel_lines(asm_path: str, kernel: str):
    lines = open(asm_path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel) and l.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    out = []  # (label or None, instruction text)
    for l in lines[start:end + 1]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            out.append((m.group(1), None))
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        out.append((None, t))
    return out


def msm_multiplicities(items, W: float):
    """Multiplicity of every instruction of cg_ed25519_msm as a function of W."""
    insts = [t for _, t in items if t]
    pos, labels = 0, {}
    for lab, t in items:
        if lab:
            labels[lab] = pos
        else:
            pos += 1
    # the closing branch of the window loop: the last s_branch whose target precedes it
    close = max(i for i, t in enumerate(insts) if t.startswith("s_branch") and labels[t.split()[1]] < i)
    header = labels[insts[close].split()[1]]
    inner_end = next(i for i, t in enumerate(insts) if t.startswith("s_cbranch_scc0") and labels[t.split()[1]] < i)
    inner_start = labels[insts[inner_end].split()[1]]
    else_at = next(i for i in range(inner_end, close) if insts[i].startswith("s_andn2_saveexec"))
    # the else arm ends at the next label (its join)
    label_pos = sorted(labels.values())
    join = next(p for p in label_pos if p > else_at + 1)
    bwin_at = max(i for i in range(join, close) if insts[i].startswith("s_cbranch_execz"))
    mult = [1.0] * len(insts)
    for i in range(len(insts)):
        if header <= i < inner_start:
            mult[i] = W  # window prologue: digit words, entry loads
        elif inner_start <= i <= inner_end:
            mult[i] = 3 * (W - 1)  # three doublings per window after the first
        elif inner_end < i <= else_at:
            mult[i] = W - 1  # 4th doubling, p1p1 -> p3, A addition
        elif else_at < i < join:
            mult[i] = 1  # first window: A added into the identity
        elif join <= i <= bwin_at:
            mult[i] = W  # R addition
        elif bwin_at < i <= close:
            mult[i] = 8  # 16-bit B windows: 2 x 128 / 16 mixed additions
    return insts, mult, dict(header=header, inner=(inner_start, inner_end), else_arm=(else_at, join),
                             bwin=(bwin_at, close))


def census(insts, mult, rates):
    cnt, cyc = collections.Counter(), collections.Counter()
    for t, m in zip(insts, mult):
        if not t.startswith("v_"):
            continue
        k = op_key(t)
        cnt[k] += m
        cyc[k] += m * cycles_of(k, rates)
    return cnt, cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=os.path.join(ROOT, "corda_amd", "csrc", "build", "ed25519_kernels.s"))
    ap.add_argument("--kernel", default="_ZN12_GLOBAL__N_114cg_ed25519_msmE")
    ap.add_argument("--rates", default=os.path.join(ROOT, "profiles", "r02a_isa_rates.json"))
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_ed25519.json"))
    ap.add_argument("--frac", type=float, default=None, help="measured fraction of the 78.6 T peak (bench roofline)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rates = load_rates(a.rates)
    items = kernel_lines(a.asm, a.kernel)
    pmc = json.load(open(a.pmc))
    msm = pmc["kernels"]["cg_ed25519_msm"] if "kernels" in pmc else pmc
    target = float(msm["valu_instr_per_unit"])
    # solve W: the VALU total is affine in W
    tot = []
    for W in (30.0, 40.0):
        insts, mult, regions = msm_multiplicities(items, W)
        tot.append(sum(m for t, m in zip(insts, mult) if t.startswith("v_")))
    W = 30.0 + 10.0 * (target - tot[0]) / (tot[1] - tot[0])
    insts, mult, regions = msm_multiplicities(items, W)
    cnt, cyc = census(insts, mult, rates)
    n, c = sum(cnt.values()), sum(cyc.values())
    four = sum(v for k, v in cnt.items() if cycles_of(k, rates) > 3.0)
    ceiling = 2.0 * n / c  # fraction of the peak the mix allows at full issue
    out = {"kernel": "cg_ed25519_msm", "asm": os.path.relpath(a.asm, ROOT), "rates": os.path.relpath(a.rates, ROOT),
           "pmc_valu_per_verify": target, "windows_W": round(W, 2), "model_valu_per_verify": round(n),
           "issue_cycles_per_verify": round(c), "avg_cycles_per_instr": round(c / n, 3),
           "four_cycle_share": round(four / n, 3), "int64_ops": round(sum(cnt[k] for k in (
               "v_mad_i64_i32", "v_mad_u64_u32", "v_ashrrev_i64", "v_lshlrev_b64", "v_lshrrev_b64", "v_lshl_add_u64",
               "v_mov_b64"))),
           "issue_ceiling_frac": round(ceiling, 4), "regions": regions,
           "opcodes": [{"op": k, "per_verify": round(v), "share": round(v / n, 4),
                        "cycles_each": round(cycles_of(k, rates), 2), "cycle_share": round(cyc[k] / c, 4)}
                       for k, v in cnt.most_common()]}
    if a.frac is not None:
        out["measured_frac"] = a.frac
        out["issue_util"] = round(a.frac / ceiling, 4)
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "opcodes"}, indent=1))
    for o in out["opcodes"][:16]:
        print(f"  {o['op']:26s} {o['per_verify']:8d}  {o['share']:.3f}  x{o['cycles_each']:.2f}  cyc {o['cycle_share']:.3f}")


if __name__ == "__main__":
    main()
