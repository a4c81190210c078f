#!/usr/bin/env python3
"""Register pressure and occupancy limit of every HIP kernel, read from the
gfx950 code-object metadata (hipcc --offload-device-only -S).

    python tools/isa_regs.py            -> profiles/isa_registers.json

For each kernel: VGPR / AGPR / SGPR counts, VGPR spills, scratch bytes per lane,
static LDS, and the waves-per-SIMD limit the registers allow. A SIMD has 512
VGPRs per lane, allocated in granules of 8, and holds at most 8 waves.
pmc_report.py joins this with the measured mean residency (SQ_WAVE_CYCLES).
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "corda_amd", "csrc")
SOURCES = ["ed25519_kernels.hip", "ecdsa_kernels.hip", "merkle_kernels.hip", "stage_kernels.hip",
           "composite_kernels.hip"]
FIELDS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
          ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill",
          ".private_segment_fixed_size": "scratch_bytes", ".group_segment_fixed_size": "lds_bytes"}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def short(name):
    base = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    return base.replace("void ", "").replace("cg::Curve", "")


def waves_limit(vgpr, agpr):
    regs = -(-(vgpr + agpr) // 8) * 8
    return min(8, 512 // max(regs, 8))


def parse(asm):
    meta = asm[asm.index("amdhsa.kernels:"):]
    kernels = []
    for block in re.split(r"\n  - ", meta)[1:]:
        e = {}
        for line in block.splitlines():
            s = line.strip()
            for key, name in FIELDS.items():
                if s.startswith(key + ":"):
                    e[name] = int(s.split(":")[1])
            if s.startswith(".name:"):
                e["symbol"] = s.split(":", 1)[1].strip()
        if "symbol" in e and "vgpr" in e:
            kernels.append(e)
    return kernels


def main():
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for src in SOURCES:
            s = os.path.join(tmp, src + ".s")
            subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                                   f"-I{ROOT}/include", f"-I{CSRC}", "--offload-device-only", "-S",
                                   os.path.join(CSRC, src), "-o", s], stderr=subprocess.DEVNULL)
            ks = parse(open(s).read())
            for k, dn in zip(ks, demangle([k["symbol"] for k in ks])):
                k.pop("symbol")
                k["source"] = src
                k["waves_per_simd_limit"] = waves_limit(k["vgpr"], k.get("agpr", 0))
                out[short(dn)] = k
    path = os.path.join(ROOT, "profiles", "isa_registers.json")
    with open(path, "w") as f:
        json.dump({"source": "tools/isa_regs.py (gfx950 code-object metadata, hipcc -O3)", "kernels": out}, f,
                  indent=1)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
