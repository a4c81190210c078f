"""Prints an e2e_sweep.py JSON as a table: one row per setting, one column per batch size
(p50 ms), and with --spans the GPU call span / host pre-work / kernels after the last
H2D / host after of each cell."""
import json
import sys

M = {"CORDA_AMD_VERIFY_CHUNKS": "K", "CORDA_AMD_VERIFY_HEAD": "h", "CORDA_AMD_VERIFY_TAIL": "t",
     "CORDA_AMD_VERIFY_LANES": "lanes", "CORDA_AMD_ED_PAIR_MAX": "pair", "CORDA_AMD_ED_QUAD_MAX": "quad",
     "CORDA_AMD_VERIFY_RING": "ring", "CORDA_AMD_VERIFY_POLICY": "policy"}


def tag(s):
    return ",".join(f"{M.get(k, k)}={v}" for k, v in s.items() if k != "CORDA_AMD_VERIFY_MIN_CHUNK") or "default"


d = json.load(open(sys.argv[1]))
rows, ns = {}, sorted({r["n"] for r in d["rows"]})
for r in d["rows"]:
    rows.setdefault(tag(r["setting"]), {})[r["n"]] = r
print("setting".ljust(36) + "".join(str(n).rjust(10) for n in ns))
for k, v in rows.items():
    print(k.ljust(36) + "".join((str(v[n]["p50_ms"]) if n in v else "").rjust(10) for n in ns))
if any("spans" in r for r in d["rows"]):
    print("\nspans (gpu call / host pre / kernels after last h2d / host after):")
    for k, v in rows.items():
        cells = []
        for n in ns:
            sp = v.get(n, {}).get("spans") or {}
            cells.append("/".join(str(sp.get(x, "-")) for x in ("call_gpu_ms", "host_pre_ms", "kernels_after_last_h2d_ms",
                                                                 "host_after_gpu_ms")))
        print(k.ljust(36) + "  ".join(c.rjust(24) for c in cells))
