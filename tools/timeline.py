#!/usr/bin/env python3
"""Print the spans of one call from a CORDA_AMD_TIMELINE file (written by
libcordagpu's collect_timings when the variable names a file), sorted by start, with
per-name totals.   python tools/timeline.py gpurun_out/r02j/timeline_k4.txt [call#]"""
import sys
from collections import defaultdict

calls = [c for c in open(sys.argv[1]).read().split("# call\n") if c.strip()]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else -1
rows = sorted((float(a), float(b), n) for n, a, b in (l.split() for l in calls[idx].splitlines()))
tot = defaultdict(float)
for a, b, n in rows:
    print(f"{n:18s} {a:8.2f} {b:8.2f} {b - a:7.2f}")
    tot[n] += b - a
print("calls:", len(calls), " span:", round(max(b for _, b, _ in rows) - min(a for a, _, _ in rows), 2), "ms")
for n, t in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {n:18s} {t:8.2f}")
