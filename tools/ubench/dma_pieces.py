"""H2D DMA from page-locked memory: one copy of a verify-pipeline chunk's bytes vs the
same bytes as the pipeline's six pieces (arena, offsets, lengths, keys, signatures,
signature lengths), timed with events on one stream.  Prints JSON."""
import json
import sys

import torch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 39424
    sizes = [n * 1024, n * 8, n * 4, n * 32, n * 68, n * 4]
    total = sum(sizes)
    src = torch.empty(total, dtype=torch.uint8).pin_memory()
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    res = {}
    for name, parts in (("one", [total]), ("six", sizes), ("one", [total]), ("six", sizes)):
        times = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                a.record()
                o = 0
                for p in parts:
                    dst[o:o + p].copy_(src[o:o + p], non_blocking=True)
                    o += p
                b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        times.sort()
        res.setdefault(name, []).append(round(times[len(times) // 2], 4))
    res["bytes"] = total
    res["GBps_one"] = round(total / (min(res["one"]) / 1e3) / 1e9, 1)
    res["GBps_six"] = round(total / (min(res["six"]) / 1e3) / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
