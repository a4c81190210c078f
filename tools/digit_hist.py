"""Histogram of the Ed25519 MSM's per-lane radix-16 digit counts (balanced split).

Runs the host build of the device's hash phase (tests/native/libcg_host.so,
`cgh_ed25519_hash_ndig`: the same cg_ed25519.h code the hash kernel compiles) over N
random (pk, sig, 32-byte msg) triples — random bytes give a uniform challenge h, the
shape of config 2's valid lanes — and reports:

  * the lane histogram of the count the kernel now stores (exact: 1 + the highest
    nonzero recoded digit of c0 or |c1|, at least 32);
  * the histogram the round-5 bit-length rule ((bitlen + 7) / 4) gave on the same lanes;
  * the windows per lane the MSM pays: the wave maximum over 64 consecutive lanes
    (dispatch order), and with lanes grouped by count (every wave one count).

    python tools/digit_hist.py [N] [out.json]
"""
import ctypes
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def digits_value(words):
    """Signed radix-16 digits (e = d + 8 per nibble, 8 words) -> integer."""
    v = 0
    for j in range(63, -1, -1):
        v = 16 * v + (((words[j >> 3] >> (4 * (j & 7))) & 15) - 8)
    return v


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    out = sys.argv[2] if len(sys.argv) > 2 else None
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libcg_host.so"))
    lib.cgh_ed25519_hash_ndig.restype = ctypes.c_uint32
    lib.cgh_ed25519_hash_ndig.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32,
                                          ctypes.c_void_p]
    rng = np.random.default_rng(0x0C0DA)
    raw = rng.integers(0, 256, size=(n, 128), dtype=np.uint8)
    dig = (ctypes.c_uint32 * 24)()
    exact, old = np.empty(n, np.int64), np.empty(n, np.int64)
    for i in range(n):
        r = raw[i].tobytes()
        exact[i] = lib.cgh_ed25519_hash_ndig(r[:32], r[32:96], r[96:128], 32, dig)
        w = list(dig)
        bl = max(abs(digits_value(w[0:8])).bit_length(), abs(digits_value(w[8:16])).bit_length())
        old[i] = max(32, min(64, (bl + 7) // 4))
    waves = n // 64
    wave_max = exact[:waves * 64].reshape(waves, 64).max(axis=1)
    old_wave_max = old[:waves * 64].reshape(waves, 64).max(axis=1)
    res = {
        "n": n,
        "lanes_exact": {int(k): int(v) for k, v in sorted(Counter(exact.tolist()).items())},
        "lanes_bitlen_rule": {int(k): int(v) for k, v in sorted(Counter(old.tolist()).items())},
        "waves_in_order_exact": {int(k): int(v) for k, v in sorted(Counter(wave_max.tolist()).items())},
        "waves_in_order_bitlen_rule": {int(k): int(v) for k, v in sorted(Counter(old_wave_max.tolist()).items())},
        "windows_per_lane": {
            "bitlen_rule_in_order": float(old_wave_max.mean()),
            "exact_in_order": float(wave_max.mean()),
            "exact_grouped_by_count": float(exact.mean()),
        },
    }
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        with open(out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
