"""North-star parity run: BASELINE.json asks for verdicts bit-exact against
Crypto.doVerify on a 10 M adversarial+valid Ed25519 mix.

Shape: config 5, i.e. signatures over 32 B tx ids with distinct keys. 10 % of
them are adversarial, spread over E1–E12 (tools/datagen). Every
chunk is verified on the GPU in both modes (Crypto.isValid, Crypto.kt:534-541;
Crypto.doVerify, Crypto.kt:472-483) and compared element by element with the
C restatement of i2p eddsa 0.2.0 (oracle/, test infrastructure only).

The default is the north star's full size: 10,000,000 Ed25519 signatures and
2,097,152 ECDSA ones (about 200 s on the box together, most of it host-side
signing and the CPU oracle). CORDA_AMD_PARITY_N / CORDA_AMD_PARITY_EC_N lower them
for quick runs. Each test writes its summary (sizes, mismatches per mode, verdict
counts, accepts per adversarial class) to gpurun_out/parity_summary_*.json and
prints it, so the result can be read after a `-q` run.
"""
from __future__ import annotations

import collections
import ctypes
import json
import os
import sys
import time

import numpy as np
import pytest

from corda_amd import crypto
from corda_amd._lib import ACCEPT, MODE_DO_VERIFY, MODE_IS_VALID, ptr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))
import datagen  # noqa: E402

pytestmark = pytest.mark.gpu

N = int(os.environ.get("CORDA_AMD_PARITY_N", 10_000_000))
CHUNK = 1 << 21
ADV = 0.10


def _oracle(oracle, w, mode, threads):
    out = np.empty(max(w.n, 1), dtype=np.uint8)
    oracle.oracle_verify_batch(ptr(w.scheme), ptr(w.pk), ctypes.c_size_t(w.pk_stride), ptr(w.sig),
                               ctypes.c_size_t(w.sig_stride), ptr(w.sig_len), ptr(w.msg), ptr(w.msg_off),
                               ptr(w.msg_len), ctypes.c_size_t(w.n), mode, threads, ptr(out))
    return out[:w.n]


def _write_summary(name, summary):
    """The summary as JSON under gpurun_out/ (merged back from a gpurun box)."""
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"parity_summary_{name}.json"), "w") as f:
        json.dump(summary, f, indent=1)


def test_adversarial_mix_vs_oracle(gpu_ctx, oracle):
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    mismatches = {MODE_IS_VALID: 0, MODE_DO_VERIFY: 0}
    verdicts = {MODE_IS_VALID: collections.Counter(), MODE_DO_VERIFY: collections.Counter()}
    accepts_by_class = collections.Counter()
    first_bad = []
    for c0 in range(0, N, CHUNK):
        n = min(CHUNK, N - c0)
        k = c0 // CHUNK
        w = datagen.make_batch(n, msg_bytes=32, seed=9000 + k, key_base=60_000_000 + c0, threads=threads)
        w = datagen.add_ed25519_adversarial(w, frac=ADV, seed=900 + k)
        b = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg,
                               w.msg_off, w.msg_len)
        cls = np.array(w.classes)
        for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
            got = crypto.verify_packed(gpu_ctx, b, mode)
            exp = _oracle(oracle, w, mode, threads)
            bad = np.flatnonzero(got != exp)
            mismatches[mode] += int(bad.size)
            first_bad += [(c0 + int(i), str(cls[i]), int(got[i]), int(exp[i])) for i in bad[:5]]
            for v, c in enumerate(np.bincount(got, minlength=5)):
                if c:
                    verdicts[mode][v] += int(c)
            if mode == MODE_IS_VALID:
                for name in np.unique(cls):
                    accepts_by_class[str(name)] += int((got[cls == name] == ACCEPT).sum())
        print(f"parity chunk {k}: {c0 + n}/{N} signatures, mismatches {mismatches}, "
              f"{time.perf_counter() - t0:.1f} s", flush=True)
    summary = {"signatures": N, "adversarial_frac": ADV, "msg_bytes": 32,
               "mismatches_is_valid": mismatches[MODE_IS_VALID],
               "mismatches_do_verify": mismatches[MODE_DO_VERIFY],
               "verdict_counts_is_valid": dict(sorted(verdicts[MODE_IS_VALID].items())),
               "verdict_counts_do_verify": dict(sorted(verdicts[MODE_DO_VERIFY].items())),
               "accepts_by_class_is_valid": dict(sorted(accepts_by_class.items())),
               "seconds": round(time.perf_counter() - t0, 1)}
    print("parity summary " + json.dumps(summary), flush=True)
    _write_summary("ed25519", summary)
    assert mismatches[MODE_IS_VALID] == 0 and mismatches[MODE_DO_VERIFY] == 0, (first_bad[:10], summary)


EC_N = int(os.environ.get("CORDA_AMD_PARITY_EC_N", 2_097_152))
EC_CHUNK = 1 << 19


def test_ecdsa_adversarial_mix_vs_oracle(gpu_ctx, oracle):
    """The same run for ECDSA: K1 and R1 interleaved, 32 B ids, 10 % adversarial
    over D1–D8, both modes, against the BC 1.57 restatement. Default 2,097,152
    (CORDA_AMD_PARITY_EC_N overrides it)."""
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    mismatches = {MODE_IS_VALID: 0, MODE_DO_VERIFY: 0}
    verdicts = {MODE_IS_VALID: collections.Counter(), MODE_DO_VERIFY: collections.Counter()}
    accepts_by_class = collections.Counter()
    first_bad = []
    for c0 in range(0, EC_N, EC_CHUNK):
        n = min(EC_CHUNK, EC_N - c0)
        k = c0 // EC_CHUNK
        scheme = np.where(np.arange(n) % 2 == 0, 2, 3).astype(np.uint8)
        w = datagen.make_batch(n, msg_bytes=32, scheme=scheme, seed=7000 + k, key_base=80_000_000 + c0,
                               threads=threads)
        w = datagen.add_ecdsa_adversarial(w, frac=ADV, seed=700 + k)
        b = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg,
                               w.msg_off, w.msg_len)
        cls = np.array(w.classes)
        for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
            got = crypto.verify_packed(gpu_ctx, b, mode)
            exp = _oracle(oracle, w, mode, threads)
            bad = np.flatnonzero(got != exp)
            mismatches[mode] += int(bad.size)
            first_bad += [(c0 + int(i), str(cls[i]), int(got[i]), int(exp[i])) for i in bad[:5]]
            for v, c in enumerate(np.bincount(got, minlength=5)):
                if c:
                    verdicts[mode][v] += int(c)
            if mode == MODE_IS_VALID:
                for name in np.unique(cls):
                    accepts_by_class[str(name)] += int((got[cls == name] == ACCEPT).sum())
        print(f"ecdsa parity chunk {k}: {c0 + n}/{EC_N} signatures, mismatches {mismatches}, "
              f"{time.perf_counter() - t0:.1f} s", flush=True)
    summary = {"signatures": EC_N, "curves": "K1/R1 interleaved", "adversarial_frac": ADV, "msg_bytes": 32,
               "mismatches_is_valid": mismatches[MODE_IS_VALID],
               "mismatches_do_verify": mismatches[MODE_DO_VERIFY],
               "verdict_counts_is_valid": dict(sorted(verdicts[MODE_IS_VALID].items())),
               "verdict_counts_do_verify": dict(sorted(verdicts[MODE_DO_VERIFY].items())),
               "accepts_by_class_is_valid": dict(sorted(accepts_by_class.items())),
               "seconds": round(time.perf_counter() - t0, 1)}
    print("ecdsa parity summary " + json.dumps(summary), flush=True)
    _write_summary("ecdsa", summary)
    assert mismatches[MODE_IS_VALID] == 0 and mismatches[MODE_DO_VERIFY] == 0, (first_bad[:10], summary)
