"""Sanitizer runs on the CPU build: the host build of the device arithmetic
(tests/native/cg_host.cpp — the very cg_*.h code the HIP kernels compile) and the C
oracle, compiled with AddressSanitizer + UndefinedBehaviorSanitizer (every finding
fatal, -fno-sanitize-recover=all) into one executable (tests/native/Makefile,
`make -C oracle asan-check`), run over:

* the Ed25519 and ECDSA golden sets (every class, a bounded sample per class) and the
  reference-held vectors (the tutorial's Ed25519 signatures and their mutants, the
  BC-signed certificates), with every input in an exactly-sized heap buffer — keys and
  signatures with no slack, messages with the 16 bytes the device arena pads;
* every device pipeline variant per Ed25519 row: both modes, the (h, 1) fallback, padded
  digit counts, the 2/4/8-lane latency splits, the key-reuse path (plain, wide, fallback);
* edge-value field (GF(2^255-19), both radix-2^26 Montgomery fields), scalar (mod L,
  half-size splits), joint-multiplication and SHA-256 leaf-streaming cases.

Verdicts must also match the golden / oracle values, so the instrumented run is the same
computation the uninstrumented tests check.  CPU only.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import random
import subprocess
from collections import defaultdict

import pytest

import ecdsa_bc as EC
import ed25519_i2p as ED

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BIN = os.path.join(NATIVE, "san_driver.bin")
P, L = ED.P, ED.L


@pytest.fixture(scope="module")
def san():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "san_driver.bin"])

    def run(lines, workers=4):
        """Feeds the lines to `workers` driver processes; returns the answers in order."""
        parts = [lines[i::workers] for i in range(workers)]

        def one(part):
            env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
                       UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
            p = subprocess.run([BIN], input="\n".join(part) + "\n", capture_output=True, text=True, env=env,
                               timeout=600)
            assert p.returncode == 0 and "runtime error" not in p.stderr and "Sanitizer" not in p.stderr, \
                p.stderr[-4000:]
            out = p.stdout.splitlines()
            assert len(out) == len(part), (len(out), len(part))
            return out

        with cf.ThreadPoolExecutor(workers) as ex:
            res = list(ex.map(one, parts))
        out = [None] * len(lines)
        for w, r in enumerate(res):
            out[w::workers] = r
        return out
    return run


def hx(b: bytes) -> str:
    return b.hex() if b else "-"


def le(x: int, n: int = 32) -> str:
    return x.to_bytes(n, "little").hex()


def words(h: str) -> int:
    return int.from_bytes(bytes.fromhex(h), "little")


def sample_by_class(rows, per_class, seed):
    by = defaultdict(list)
    for r in rows:
        by[r["cls"]].append(r)
    rnd = random.Random(seed)
    out = []
    for cls in sorted(by):
        out += rnd.sample(by[cls], min(per_class, len(by[cls])))
    return out


def test_sanitized_ed25519_pipeline_variants(san, golden_ed25519, ref_ed25519_cases):
    """Every Ed25519 golden class (<= 12 rows each) and every reference-artefact case through
    the instrumented oracle and all instrumented device-pipeline variants: no sanitizer
    finding, and every variant gives the golden / oracle verdict."""
    rows = [(bytes.fromhex(e["pk"]), bytes.fromhex(e["sig"]), bytes.fromhex(e["msg"]), e["cls"],
             (e["is_valid"], e["do_verify"])) for e in sample_by_class(golden_ed25519, 12, 1)]
    rows += [(c["pk"], c["sig"], c["msg"], c["cls"], None) for c in ref_ed25519_cases[::2]]
    out = san([f"E {hx(pk)} {hx(sig)} {hx(msg)}" for pk, sig, msg, _, _ in rows])
    n = 0
    for (pk, sig, msg, cls, exp), line in zip(rows, out):
        f = line.split()
        if f[1] == "skip":
            continue
        v = list(map(int, f[1:]))
        iv, dv = v[0], v[1]
        if exp is not None:
            assert (iv, dv) == exp, (cls, v)
        # host: both modes, fallback, padded digits, pair, quad, oct (doVerify, padded), reuse x3
        assert v[2:] == [iv, dv, iv, iv, iv, iv, dv, iv, iv, dv], (cls, v)
        n += 1
    assert n >= 200


def test_sanitized_ecdsa_and_der(san, golden_ecdsa, ref_cert_cases):
    """ECDSA golden classes (<= 10 rows each, both curves) and the reference's BC-signed
    certificates with their mutants through the instrumented oracle, the instrumented
    device verify (both modes) and the K4 DER parser: no finding, verdicts equal, and a
    DER row that parses gives the oracle's (r, s)."""
    rows = [(e["scheme"], e["q"] if isinstance(e["q"], str) else bytes(e["q"]).hex(), bytes.fromhex(e["sig"]),
             bytes.fromhex(e["msg"]), e["cls"], (e["is_valid"], e["do_verify"]))
            for e in sample_by_class(golden_ecdsa, 10, 2)]
    rows += [(c["scheme"], c["q"], c["sig"], c["msg"], c["cls"], None) for c in ref_cert_cases]
    out = san([f"C {s} {q} {hx(sig)} {hx(msg)}" for s, q, sig, msg, _, _ in rows])
    n = 0
    for (scheme, q, sig, msg, cls, exp), line in zip(rows, out):
        f = line.split()
        if f[1] == "skip":
            continue
        o0, o1, h0, h1, der = map(int, f[1:6])
        if exp is not None:
            assert (o0, o1) == exp, (cls, f)
        assert (h0, h1) == (o0, o1), (cls, f)
        if der == 0:  # parsed and in range: (r, s) as the oracle decodes them
            r, s = EC.der_decode(sig)
            assert (words(f[6]), words(f[7])) == (r, s), cls
        n += 1
    assert n >= 200


def test_sanitized_field_scalar_and_hash_edges(san):
    """Edge values through the instrumented arithmetic: GF(2^255-19) products, squares and
    inverses at 0, 1, p - 1, p .. 2^255 - 1 and limb-boundary patterns; both radix-2^26
    Montgomery fields (ops 0..4 of cgh_f26_op) at 0, p - 1, 2^256 - 1; sc_reduce512 at 0,
    L, 2^512 - 1; the half-size splits (TB 128 / 192) at 0, 1, L - 1, 2^128, 2^192;
    joint multiplications with u1 = 0 / n - 1; SHA-256 leaf streaming around every block
    boundary — all against Python big ints / hashlib."""
    import hashlib
    rnd = random.Random(55)
    fe_edge = [0, 1, 2, 19, P - 1, P, P + 1, 2**255 - 1, 2**255 - 20, 2**254, 2**26 - 1, 2**25, 2**51 - 1,
               sum(1 << (26 * i) for i in range(9))]
    lines, checks = [], []
    for a in fe_edge:
        for b in (fe_edge[rnd.randrange(len(fe_edge))], rnd.getrandbits(255)):
            lines.append(f"F {le(a)} {le(b)}")
            checks.append(("F", a, b))
    for scheme in (2, 3):
        p = EC.CURVES[scheme].p
        for a in (0, 1, p - 1, p, 2**256 - 1, 2**255, rnd.getrandbits(256)):
            b = rnd.choice([0, 1, p - 1, 2**256 - 1, rnd.getrandbits(256)])
            lines.append(f"P {scheme} {le(a)} {le(b)}")
            checks.append(("P", scheme, a, b))
    for x in (0, 1, L - 1, L, 2 * L, 2**512 - 1, 2**256, rnd.getrandbits(512)):
        lines.append(f"S {le(x, 64)}")
        checks.append(("S", x))
    for h in (0, 1, 2, L - 1, 2**128 - 1, 2**128, 2**192, 2**252, rnd.randrange(L), rnd.randrange(L)):
        lines.append(f"H {le(h)}")
        checks.append(("H", h))
    for scheme in (2, 3):
        c = EC.CURVES[scheme]
        for u1, u2 in ((0, 1), (c.n - 1, 1), (1, c.n - 1), (rnd.randrange(c.n), rnd.randrange(1, c.n))):
            d = rnd.randrange(1, c.n)
            q = EC._mul(c, d, c.g)
            lines.append(f"J {scheme} {le(u1)} {le(u2)} {le(q[0])} {le(q[1])}")
            checks.append(("J", scheme, u1, u2, q))
    buf = rnd.randbytes(300)
    for n in list(range(0, 130, 3)) + [183, 184, 191, 192, 247, 248, 255, 256, 299]:
        tail = rnd.randbytes(32) if n % 2 else b""
        lines.append(f"T {hx(buf[:n])} {hx(tail)}")
        checks.append(("T", buf[:n], tail))
    out = san(lines, workers=2)
    N8 = 8 * L
    for chk, line in zip(checks, out):
        f = line.split()
        if chk[0] == "F":
            _, a, b = chk
            assert [words(x) for x in f[1:4]] == [a * b % P, a * a % P, pow(a, P - 2, P)], (hex(a), hex(b))
        elif chk[0] == "P":
            _, scheme, a, b = chk
            p = EC.CURVES[scheme].p
            got = [words(x) for x in f[1:6]]
            assert got[0] == a * b % p and got[1] == a * a % p and got[3] == int((a - b) % p == 0), (scheme, hex(a))
            assert got[2] == (pow(a, p - 2, p) if a % p else 0) and got[4] == (3 * a - 2 * b) * (7 * b - 7 * a) % p
        elif chk[0] == "S":
            assert words(f[1]) == chk[1] % L
        elif chk[0] == "H":
            h = chk[1]
            for ok, c0, c1, neg in ((f[1], f[2], f[3], f[4]), (f[5], f[6], f[7], f[8])):
                C0, C1 = words(c0), words(c1) * (-1 if int(neg) else 1)
                assert C1 % 2 == 1 and (C0 - C1 * h) % N8 == 0 and C0 >= 0, hex(h)
                if not int(ok):
                    assert (C0, C1) == (h, 1), hex(h)
        elif chk[0] == "J":
            _, scheme, u1, u2, q = chk
            c = EC.CURVES[scheme]
            exp = EC._add(c, EC._mul(c, u1, c.g), EC._mul(c, u2, q))
            if exp is None:
                assert f[1] == "1"
            else:
                assert f[1] == "0" and words(f[2][:64]) == exp[0] and words(f[2][64:]) == exp[1], (scheme, u1)
        else:
            _, msg, tail = chk
            assert f[1] == hashlib.sha256(msg + tail).hexdigest(), len(msg)


def test_sanitizer_catches_an_overread():
    """Negative control: the instrumented build does report a heap overread (the driver's X
    command hands the oracle's key decode a 31-byte buffer for a 32-byte key)."""
    subprocess.check_call(["make", "-s", "-C", NATIVE, "san_driver.bin"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")
    p = subprocess.run([BIN], input="X\n", capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode != 0 and "heap-buffer-overflow" in p.stderr, p.stderr[-2000:]
