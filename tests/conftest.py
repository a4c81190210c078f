"""Shared pytest configuration.

Markers: ``gpu`` — needs a gfx950 device (run on the MI355X box); everything else
runs on the CPU-only container.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def oracle():
    """The C oracle (test infrastructure; built by __graft_entry__.build())."""
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.oracle_verify_batch.restype = ctypes.c_int
    lib.oracle_verify_batch.argtypes = [vp, vp, sz, vp, sz, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, vp]
    lib.oracle_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_int]
    lib.oracle_ecdsa_verify.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz,
                                        ctypes.c_int]
    lib.oracle_txid_batch.argtypes = [vp, vp, vp, vp, vp, sz, vp]
    lib.oracle_ftx_verify_batch.argtypes = [vp] * 9 + [sz, vp]
    return lib


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_ed25519():
    return load_golden("ed25519_golden.json")


@pytest.fixture(scope="session")
def golden_ecdsa():
    return load_golden("ecdsa_golden.json")


@pytest.fixture(scope="session")
def golden_merkle():
    return load_golden("merkle_golden.json")


@pytest.fixture(scope="session")
def golden_ftx():
    return load_golden("ftx_golden.json")


@pytest.fixture(scope="session")
def golden_composite():
    return load_golden("composite_golden.json")


@pytest.fixture(scope="session")
def gpu_ctx():
    from corda_amd import Context
    ctx = Context(int(os.environ.get("LOCAL_RANK", "0")))
    yield ctx
    ctx.close()


@pytest.fixture
def knobs(gpu_ctx):
    """The session context's CORDA_AMD_* run-time options (cg_set_option), with
    monkeypatch's setenv / delenv names; every option a test touched is unset again after
    it.  The library reads the environment only at cg_open, never per call."""
    class Knobs:
        def __init__(self):
            self.touched = set()

        def setenv(self, key, value):
            gpu_ctx.set_option(key, value)
            self.touched.add(key)

        def delenv(self, key, raising=False):
            gpu_ctx.set_option(key, None)
            self.touched.add(key)

    k = Knobs()
    yield k
    for key in k.touched:
        gpu_ctx.set_option(key, None)


def _der_with(r: int, s: int, pad_r: bool = False) -> bytes:
    def integer(v, pad=False):
        b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")  # minimal two's complement (v >= 0)
        if pad:
            b = b"\0" + b
        return b"\x02" + bytes([len(b)]) + b
    body = integer(r, pad_r) + integer(s)
    return b"\x30" + bytes([len(body)]) + body


@pytest.fixture(scope="session")
def ref_cert_cases():
    """The reference's own BC-signed certificate signatures (tests/golden/ref_cert_vectors.json,
    extracted by make_ref_cert_vectors.py) plus mutants derived from each: TBS bit flip, sig[0]++
    (CryptoUtilsTest.kt's corruption), high-S (n - s, BC has no low-S rule), r + n, a non-minimal
    r INTEGER, an empty message and the key presented under the other curve's scheme.  Each case:
    dict(cls, scheme, q (hex X||Y), sig, msg)."""
    import ecdsa_bc as EC
    rows = load_golden("ref_cert_vectors.json")["rows"]
    out = []
    for r in rows:
        sig, msg = bytes.fromhex(r["sig"]), bytes.fromhex(r["msg"])
        base = dict(scheme=r["scheme"], q=r["q"])
        out.append(dict(base, cls=r["cls"], sig=sig, msg=msg))
        if r["cls"] != "ref_cert":
            continue
        n = EC.CURVES[r["scheme"]].n
        rr, ss = EC.der_decode(sig)
        flip = bytearray(msg)
        flip[len(flip) // 2] ^= 0x10
        bump = bytearray(sig)
        bump[0] = (bump[0] + 1) & 0xFF
        out += [dict(base, cls="ref_tbs_flip", sig=sig, msg=bytes(flip)),
                dict(base, cls="ref_sig0_inc", sig=bytes(bump), msg=msg),
                dict(base, cls="ref_high_s", sig=_der_with(rr, n - ss), msg=msg),
                dict(base, cls="ref_r_plus_n", sig=_der_with(rr + n, ss), msg=msg),
                dict(base, cls="ref_nonminimal_r", sig=_der_with(rr, ss, pad_r=True), msg=msg),
                dict(base, cls="ref_empty_msg", sig=sig, msg=b""),
                dict(base, cls="ref_other_curve", scheme=5 - r["scheme"], sig=sig, msg=msg)]
    return out


# (is_valid, do_verify) the structure of each reference-Ed25519 case implies; None = decided by the
# restatement alone (i2p-specific rules A.6/A.7 and mixed-order keys: no reference artefact pins them)
REF_ED_EXPECT = {"ref_sig": (0, 0), "ref_wrong_key": (1, 1), "ref_id_flip": (1, 1), "ref_sig0_inc": (1, 1),
                 "ref_R_signflip": (1, 1), "ref_key_signflip": (1, 1), "ref_sig_len63": (2, 2),
                 "ref_sig_len65": (2, 2), "ref_empty_msg": (1, 4), "ref_empty_sig": (2, 4),
                 "ref_entropy_signed": (0, 0), "ref_S_plus_L": None, "ref_S_plus_kL": None,
                 "ref_entropy_mixed_order": None}


@pytest.fixture(scope="session")
def ref_ed25519_cases():
    """The reference's own Ed25519 artefacts (tests/golden/ref_ed25519_vectors.json, extracted by
    make_ref_ed25519_vectors.py): the two signatures of the tutorial's verifiedTransactions dump
    over its tx id (docs/source/tutorial-cordapp.rst:472-476) and mutants of them, every signature
    under every other reference key, and signatures made with the two trade.json keys, which are
    entropyToKeyPair(1)/(2) (Crypto.kt:733-739): over the tutorial id, 100 zero bytes and 1 KB
    (CryptoUtilsTest.kt's shapes), plus E8-style mixed-order variants of those keys (a·B + T signed
    with a).  Each case: dict(cls, pk, sig, msg); expected verdicts in REF_ED_EXPECT."""
    import hashlib
    import random

    import ed25519_i2p as ED
    g = load_golden("ref_ed25519_vectors.json")
    keys = [bytes.fromhex(k["a"]) for k in g["keys"]]
    out = []
    for row in g["sigs"]:
        a, sig, msg = bytes.fromhex(row["a"]), bytes.fromhex(row["sig"]), bytes.fromhex(row["msg"])
        out.append(dict(cls="ref_sig", pk=a, sig=sig, msg=msg))
        out += [dict(cls="ref_wrong_key", pk=k, sig=sig, msg=msg) for k in keys if k != a]
        flip = bytearray(msg)
        flip[5] ^= 0x01
        bump = bytearray(sig)
        bump[0] = (bump[0] + 1) & 0xFF
        rsign = bytearray(sig)
        rsign[31] ^= 0x80
        ksign = bytearray(a)
        ksign[31] ^= 0x80
        s = int.from_bytes(sig[32:], "little")
        out += [dict(cls="ref_id_flip", pk=a, sig=sig, msg=bytes(flip)),
                dict(cls="ref_sig0_inc", pk=a, sig=bytes(bump), msg=msg),
                dict(cls="ref_R_signflip", pk=a, sig=bytes(rsign), msg=msg),
                dict(cls="ref_key_signflip", pk=bytes(ksign), sig=sig, msg=msg),
                dict(cls="ref_sig_len63", pk=a, sig=sig[:63], msg=msg),
                dict(cls="ref_sig_len65", pk=a, sig=sig + b"\0", msg=msg),
                dict(cls="ref_empty_msg", pk=a, sig=sig, msg=b""),
                dict(cls="ref_empty_sig", pk=a, sig=b"", msg=msg),
                dict(cls="ref_S_plus_L", pk=a, sig=sig[:32] + (s + ED.L).to_bytes(32, "little"), msg=msg)]
        out += [dict(cls="ref_S_plus_kL", pk=a, sig=sig[:32] + (s + k * ED.L).to_bytes(32, "little"), msg=msg)
                for k in range(1, 16) if 2**255 <= s + k * ED.L < 2**256]
    tutorial_id = bytes.fromhex(g["sigs"][0]["msg"])
    rnd = random.Random(20170707)
    tors = None
    for k in g["keys"]:
        if k["entropy_k"] is None:
            continue
        seed = ED.entropy_seed(k["entropy_k"])
        for msg in (tutorial_id, bytes(100), rnd.randbytes(1024)):
            pk, sig = ED.sign(seed, msg)
            assert pk.hex() == k["a"]
            out.append(dict(cls="ref_entropy_signed", pk=pk, sig=sig, msg=msg))
        if tors is None:  # the order-8 subgroup, from a point of order 8L·k
            y = 2
            while True:
                try:
                    t = ED.scalarmult(ED.decode_point_i2p(y.to_bytes(32, "little")), ED.L)
                except ED.KeyInvalid:
                    y += 1
                    continue
                if not ED.point_equal(ED.scalarmult(t, 4), ED.IDENTITY):
                    break
                y += 1
            tors = [ED.scalarmult(t, j) for j in range(8)]
        a_sc, prefix, _ = ED.seed_to_keypair(seed)
        for j in (1, 2, 4):  # torsion components of order 8, 4, 2
            aenc = ED.encode_point(ED._add(ED.scalarmult(ED.BASE, a_sc), tors[j]))
            for msg in (tutorial_id, rnd.randbytes(40)):
                r = ED.sc_reduce(hashlib.sha512(prefix + msg).digest())
                rb = ED.encode_point(ED.scalarmult(ED.BASE, r))
                h = ED.sc_reduce(hashlib.sha512(rb + aenc + msg).digest())
                out.append(dict(cls="ref_entropy_mixed_order", pk=aenc,
                                sig=rb + ((r + h * a_sc) % ED.L).to_bytes(32, "little"), msg=msg))
    return out
