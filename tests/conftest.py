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
