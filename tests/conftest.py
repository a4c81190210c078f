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
