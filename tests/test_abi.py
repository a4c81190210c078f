"""The C ABI boundary (CPU-only checks): libcordagpu.so loads, exports every
function include/cordagpu.h declares with plain-C signatures, and refuses to run
without a gfx950 device (no CPU fallback)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cordagpu.h")
LIB = os.path.join(ROOT, "corda_amd", "libcordagpu.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cg_[a-z_0-9]+)\s*\(", text)))


def test_header_is_plain_c():
    # the header must compile as C (no C++ / torch types cross the boundary)
    subprocess.check_call(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Werror", "-x", "c", HEADER])


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "libcordagpu.so not built (__graft_entry__.build())"
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    assert len(declared_functions()) >= 15


def test_python_binding_covers_header():
    from corda_amd import _lib
    assert set(declared_functions()) == set(_lib.PROTOTYPES)


def test_abi_version_and_no_fallback_without_gpu():
    from corda_amd import _lib
    lib = _lib.load()
    assert lib.cg_abi_version() == _lib.ABI_VERSION == 4
    if lib.cg_device_count() > 0:
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    assert lib.cg_open(0, ctypes.byref(h)) == _lib.CG_E_NO_DEVICE
    with pytest.raises(_lib.CordaGpuError):
        _lib.Context(0)


def test_null_context_is_an_error_not_a_crash():
    from corda_amd import _lib
    lib = _lib.load()
    assert lib.cg_set_profiling(None, 1) == _lib.CG_E_INVALID_ARGUMENT
    assert lib.cg_reset_stats(None) == _lib.CG_E_INVALID_ARGUMENT
    assert lib.cg_last_error(None) == b"null context"


def test_product_does_not_link_the_oracle():
    out = subprocess.check_output(["nm", "-D", LIB], text=True)
    assert "oracle_" not in out
    deps = subprocess.check_output(["readelf", "-d", LIB], text=True)
    assert "liboracle" not in deps and "libcrypto" not in deps


def test_single_hip_runtime_per_process():
    """libcordagpu and torch must share one HIP runtime (two in one process
    leave the second without a GPU); see corda_amd._lib._share_torch_hip_runtime."""
    import re
    import subprocess
    import sys
    code = ("from corda_amd import _lib; _lib.load(); import torch, re;"
            "print(sorted(set(re.findall(r'/\\S*libamdhip64\\S*', open('/proc/self/maps').read()))))")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    libs = eval(out.stdout.strip().splitlines()[-1])
    assert len(libs) == 1, libs


def _native(name):
    path = os.path.join(ROOT, "tests", "native", name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not built (__graft_entry__.build())")
    return path


def test_c_program_error_paths_without_device():
    """A plain C99 caller linked through include/cordagpu.h: null contexts and the
    missing device come back as statuses (tests/native/abi_errors.c)."""
    out = subprocess.run([_native("abi_errors.bin"), "cpu"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr


def test_jni_glue_compiles_and_runs_against_stub_env():
    """integration/jvm/cordagpu_jni.c compiled against the stub jni.h and driven by a
    fake JNIEnv (tests/native/jni_harness.c): handles, statuses, error strings."""
    out = subprocess.run([_native("jni_harness.bin"), "cpu"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
