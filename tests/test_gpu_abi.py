"""C-ABI error paths on the device (tests/native/abi_errors.c, jni_harness.c): a
plain C caller and the JNI glue see statuses — argument errors, an injected
allocation failure at every allocation point of a mixed batch, an injected C++
exception — and correct verdicts right after each failure."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("prog", ["abi_errors.bin", "jni_harness.bin"])
def test_native_callers_on_device(prog):
    path = os.path.join(ROOT, "tests", "native", prog)
    assert os.path.exists(path), f"{prog} not built (__graft_entry__.build())"
    out = subprocess.run([path, "gpu"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ok" in out.stdout
