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


@pytest.mark.gpu
def test_host_paths_under_asan_ubsan():
    """The library's host code (cordagpu.cpp: plan, partition, bounds pass and async arena on
    the upload thread, split / early points, the chunked pipeline with its upload thread and
    staging ring, tx / ftx pipelines, profiling spans, error exits) built with host ASan +
    UBSan (tests/native/Makefile `asan-lib`; device code unchanged) and driven by
    tests/native/host_paths.c: every call's status as expected, verdicts identical across
    repeats, layouts and tuning options, and no sanitizer finding (any aborts the run)."""
    path = os.path.join(ROOT, "tests", "native", "host_paths_asan.bin")
    assert os.path.exists(path), "host_paths_asan.bin not built (make -C tests/native asan-lib)"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    out = subprocess.run([path, "gpu"], capture_output=True, text=True, timeout=500, env=env)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "ok" in out.stdout
