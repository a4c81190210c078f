"""cg_verify_batch's host plan without a GPU (cg_plan.h, the functions cordagpu.cpp calls):
copy-bound or compute-bound by bytes per element, chunk bounds, latency lanes, early /
split points, async arena, the key-sample hinge, grouped MSM — at one below and one past
every boundary tests/test_gpu_ed25519.py::test_host_verify_plan_boundaries_vs_oracle
crosses on the GPU (plus 20,480 / 20,481 x 32 B and 32,768 / 32,769 x 1 KB, the one-chunk
latency thresholds), under option overrides, and the whole table again through the
ASan + UBSan build (tests/native/san_driver.bin, command Q).  Also: the options are read
only at cg_open — no call path of the library reads the environment."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
SO = os.path.join(NATIVE, "libcg_host.so")
FIELDS = ("copy_bound", "chunks", "pair_max", "defer_arena", "defer_meta", "async_arena", "rows_direct",
          "needs_key_sample", "early_parts", "split_points", "key_dedupe", "lanes", "grouped_msm")

# the GPU tests' layout (datagen rows: 64-byte key rows, 72-byte signature rows, sig_len)
PK, SG = 64, 72


@pytest.fixture(scope="module")
def host():
    src = os.path.join(NATIVE, "cg_host.cpp")
    hdrs = [os.path.join(ROOT, "corda_amd", "csrc", f) for f in os.listdir(os.path.join(ROOT, "corda_amd", "csrc"))
            if f.endswith(".h")]
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(map(os.path.getmtime, hdrs + [src])):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I",
                               os.path.join(ROOT, "corda_amd", "csrc"), src, "-o", SO])
    lib = ctypes.CDLL(SO)
    u64 = ctypes.c_uint64
    lib.cgh_plan_verify.argtypes = [u64, u64, u64, u64, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.c_int]
    return lib


def plan(host, n, msg_bytes, *, n_ed=None, pk=PK, sg=SG, sl=True, ecdsa=False, in_order=True, keys=0, opts=""):
    out, bounds = (ctypes.c_uint64 * 13)(), (ctypes.c_uint64 * 16)()
    nb = host.cgh_plan_verify(n, n if n_ed is None else n_ed, n * msg_bytes, pk, sg, int(sl), int(ecdsa),
                              int(in_order), keys, opts.encode(), out, bounds, 16)
    assert nb >= 2, (nb, opts)
    p = dict(zip(FIELDS, (int(x) for x in out)))
    p["bounds"] = [int(bounds[i]) for i in range(min(nb, 16))]
    return p


# (n, message bytes) -> the plan's choices on the GPU tests' layout, distinct keys
ONE = {"chunks": 1, "defer_arena": 1, "defer_meta": 1, "rows_direct": 1, "key_dedupe": 0, "needs_key_sample": 0}
CASES = [
    # tiny ragged calls: the eight-lane latency mode
    ((1, 32), dict(ONE, copy_bound=0, pair_max=20480, lanes=8, split_points=0, early_parts=0, grouped_msm=0)),
    ((63, 1024), dict(ONE, copy_bound=1, pair_max=32768, lanes=8, split_points=0, grouped_msm=0)),
    ((65, 32), dict(ONE, copy_bound=0, lanes=8)),
    ((257, 1024), dict(ONE, copy_bound=1, lanes=8)),
    ((7168, 32), dict(ONE, lanes=8)),
    ((7169, 32), dict(ONE, lanes=4)),
    # the one-chunk latency thresholds: 20,480 (compute-bound, 32 B ids), 32,768 (copy-bound, 1 KB)
    ((20480, 32), dict(ONE, copy_bound=0, lanes=4, split_points=0, grouped_msm=0)),
    ((20481, 32), dict(ONE, copy_bound=0, lanes=1, split_points=1, early_parts=0, grouped_msm=1)),
    ((32768, 1024), dict(ONE, copy_bound=1, lanes=4, split_points=0, async_arena=1, grouped_msm=0)),
    ((32769, 1024), dict(ONE, copy_bound=1, lanes=1, split_points=1, async_arena=1, grouped_msm=1)),
    ((40000, 32), dict(ONE, lanes=1, split_points=1)),
    ((40001, 32), dict(ONE, lanes=1, split_points=1, async_arena=1, grouped_msm=1)),
    # an arena from 1 MB goes up from the upload thread once the bounds pass runs there (n >= 32,768)
    ((32767, 32), dict(ONE, lanes=1, async_arena=0)),
    ((32768, 32), dict(ONE, lanes=1, async_arena=1)),
    # the early-points part size (65,536): one part is split points, two parts early points
    ((65536, 32), dict(ONE, lanes=1, early_parts=1, split_points=1, async_arena=1)),
    ((65537, 32), dict(ONE, lanes=1, early_parts=1, split_points=1)),
    ((131071, 32), dict(ONE, lanes=1, early_parts=1, split_points=1, async_arena=1)),
    ((131073, 32), dict(ONE, lanes=1, early_parts=2, split_points=0, async_arena=0)),
    # copy-bound calls from 2^17 run the chunked pipeline
    ((131071, 1024), dict(ONE, copy_bound=1, lanes=1, early_parts=1, split_points=1, async_arena=1)),
    ((131073, 1024), {"copy_bound": 1, "chunks": 4}),
    ((262145, 1024), {"copy_bound": 1, "chunks": 8}),
    # compute-bound ones from 2^20
    (((1 << 20) - 1, 32), dict(ONE, copy_bound=0, lanes=1, early_parts=4, split_points=0, grouped_msm=1)),
    ((1 << 20, 32), {"copy_bound": 0, "chunks": 8}),
    (((1 << 20) + 1, 32), {"copy_bound": 0, "chunks": 8}),
]


@pytest.mark.parametrize("shape,want", CASES, ids=[f"{n}x{m}" for (n, m), _ in CASES])
def test_plan_at_every_boundary(host, shape, want):
    p = plan(host, *shape)
    got = {k: p[k] for k in want}
    assert got == want, p
    b = p["bounds"]
    assert b[0] == 0 and b[-1] == shape[0] and all(x <= y for x, y in zip(b, b[1:]))
    assert all(x % 64 == 0 for x in b[1:-1])  # whole waves per chunk
    if p["chunks"] > 1:  # head and tail a quarter of a regular chunk
        mid = b[2] - b[1]
        assert abs((b[1] - b[0]) - mid / 4) <= 64 and abs((b[-1] - b[-2]) - mid / 4) <= 128


def test_plan_bytes_per_element_rule(host):
    """Copy-bound iff bytes per element > 475 (PCIe ~50 GB/s against ~9.5 ns of kernels
    per verify): 32 B ids with 152-byte rows are compute-bound, 1 KB messages copy-bound,
    and the boundary sits at 475 - 152 = 323 message bytes."""
    assert plan(host, 10000, 323)["copy_bound"] == 0
    assert plan(host, 10000, 324)["copy_bound"] == 1
    assert plan(host, 10000, 323, opts="CORDA_AMD_VERIFY_POLICY=0")["copy_bound"] == 1


def test_plan_key_sample_hinge(host):
    """Early / split points need distinct keys and the device dedupe repeating ones: with
    the sample not taken (-1) above the latency threshold the plan asks for it; forced key
    reuse (1) or its absence (0) never do."""
    p = plan(host, 100000, 32, keys=-1)
    assert p["needs_key_sample"] == 1 and p["split_points"] == 0 and p["key_dedupe"] == 0
    p = plan(host, 100000, 32, keys=1)
    assert p["needs_key_sample"] == 0 and p["key_dedupe"] == 1 and p["split_points"] == 0
    assert plan(host, 100000, 32, keys=0)["split_points"] == 1
    assert plan(host, 1000, 32, keys=-1)["needs_key_sample"] == 0  # below the latency threshold: no sample
    p = plan(host, 100000, 32, keys=-1, opts="CORDA_AMD_KEY_REUSE=0")
    assert p["needs_key_sample"] == 0 and p["split_points"] == 1 and p["key_dedupe"] == 0
    p = plan(host, 100, 32, keys=-1, opts="CORDA_AMD_KEY_REUSE=1")
    assert p["needs_key_sample"] == 0 and p["key_dedupe"] == 1 and p["lanes"] == 1 and p["grouped_msm"] == 0


@pytest.mark.parametrize("opts,n,m,want", [
    ("CORDA_AMD_ED_PAIR_MAX=0", 100, 32, {"lanes": 1, "split_points": 1, "grouped_msm": 0}),
    ("CORDA_AMD_ED_PAIR_MAX=0;CORDA_AMD_ED_BUCKET_MIN=1", 5000, 32, {"lanes": 1, "grouped_msm": 1}),
    ("CORDA_AMD_ED_PAIR_MAX=0;CORDA_AMD_ED_BUCKET_MIN=1", 4095, 32, {"lanes": 1, "grouped_msm": 0}),
    ("CORDA_AMD_ED_BUCKET_MIN=0", 100000, 32, {"grouped_msm": 0}),
    ("CORDA_AMD_ED_QUAD_MAX=0", 1000, 32, {"lanes": 2}),
    ("CORDA_AMD_ED_OCT_MAX=0", 1000, 32, {"lanes": 4}),
    ("CORDA_AMD_EARLY_POINTS=0", 200000, 32, {"early_parts": 0, "split_points": 1}),
    ("CORDA_AMD_EARLY_POINTS=0;CORDA_AMD_SPLIT_POINTS=0", 200000, 32, {"early_parts": 0, "split_points": 0}),
    ("CORDA_AMD_ED_SPLIT=2", 200000, 32, {"early_parts": 0, "split_points": 0}),
    ("CORDA_AMD_ED_SPLIT=1", 12000, 1024, {"async_arena": 0}),
    ("CORDA_AMD_ASYNC_ARENA=0", 12000, 1024, {"async_arena": 0}),
    ("", 12000, 1024, {"async_arena": 1}),
    ("", 7000, 1024, {"async_arena": 0}),  # 7 MB < 8 MB
    ("CORDA_AMD_ED_OVERLAP=0", 100000, 32, {"split_points": 0, "early_parts": 0}),
    ("CORDA_AMD_VERIFY_CHUNKS=3", 100000, 32, {"chunks": 3}),
    ("CORDA_AMD_VERIFY_MIN_CHUNK=500;CORDA_AMD_VERIFY_CHUNKS=6", 4000, 96, {"chunks": 6}),
])
def test_plan_under_options(host, opts, n, m, want):
    p = plan(host, n, m, opts=opts)
    assert {k: p[k] for k in want} == want, p


def test_plan_shapes_that_defer_nothing(host):
    """ECDSA among the elements: the arena goes up at staging (an ECDSA kernel reads it
    first); a mixed or reordered Ed25519 subset keeps its offsets with the staging and its
    points kernel on the staged SoA rows; unaligned row strides the same."""
    p = plan(host, 50000, 32, n_ed=40000, ecdsa=True, in_order=False)
    assert p["defer_arena"] == 0 and p["defer_meta"] == 0 and p["rows_direct"] == 0 and p["split_points"] == 0
    p = plan(host, 50000, 32, in_order=False)
    assert p["defer_arena"] == 1 and p["defer_meta"] == 0 and p["rows_direct"] == 0
    assert plan(host, 50000, 32, sg=66)["rows_direct"] == 0
    assert plan(host, 50000, 0)["defer_arena"] == 0  # no message bytes at all


def test_unknown_option_is_rejected(host):
    out, bounds = (ctypes.c_uint64 * 13)(), (ctypes.c_uint64 * 16)()
    assert host.cgh_plan_verify(10, 10, 320, PK, SG, 1, 0, 1, 0, b"CORDA_AMD_NOT_A_KNOB=1", out, bounds, 16) == -1


def test_plan_under_asan_ubsan():
    """The same table through the ASan + UBSan build of the plan (san_driver.bin, Q):
    identical answers, no sanitizer report."""
    subprocess.check_call(["make", "-s", "-C", NATIVE, "san_driver.bin"])
    lines = []
    for (n, m), _ in CASES:
        for keys in (-1, 0, 1):
            for opts in ("-", "CORDA_AMD_ED_PAIR_MAX=0", "CORDA_AMD_VERIFY_POLICY=0", "CORDA_AMD_KEY_REUSE=1",
                         "CORDA_AMD_VERIFY_CHUNKS=5;CORDA_AMD_VERIFY_MIN_CHUNK=1000;CORDA_AMD_VERIFY_TAIL=0.1"):
                lines.append((n, m, keys, opts))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    inp = "".join(f"Q {n} {n} {n * m} {PK} {SG} 1 0 1 {k} {o}\n" for n, m, k, o in lines)
    r = subprocess.run([os.path.join(NATIVE, "san_driver.bin")], input=inp, capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-3000:]
    out = r.stdout.splitlines()
    assert len(out) == len(lines)
    lib = ctypes.CDLL(SO) if os.path.exists(SO) else None
    if lib is None:
        pytest.skip("host build missing")
    u64 = ctypes.c_uint64
    lib.cgh_plan_verify.argtypes = [u64, u64, u64, u64, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.c_int]
    for (n, m, keys, opts), line in zip(lines, out):
        p = plan(lib, n, m, keys=keys, opts="" if opts == "-" else opts)
        vals = [int(x) for x in line.split()[1:]]
        assert vals[0] == len(p["bounds"]) and vals[1:14] == [p[f] for f in FIELDS] and vals[14:] == p["bounds"], \
            (n, m, keys, opts, line)


def test_no_environment_reads_on_the_call_path():
    """The CORDA_AMD_* knobs are read once, at cg_open (cg_plan.h Options::from_env); the
    library's sources hold no other getenv but GPU_MAX_HW_QUEUES, read at cg_open too."""
    src = open(os.path.join(ROOT, "corda_amd", "csrc", "cordagpu.cpp")).read()
    calls = re.findall(r"getenv\(\s*\"?([A-Za-z_]*)", src)
    assert calls == ["GPU_MAX_HW_QUEUES"], calls
    open_fn = src[src.index("cg_status cg_open("):src.index("void cg_close(")]
    assert "getenv(\"GPU_MAX_HW_QUEUES\")" in open_fn and "opts.from_env()" in open_fn
    plan_h = open(os.path.join(ROOT, "corda_amd", "csrc", "cg_plan.h")).read()
    assert plan_h.count("std::getenv(") == 1 and "void from_env()" in plan_h
    for f in os.listdir(os.path.join(ROOT, "corda_amd", "csrc")):
        if f.endswith((".hip", ".h")) and f != "cg_plan.h":
            assert "getenv" not in open(os.path.join(ROOT, "corda_amd", "csrc", f)).read(), f
