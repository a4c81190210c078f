"""GPU parity: Ed25519 verdicts of libcordagpu (HIP, gfx950) vs the CPU oracle.

Bar: bit-exact verdict codes (integer work).  Inputs: the committed golden
fixtures (every adversarial class of SURVEY.md §8d, RFC 8032 KATs, reference test
keys), seeded random valid + mutated batches checked element-wise against the C
oracle, and at config scale (1M signatures) size-independent properties
(every untouched signature accepts; verdict histogram of the mutated 1% equals
the oracle's on the same subset).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import pytest

from corda_amd import crypto
from corda_amd._lib import ACCEPT, MODE_DO_VERIFY, MODE_IS_VALID, ptr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "datagen"))
import datagen  # noqa: E402

pytestmark = pytest.mark.gpu


def oracle_verdicts(oracle, w, mode, threads=16):
    out = np.empty(max(w.n, 1), dtype=np.uint8)
    oracle.oracle_verify_batch(ptr(w.scheme), ptr(w.pk), ctypes.c_size_t(w.pk_stride), ptr(w.sig),
                               ctypes.c_size_t(w.sig_stride), ptr(w.sig_len), ptr(w.msg), ptr(w.msg_off),
                               ptr(w.msg_len), ctypes.c_size_t(w.n), mode, threads, ptr(out))
    return out[:w.n]


def gpu_verdicts(ctx, w, mode):
    b = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                           w.msg_len)
    return crypto.verify_packed(ctx, b, mode)


def test_golden_fixtures(gpu_ctx, golden_ed25519):
    g = golden_ed25519
    pks = [bytes.fromhex(e["pk"]) for e in g]
    sigs = [bytes.fromhex(e["sig"]) for e in g]
    msgs = [bytes.fromhex(e["msg"]) for e in g]
    for mode, key in ((MODE_IS_VALID, "is_valid"), (MODE_DO_VERIFY, "do_verify")):
        b = crypto.pack(crypto.EDDSA_ED25519_SHA512, pks, sigs, msgs)
        v = crypto.verify_packed(gpu_ctx, b, mode)
        exp = np.array([e[key] for e in g], dtype=np.uint8)
        bad = np.flatnonzero(v != exp)
        assert bad.size == 0, [(g[i]["cls"], int(v[i]), int(exp[i])) for i in bad[:10]]


def test_random_and_mutated_vs_oracle(gpu_ctx, oracle):
    w = datagen.make_batch(6000, msg_bytes=97, seed=11, key_base=1000)
    w = datagen.add_ed25519_adversarial(w, frac=0.25, seed=3)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        got = gpu_verdicts(gpu_ctx, w, mode)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, [(w.classes[i], int(got[i]), int(exp[i])) for i in bad[:10]]
    assert (exp == ACCEPT).sum() > 0.7 * w.n


def test_message_lengths_and_alignment(gpu_ctx, oracle):
    # every length 0..300 (SHA-512 block boundaries at 64/111/112/128+...), odd arena offsets
    lens = list(range(0, 301))
    rng = np.random.default_rng(5)
    base = datagen.make_batch(len(lens), msg_bytes=301, seed=99, key_base=50_000)
    # re-sign at the exact lengths with an unaligned arena
    n = len(lens)
    msg_len = np.array(lens, dtype=np.uint32)
    msg_off = np.zeros(n, dtype=np.uint64)
    pos = 1
    for i in range(n):
        msg_off[i] = pos
        pos += lens[i] + int(rng.integers(0, 4))
    arena = np.zeros(pos + 8, dtype=np.uint8)
    for i in range(n):
        arena[int(msg_off[i]):int(msg_off[i]) + lens[i]] = base.msg[i * 301:i * 301 + lens[i]]
    c = datagen.lib()
    pk = np.zeros((n, 64), np.uint8)
    sig = np.zeros((n, 72), np.uint8)
    sl = np.zeros(n, np.uint32)
    sch = np.full(n, 4, np.uint8)
    assert c.dg_sign_batch(n, sch.ctypes.data, 77, pk.ctypes.data, 64, sig.ctypes.data, 72, sl.ctypes.data,
                           arena.ctypes.data, msg_off.ctypes.data, msg_len.ctypes.data, 8) == 0
    w = datagen.Workload(n, sch, pk, 64, sig, 72, sl, arena, msg_off, msg_len)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        got = gpu_verdicts(gpu_ctx, w, mode)
        assert np.array_equal(got, exp)
    assert (gpu_verdicts(gpu_ctx, w, MODE_IS_VALID) == ACCEPT).all()


def test_prepared_batch_and_bitmap(gpu_ctx, oracle):
    w = datagen.make_batch(3000, msg_bytes=32, seed=3, key_base=9)
    w = datagen.add_ed25519_adversarial(w, frac=0.1, seed=9)
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    b = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                           w.msg_len)
    pb = crypto.PreparedBatch(gpu_ctx, b)
    v1 = pb.verify(MODE_IS_VALID)
    v2 = pb.verify(MODE_IS_VALID)
    assert np.array_equal(v1, exp) and np.array_equal(v2, exp)
    v, bm = crypto.verify_packed(gpu_ctx, b, MODE_IS_VALID, bitmap=True)
    bits = np.unpackbits(bm.view(np.uint8), bitorder="little")[:w.n]
    assert np.array_equal(bits.astype(bool), exp == ACCEPT)
    pb.close()


def test_do_verify_batch_raises_like_loop(gpu_ctx, golden_ed25519):
    g = [e for e in golden_ed25519 if e["cls"] == "valid" and e["msg"]][:20]
    pks = [bytes.fromhex(e["pk"]) for e in g]
    sigs = [bytes.fromhex(e["sig"]) for e in g]
    msgs = [bytes.fromhex(e["msg"]) for e in g]
    assert crypto.do_verify_batch(gpu_ctx, crypto.EDDSA_ED25519_SHA512, pks, sigs, msgs)
    bad = list(sigs)
    bad[7] = bytes([bad[7][0] ^ 1]) + bad[7][1:]
    bad[12] = b""
    with pytest.raises(crypto.SignatureException) as ei:
        crypto.do_verify_batch(gpu_ctx, crypto.EDDSA_ED25519_SHA512, pks, bad, msgs)
    assert ei.value.index == 7
    bad[3] = b""
    with pytest.raises(crypto.IllegalArgumentException) as ei:
        crypto.do_verify_batch(gpu_ctx, crypto.EDDSA_ED25519_SHA512, pks, bad, msgs)
    assert ei.value.index == 3


def test_config2_scale_properties(gpu_ctx, oracle):
    """BASELINE config 2 exactly as bench.py builds it on rank 0 (1M Ed25519, 1 KB
    messages, distinct keys with every 4,096th one a reference test key
    entropyToKeyPair(20..110), 1% adversarial over E1-E12), verified from host buffers
    (cg_verify_batch's chunked upload pipeline): untouched elements all accept; the
    adversarial subset and every reference-test-key element match the oracle
    element-wise."""
    n = 1 << 20
    w = datagen.make_batch(n, msg_bytes=1024, seed=42, key_base=0, ref_seed_stride=4096)
    w = datagen.add_ed25519_adversarial(w, frac=0.01, seed=1)
    got = gpu_verdicts(gpu_ctx, w, MODE_IS_VALID)
    adv = np.array([c != "valid" for c in w.classes])
    assert (got[~adv] == ACCEPT).all()
    ref = np.arange(0, n, 4096)
    check = np.union1d(np.flatnonzero(adv), ref)
    exp = oracle_verdicts(oracle, w.subset(check), MODE_IS_VALID)
    assert np.array_equal(got[check], exp)
    assert ref.size == 256 and (got[ref] == ACCEPT).sum() >= 250


def test_reference_message_shapes_all_schemes(gpu_ctx, oracle):
    """CryptoUtilsTest.kt:123-286 shapes for all three schemes in one ragged batch:
    a 1 MB message, 100 zero bytes, a 1-byte message, a 1 KB message; each signed
    (valid), with sig[0] incremented (reject / malformed DER), an empty signature and
    empty clear data (doVerify: IllegalArgumentException; isValid: engine outcome)."""
    rng = np.random.default_rng(17)
    msgs = [rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes(), bytes(100), b"\x07",
            rng.integers(0, 256, 1024, dtype=np.uint8).tobytes()]
    schemes = [4, 3, 2]
    rows = [(s, m) for s in schemes for m in msgs]
    n = len(rows)
    arena = np.frombuffer(b"".join(m for _, m in rows) + bytes(8), dtype=np.uint8).copy()
    msg_len = np.array([len(m) for _, m in rows], dtype=np.uint32)
    msg_off = np.concatenate([[0], np.cumsum(msg_len[:-1])]).astype(np.uint64)
    sch = np.array([s for s, _ in rows], dtype=np.uint8)
    pk = np.zeros((n, 64), np.uint8)
    sig = np.zeros((n, 72), np.uint8)
    sl = np.zeros(n, np.uint32)
    assert datagen.lib().dg_sign_batch(n, sch.ctypes.data, 4242, pk.ctypes.data, 64, sig.ctypes.data, 72,
                                       sl.ctypes.data, arena.ctypes.data, msg_off.ctypes.data, msg_len.ctypes.data,
                                       8) == 0
    # variants: valid, sig[0]++, empty signature, empty message
    reps = 4
    sch4, pk4, sig4 = np.tile(sch, reps), np.tile(pk, (reps, 1)), np.tile(sig, (reps, 1))
    sl4, off4, len4 = np.tile(sl, reps), np.tile(msg_off, reps), np.tile(msg_len, reps)
    sig4[n:2 * n, 0] += 1
    sl4[2 * n:3 * n] = 0
    len4[3 * n:] = 0
    w = datagen.Workload(4 * n, sch4, pk4, 64, sig4, 72, sl4, arena, off4, len4)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        got = gpu_verdicts(gpu_ctx, w, mode)
        assert np.array_equal(got, exp), (mode, got.tolist(), exp.tolist())
        assert (got[:n] == ACCEPT).all() and (got[n:2 * n] != ACCEPT).all()
        if mode == MODE_DO_VERIFY:
            assert (got[2 * n:] == 4).all()  # ARG_EMPTY for empty signature / clear data


def test_empty_batch_is_ok(gpu_ctx):
    v = np.zeros(1, np.uint8)
    st = gpu_ctx.lib.cg_verify_batch(gpu_ctx.h, 0, MODE_IS_VALID, None, None, 64, None, 64, None, None, 0, None, None,
                                     ptr(v), None)
    assert st == 0


@pytest.mark.parametrize("mod", [7, 1])
def test_forced_full_length_fallback_vs_oracle(gpu_ctx, oracle, golden_ed25519, mod):
    """The half-size reduction's fallback (c0, c1) = (h, 1) (cg_halfscalar.h; taken
    when the Lehmer quotient overflows, ~1e-8 of hash-derived h) forced on the device
    through cg_set_debug for every mod-th element — golden E1-E12 fixtures plus a
    mutated random batch — must give the oracle's verdicts (the full-length loop
    decides the same i2p predicate).  The waves holding a forced lane run 64 radix-16
    digits instead of ~33."""
    from corda_amd._lib import DEBUG_FORCE_FULL_LENGTH
    g = golden_ed25519
    pks = [bytes.fromhex(e["pk"]) for e in g]
    sigs = [bytes.fromhex(e["sig"]) for e in g]
    msgs = [bytes.fromhex(e["msg"]) for e in g]
    w = datagen.add_ed25519_adversarial(datagen.make_batch(4000, msg_bytes=64, seed=21, key_base=777), frac=0.3,
                                        seed=9)
    gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, mod)
    try:
        for mode, key in ((MODE_IS_VALID, "is_valid"), (MODE_DO_VERIFY, "do_verify")):
            v = crypto.verify_packed(gpu_ctx, crypto.pack(crypto.EDDSA_ED25519_SHA512, pks, sigs, msgs), mode)
            exp = np.array([e[key] for e in g], dtype=np.uint8)
            bad = np.flatnonzero(v != exp)
            assert bad.size == 0, [(g[i]["cls"], int(v[i]), int(exp[i])) for i in bad[:10]]
            got = gpu_verdicts(gpu_ctx, w, mode)
            assert np.array_equal(got, oracle_verdicts(oracle, w, mode))
        assert (got == ACCEPT).sum() > 2000
    finally:
        gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 0)


@pytest.mark.parametrize("bucket_min", ["0", "1", None])
@pytest.mark.parametrize("mixed", [False, True])
def test_grouped_msm_vs_oracle(gpu_ctx, oracle, golden_ed25519, knobs, bucket_min, mixed):
    """The balanced MSM over lanes grouped by digit count (cg_ed25519_bucket; round 6)
    against the oracle: off ('0'), from 4,096 signatures ('1'), and
    the default threshold (every piece of at least 4,096 grouped with '1').  Latency lanes off so the balanced MSM runs; every 97th lane
    takes the 64-digit (h, 1) fallback, so class 0 holds long lanes; 30 % mutations put
    hash- and points-phase verdicts (written by the bucket kernel) among them; the mixed
    batch scatters the Ed25519 verdicts through the scheme partition's index."""
    from corda_amd._lib import DEBUG_FORCE_FULL_LENGTH
    knobs.setenv("CORDA_AMD_ED_PAIR_MAX", "0")
    if bucket_min is not None:
        knobs.setenv("CORDA_AMD_ED_BUCKET_MIN", bucket_min)
    g = golden_ed25519
    gb = crypto.pack(crypto.EDDSA_ED25519_SHA512, [bytes.fromhex(e["pk"]) for e in g],
                     [bytes.fromhex(e["sig"]) for e in g], [bytes.fromhex(e["msg"]) for e in g])
    n = 40_000
    scheme = 4
    if mixed:
        scheme = np.random.default_rng(3).choice(np.array([4, 4, 4, 2, 3], np.uint8), size=n)
    w = datagen.make_batch(n, msg_bytes=48, scheme=scheme, seed=31, key_base=4_400)
    w = datagen.add_ed25519_adversarial(w, frac=0.3, seed=13)
    gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 97)
    try:
        for mode, key in ((MODE_IS_VALID, "is_valid"), (MODE_DO_VERIFY, "do_verify")):
            v = crypto.verify_packed(gpu_ctx, gb, mode)
            exp = np.array([e[key] for e in g], dtype=np.uint8)
            bad = np.flatnonzero(v != exp)
            assert bad.size == 0, [(g[i]["cls"], int(v[i]), int(exp[i])) for i in bad[:10]]
            got = gpu_verdicts(gpu_ctx, w, mode)
            want = oracle_verdicts(oracle, w, mode)
            bad = np.flatnonzero(got != want)
            assert bad.size == 0, (bad[:10].tolist(), got[bad[:10]].tolist(), want[bad[:10]].tolist())
        assert (got == ACCEPT).sum() > n // 3
    finally:
        gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 0)


@pytest.fixture
def key_reuse(knobs, request):
    """CORDA_AMD_KEY_REUSE: '1' forces the key-reuse path, '0' the balanced one,
    unset = automatic (distinct keys <= n / 8)."""
    if request.param is None:
        knobs.delenv("CORDA_AMD_KEY_REUSE", raising=False)
    else:
        knobs.setenv("CORDA_AMD_KEY_REUSE", request.param)
    return request.param


@pytest.mark.parametrize("key_reuse", ["1"], indirect=True)
def test_key_reuse_path_golden_fixtures(gpu_ctx, golden_ed25519, key_reuse):
    """Every golden class E1-E12 through the key-reuse path (device key dedupe,
    per-key decode + tables 2^(64 t)(-A), R-only points kernel, 64-doubling msm):
    torsion / mixed-order / non-canonical keys, KEY_INVALID from the per-key decode
    taking precedence over ARG_EMPTY / SIG_MALFORMED of each signature."""
    g = golden_ed25519 * 3  # every key at least three times
    pks = [bytes.fromhex(e["pk"]) for e in g]
    sigs = [bytes.fromhex(e["sig"]) for e in g]
    msgs = [bytes.fromhex(e["msg"]) for e in g]
    for mode, key in ((MODE_IS_VALID, "is_valid"), (MODE_DO_VERIFY, "do_verify")):
        v = crypto.verify_packed(gpu_ctx, crypto.pack(crypto.EDDSA_ED25519_SHA512, pks, sigs, msgs), mode)
        exp = np.array([e[key] for e in g], dtype=np.uint8)
        bad = np.flatnonzero(v != exp)
        assert bad.size == 0, [(g[i]["cls"], int(v[i]), int(exp[i])) for i in bad[:10]]


@pytest.mark.parametrize("key_reuse", [None, "1"], indirect=True)
@pytest.mark.parametrize("n_keys", [1, 16, 300])
def test_key_reuse_random_signers_vs_oracle(gpu_ctx, oracle, key_reuse, n_keys):
    """A notary-backlog shape: 48k signatures by n_keys signers (automatic mode picks
    the key-reuse path: the batch is above the latency mode's 40k, below which the
    balanced two-lane path is the shorter chain), 25 % mutated over E1-E12, both modes,
    against the oracle; and again with the (h, 1) fallback forced on every 5th
    signature (wide waves)."""
    from corda_amd._lib import DEBUG_FORCE_FULL_LENGTH
    w = datagen.make_batch(48_000, msg_bytes=48, seed=n_keys, key_base=4_000_000, key_reuse=n_keys)
    w = datagen.add_ed25519_adversarial(w, frac=0.25, seed=n_keys + 1)
    for mod in (0, 5):
        gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, mod)
        try:
            for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
                got = gpu_verdicts(gpu_ctx, w, mode)
                assert np.array_equal(got, oracle_verdicts(oracle, w, mode)), (mod, mode)
        finally:
            gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 0)
    assert (got == ACCEPT).sum() > 33000


@pytest.mark.parametrize("key_reuse", [None], indirect=True)
def test_key_reuse_prepared_batch_bitmap(gpu_ctx, oracle, key_reuse):
    """Prepared batch on the reuse path verified twice (per-key tables rebuilt each
    call) with the device bitmap, plus a distinct-key batch in the same context
    (balanced path) in between."""
    w = datagen.add_ed25519_adversarial(datagen.make_batch(70_001, msg_bytes=32, seed=3, key_reuse=40), 0.02, seed=2)
    pb = crypto.PreparedBatch(gpu_ctx, crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride,
                                                          w.sig_len, w.msg, w.msg_off, w.msg_len))
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    assert np.array_equal(pb.verify(MODE_IS_VALID), exp)
    d = datagen.make_batch(3000, msg_bytes=32, seed=4, key_base=99)
    assert (gpu_verdicts(gpu_ctx, d, MODE_IS_VALID) == ACCEPT).all()
    assert np.array_equal(pb.verify(MODE_IS_VALID), exp)
    pb.close()


@pytest.mark.parametrize("chunks,min_chunk,tail,variant", [("9", "700", "0.3", "default"), ("3", "1", "1.0", "default"),
                                                          ("9", "700", "0.3", "one_dma_off"),
                                                          ("9", "700", "0.3", "small_slices"),
                                                          ("9", "700", "0.3", "upload_on_caller"),
                                                          ("9", "700", "0.3", "ring"),
                                                          ("4", "700", "0.4", "pinned_in")])
def test_host_verify_pipeline_small_chunks_vs_oracle(gpu_ctx, oracle, knobs, chunks, min_chunk, tail, variant):
    """cg_verify_batch's pipeline (chunk k's upload on the copy stream beside chunk k-1's
    kernels) forced onto small, ragged chunks: a mixed batch — Ed25519 from distinct and
    from 12 repeated signers (the key-reuse path inside a chunk), secp256k1, P-256, an
    unsupported scheme id and wrong-length keys — whose arena is packed in REVERSE element
    order (the first chunk's messages sit at the end, so its prefix is the whole arena),
    in both modes, verdicts and accept bitmap against the oracle.  Variants: the default
    (the runtime's pageable copies, issued by the upload thread); the page-locked staging
    ring instead (CORDA_AMD_VERIFY_RING=1), with each staged chunk's rows as one DMA per
    staging slice (12 MB slices, so one here) or one per array (CORDA_AMD_VERIFY_ONE_DMA=0)
    or 4 KB staging slices, one DMA each (CORDA_AMD_VERIFY_SLICE_KB=4: slices straddle the
    arena / rows boundary of the slot); the uploads issued on the calling thread
    (CORDA_AMD_VERIFY_UPLOAD_THREAD=0); and page-locked inputs (cg_register_host: direct
    DMAs; the pageable verdict buffers then come back through the bounce buffer)."""
    from corda_amd import dist as D
    from corda_amd._lib import KEY_INVALID, UNSUPPORTED
    knobs.setenv("CORDA_AMD_VERIFY_CHUNKS", chunks)
    knobs.setenv("CORDA_AMD_VERIFY_MIN_CHUNK", min_chunk)
    knobs.setenv("CORDA_AMD_VERIFY_TAIL", tail)
    if variant in ("one_dma_off", "small_slices"):  # (ring staging options)
        knobs.setenv("CORDA_AMD_VERIFY_RING", "1")
    if variant == "one_dma_off":
        knobs.setenv("CORDA_AMD_VERIFY_ONE_DMA", "0")
    if variant == "upload_on_caller":
        knobs.setenv("CORDA_AMD_VERIFY_UPLOAD_THREAD", "0")
    if variant == "ring":
        knobs.setenv("CORDA_AMD_VERIFY_RING", "1")
    if variant == "small_slices":
        knobs.setenv("CORDA_AMD_VERIFY_SLICE_KB", "4")
    sch = np.random.default_rng(12).choice(np.array([2, 3, 4, 4, 4], np.uint8), size=5200)
    w = datagen.make_batch(len(sch), msg_bytes=70, scheme=sch, seed=23, key_base=620_000)
    w = datagen.add_ecdsa_adversarial(w, frac=0.2, seed=4)
    reuse = datagen.add_ed25519_adversarial(datagen.make_batch(1400, msg_bytes=33, seed=29, key_base=640_000,
                                                               key_reuse=12), frac=0.2, seed=6)
    ed = datagen.add_ed25519_adversarial(datagen.make_batch(1500, msg_bytes=120, seed=31, key_base=650_000),
                                         frac=0.2, seed=8)
    parts = [w, reuse, ed]
    keys, sigs, msgs, schemes = [], [], [], []
    for p in parts:
        for i in range(p.n):
            s = int(p.scheme[i])
            keys.append(bytes(p.pk[i, :64 if s in (2, 3) else 32]))
            sigs.append(bytes(p.sig[i, :p.sig_len[i]]))
            msgs.append(bytes(p.msg[p.msg_off[i]:p.msg_off[i] + p.msg_len[i]]))
            schemes.append(s)
    n = len(keys)
    bad_key = list(range(5, n, 997))
    for i in bad_key:
        keys[i] = keys[i][:-1]
    unsup = list(range(11, n, 1301))
    for i in unsup:
        schemes[i] = 9
    b = crypto.pack(schemes, keys, sigs, msgs)
    # reverse the arena: element i's message moves to the mirrored position
    ln = b.msg_len[:n].astype(np.uint64)
    new_off = np.zeros(n, np.uint64)
    new_off[::-1] = np.concatenate([[0], np.cumsum(ln[::-1])[:-1]]).astype(np.uint64)
    arena = np.zeros(len(b.msg) + 1, np.uint8)
    for i in range(n):
        arena[int(new_off[i]):int(new_off[i] + ln[i])] = b.msg[int(b.msg_off[i]):int(b.msg_off[i] + ln[i])]
    b2 = crypto.PackedBatch(n, b.scheme, b.pk, b.pk_stride, b.sig, b.sig_stride, b.sig_len, arena, new_off,
                            b.msg_len)
    oracle_w = datagen.Workload(n, b.scheme & 0x7F, b.pk, b.pk_stride, b.sig, b.sig_stride, b.sig_len, arena,
                                new_off, b.msg_len)
    pinned = (b2.scheme, b2.pk, b2.sig, b2.sig_len, arena, new_off, b2.msg_len) if variant == "pinned_in" else ()
    gpu_ctx.register_host(*pinned)
    try:
        for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
            exp = oracle_verdicts(oracle, oracle_w, mode)
            exp[bad_key] = KEY_INVALID
            exp[unsup] = UNSUPPORTED
            got, bm = crypto.verify_packed(gpu_ctx, b2, mode, bitmap=True)
            bad = np.flatnonzero(got != exp)
            assert bad.size == 0, [(int(i), int(schemes[i]), int(got[i]), int(exp[i])) for i in bad[:10]]
            assert np.array_equal(bm.view(np.int32), D.pack_bits(exp == ACCEPT).view(np.int32))
    finally:
        gpu_ctx.unregister_host(*pinned)
    assert (exp == ACCEPT).sum() > 0.6 * n


@pytest.mark.parametrize("beside", [None, "0"])
def test_one_chunk_large_arena_and_pinned_outputs_vs_oracle(gpu_ctx, oracle, knobs, beside):
    """The one-chunk host verify with an arena large enough (8,192 x 1 KB) that its deferred
    copy runs on its own stream beside the staging and points kernels (and with that
    turned off, CORDA_AMD_ARENA_BESIDE=0), 25 % mutated, in both modes; then the same call
    with page-locked verdict and bitmap buffers (the download's direct path instead of
    the bounce buffer) — verdicts and bitmap against the oracle."""
    from corda_amd import dist as D
    if beside is not None:
        knobs.setenv("CORDA_AMD_ARENA_BESIDE", beside)
    w = datagen.add_ed25519_adversarial(datagen.make_batch(8192, msg_bytes=1024, seed=83, key_base=970_000),
                                        frac=0.25, seed=13)
    assert len(w.msg) >= 6 << 20
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        got = gpu_verdicts(gpu_ctx, w, mode)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, [(w.classes[i], int(got[i]), int(exp[i])) for i in bad[:10]]
    verdict = np.empty(w.n, np.uint8)
    bm = np.zeros((w.n + 31) // 32, np.uint32)
    gpu_ctx.register_host(verdict, bm)
    try:
        gpu_ctx.check(gpu_ctx.lib.cg_verify_batch(gpu_ctx.h, w.n, MODE_IS_VALID, ptr(w.scheme), ptr(w.pk), w.pk_stride,
                                                  ptr(w.sig), w.sig_stride, ptr(w.sig_len), ptr(w.msg), len(w.msg),
                                                  ptr(w.msg_off), ptr(w.msg_len), ptr(verdict), ptr(bm)))
    finally:
        gpu_ctx.unregister_host(verdict, bm)
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    assert np.array_equal(verdict, exp)
    assert np.array_equal(bm.view(np.int32), D.pack_bits(exp == ACCEPT).view(np.int32))


@pytest.mark.parametrize("chunks", [None, "5"])
def test_compact_ed25519_layout_vs_oracle(gpu_ctx, oracle, knobs, chunks):
    """The layout an Ed25519-only JVM caller packs (and bench.py's end-to-end line times):
    scheme_id NULL, 32-byte key rows, 64-byte R||S rows and sig_len NULL — and the same
    with sig_len given when some rows are ragged (E12: 0 / 63 / 65 bytes, sig_stride 68).
    Verdicts in both modes against the oracle on the full-layout rows."""
    if chunks:
        knobs.setenv("CORDA_AMD_VERIFY_CHUNKS", chunks)
        knobs.setenv("CORDA_AMD_VERIFY_MIN_CHUNK", "300")
    w = datagen.add_ed25519_adversarial(datagen.make_batch(4000, msg_bytes=200, seed=41, key_base=700_000),
                                        frac=0.2, seed=13)
    sl = w.sig_len[:w.n].astype(np.uint32)
    ragged = sl != 64
    assert ragged.any()
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        # every row 64 bytes: the ragged rows leave, so the layout with sig_len NULL is exact
        keep = np.flatnonzero(~ragged)
        s = w.subset(keep)
        b = crypto.PackedBatch(s.n, None, np.ascontiguousarray(s.pk[:, :32]), 32,
                               np.ascontiguousarray(s.sig[:, :64]), 64, None, s.msg, s.msg_off, s.msg_len)
        got = crypto.verify_packed(gpu_ctx, b, mode)
        assert np.array_equal(got, exp[keep]), np.flatnonzero(got != exp[keep])[:10]
        # ragged rows with their lengths (65-byte rows need a wider stride)
        sg = np.zeros((w.n, 68), np.uint8)
        sg[:, :min(68, w.sig_stride)] = w.sig[:w.n, :min(68, w.sig_stride)]
        b = crypto.PackedBatch(w.n, None, np.ascontiguousarray(w.pk[:w.n, :32]), 32, sg, 68, sl, w.msg, w.msg_off,
                               w.msg_len)
        got = crypto.verify_packed(gpu_ctx, b, mode)
        assert np.array_equal(got, exp), np.flatnonzero(got != exp)[:10]


@pytest.mark.parametrize("split,overlap,signers", [("2", "1", 0), ("3", "0", 0), ("2", "2", 40), ("1", "2", 0),
                                                   ("1", "1", 0)])
def test_prepared_batch_split_and_overlap_vs_oracle(gpu_ctx, oracle, knobs, split, overlap, signers):
    """cg_batch_verify's scheduling variants on one prepared batch: the Ed25519 subset as
    index pieces on two streams (CORDA_AMD_ED_SPLIT, pieces >= 65,536), the points kernel
    after the hash kernel (CORDA_AMD_ED_OVERLAP 0, and 1 — the default — for a resident
    batch) or beside it (2), distinct signers and 40
    repeated ones (the key-reuse path: both lanes wait for the per-key tables) — verdicts
    and accept bitmap identical to the oracle's, verified twice."""
    knobs.setenv("CORDA_AMD_ED_SPLIT", split)
    knobs.setenv("CORDA_AMD_ED_OVERLAP", overlap)
    n = 3 * 65536 + 777
    w = datagen.make_batch(n, msg_bytes=32, seed=51, key_base=800_000, key_reuse=signers)
    w = datagen.add_ed25519_adversarial(w, frac=0.02, seed=19)
    adv = np.array([c != "valid" for c in w.classes])
    check = np.union1d(np.flatnonzero(adv), np.arange(0, n, 997))
    exp_sub = oracle_verdicts(oracle, w.subset(check), MODE_IS_VALID)
    b = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                           w.msg_len)
    pb = crypto.PreparedBatch(gpu_ctx, b)
    for _ in range(2):
        got = pb.verify(MODE_IS_VALID)
        assert (got[~adv] == ACCEPT).all()
        assert np.array_equal(got[check], exp_sub)
    pb.close()


@pytest.mark.parametrize("lanes", [1, 2, 4, 8])
@pytest.mark.parametrize("mode", [MODE_IS_VALID, MODE_DO_VERIFY])
def test_latency_mode_on_and_off_vs_oracle(gpu_ctx, oracle, golden_ed25519, knobs, lanes, mode):
    """The latency mode (cg_ed25519_points_lanes / cg_ed25519_msm_lanes: two, four or eight
    lanes per signature, used for small pieces, CORDA_AMD_ED_PAIR_MAX / _QUAD_MAX / _OCT_MAX)
    forced on for every size with 2, 4 and 8 lanes, and forced off: every golden class
    and a mutated 4,096-signature batch (the serving size it is for) against the golden
    verdicts and the oracle, plus the forced (h, 1) fallback on every 3rd lane (64-window
    loops beside ~33-window ones in one wave).  The library's per-kernel counters confirm
    which MSM kernel ran."""
    from corda_amd._lib import DEBUG_FORCE_FULL_LENGTH
    knobs.setenv("CORDA_AMD_ED_PAIR_MAX", "0" if lanes == 1 else "1000000")
    knobs.setenv("CORDA_AMD_ED_QUAD_MAX", "1000000" if lanes >= 4 else "0")
    knobs.setenv("CORDA_AMD_ED_OCT_MAX", "1000000" if lanes == 8 else "0")
    msm = {1: "ed25519_msm", 2: "ed25519_msm_pair", 4: "ed25519_msm_quad", 8: "ed25519_msm_oct"}[lanes]
    gpu_ctx.set_profiling(True)
    gpu_ctx.reset_stats()
    g = golden_ed25519
    b = crypto.pack(crypto.EDDSA_ED25519_SHA512, [bytes.fromhex(e["pk"]) for e in g],
                    [bytes.fromhex(e["sig"]) for e in g], [bytes.fromhex(e["msg"]) for e in g])
    key = "is_valid" if mode == MODE_IS_VALID else "do_verify"
    exp_g = np.array([e[key] for e in g], dtype=np.uint8)
    got_g = crypto.verify_packed(gpu_ctx, b, mode)
    assert np.array_equal(got_g, exp_g), [(g[i]["cls"], int(got_g[i]), int(exp_g[i]))
                                          for i in np.flatnonzero(got_g != exp_g)[:10]]
    w = datagen.add_ed25519_adversarial(datagen.make_batch(4096, msg_bytes=1024, seed=71, key_base=950_000),
                                        frac=0.25, seed=9)
    exp = oracle_verdicts(oracle, w, mode)
    got = gpu_verdicts(gpu_ctx, w, mode)
    assert np.array_equal(got, exp), [(w.classes[i], int(got[i]), int(exp[i])) for i in np.flatnonzero(got != exp)[:10]]
    gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 3)
    try:
        assert np.array_equal(gpu_verdicts(gpu_ctx, w, mode), exp)
        assert np.array_equal(crypto.verify_packed(gpu_ctx, b, mode), exp_g)
    finally:
        gpu_ctx.set_debug(DEBUG_FORCE_FULL_LENGTH, 0)
        launches = {k: gpu_ctx.kernel_stats(k)[1]
                    for k in ("ed25519_msm", "ed25519_msm_pair", "ed25519_msm_quad", "ed25519_msm_oct")}
        gpu_ctx.set_profiling(False)
    assert launches[msm] >= 4 and sum(launches.values()) == launches[msm], launches


@pytest.mark.parametrize("path", ["auto", "lanes1", "key_reuse"])
def test_reference_ed25519_artefacts(gpu_ctx, oracle, ref_ed25519_cases, knobs, path):
    """The reference's own Ed25519 artefacts (tests/golden/ref_ed25519_vectors.json): the
    tutorial's two signatures over its tx id (docs/source/tutorial-cordapp.rst:472-476), the
    four Kryo-wire keys (trade.json:3,25 = entropyToKeyPair(1)/(2); tutorial-cordapp.rst:498-499)
    and the mutants of conftest.ref_ed25519_cases through cg_verify_batch in both modes: the
    device gives the verdicts their structure implies (REF_ED_EXPECT) and the oracle's on every
    row (the S + L / S + kL / mixed-order rows are restatement-only).  Then the rows tiled 300×
    among a 25 %-mutated random batch so they sit in every lane position.  Paths: automatic
    (the small call runs the eight-lane latency kernels), latency mode off (one lane per
    signature), and the key-reuse path forced (each reference key decoded once per call)."""
    from conftest import REF_ED_EXPECT
    if path == "lanes1":
        for v in ("CORDA_AMD_ED_PAIR_MAX", "CORDA_AMD_ED_QUAD_MAX", "CORDA_AMD_ED_OCT_MAX"):
            knobs.setenv(v, "0")
    elif path == "key_reuse":
        knobs.setenv("CORDA_AMD_KEY_REUSE", "1")
    cases = ref_ed25519_cases
    b = crypto.pack(crypto.EDDSA_ED25519_SHA512, [c["pk"] for c in cases], [c["sig"] for c in cases],
                    [c["msg"] for c in cases])
    w_cases = datagen.Workload(len(cases), b.scheme & 0x7F, b.pk, b.pk_stride, b.sig, b.sig_stride, b.sig_len, b.msg,
                               b.msg_off, b.msg_len)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        got = crypto.verify_packed(gpu_ctx, b, mode)
        exp = oracle_verdicts(oracle, w_cases, mode)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, [(cases[i]["cls"], int(got[i]), int(exp[i])) for i in bad]
        for i, c in enumerate(cases):
            e = REF_ED_EXPECT[c["cls"]]
            assert e is None or got[i] == e[mode], (c["cls"], int(got[i]), e)
        assert (got[[i for i, c in enumerate(cases) if c["cls"] == "ref_sig"]] == ACCEPT).all()
    rep = 300
    w = datagen.add_ed25519_adversarial(datagen.make_batch(4000, msg_bytes=32, seed=43, key_base=430_000),
                                        frac=0.25, seed=21)
    keys, sigs, msgs = [], [], []
    for j in range(w.n):
        keys.append(bytes(w.pk[j, :32]))
        sigs.append(bytes(w.sig[j, :w.sig_len[j]]))
        msgs.append(bytes(w.msg[w.msg_off[j]:w.msg_off[j] + w.msg_len[j]]))
    for _ in range(rep):
        for c in cases:
            keys.append(c["pk"])
            sigs.append(c["sig"])
            msgs.append(c["msg"])
    order = np.argsort(np.random.default_rng(6).permutation(len(keys)))
    bt = crypto.pack(crypto.EDDSA_ED25519_SHA512, [keys[i] for i in order], [sigs[i] for i in order],
                     [msgs[i] for i in order])
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        got = crypto.verify_packed(gpu_ctx, bt, mode)
        exp = np.concatenate([oracle_verdicts(oracle, w, mode), np.tile(oracle_verdicts(oracle, w_cases, mode), rep)])
        assert np.array_equal(got, exp[order]), np.flatnonzero(got != exp[order])[:10]


@pytest.mark.parametrize("split", ["2", "3"])
def test_one_chunk_verify_split_pieces_vs_oracle(gpu_ctx, oracle, knobs, split):
    """cg_verify_batch as ONE chunk (CORDA_AMD_VERIFY_CHUNKS=1) of an Ed25519-only batch —
    whose message arena is uploaded late, from launch_verify — with the index pieces on two
    streams (CORDA_AMD_ED_SPLIT): the arena must be on the device before any piece's hash
    kernel runs on the second stream (round-4 advisor finding).  Verdicts against the oracle
    on the mutated subset and a stride sample; every untouched signature accepts."""
    knobs.setenv("CORDA_AMD_VERIFY_CHUNKS", "1")
    knobs.setenv("CORDA_AMD_ED_SPLIT", split)
    n = 2 * 65536 + 8191 if split == "2" else 3 * 65536 + 100
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=256, seed=93, key_base=1_300_000),
                                        frac=0.02, seed=23)
    adv = np.array([c != "valid" for c in w.classes])
    check = np.union1d(np.flatnonzero(adv), np.arange(0, n, 331))
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        got = gpu_verdicts(gpu_ctx, w, mode)
        assert (got[~adv] == ACCEPT).all(), np.flatnonzero(got[~adv] != ACCEPT)[:10]
        assert np.array_equal(got[check], oracle_verdicts(oracle, w.subset(check), mode))


@pytest.mark.parametrize("n,reverse,env,msg_bytes", [(160_000, True, "", 32), (160_000, False, "CORDA_AMD_EARLY_POINTS=0", 32),
                                                     (160_000, True, "CORDA_AMD_EARLY_POINTS=0,CORDA_AMD_SPLIT_POINTS=0", 32),
                                                     (50_000, True, "", 32),
                                                     (20_000, False, "", 32), (6_000, True, "", 1024),
                                                     (12_000, True, "", 1024), (12_000, False, "CORDA_AMD_ASYNC_ARENA=0", 1024)])
def test_compute_bound_one_chunk_deferred_offsets_vs_oracle(gpu_ctx, oracle, knobs, n, reverse, env, msg_bytes):
    """A compute-bound host-buffer call (32-byte tx ids: ~140 B per element) runs as ONE chunk
    up to 2^20 elements, and for an Ed25519-only in-order batch its offsets and lengths go
    up with the arena, after the key and signature rows (the points kernel starts first,
    reading the raw 68-byte signature rows; the hash kernel reads the offsets through the
    batch's own arrays).  160,000 signatures: the rows go up in two parts (65,536-aligned
    boundary at 79,872) with each part's points kernel started on its arrival (early
    points).  Below that (50,000, and 160,000 with EARLY_POINTS=0) the key rows go up first
    and the keys are decoded beside the signature rows' copy, then R (split points;
    SPLIT_POINTS=0: one points kernel on the raw rows after both copies).  Arena in
    reverse element order (offsets far from monotone), ragged E12 rows with sig_len, 20 %
    mutated, both modes, against the oracle; the larger call's deferred copy (>= 6 MB)
    runs beside the points kernel.  6,000 x 1 KB: a copy-bound call below the pipeline's
    threshold, one chunk in the eight-lane latency mode, its 6 MB arena deferred; 12,000 x 1 KB (12 MB)
    the same with the arena and its offsets / lengths issued from the upload thread beside
    the row copies (async arena; ASYNC_ARENA=0: after them)."""
    for kv in filter(None, env.split(",")):
        knobs.setenv(*kv.split("=", 1))
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=msg_bytes, seed=101, key_base=1_700_000),
                                        frac=0.2, seed=31)
    ln = w.msg_len[:n].astype(np.uint64)
    off = w.msg_off[:n].astype(np.uint64)
    if reverse:
        new_off = np.zeros(n, np.uint64)
        new_off[::-1] = np.concatenate([[0], np.cumsum(ln[::-1])[:-1]]).astype(np.uint64)
        arena = np.zeros(int(ln.sum()) + 1, np.uint8)
        for i in range(n):
            arena[int(new_off[i]):int(new_off[i] + ln[i])] = w.msg[int(off[i]):int(off[i] + ln[i])]
    else:
        new_off, arena = off, w.msg
    sl = w.sig_len[:n].astype(np.uint32)
    sg = np.zeros((n, 68), np.uint8)
    sg[:, :min(68, w.sig_stride)] = w.sig[:n, :min(68, w.sig_stride)]
    b = crypto.PackedBatch(n, None, np.ascontiguousarray(w.pk[:n, :32]), 32, sg, 68, sl, arena, new_off, w.msg_len[:n])
    ow = datagen.Workload(n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, arena, new_off,
                          w.msg_len)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, ow, mode)
        got = crypto.verify_packed(gpu_ctx, b, mode)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, [(w.classes[i], int(got[i]), int(exp[i])) for i in bad[:10]]


@pytest.mark.parametrize("upload_thread", ["1", "0"])
def test_pipeline_errors_then_recovery(gpu_ctx, oracle, knobs, upload_thread):
    """A chunked host-buffer call (forced into six chunks) whose fifth chunk holds a message
    outside the arena returns CG_E_INVALID_ARGUMENT: the chunk's inputs are checked on the
    calling thread before its kernels go out, the upload thread (CORDA_AMD_VERIFY_UPLOAD_THREAD)
    is stopped and joined, the call's streams drained.  Then allocation failures injected at
    the k-th device allocation (CG_DEBUG_FAIL_ALLOC) return CG_E_OUT_OF_MEMORY (or, past the
    call's last allocation, nothing).  After every failure the same context verifies the
    intact batch against the oracle."""
    from corda_amd._lib import DEBUG_FAIL_ALLOC, CordaGpuError
    knobs.setenv("CORDA_AMD_VERIFY_CHUNKS", "6")
    knobs.setenv("CORDA_AMD_VERIFY_MIN_CHUNK", "500")
    knobs.setenv("CORDA_AMD_VERIFY_UPLOAD_THREAD", upload_thread)
    n = 4000
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=96, seed=77, key_base=1_900_000),
                                        frac=0.2, seed=13)
    mk = lambda off: crypto.PackedBatch(n, None, np.ascontiguousarray(w.pk[:n, :32]), 32, np.ascontiguousarray(
        w.sig[:n, :w.sig_stride]), w.sig_stride, w.sig_len[:n].astype(np.uint32), w.msg, off, w.msg_len[:n])
    good = mk(w.msg_off[:n].astype(np.uint64))
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    assert np.array_equal(crypto.verify_packed(gpu_ctx, good, MODE_IS_VALID), exp)
    off = w.msg_off[:n].astype(np.uint64).copy()
    off[3400] = np.uint64(len(w.msg))  # (chunk 5 of 6) past the arena's end
    with pytest.raises(CordaGpuError):
        crypto.verify_packed(gpu_ctx, mk(off), MODE_IS_VALID)
    assert np.array_equal(crypto.verify_packed(gpu_ctx, good, MODE_IS_VALID), exp)
    for k in (1, 2, 4, 7, 11, 16, 24):
        gpu_ctx.set_debug(DEBUG_FAIL_ALLOC, k)
        try:
            crypto.verify_packed(gpu_ctx, good, MODE_IS_VALID)
        except CordaGpuError:
            pass
        finally:
            gpu_ctx.set_debug(DEBUG_FAIL_ALLOC, 0)
        assert np.array_equal(crypto.verify_packed(gpu_ctx, good, MODE_IS_VALID), exp), k


@pytest.mark.parametrize("n,msg_bytes", [(32_767, 32), (32_768, 32), (65_536, 32), (40_000, 1024), (262_144, 32)])
def test_host_verify_arena_bounds_beside_row_copies(gpu_ctx, oracle, n, msg_bytes):
    """One-chunk Ed25519-only host calls from 32,768 elements check msg_off / msg_len against
    the arena on the upload thread while the rows go up and the points kernels run
    (create_batch's BoundsBeside): an element outside the arena — first, middle or last,
    offset past the end or length over it — still returns CG_E_INVALID_ARGUMENT naming that
    element (as the synchronous check below 32,768 does), and the same context then
    verifies the intact batch against the oracle."""
    from corda_amd._lib import CordaGpuError
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=msg_bytes, seed=n % 997 + 3,
                                                           key_base=3_400_000 + n % 7919), frac=0.02, seed=31)
    sl = w.sig_len[:n].astype(np.uint32)
    ss = max(64, (int(sl.max()) + 3) // 4 * 4)
    sg = np.zeros((n, ss), dtype=np.uint8)
    sg[:, :min(ss, w.sig_stride)] = w.sig[:n, :min(ss, w.sig_stride)]
    mk = lambda off, ln: crypto.PackedBatch(n, None, np.ascontiguousarray(w.pk[:n, :32]), 32, sg, ss, sl, w.msg,
                                            off, ln)
    off0, len0 = w.msg_off[:n].astype(np.uint64), w.msg_len[:n].astype(np.uint32)
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    for i, kind in ((0, "off"), (n // 2, "len"), (n - 1, "off")):
        off, ln = off0.copy(), len0.copy()
        if kind == "off":
            off[i] = np.uint64(len(w.msg) + 1)
        else:
            ln[i] = np.uint32(len(w.msg) - int(off[i]) + 1)
        with pytest.raises(CordaGpuError, match=f"element {i}$"):
            crypto.verify_packed(gpu_ctx, mk(off, ln), MODE_IS_VALID)
        got = crypto.verify_packed(gpu_ctx, mk(off0, len0), MODE_IS_VALID)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, (i, [(w.classes[j], int(got[j]), int(exp[j])) for j in bad[:10]])


@pytest.mark.parametrize("n", [4096, 65_536])
def test_all_ed25519_scheme_array_equals_null(gpu_ctx, oracle, n):
    """A scheme array naming Ed25519 for every element takes the scheme_id = NULL host path
    (cordagpu.cpp ed25519_only); the verdicts equal the oracle's with the array, without it,
    and with one element flagged CG_SCHEME_FLAG_KEY_INVALID (which keeps the per-element
    path: that element KEY_INVALID, the rest unchanged); an out-of-arena message is the same
    error either way."""
    from corda_amd._lib import CordaGpuError
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=1024, seed=n % 991 + 7,
                                                           key_base=3_700_000 + n % 7919), frac=0.02, seed=37)
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    mk = lambda sch, off=None: crypto.PackedBatch(n, sch, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg,
                                                  w.msg_off if off is None else off, w.msg_len)
    assert np.array_equal(crypto.verify_packed(gpu_ctx, mk(w.scheme), MODE_IS_VALID), exp)
    assert np.array_equal(crypto.verify_packed(gpu_ctx, mk(None), MODE_IS_VALID), exp)
    flagged = w.scheme.copy()
    flagged[n // 3] |= 0x80  # CG_SCHEME_FLAG_KEY_INVALID
    want = exp.copy()
    want[n // 3] = 3  # CG_KEY_INVALID
    assert np.array_equal(crypto.verify_packed(gpu_ctx, mk(flagged), MODE_IS_VALID), want)
    off = w.msg_off.astype(np.uint64).copy()
    off[n - 2] = np.uint64(len(w.msg) + 5)
    for sch in (w.scheme, None):
        with pytest.raises(CordaGpuError, match=f"element {n - 2}$"):
            crypto.verify_packed(gpu_ctx, mk(sch, off), MODE_IS_VALID)


@pytest.mark.parametrize("n,msg_bytes", [(1, 32), (63, 1024), (65, 32), (257, 1024), (20_480, 32), (20_481, 32),
                                         (32_768, 1024), (32_769, 1024), (40_001, 32), (65_537, 32),
                                         (131_073, 32), (131_073, 1024), (262_145, 1024), ((1 << 20) + 1, 32)])
def test_host_verify_plan_boundaries_vs_oracle(gpu_ctx, oracle, n, msg_bytes):
    """cg_verify_batch from pageable host buffers at sizes one past each plan boundary:
    the latency-mode thresholds (one-chunk calls: 20,480 for 32 B ids, 32,768 for 1 KB
    messages — each at and one past; pieces: 40,000), the early-points part size (65,536), the
    pipeline's start for copy-bound calls (2^17) and for compute-bound ones (2^20: 2^20 + 1
    32-byte ids run as eight chunks), and small ragged calls; 32 B ids and 1 KB messages, 2 %
    mutated, every verdict against the oracle."""
    w = datagen.add_ed25519_adversarial(datagen.make_batch(n, msg_bytes=msg_bytes, seed=n % 1000 + 5,
                                                           key_base=3_000_000 + n % 7919), frac=0.02, seed=29)
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)
    got = gpu_verdicts(gpu_ctx, w, MODE_IS_VALID)
    bad = np.flatnonzero(got != exp)
    assert bad.size == 0, [(w.classes[i], int(got[i]), int(exp[i])) for i in bad[:10]]


def test_options_are_read_at_open_and_set_per_context(gpu_ctx, oracle, knobs):
    """The CORDA_AMD_* knobs (cg_plan.h Options): an environment change after cg_open has
    no effect on the open context, cg_set_option has (the library's per-kernel counters say
    which MSM ran), an unknown key is an error naming it, and the verdicts never change."""
    from corda_amd._lib import CordaGpuError
    w = datagen.add_ed25519_adversarial(datagen.make_batch(1000, msg_bytes=32, seed=8, key_base=2_600_000), frac=0.1,
                                        seed=4)
    exp = oracle_verdicts(oracle, w, MODE_IS_VALID)

    def msm_kernels():
        gpu_ctx.set_profiling(True)
        gpu_ctx.reset_stats()
        try:
            assert np.array_equal(gpu_verdicts(gpu_ctx, w, MODE_IS_VALID), exp)
            return {k for k in ("ed25519_msm", "ed25519_msm_pair", "ed25519_msm_quad", "ed25519_msm_oct")
                    if gpu_ctx.kernel_stats(k)[1]}
        finally:
            gpu_ctx.set_profiling(False)

    assert msm_kernels() == {"ed25519_msm_oct"}  # 1,000 signatures: eight lanes per signature
    old = os.environ.get("CORDA_AMD_ED_PAIR_MAX")
    os.environ["CORDA_AMD_ED_PAIR_MAX"] = "0"
    try:
        assert msm_kernels() == {"ed25519_msm_oct"}  # read at cg_open only
    finally:
        if old is None:
            os.environ.pop("CORDA_AMD_ED_PAIR_MAX")
        else:
            os.environ["CORDA_AMD_ED_PAIR_MAX"] = old
    knobs.setenv("CORDA_AMD_ED_PAIR_MAX", "0")
    assert msm_kernels() == {"ed25519_msm"}
    knobs.setenv("CORDA_AMD_ED_PAIR_MAX", None)
    assert msm_kernels() == {"ed25519_msm_oct"}
    with pytest.raises(CordaGpuError, match="CORDA_AMD_NO_SUCH_KNOB"):
        gpu_ctx.set_option("CORDA_AMD_NO_SUCH_KNOB", "1")
