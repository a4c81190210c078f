"""GPU parity: ECDSA secp256k1 / secp256r1 (BC 1.57 semantics) and the DER
pre-pass of libcordagpu vs the CPU oracle — golden fixtures (D1–D8 + DER
variants, RFC 6979 KATs), seeded random batches, mixed-scheme batches, and a
config-3-shaped batch (size-independent property: every untouched signature
accepts; the mutated subset matches the oracle element-wise)."""
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
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datagen  # noqa: E402
from test_gpu_ed25519 import gpu_verdicts, oracle_verdicts  # noqa: E402

pytestmark = pytest.mark.gpu


def test_golden_fixtures(gpu_ctx, golden_ecdsa):
    g = golden_ecdsa
    for mode, key in ((MODE_IS_VALID, "is_valid"), (MODE_DO_VERIFY, "do_verify")):
        b = crypto.pack([e["scheme"] for e in g], [bytes.fromhex(e["q"]) for e in g],
                        [bytes.fromhex(e["sig"]) for e in g], [bytes.fromhex(e["msg"]) for e in g])
        v = crypto.verify_packed(gpu_ctx, b, mode)
        exp = np.array([e[key] for e in g], dtype=np.uint8)
        bad = np.flatnonzero(v != exp)
        assert bad.size == 0, [(g[i]["cls"], g[i]["scheme"], int(v[i]), int(exp[i])) for i in bad[:10]]


@pytest.mark.parametrize("scheme", [2, 3])
def test_random_and_mutated_vs_oracle(gpu_ctx, oracle, scheme):
    w = datagen.make_batch(4000, msg_bytes=77, scheme=scheme, seed=5 + scheme, key_base=70_000)
    w = datagen.add_ecdsa_adversarial(w, frac=0.3, seed=scheme)
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        got = gpu_verdicts(gpu_ctx, w, mode)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, [(w.classes[i], int(got[i]), int(exp[i])) for i in bad[:10]]


def test_mixed_scheme_batch(gpu_ctx, oracle):
    rng = np.random.default_rng(4)
    sch = rng.choice(np.array([2, 3, 4], dtype=np.uint8), size=6000, p=[0.15, 0.15, 0.7])
    w = datagen.make_batch(len(sch), msg_bytes=32, scheme=sch, seed=21, key_base=123_456)
    w = datagen.add_ecdsa_adversarial(w, frac=0.2, seed=3)
    for j in np.flatnonzero(sch == 4)[:200]:
        w.sig[j, 5] ^= 1
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        exp = oracle_verdicts(oracle, w, mode)
        got = gpu_verdicts(gpu_ctx, w, mode)
        assert np.array_equal(got, exp)


def test_der_parse_batch(gpu_ctx, oracle, golden_ecdsa):
    g = golden_ecdsa
    sigs = [bytes.fromhex(e["sig"]) for e in g]
    stride = (max(len(s) for s in sigs) + 3) // 4 * 4
    buf = np.zeros((len(g), stride), np.uint8)
    sl = np.zeros(len(g), np.uint32)
    for i, s in enumerate(sigs):
        buf[i, :len(s)] = np.frombuffer(s, np.uint8)
        sl[i] = len(s)
    sch = np.array([e["scheme"] for e in g], np.uint8)
    rs = np.zeros((len(g), 64), np.uint8)
    st = np.zeros(len(g), np.uint8)
    gpu_ctx.check(gpu_ctx.lib.cg_der_parse_batch(gpu_ctx.h, len(g), ptr(sch), ptr(buf), stride, ptr(sl), ptr(rs),
                                                 ptr(st)))
    oracle.oracle_der_decode.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                         ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    for i, s in enumerate(sigs):
        r, ss, fl = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32), ctypes.c_int()
        rc = oracle.oracle_der_decode(int(sch[i]), s, len(s), r, ss, ctypes.byref(fl))
        if rc != 0:
            assert st[i] == 2, g[i]["cls"]
        else:
            assert st[i] == (1 if fl.value else 0), g[i]["cls"]
            if not fl.value:
                assert bytes(rs[i]) == r.raw + ss.raw


def test_config3_shape(gpu_ctx, oracle):
    n = 1 << 17
    for scheme in (2, 3):
        w = datagen.make_batch(n, msg_bytes=1024, scheme=scheme, seed=scheme * 7, key_base=5_000_000)
        w = datagen.add_ecdsa_adversarial(w, frac=0.01, seed=scheme)
        got = gpu_verdicts(gpu_ctx, w, MODE_IS_VALID)
        adv = np.array([c != "valid" for c in w.classes])
        assert (got[~adv] == ACCEPT).all()
        sub = w.subset(np.flatnonzero(adv))
        assert np.array_equal(got[adv], oracle_verdicts(oracle, sub, MODE_IS_VALID))


def test_config3_full_size_mixed_batch(gpu_ctx, oracle):
    """BASELINE config 3 at full size in ONE batch: 2^20 secp256k1 + 2^20 P-256
    signatures, 1 KB messages, 1 % adversarial over D1-D8 (both curves' pipelines
    concurrently on their streams, several ECDSA scratch chunks).  Size-independent
    properties at full size: every untouched signature accepts; the adversarial
    subset's verdicts equal the oracle's element for element.  Each curve's 2^20
    signatures tile 2^18 distinct (key, message, signature) tuples."""
    n, pool = 1 << 20, 1 << 18
    p = datagen.make_batch(2 * pool, msg_bytes=1024, scheme=np.repeat(np.array([2, 3], np.uint8), pool), seed=77,
                           key_base=7_000_000)
    k1 = p.subset(np.arange(pool)).tiled(n)
    r1 = p.subset(np.arange(pool, 2 * pool)).tiled(n)
    w = datagen.Workload(2 * n, np.concatenate([k1.scheme, r1.scheme]), np.concatenate([k1.pk, r1.pk]), 64,
                         np.concatenate([k1.sig, r1.sig]), k1.sig_stride, np.concatenate([k1.sig_len, r1.sig_len]),
                         np.concatenate([k1.msg[:-16], r1.msg]),
                         np.concatenate([k1.msg_off, r1.msg_off + np.uint64(len(k1.msg) - 16)]),
                         np.concatenate([k1.msg_len, r1.msg_len]), ["valid"] * (2 * n))
    del k1, r1, p
    w = datagen.add_ecdsa_adversarial(w, frac=0.01, seed=13)
    got = gpu_verdicts(gpu_ctx, w, MODE_IS_VALID)
    adv = np.array([c != "valid" for c in w.classes])
    assert (got[~adv] == ACCEPT).all()
    idx = np.flatnonzero(adv)
    assert np.array_equal(got[idx], oracle_verdicts(oracle, w.subset(idx), MODE_IS_VALID))
    assert idx.size > 15000 and (w.scheme[idx] == 2).any() and (w.scheme[idx] == 3).any()


@pytest.mark.parametrize("mod", [3, 1])
def test_forced_glv_fallback_vs_oracle(gpu_ctx, oracle, golden_ecdsa, mod):
    """secp256k1's GLV split falls back to the full-length pair (|u2|, 0) when a half
    exceeds 129 bits (cg_ecdsa.h glv_split; never observed on real scalars).  Forced on
    the device through cg_set_debug for every mod-th K1 element — the golden D1-D8 and
    B.4 rows plus a mutated random K1 batch — the verdicts must stay the oracle's (the
    waves holding a forced lane run 65 digits instead of ~33)."""
    from corda_amd._lib import DEBUG_FORCE_GLV_FALLBACK
    g = [e for e in golden_ecdsa if e["scheme"] == 2]
    w = datagen.add_ecdsa_adversarial(datagen.make_batch(3000, msg_bytes=77, scheme=2, seed=31, key_base=90_000),
                                      frac=0.3, seed=5)
    gpu_ctx.set_debug(DEBUG_FORCE_GLV_FALLBACK, mod)
    try:
        for mode, key in ((MODE_IS_VALID, "is_valid"), (MODE_DO_VERIFY, "do_verify")):
            b = crypto.pack([e["scheme"] for e in g], [bytes.fromhex(e["q"]) for e in g],
                            [bytes.fromhex(e["sig"]) for e in g], [bytes.fromhex(e["msg"]) for e in g])
            v = crypto.verify_packed(gpu_ctx, b, mode)
            exp = np.array([e[key] for e in g], dtype=np.uint8)
            bad = np.flatnonzero(v != exp)
            assert bad.size == 0, [(g[i]["cls"], int(v[i]), int(exp[i])) for i in bad[:10]]
            got = gpu_verdicts(gpu_ctx, w, mode)
            exp = oracle_verdicts(oracle, w, mode)
            bad = np.flatnonzero(got != exp)
            assert bad.size == 0, [(w.classes[i], int(got[i]), int(exp[i])) for i in bad[:10]]
        assert (got == ACCEPT).sum() > 1500
    finally:
        gpu_ctx.set_debug(DEBUG_FORCE_GLV_FALLBACK, 0)


def test_prepared_batch_reparses_der_every_verify(gpu_ctx, oracle, golden_ecdsa):
    """A staged batch keeps its raw DER rows and every cg_batch_verify re-runs the K4
    parse before the ECDSA kernels (BC decodes inside each engineVerify).  The same
    staged mixed batch — golden D1-D8 rows (malformed and out-of-range DER among
    them), mutated random K1/R1 and Ed25519 elements — verified repeatedly in both
    modes must give the oracle's verdicts every time."""
    g = golden_ecdsa
    gold = crypto.pack([e["scheme"] for e in g], [bytes.fromhex(e["q"]) for e in g],
                       [bytes.fromhex(e["sig"]) for e in g], [bytes.fromhex(e["msg"]) for e in g])
    sch = np.random.default_rng(9).choice(np.array([2, 3, 4], np.uint8), size=3000)
    w = datagen.add_ecdsa_adversarial(datagen.make_batch(len(sch), msg_bytes=41, scheme=sch, seed=19,
                                                         key_base=310_000), frac=0.3, seed=11)
    rand = crypto.PackedBatch(w.n, w.scheme, w.pk, w.pk_stride, w.sig, w.sig_stride, w.sig_len, w.msg, w.msg_off,
                              w.msg_len)
    for b, exp_of in ((gold, lambda mode: np.array([e["is_valid" if mode == MODE_IS_VALID else "do_verify"]
                                                    for e in g], np.uint8)),
                      (rand, lambda mode: oracle_verdicts(oracle, w, mode))):
        pb = crypto.PreparedBatch(gpu_ctx, b)
        try:
            for mode in (MODE_IS_VALID, MODE_DO_VERIFY, MODE_IS_VALID):
                got, exp = pb.verify(mode), exp_of(mode)
                bad = np.flatnonzero(got != exp)
                assert bad.size == 0, [(int(i), int(got[i]), int(exp[i])) for i in bad[:10]]
        finally:
            pb.close()


def test_reference_certificate_signatures(gpu_ctx, oracle, ref_cert_cases):
    """The reference's own BC-signed ecdsa-with-SHA256 certificates (dev CA / sample
    keystores; tests/golden/ref_cert_vectors.json) and their mutants through
    cg_verify_batch in both modes, and the K4 DER pre-pass on their signature rows:
    the device gives the verdicts the structure implies (test_oracle.REF_EXPECT), which
    the oracle and OpenSSL also give.  The rows are also tiled 300× into one batch with
    mutated random K1/R1 signatures, so they sit in every lane position of a wave."""
    from test_oracle import REF_EXPECT
    cases = ref_cert_cases
    b = crypto.pack([c["scheme"] for c in cases], [bytes.fromhex(c["q"]) for c in cases], [c["sig"] for c in cases],
                    [c["msg"] for c in cases])
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        v = crypto.verify_packed(gpu_ctx, b, mode)
        exp = np.array([REF_EXPECT[c["cls"]][mode] for c in cases], np.uint8)
        bad = np.flatnonzero(v != exp)
        assert bad.size == 0, [(cases[i]["cls"], cases[i]["scheme"], int(v[i]), int(exp[i])) for i in bad]
    # K4 alone: the reference rows parse to the oracle's (r, s); the malformed mutants fail
    sigs = [c["sig"] for c in cases]
    stride = (max(len(s) for s in sigs) + 3) // 4 * 4
    buf = np.zeros((len(sigs), stride), np.uint8)
    sl = np.array([len(s) for s in sigs], np.uint32)
    for i, s in enumerate(sigs):
        buf[i, :len(s)] = np.frombuffer(s, np.uint8)
    sch = np.array([c["scheme"] for c in cases], np.uint8)
    rs, st = np.zeros((len(sigs), 64), np.uint8), np.zeros(len(sigs), np.uint8)
    gpu_ctx.check(gpu_ctx.lib.cg_der_parse_batch(gpu_ctx.h, len(sigs), ptr(sch), ptr(buf), stride, ptr(sl), ptr(rs),
                                                 ptr(st)))
    oracle.oracle_der_decode.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                         ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    for i, s in enumerate(sigs):
        r, ss, fl = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32), ctypes.c_int()
        rc = oracle.oracle_der_decode(int(sch[i]), s, len(s), r, ss, ctypes.byref(fl))
        assert (st[i] == 2) == (rc != 0) == (cases[i]["cls"] in ("ref_sig0_inc", "ref_nonminimal_r")), cases[i]["cls"]
        if rc == 0:
            assert st[i] == (1 if fl.value else 0), cases[i]["cls"]
            if not fl.value:
                assert bytes(rs[i]) == r.raw + ss.raw, cases[i]["cls"]
    # tiled among random mutated ECDSA signatures
    rep = 300
    w = datagen.add_ecdsa_adversarial(datagen.make_batch(4000, msg_bytes=300, scheme=np.array([2, 3] * 2000, np.uint8),
                                                         seed=41, key_base=410_000), frac=0.3, seed=17)
    pos = np.random.default_rng(5).permutation(w.n + rep * len(cases))
    all_s, all_q, all_sig, all_m = [], [], [], []
    for j in range(w.n):
        all_s.append(int(w.scheme[j]))
        all_q.append(bytes(w.pk[j, :64]))
        all_sig.append(bytes(w.sig[j, :w.sig_len[j]]))
        all_m.append(bytes(w.msg[w.msg_off[j]:w.msg_off[j] + w.msg_len[j]]))
    for _ in range(rep):
        for c in cases:
            all_s.append(c["scheme"])
            all_q.append(bytes.fromhex(c["q"]))
            all_sig.append(c["sig"])
            all_m.append(c["msg"])
    order = np.argsort(pos)
    bt = crypto.pack([all_s[i] for i in order], [all_q[i] for i in order], [all_sig[i] for i in order],
                     [all_m[i] for i in order])
    for mode in (MODE_IS_VALID, MODE_DO_VERIFY):
        got = crypto.verify_packed(gpu_ctx, bt, mode)
        exp_r = oracle_verdicts(oracle, w, mode)
        exp = np.concatenate([exp_r, np.tile(np.array([REF_EXPECT[c["cls"]][mode] for c in cases], np.uint8), rep)])
        assert np.array_equal(got, exp[order])
