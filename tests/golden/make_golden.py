#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

The reference path cannot run here (JVM + un-vendored i2p 0.2.0 / BC 1.57 jars,
SURVEY.md §8c) and the reference tests hold no fixed vectors, so the fixtures are
produced by the oracle's Python twin (oracle/py) and every verdict is
cross-checked, at generation time, against the independent C restatement
(oracle/liboracle.so) and — on the semantic overlap only — against OpenSSL 3.
Known-answer anchors: RFC 8032 §7.1 tests 1-3 (Ed25519) and RFC 6979 A.2.5
(P-256, "sample"/"test").

    python tests/golden/make_golden.py      # rewrites the *.json fixtures
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))

import ecdsa_bc as EC  # noqa: E402
import ed25519_i2p as ED  # noqa: E402
import merkle_tx as MK  # noqa: E402
import openssl_xcheck as OSSL  # noqa: E402

ORACLE = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
ORACLE.oracle_ftx_verify_batch.argtypes = [ctypes.c_void_p] * 9 + [ctypes.c_size_t, ctypes.c_void_p]

RFC8032 = [  # (secret, public, message, signature) — RFC 8032 §7.1 TEST 1..3
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]

RFC6979_P256 = {  # RFC 6979 A.2.5, SHA-256
    "x": 0xC9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721,
    "Ux": 0x60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6,
    "Uy": 0x7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299,
    "sample": (0xEFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716,
               0xF7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8),
    "test": (0xF1ABB023518351CD71D881567B1EA663ED3EFCF6C5132B354F28D3B0B7D38367,
             0x019F4113742A2B14BD25926B49C649155F267E60D3814B4C0CC84250E46F0083),
}


def c_ed(pk, sig, msg, mode):
    return ORACLE.oracle_ed25519_verify(pk, sig, len(sig), msg, len(msg), mode)


def c_ec(scheme, q, sig, msg, mode):
    qb = q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")
    return ORACLE.oracle_ecdsa_verify(scheme, qb, sig, len(sig), msg, len(msg), mode)


# ------------------------------------------------------------------- Ed25519
def torsion_points():
    """The 8 points of order dividing 8 (as extended coordinates)."""
    rnd = random.Random(7)
    while True:
        y = rnd.randrange(ED.P)
        try:
            pt = ED.decode_point_i2p(y.to_bytes(32, "little"))
        except ED.KeyInvalid:
            continue
        t = ED.scalarmult(pt, ED.L)
        t4 = ED.scalarmult(t, 4)
        if not ED.point_equal(t4, ED.IDENTITY):  # order exactly 8
            return [ED.scalarmult(t, k) for k in range(8)]


def order_of(pt):
    for k in (1, 2, 4, 8):
        if ED.point_equal(ED.scalarmult(pt, k), ED.IDENTITY):
            return k
    return None


def forge_small_order(a_enc: bytes, order: int, rnd, r_enc: bytes | None = None):
    """Signature (R = identity, S = 0 or L) accepted for a key of small order:
    [S]B - [h]A = -[h]A = O whenever order | h.  Searches a message."""
    r = r_enc if r_enc is not None else (1).to_bytes(32, "little")
    ab = ED.abyte(a_enc)
    while True:
        msg = rnd.randbytes(rnd.randint(1, 48))
        h = ED.sc_reduce(hashlib.sha512(r + ab + msg).digest())
        if h % order == 0:
            return msg, r + bytes(32)


def ed25519_cases():
    rnd = random.Random(20170614)
    cases = []

    def add(cls, pk, sig, msg):
        vi, vd = ED.is_valid(pk, sig, msg), ED.do_verify(pk, sig, msg)
        ci, cd = c_ed(pk, sig, msg, 0), c_ed(pk, sig, msg, 1)
        assert (vi, vd) == (ci, cd), (cls, pk.hex(), sig.hex(), msg.hex(), vi, vd, ci, cd)
        cases.append({"cls": cls, "pk": pk.hex(), "sig": sig.hex(), "msg": msg.hex(), "is_valid": vi,
                      "do_verify": vd})

    # RFC 8032 known answers: the twin must reproduce them and OpenSSL must agree
    for sk, pk, m, sig in RFC8032:
        spk, ssig = ED.sign(bytes.fromhex(sk), bytes.fromhex(m))
        assert spk.hex() == pk and ssig.hex() == sig, "RFC 8032 KAT mismatch"
        assert OSSL.ed25519_verify(spk, ssig, bytes.fromhex(m))
        add("rfc8032", spk, ssig, bytes.fromhex(m))
    # reference test keys entropyToKeyPair(20..110) (TestConstants.kt:32-71)
    for k in range(20, 111, 10):
        seed = ED.entropy_seed(k)
        for msg in (bytes(100), rnd.randbytes(32), b"corda"):
            pk, sig = ED.sign(seed, msg)
            add("testkey", pk, sig, msg)
    valid = []
    for t in range(120):
        seed = rnd.randbytes(32)
        msg = rnd.randbytes(rnd.choice([0, 1, 31, 32, 33, 63, 64, 65, 111, 112, 127, 128, 129, 200, 1024]))
        pk, sig = ED.sign(seed, msg)
        if msg:
            assert OSSL.ed25519_sign(seed, msg) == sig and OSSL.ed25519_verify(pk, sig, msg)
        valid.append((seed, pk, sig, msg))
        add("valid", pk, sig, msg)
    for seed, pk, sig, msg in valid[:40]:
        b = bytearray(sig); b[rnd.randrange(32)] ^= 1 << rnd.randrange(8); add("E1_flip_R", pk, bytes(b), msg)
        b = bytearray(sig); b[32 + rnd.randrange(32)] ^= 1 << rnd.randrange(8); add("E2_flip_S", pk, bytes(b), msg)
        if msg:
            b = bytearray(msg); b[rnd.randrange(len(b))] ^= 1 << rnd.randrange(8); add("E3_flip_M", pk, sig, bytes(b))
        other = ED.sign(rnd.randbytes(32), b"x")[0]
        add("E4_wrong_key", other, sig, msg)
        s = int.from_bytes(sig[32:], "little")
        add("E5_S_plus_L", pk, sig[:32] + (s + ED.L).to_bytes(32, "little"), msg)
        k_hi = [k for k in range(1, 16) if s + k * ED.L >= 2**255 and s + k * ED.L < 2**256]
        for k in k_hi[:2]:
            add("E6_S_plus_kL", pk, sig[:32] + (s + k * ED.L).to_bytes(32, "little"), msg)
    # E6 with the slide() carry forced off the top: S with long runs of ones near bit 255
    for _ in range(24):
        seed, pk, sig, msg = valid[rnd.randrange(len(valid))]
        s = (2**256 - 1) ^ (rnd.getrandbits(16) << rnd.randrange(0, 240))
        add("E6_slide_drop", pk, sig[:32] + s.to_bytes(32, "little"), msg)
    # E7 small-order keys with forged accepting signatures (+ rejecting ones)
    tors = torsion_points()
    for t in tors:
        enc = ED.encode_point(t)
        o = order_of(t)
        msg, sig = forge_small_order(enc, o, rnd)
        add("E7_small_order_forged", enc, sig, msg)
        add("E7_small_order_forged_SL", enc, sig[:32] + ED.L.to_bytes(32, "little"), msg)
        add("E7_small_order_random", enc, rnd.randbytes(64), rnd.randbytes(16))
    # E8 mixed-order A = aB + T, signed with a (accepts iff [h]T = O)
    for i in range(16):
        seed = rnd.randbytes(32)
        a, prefix, _ = ED.seed_to_keypair(seed)
        t = tors[1 + i % 7]
        apt = ED._add(ED.scalarmult(ED.BASE, a), t)
        aenc = ED.encode_point(apt)
        msg = rnd.randbytes(20)
        r = ED.sc_reduce(hashlib.sha512(prefix + msg).digest())
        rb = ED.encode_point(ED.scalarmult(ED.BASE, r))
        h = ED.sc_reduce(hashlib.sha512(rb + aenc + msg).digest())
        add("E8_mixed_order", aenc, rb + ((r + h * a) % ED.L).to_bytes(32, "little"), msg)
    # E9 non-canonical A encodings: y + p (y < 19) and x = 0 with the sign bit set
    for y in range(0, 19):
        for sign in (0, 1):
            enc = bytearray((y + ED.P).to_bytes(32, "little"))
            enc[31] |= sign << 7
            enc = bytes(enc)
            try:
                apt = ED.decode_point_i2p(enc)
            except ED.KeyInvalid:
                add("E9_noncanon_A_invalid", enc, rnd.randbytes(64), b"m")
                continue
            o = order_of(apt)
            if o:
                msg, sig = forge_small_order(enc, o, rnd)
                add("E9_noncanon_A_forged", enc, sig, msg)
            else:
                add("E9_noncanon_A", enc, rnd.randbytes(64), b"m")
    for enc_hex in ("0100000000000000000000000000000000000000000000000000000000000080",
                    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff"):
        enc = bytes.fromhex(enc_hex)
        apt = ED.decode_point_i2p(enc)
        msg, sig = forge_small_order(enc, order_of(apt), rnd)
        add("E9_x0_signbit", enc, sig, msg)
    # E10 non-canonical R: identity encoded as y = 1 + p never verifies
    for t in tors[:4]:
        enc = ED.encode_point(t)
        msg, sig = forge_small_order(enc, order_of(t), rnd, r_enc=(1 + ED.P).to_bytes(32, "little"))
        add("E10_noncanon_R", enc, sig, msg)
    # E11 keys with no square root
    n11 = 0
    while n11 < 12:
        enc = rnd.randbytes(32)
        try:
            ED.decode_point_i2p(enc)
        except ED.KeyInvalid:
            add("E11_no_sqrt_key", enc, rnd.randbytes(64), rnd.randbytes(8))
            n11 += 1
    # E12 signature length != 64 (and the doVerify empty-argument cases)
    seed, pk, sig, msg = valid[3]
    for ln in (0, 1, 63, 65, 72, 128):
        add("E12_sig_len", pk, (sig * 3)[:ln], msg)
    add("empty_msg", *ED.sign(rnd.randbytes(32), b""), b"")
    return cases


# --------------------------------------------------------------------- ECDSA
def ecdsa_cases():
    rnd = random.Random(1979)
    cases = []

    def add(cls, scheme, q, sig, msg):
        vi, vd = EC.is_valid(scheme, q, sig, msg), EC.do_verify(scheme, q, sig, msg)
        ci, cd = c_ec(scheme, q, sig, msg, 0), c_ec(scheme, q, sig, msg, 1)
        assert (vi, vd) == (ci, cd), (cls, scheme, sig.hex(), vi, vd, ci, cd)
        if vi == EC.ACCEPT:  # the overlap: OpenSSL must accept too
            assert OSSL.ecdsa_verify(scheme, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), sig,
                                     hashlib.sha256(msg).digest()), (cls, scheme)
        cases.append({"cls": cls, "scheme": scheme, "q": q[0].to_bytes(32, "big").hex() + q[1].to_bytes(32, "big").hex(),
                      "sig": sig.hex(), "msg": msg.hex(), "is_valid": vi, "do_verify": vd})

    # RFC 6979 A.2.5 known answers
    K = RFC6979_P256
    q = EC.pubkey(3, K["x"])
    assert q == (K["Ux"], K["Uy"])
    for m in ("sample", "test"):
        r, s = EC.sign_rs(3, K["x"], m.encode())
        assert (r, s) == K[m], "RFC 6979 KAT mismatch"
        add("rfc6979", 3, q, EC.der_encode(r, s), m.encode())
    for scheme in (2, 3):
        c = EC.CURVES[scheme]
        for t in range(40):
            d = rnd.randrange(1, c.n)
            q = EC.pubkey(scheme, d)
            msg = rnd.randbytes(1024 if t % 10 == 0 else rnd.choice([1, 32, 100]))
            r, s = EC.sign_rs(scheme, d, msg)
            sig = EC.der_encode(r, s)
            add("valid", scheme, q, sig, msg)
            if t >= 20:
                continue
            b = bytearray(sig); b[rnd.randrange(6, len(b))] ^= 1 << rnd.randrange(8); add("D1_flip_sig", scheme, q, bytes(b), msg)
            b = bytearray(msg); b[rnd.randrange(len(b))] ^= 1; add("D1_flip_msg", scheme, q, sig, bytes(b))
            add("D2_r_zero", scheme, q, EC.der_encode(0, s), msg)
            add("D2_s_zero", scheme, q, EC.der_encode(r, 0), msg)
            add("D3_r_ge_n", scheme, q, EC.der_encode(r + c.n, s), msg)
            add("D3_s_ge_n", scheme, q, EC.der_encode(r, s + c.n), msg)
            add("D4_negative", scheme, q, EC.der_encode(-r, s), msg)
            body_r = EC.der_int(r)
            padded = b"\x02" + bytes([body_r[1] + 1]) + b"\x00" + body_r[2:]
            body = padded + EC.der_int(s)
            add("D5_nonminimal_int", scheme, q, b"\x30" + bytes([len(body)]) + body, msg)
            body = EC.der_int(r) + EC.der_int(s)
            add("D6_ber_long_len", scheme, q, b"\x30\x81" + bytes([len(body)]) + body, msg)
            add("D7_trailing", scheme, q, sig + b"\x00", msg)
            add("D8_high_s", scheme, q, EC.der_encode(r, c.n - s), msg)
            add("D_three_elems", scheme, q, b"\x30" + bytes([len(body) + 3]) + body + b"\x02\x01\x01", msg)
            add("D_indefinite", scheme, q, b"\x30\x80" + body + b"\x00\x00", msg)
            add("D_empty_int", scheme, q, b"\x30" + bytes([len(EC.der_int(s)) + 2]) + b"\x02\x00" + EC.der_int(s), msg)
            add("D_octet_string", scheme, q, b"\x30" + bytes([len(body)]) + b"\x04" + body[1:], msg)
            add("D_empty", scheme, q, b"", msg)
            add("empty_msg", scheme, q, sig, b"")
            add("wrong_key", scheme, EC.pubkey(scheme, rnd.randrange(1, c.n)), sig, msg)
        # long (but DER-valid) integer -> REJECT, not malformed
        d = rnd.randrange(1, c.n); q = EC.pubkey(scheme, d); msg = b"long-int"
        r, s = EC.sign_rs(scheme, d, msg)
        add("D3_huge_int", scheme, q, EC.der_encode(r + (1 << 600), s), msg)
        # off-curve / out-of-range keys -> KEY_INVALID
        add("key_off_curve", scheme, (q[0], (q[1] + 1) % c.p), EC.der_encode(r, s), msg)
        add("key_x_ge_p", scheme, (q[0] + c.p, q[1]), EC.der_encode(r, s), msg) if q[0] + c.p < 2**256 else None
        add("key_zero", scheme, (0, 0), EC.der_encode(r, s), msg)
    # Appendix B.4 exceptional points, realised as signatures (a separate RNG keeps the
    # rows above unchanged).  With e = SHA-256(M) mod n, (r, s) fixes u1 = e/s and
    # u2 = r/s exactly, so any (u1, u2, Q = dG) relation maps to a signature:
    rx = random.Random(4242)
    for scheme in (2, 3):
        c = EC.CURVES[scheme]
        for t in range(4):
            msg = b"B4-%d-%d" % (scheme, t)
            e = int.from_bytes(hashlib.sha256(msg).digest(), "big") % c.n
            # u1 G + u2 Q = infinity (u1 + d u2 = 0 mod n: r = -e/d) -> REJECT (B.4)
            for d in (1, 2, 3, c.n - 1):
                r = (-e * pow(d, -1, c.n)) % c.n
                add("B4_infinity", scheme, EC.pubkey(scheme, d), EC.der_encode(r, rx.randrange(1, c.n)), msg)
            # u1 = u2 with Q = G (r = e): every Q addition of the device's joint
            # multiplication meets an equal partial sum (its doubling branch;
            # tests/test_native_host.py::test_ecdsa_joint_exceptional_cases)
            add("B4_doubling_q_eq_g", scheme, EC.pubkey(scheme, 1), EC.der_encode(e, rx.randrange(1, c.n)), msg)
            # Q = -G, u1 = u2: partial sums cancel to infinity mid-loop, then grow again
            add("B4_cancel_q_eq_minus_g", scheme, EC.pubkey(scheme, c.n - 1),
                EC.der_encode(e, rx.randrange(1, c.n)), msg)
            # Q = 2G, u1 = 2 u2 (r = e/2)
            add("B4_q_eq_2g_u1_eq_2u2", scheme, EC.pubkey(scheme, 2),
                EC.der_encode(e * pow(2, -1, c.n) % c.n, rx.randrange(1, c.n)), msg)
            # a VALID signature whose two halves are the same point, u1 G == u2 Q:
            # key d = e/r, s = k^-1 (e + r d) = 2e/k -> ACCEPT
            k = rx.randrange(1, c.n)
            r = EC._mul(c, k, c.g)[0] % c.n
            d = e * pow(r, -1, c.n) % c.n
            s2 = 2 * e * pow(k, -1, c.n) % c.n
            add("B4_equal_halves_valid", scheme, EC.pubkey(scheme, d), EC.der_encode(r, s2), msg)
            assert EC.is_valid(scheme, EC.pubkey(scheme, d), EC.der_encode(r, s2), msg) == EC.ACCEPT
    return cases


# -------------------------------------------------------------------- Merkle
def merkle_cases():
    rnd = random.Random(42)
    header = b"corda\x00\x00\x01"  # SerializationScheme.kt:216
    txs = []
    # structure cases of PartialMerkleTreeTest.kt:60-84 (1, 3, 6, 8 leaves) + random shapes
    for k in (1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16, 17):
        salt = rnd.randbytes(32)
        comps = [header + rnd.randbytes(rnd.randint(0, 700)) for _ in range(k - 1)]
        comps.append(header + b"\x01" + salt + bytes(3))  # serialized PrivacySalt (44 B)
        tid = MK.tx_id(comps, salt)
        txs.append({"salt": salt.hex(), "components": [c.hex() for c in comps], "id": tid.hex()})
    roots = {}
    leaves = [rnd.randbytes(32) for _ in range(8)]
    for k in (1, 3, 6, 8):
        roots[str(k)] = {"leaves": [x.hex() for x in leaves[:k]], "root": MK.merkle_root(leaves[:k]).hex()}
    # PartialMerkleTreeTest.kt:77-84: 3 leaves give h(h(l0,l1), h(l2,0))
    l = leaves[:3]
    assert MK.merkle_root(l) == MK.sha256(MK.sha256(l[0] + l[1]) + MK.sha256(l[2] + MK.ZERO_HASH))
    assert MK.merkle_root(leaves[:1]) == leaves[0]
    # cross-check with the C oracle
    for t in txs:
        comps = [bytes.fromhex(c) for c in t["components"]]
        arena = b"".join(comps)
        offs, o = [], 0
        for c in comps:
            offs.append(o); o += len(c)
        out = ctypes.create_string_buffer(32)
        ORACLE.oracle_txid_batch(arena, (ctypes.c_uint64 * len(offs))(*offs),
                                 (ctypes.c_uint32 * len(comps))(*[len(c) for c in comps]),
                                 (ctypes.c_uint32 * 2)(0, len(comps)), bytes.fromhex(t["salt"]), 1, out)
        assert out.raw.hex() == t["id"]
    return {"txs": txs, "roots": roots}


# ------------------------------------------------------- FilteredTransaction
def _ftx_row(cls, comps, nonces, prog, root, result):
    return {"cls": cls, "components": [c.hex() for c in comps], "nonces": [n.hex() for n in nonces],
            "program": [[k, h.hex()] for k, h in prog], "root": root.hex(), "result": result}


def _ftx_expected(comps, nonces, prog, root):
    tree = MK.pmt_from_postorder(prog)
    if not comps:
        return 2
    if tree is None:
        return 3
    return 0 if MK.ftx_verify(comps, nonces, tree, root) else 1


def ftx_cases():
    """FilteredTransaction.verify fixtures: the PartialMerkleTreeTest.kt:159-230 cases
    recast as filtered transactions (components + nonces whose leaf hashes are the
    test's `hashed`), plus adversarial node programs."""
    rnd = random.Random(77)
    header = b"corda\x00\x00\x01"
    salt = rnd.randbytes(32)
    comps = [header + bytes([ord(ch)]) + rnd.randbytes(rnd.randint(20, 300)) for ch in "abcdef"]
    nonces = [MK.compute_nonce(salt, i) for i in range(6)]
    hashed = [MK.filtered_leaf_hash(c, n) for c, n in zip(comps, nonces)]
    mt = MK.get_merkle_tree(hashed)
    rows = []

    def add(cls, idx, tree, root, comp_override=None):
        cs = comp_override if comp_override is not None else [comps[i] for i in idx]
        ns = [nonces[i] for i in idx]
        prog = MK.pmt_postorder(tree) if not isinstance(tree, list) else tree
        rows.append(_ftx_row(cls, cs, ns, prog, root, _ftx_expected(cs, ns, prog, root)))

    t35 = MK.pmt_build(mt, [hashed[3], hashed[5]])
    add("only_left_branch", [3, 5], t35, mt.hash)
    add("order_swapped", [5, 3], t35, mt.hash)
    add("include_zero_leaves", [], MK.pmt_build(mt, []), mt.hash)
    add("include_all", range(6), MK.pmt_build(mt, hashed), mt.hash)
    add("too_many_leaves", [3, 5, 0], t35, mt.hash)
    add("too_little_leaves", [3, 5], MK.pmt_build(mt, [hashed[3], hashed[5], hashed[0]]), mt.hash)
    mt5 = MK.get_merkle_tree(hashed[:5])
    add("duplicate_leaves", [3, 4, 4], MK.pmt_build(mt5, [hashed[3], hashed[4]]), mt5.hash)
    add("different_leaves", [2, 4], t35, mt.hash)
    add("wrong_root", [3, 5], t35, MK.sha256(hashed[3] + hashed[5]))
    add("same_count_other_multiset", [3, 3], t35, mt.hash)
    tampered = bytearray(comps[5]); tampered[9] ^= 1
    add("tampered_component", [3, 5], t35, mt.hash, [comps[3], bytes(tampered)])
    add("single_leaf_tree", [2], MK.PTIncluded(hashed[2]), hashed[2])
    add("malformed_node_only", [3], [(2, MK.ZERO_HASH)], mt.hash)
    add("malformed_two_roots", [3], [(0, hashed[3]), (1, hashed[4])], mt.hash)
    add("malformed_empty", [3], [], mt.hash)
    add("malformed_bad_kind", [3], [(7, hashed[3])], mt.hash)
    add("no_leaves_beats_malformed", [], [(2, MK.ZERO_HASH)], mt.hash)
    # identical leaves (PartialMerkleTreeTest.kt:185-190 "aaa")
    same = [comps[0]] * 3
    hs = [MK.filtered_leaf_hash(c, nonces[0]) for c in same]
    mta = MK.get_merkle_tree(hs)
    ta = MK.pmt_build(mta, hs)
    rows.append(_ftx_row("identical_leaves_all", same, [nonces[0]] * 3, MK.pmt_postorder(ta), mta.hash,
                         _ftx_expected(same, [nonces[0]] * 3, MK.pmt_postorder(ta), mta.hash)))
    rows.append(_ftx_row("identical_leaves_fewer", same[:2], [nonces[0]] * 2, MK.pmt_postorder(ta), mta.hash,
                         _ftx_expected(same[:2], [nonces[0]] * 2, MK.pmt_postorder(ta), mta.hash)))
    # a deep chain (adversarial shape, depth 40): root computed along the chain
    tree, root = MK.PTIncluded(hashed[1]), hashed[1]
    for d in range(40):
        sib = rnd.randbytes(32)
        tree, root = (MK.PTNode(tree, MK.PTLeaf(sib)), MK.sha256(root + sib)) if d % 2 else \
            (MK.PTNode(MK.PTLeaf(sib), tree), MK.sha256(sib + root))
    add("deep_chain_40", [1], tree, root)
    # more included leaves than one lane compares (the library's host multiset path)
    big_c = [header + rnd.randbytes(40) for _ in range(300)]
    big_n = [MK.compute_nonce(salt, i) for i in range(300)]
    big_h = [MK.filtered_leaf_hash(c, n) for c, n in zip(big_c, big_n)]
    mtb = MK.get_merkle_tree(big_h)
    pb = MK.pmt_postorder(MK.pmt_build(mtb, big_h))
    rows.append(_ftx_row("many_leaves_300", big_c, big_n, pb, mtb.hash, _ftx_expected(big_c, big_n, pb, mtb.hash)))
    swap_c = list(big_c); swap_c[7] = big_c[8]
    swap_n = list(big_n); swap_n[7] = big_n[8]
    rows.append(_ftx_row("many_leaves_300_other_multiset", swap_c, swap_n, pb, mtb.hash,
                         _ftx_expected(swap_c, swap_n, pb, mtb.hash)))
    # cross-check with the C oracle
    for r in rows:
        cs = [bytes.fromhex(c) for c in r["components"]]
        arena = b"".join(cs) or b"\0"
        offs, o = [], 0
        for c in cs:
            offs.append(o); o += len(c)
        prog = r["program"]
        out = ctypes.create_string_buffer(1)
        ORACLE.oracle_ftx_verify_batch(arena, (ctypes.c_uint64 * max(1, len(cs)))(*offs),
                                       (ctypes.c_uint32 * max(1, len(cs)))(*[len(c) for c in cs]),
                                       (ctypes.c_uint32 * 2)(0, len(cs)),
                                       b"".join(bytes.fromhex(n) for n in r["nonces"]) or bytes(32),
                                       (ctypes.c_uint32 * 2)(0, len(prog)), bytes([k for k, _ in prog]) or b"\0",
                                       b"".join(bytes.fromhex(h) for _, h in prog) or bytes(32),
                                       bytes.fromhex(r["root"]), 1, out)
        assert out.raw[0] == r["result"], r["cls"]
    return rows


# ------------------------------------------------------- CompositeKey fulfilment
def composite_cases():
    """CompositeKey fulfilment fixtures: the CompositeKeyTests.kt:45-82,126-174,284-305
    cases plus random trees and signer subsets, each as the flat op program of
    cg_composite_eval_batch with its expected out byte (oracle/py/composite.py)."""
    import composite as CK
    rnd = random.Random(99)
    alice, bob, charlie, dave, eve = (bytes([0x30 + i]) * 32 for i in range(5))
    rows = []

    def add(cls, key, signers, verdicts=None):
        idx = {}
        for i, k in enumerate(signers):
            idx.setdefault(k, i)
        prog = CK.program(key, idx)
        vs = verdicts if verdicts is not None else [0] * len(signers)
        exp = int(CK.is_fulfilled_by(key, signers)) | (int(all(v == 0 for v in vs)) << 1)
        rows.append({"cls": cls, "prog": [list(o) for o in prog], "n_sig": len(signers), "verdicts": vs,
                     "out": exp})

    B = CK.Builder
    add("alice_by_alice", alice, [alice])
    add("alice_by_charlie", alice, [charlie])
    a_or_b = B().add_keys(alice, bob).build(1)
    for sg in ([alice], [bob], [alice, bob], [charlie], []):
        add("alice_or_bob", a_or_b, sg)
    a_and_b = B().add_keys(alice, bob).build()
    for sg in ([alice], [bob], [alice, bob], [bob, alice, charlie]):
        add("alice_and_bob", a_and_b, sg)
    ab_or_c = B().add_keys(a_and_b, charlie).build(1)
    for sg in ([alice, bob], [charlie], [alice], [bob, charlie]):
        add("alice_and_bob_or_charlie", ab_or_c, sg)
    node2 = B().add_keys(alice, bob).build(2)
    add("node2_by_alice", node2, [alice])
    two_of_three = B().add_keys(alice, bob, charlie).build(2)
    for sg, vs in (([alice], [0]), ([alice, bob], [0, 0]), ([alice, charlie], [0, 0]),
                   ([alice, bob, charlie], [0, 0, 0]), ([alice, bob], [0, 1]), ([alice, bob, charlie], [0, 0, 2])):
        add("two_of_three_composite_signature", two_of_three, sg, vs)
    weighted = B().add_key(B().add_keys(alice, bob).build(), 3).add_key(charlie, 2).add_key(dave, 1).build(3)
    for sg in ([alice, bob], [charlie], [charlie, dave], [alice, dave], [eve]):
        add("weighted_tree", weighted, sg)
    five = B().add_keys(alice, bob, charlie, dave, eve).build()
    add("all_five", five, [eve, dave, charlie, bob, alice])
    add("all_five_minus_one", five, [eve, dave, charlie, bob])
    # random trees
    keys = [bytes([i]) * 31 + b"k" for i in range(24)]

    def rand_tree(depth):
        n = rnd.randint(2, 4)
        kids = rnd.sample(keys, n)
        b = B()
        for k in kids:
            if depth > 0 and rnd.random() < 0.3:
                b.add_key(rand_tree(depth - 1), rnd.randint(1, 4))
            else:
                b.add_key(k, rnd.randint(1, 4))
        tot = sum(w for _, w in b.children)
        return b.build(rnd.randint(1, tot))
    for t in range(300):
        key = rand_tree(3)
        leaves = sorted(key.leaf_keys)
        sg = rnd.sample(leaves, rnd.randint(0, len(leaves))) + ([keys[-1]] if t % 7 == 0 else [])
        vs = [0 if rnd.random() < 0.9 else 1 for _ in sg]
        add("random_tree", key, sg, vs)
    # programs violating CompositeKey's constraints (IllegalArgumentException)
    bad = [[[0, -1, 1, 0], [1, 1, 1, 1]],                       # arity 1
           [[0, -1, 1, 0], [0, -1, 0, 0], [1, 2, 1, 1]],         # zero weight
           [[0, -1, 2, 0], [0, -1, 2, 0], [1, 2, 1, 5]],         # threshold > total weight
           [[0, -1, 1, 0], [0, -1, 1, 0], [1, 2, 1, 0]],         # threshold 0
           [[0, -1, 2**31 - 1, 0], [0, -1, 2**31 - 1, 0], [1, 2, 1, 1]],  # Int overflow of the total
           [[0, -1, 1, 0], [0, -1, 1, 0]],                       # two roots
           [[1, 2, 1, 1]],                                       # node without children
           []]                                                   # empty
    for i, prog in enumerate(bad):
        rows.append({"cls": f"invalid_{i}", "prog": prog, "n_sig": 0, "verdicts": [], "out": 0x80})
    return rows


def main():
    if "--only-composite" in sys.argv:
        rows = composite_cases()
        with open(os.path.join(HERE, "composite_golden.json"), "w") as f:
            json.dump(rows, f, indent=0)
        print("composite", len(rows))
        return
    if "--only-ftx" in sys.argv:
        fx = ftx_cases()
        with open(os.path.join(HERE, "ftx_golden.json"), "w") as f:
            json.dump(fx, f, indent=0)
        from collections import Counter
        print("ftx", len(fx), Counter(r["result"] for r in fx))
        return
    ed = ed25519_cases()
    with open(os.path.join(HERE, "ed25519_golden.json"), "w") as f:
        json.dump(ed, f, indent=0)
    ec = ecdsa_cases()
    with open(os.path.join(HERE, "ecdsa_golden.json"), "w") as f:
        json.dump(ec, f, indent=0)
    mk = merkle_cases()
    with open(os.path.join(HERE, "merkle_golden.json"), "w") as f:
        json.dump(mk, f, indent=0)
    from collections import Counter
    print("ed25519", len(ed), Counter(c["is_valid"] for c in ed))
    print("ecdsa", len(ec), Counter(c["is_valid"] for c in ec))
    print("merkle", len(mk["txs"]))
    fx = ftx_cases()
    with open(os.path.join(HERE, "ftx_golden.json"), "w") as f:
        json.dump(fx, f, indent=0)
    rows = composite_cases()
    with open(os.path.join(HERE, "composite_golden.json"), "w") as f:
        json.dump(rows, f, indent=0)


if __name__ == "__main__":
    main()
