"""Host logic of the Crypto batch mirror (no GPU): packing into the C-ABI
layout, scheme lookup and the doVerify exception mapping (Crypto.kt:472-483)."""
from __future__ import annotations

import numpy as np
import pytest

from corda_amd import crypto
from corda_amd._lib import ACCEPT, ARG_EMPTY, KEY_INVALID, REJECT, SIG_MALFORMED, UNSUPPORTED


def test_pack_layout():
    b = crypto.pack(crypto.EDDSA_ED25519_SHA512, [b"\1" * 32, b"\2" * 32], [b"\3" * 64, b"\4" * 70],
                    [b"hello", b""])
    assert b.n == 2 and b.pk_stride == 64 and b.sig_stride == 72
    assert list(b.scheme) == [4, 4]
    assert list(b.sig_len) == [64, 70]
    assert list(b.msg_off) == [0, 5] and list(b.msg_len) == [5, 0]
    assert bytes(b.msg[:5]) == b"hello"
    assert bytes(b.pk[1, :32]) == b"\2" * 32 and not b.pk[1, 32:].any()


def test_scheme_lookup_like_find_signature_scheme():
    assert crypto._scheme_id("ECDSA_SECP256R1_SHA256") == 3
    assert crypto._scheme_id(crypto.ECDSA_SECP256K1_SHA256) == 2
    with pytest.raises(crypto.IllegalArgumentException):
        crypto._scheme_id("RSA_SHA256")


@pytest.mark.parametrize("code,exc", [(REJECT, crypto.SignatureException), (SIG_MALFORMED, crypto.SignatureException),
                                      (KEY_INVALID, crypto.InvalidKeyException),
                                      (ARG_EMPTY, crypto.IllegalArgumentException),
                                      (UNSUPPORTED, crypto.IllegalArgumentException)])
def test_exception_mapping(code, exc):
    with pytest.raises(exc) as ei:
        crypto.raise_for_verdict(code, 5)
    assert ei.value.index == 5
    crypto.raise_for_verdict(ACCEPT, 0)  # no exception


def test_mixed_scheme_pack():
    b = crypto.pack([2, 3, 4], [b"\0" * 64] * 2 + [b"\0" * 32], [b"\x30\x06\x02\x01\x01\x02\x01\x01", b"", b"\0" * 64],
                    [b"a"] * 3)
    assert list(b.scheme) == [2, 3, 4]
    assert np.array_equal(b.sig_len, [8, 0, 64])


def test_wrong_length_keys_are_key_invalid_not_truncated():
    """A 31/33-byte Ed25519 key or a 65-byte ECDSA key cannot be a key object: its
    verdict is KEY_INVALID (never verified as a truncated / zero-padded key)."""
    b = crypto.pack([4, 4, 4, 3], [b"\1" * 31, b"\1" * 33, b"\1" * 32, b"\2" * 65], [b"\3" * 64] * 4, [b"m"] * 4)
    assert list(b.key_invalid) == [0, 1, 3]
    # flagged in the scheme id, so the library reports KEY_INVALID on every path
    # (verify, prepared batches and their device bitmaps, shards, transactions)
    assert list(b.scheme) == [4 | 0x80, 4 | 0x80, 4, 3 | 0x80]
    assert not b.pk[0].any() and not b.pk[1].any() and not b.pk[3].any()
    from corda_amd import dist as D
    sh = D.slice_batch(b, 1, 4)
    assert list(sh.scheme) == [4 | 0x80, 4, 3 | 0x80]
    assert crypto.key_length_ok(4, b"x" * 32) and not crypto.key_length_ok(2, b"x" * 32)


def test_host_schemes_need_a_host_verifier():
    """RSA / SPHINCS / COMPOSITE (Crypto.kt:176-183) are supported by the reference
    through JCA: the batch routes them to the caller's host verifier instead of
    reporting them UNSUPPORTED, and refuses to guess without one."""
    with pytest.raises(crypto.IllegalArgumentException) as ei:
        crypto._verify_mixed(None, [4, 1], [b"\1" * 32, b"k"], [b"s" * 64, b"s"], [b"m", b"m"], 0, None)
    assert ei.value.index == 1


def _fake_verifier(monkeypatch, codes):
    """Replace the device batch with fixed verdict codes, to check the loop semantics of
    corda_amd.signatures without a GPU."""
    from corda_amd import signatures
    calls = []

    def fake(ctx, schemes, keys, sigs, data, mode, host_verify):
        calls.append((list(schemes), list(keys), list(sigs), list(data), mode))
        return np.array(codes[:len(sigs)], dtype=np.uint8)
    monkeypatch.setattr(signatures, "_verify_mixed", fake)
    monkeypatch.setattr(crypto, "_verify_mixed", fake)
    return calls


def test_public_key_is_valid_loop_semantics(monkeypatch):
    """PublicKey.isValid (CryptoUtils.kt:63-67): bools for ACCEPT/REJECT, Crypto.isValid's exception
    at the first throwing element, IllegalStateException at the first CompositeKey — whichever the
    loop meets first; elements past a composite key are never verified."""
    from corda_amd import signatures as S
    ed = lambda b: S.PublicKey(crypto.EDDSA_ED25519_SHA512, bytes([b]) * 32)  # noqa: E731
    comp = S.PublicKey(6, b"composite")
    calls = _fake_verifier(monkeypatch, [ACCEPT, REJECT, ACCEPT])
    got = S.public_key_is_valid_batch(None, [ed(1), ed(2), ed(3)], [b"a", b"b", b"c"], [b"s"] * 3)
    assert got.tolist() == [True, False, True] and calls[-1][4] == crypto._lib.MODE_IS_VALID
    with pytest.raises(S.IllegalStateException) as ei:
        S.public_key_is_valid_batch(None, [ed(1), ed(2), comp, ed(3)], [b"a"] * 4, [b"s"] * 4)
    assert ei.value.index == 2 and len(calls[-1][2]) == 2
    _fake_verifier(monkeypatch, [ACCEPT, SIG_MALFORMED])
    with pytest.raises(crypto.SignatureException) as ei:
        S.public_key_is_valid_batch(None, [ed(1), ed(2), comp], [b"a"] * 3, [b"s"] * 3)
    assert ei.value.index == 1
    _fake_verifier(monkeypatch, [KEY_INVALID])
    with pytest.raises(crypto.InvalidKeyException):
        S.with_key_is_valid_batch(None, [S.WithKey(ed(1), b"s")], [b"a"])
    _fake_verifier(monkeypatch, [ACCEPT, ARG_EMPTY])  # isValid has no empty-data rule of its own
    with pytest.raises(crypto.IllegalArgumentException):
        S.public_key_is_valid_batch(None, [ed(1), ed(2)], [b"a", b""], [b"s"] * 2)


def test_transaction_signature_mirrors(monkeypatch):
    """TransactionSignature.verify (TransactionSignature.kt:20) verifies under metaData.publicKey;
    Crypto.doVerify(publicKey, txSig) (Crypto.kt:497-501) under the PASSED key, over
    metaData.bytes(), and a key differing from metaData.publicKey is not an error by itself."""
    from corda_amd import signatures as S
    ka = S.PublicKey(crypto.EDDSA_ED25519_SHA512, b"A" * 32)
    kb = S.PublicKey(crypto.ECDSA_SECP256R1_SHA256, b"B" * 64)
    ts = S.TransactionSignature(b"sig", b"metadata-bytes", ka)
    calls = _fake_verifier(monkeypatch, [ACCEPT])
    assert S.transaction_signatures_verify(None, [ts])
    assert calls[-1][:4] == ([4], [b"A" * 32], [b"sig"], [b"metadata-bytes"])
    assert calls[-1][4] == crypto._lib.MODE_DO_VERIFY
    assert S.do_verify_transaction_signatures(None, [kb], [ts])
    assert calls[-1][:4] == ([3], [b"B" * 64], [b"sig"], [b"metadata-bytes"])
    _fake_verifier(monkeypatch, [ACCEPT, REJECT])
    with pytest.raises(crypto.SignatureException) as ei:
        S.transaction_signatures_verify(None, [ts, ts])
    assert ei.value.index == 1
    with pytest.raises(ValueError):
        S.do_verify_transaction_signatures(None, [ka], [ts, ts])


def test_host_scheme_keys_of_any_length(monkeypatch):
    """RSA / SPHINCS keys are long (X.509 SPKI of a 2048-bit RSA key ~294 B, SPHINCS-256
    ~1 KB): the device never reads their rows, so pack() leaves them empty instead of
    failing to fit them into the 64-byte row, and host_verify gets the full key bytes."""
    rsa, sphincs = b"R" * 294, b"S" * 1056
    b = crypto.pack([1, 5, 4], [rsa, sphincs, b"\1" * 32], [b"s"] * 3, [b"m"] * 3)
    assert b.key_invalid is None and list(b.scheme) == [1, 5, 4] and not b.pk[:2].any()
    monkeypatch.setattr(crypto, "verify_packed", lambda ctx, bb, mode: np.full(bb.n, UNSUPPORTED, np.uint8))
    seen = []

    def host_verify(sid, key, sig, data, mode):
        seen.append((sid, len(key)))
        return ACCEPT
    v = crypto._verify_mixed(None, [1, 5, 4], [rsa, sphincs, b"\1" * 32], [b"s"] * 3, [b"m"] * 3, 0, host_verify)
    assert seen == [(1, 294), (5, 1056)] and v.tolist() == [ACCEPT, ACCEPT, UNSUPPORTED]


def test_tx_pack_flags_wrong_length_keys_per_signature():
    """A wrong-length key makes only its own signature KEY_INVALID (no batch-wide raise),
    so the first failing signature in tx order still decides the exception."""
    from corda_amd import transactions as T
    stx = T.SignedTx(T.WireTx([b"c"], bytes(32)), [(4, b"\1" * 32, b"s" * 64), (4, b"\1" * 31, b"s" * 64)])
    sig_start, scheme, pk, sig, sig_stride, sig_len, n_sig = T._pack_sigs([stx])
    assert n_sig == 2 and list(scheme) == [4, 4 | 0x80] and not pk[1].any()
