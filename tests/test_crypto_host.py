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
    b = crypto.pack([2, 3, 4], [b"\0" * 64] * 3, [b"\x30\x06\x02\x01\x01\x02\x01\x01", b"", b"\0" * 64], [b"a"] * 3)
    assert list(b.scheme) == [2, 3, 4]
    assert np.array_equal(b.sig_len, [8, 0, 64])


def test_wrong_length_keys_are_key_invalid_not_truncated():
    """A 31/33-byte Ed25519 key or a 65-byte ECDSA key cannot be a key object: its
    verdict is KEY_INVALID (never verified as a truncated / zero-padded key)."""
    b = crypto.pack([4, 4, 4, 3], [b"\1" * 31, b"\1" * 33, b"\1" * 32, b"\2" * 65], [b"\3" * 64] * 4, [b"m"] * 4)
    assert list(b.key_invalid) == [0, 1, 3]
    assert not b.pk[0].any() and not b.pk[1].any() and not b.pk[3].any()
    assert crypto.key_length_ok(4, b"x" * 32) and not crypto.key_length_ok(2, b"x" * 32)


def test_host_schemes_need_a_host_verifier():
    """RSA / SPHINCS / COMPOSITE (Crypto.kt:176-183) are supported by the reference
    through JCA: the batch routes them to the caller's host verifier instead of
    reporting them UNSUPPORTED, and refuses to guess without one."""
    with pytest.raises(crypto.IllegalArgumentException) as ei:
        crypto._verify_mixed(None, [4, 1], [b"\1" * 32, b"k"], [b"s" * 64, b"s"], [b"m", b"m"], 0, None)
    assert ei.value.index == 1
