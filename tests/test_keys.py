"""SubjectPublicKeyInfo decoding (corda_amd.keys) on fixed points: the curve
generators, compressed and uncompressed, and the standard DER prefixes JCA emits for
P-256 / Ed25519 keys (Crypto.kt:347-355 decodePublicKey)."""
from __future__ import annotations

import pytest

from corda_amd import keys
from corda_amd.crypto import IllegalArgumentException

P256_G = bytes.fromhex(
    "6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296"
    "4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5")
K1_G = bytes.fromhex(
    "79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798"
    "483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8")


@pytest.mark.parametrize("scheme,g", [(3, P256_G), (2, K1_G)])
@pytest.mark.parametrize("compressed", [False, True])
def test_ec_roundtrip(scheme, g, compressed):
    der = keys.encode_ec_spki(scheme, g, compressed)
    assert keys.decode_spki(der) == (scheme, g)


def test_jca_prefixes():
    p256 = bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200") + b"\x04" + P256_G
    assert keys.encode_ec_spki(3, P256_G) == p256
    assert keys.decode_spki(p256) == (3, P256_G)
    a = bytes(range(32))
    ed = bytes.fromhex("302a300506032b6570032100") + a
    assert keys.decode_spki(ed) == (4, a)


def test_rejects():
    good = keys.encode_ec_spki(3, P256_G)
    with pytest.raises(IllegalArgumentException):
        keys.decode_spki(good[:-1])                      # truncated
    with pytest.raises(IllegalArgumentException):
        keys.decode_spki(good + b"\x00")                 # trailing bytes
    bad_prefix = bytearray(good)
    bad_prefix[-65] = 5
    with pytest.raises(IllegalArgumentException):
        keys.decode_spki(bytes(bad_prefix))              # unknown point encoding
    # a compressed x whose x^3 - 3x + b is a non-residue on P-256
    p = 2**256 - 2**224 + 2**192 + 2**96 - 1
    b = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
    x = next(x for x in range(1, 100) if pow((x ** 3 - 3 * x + b) % p, (p - 1) // 2, p) != 1)
    comp = keys.encode_ec_spki(3, x.to_bytes(32, "big") + bytes(32), compressed=True)
    with pytest.raises(IllegalArgumentException):
        keys.decode_spki(comp)
