"""Host-side key decoding for the batch ABI: X.509 SubjectPublicKeyInfo (the
``PublicKey.encoded`` bytes Corda carries for EC keys, Kryo.kt:388-398 ->
Crypto.decodePublicKey, Crypto.kt:347-355) to the 64-byte big-endian X||Y the
ECDSA kernels take, and the 32-byte Ed25519 ``A`` (Kryo.kt:330-340 carries it raw;
its SPKI form is unwrapped too).

Key construction is not the hot path (a JVM caller holds decoded key objects); this
mirrors what the JNI glue does before packing a batch.  Off-curve points are left to
the kernels, which report them as CG_KEY_INVALID exactly as the JVM would fail to
build the key.  Compressed points (02/03 prefix) are decompressed here, as BC's
ECCurve.decodePoint does; a compressed x with no square root raises.
"""
from __future__ import annotations

from .crypto import IllegalArgumentException

OID_EC_PUBLIC_KEY = bytes.fromhex("2a8648ce3d0201")      # 1.2.840.10045.2.1
OID_SECP256R1 = bytes.fromhex("2a8648ce3d030107")        # 1.2.840.10045.3.1.7
OID_SECP256K1 = bytes.fromhex("2b8104000a")              # 1.3.132.0.10
OID_ED25519 = bytes.fromhex("2b6570")                    # 1.3.101.112

_CURVES = {
    OID_SECP256K1: (2, 2**256 - 2**32 - 977, 0, 7),
    OID_SECP256R1: (3, 2**256 - 2**224 + 2**192 + 2**96 - 1, -3,
                    0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B),
}


def _tlv(buf: bytes, i: int) -> tuple[int, bytes, int]:
    """(tag, value, next index) of one DER element."""
    if i + 2 > len(buf):
        raise IllegalArgumentException("truncated DER")
    tag, ln = buf[i], buf[i + 1]
    i += 2
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or nb > 4 or i + nb > len(buf):
            raise IllegalArgumentException("bad DER length")
        ln = int.from_bytes(buf[i:i + nb], "big")
        i += nb
    if i + ln > len(buf):
        raise IllegalArgumentException("truncated DER")
    return tag, buf[i:i + ln], i + ln


def _sqrt_mod(a: int, p: int) -> int | None:
    # both primes are 3 mod 4
    r = pow(a, (p + 1) // 4, p)
    return r if r * r % p == a % p else None


def decode_spki(der: bytes) -> tuple[int, bytes]:
    """SubjectPublicKeyInfo -> (scheme id, kernel key bytes): (2|3, X||Y 64 B) for EC
    keys, (4, A 32 B) for Ed25519."""
    tag, body, end = _tlv(der, 0)
    if tag != 0x30 or end != len(der):
        raise IllegalArgumentException("not a SubjectPublicKeyInfo")
    tag, alg, i = _tlv(body, 0)
    tag2, bits, j = _tlv(body, i)
    if tag != 0x30 or tag2 != 0x03 or j != len(body) or not bits or bits[0] != 0:
        raise IllegalArgumentException("not a SubjectPublicKeyInfo")
    point = bits[1:]
    t, oid, k = _tlv(alg, 0)
    if t != 0x06:
        raise IllegalArgumentException("bad algorithm identifier")
    if oid == OID_ED25519:
        if len(point) != 32:
            raise IllegalArgumentException("Ed25519 key must be 32 bytes")
        return 4, bytes(point)
    if oid != OID_EC_PUBLIC_KEY:
        raise IllegalArgumentException("unsupported key algorithm")
    t, curve, _ = _tlv(alg, k)
    if t != 0x06 or curve not in _CURVES:
        raise IllegalArgumentException("unsupported curve")
    scheme, p, a, b = _CURVES[curve]
    if len(point) == 65 and point[0] == 4:
        return scheme, bytes(point[1:])
    if len(point) == 33 and point[0] in (2, 3):
        x = int.from_bytes(point[1:], "big")
        if x >= p:
            raise IllegalArgumentException("x out of range")
        y = _sqrt_mod((x * x * x + a * x + b) % p, p)
        if y is None:
            raise IllegalArgumentException("Invalid point compression")
        if (y & 1) != (point[0] & 1):
            y = p - y
        return scheme, x.to_bytes(32, "big") + y.to_bytes(32, "big")
    raise IllegalArgumentException("Invalid point encoding")


def encode_ec_spki(scheme: int, xy: bytes, compressed: bool = False) -> bytes:
    """Inverse of decode_spki for EC keys (test / tooling helper)."""
    curve = OID_SECP256K1 if scheme == 2 else OID_SECP256R1
    if compressed:
        point = bytes([2 | (xy[63] & 1)]) + xy[:32]
    else:
        point = b"\x04" + xy
    alg = b"\x06" + bytes([len(OID_EC_PUBLIC_KEY)]) + OID_EC_PUBLIC_KEY + b"\x06" + bytes([len(curve)]) + curve
    alg = b"\x30" + bytes([len(alg)]) + alg
    bits = b"\x03" + bytes([len(point) + 1]) + b"\x00" + point
    body = alg + bits
    return b"\x30" + bytes([len(body)]) + body
