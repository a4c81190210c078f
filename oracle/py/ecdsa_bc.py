"""TEST INFRASTRUCTURE ONLY — pure-Python twin of the ECDSA oracle.

Restates BouncyCastle 1.57 ``SHA256withECDSA`` verification as driven by Corda's
``Crypto.isValid`` (/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541)
for ``ECDSA_SECP256K1_SHA256`` (scheme id 2, Crypto.kt:91-102) and
``ECDSA_SECP256R1_SHA256`` (scheme id 3, Crypto.kt:105-116).  bcprov-jdk15on:1.57
(/root/reference/constants.properties:4) is not vendored, so the semantics are
restated from SURVEY.md Appendix B:

* B.1 strict DER: exactly ``30 L 02 Lr r 02 Ls s`` with minimal definite lengths,
  minimal non-empty two's-complement INTEGERs and no trailing bytes; anything else
  -> SignatureException (SIG_MALFORMED).
* B.2 r, s outside [1, n-1] (negative included) -> false.
* B.3 e = SHA-256(M) as a 256-bit integer (no truncation, not pre-reduced).
* B.4 P = (e/s)G + (r/s)Q; infinity -> false.
* B.5 accept iff x(P) mod n == r.
* B.6 Q must be a valid affine point (x, y < p, on the curve) else the key cannot
  be built (KEY_INVALID).  High-S is accepted.
"""
from __future__ import annotations

import hashlib
import hmac

ACCEPT, REJECT, SIG_MALFORMED, KEY_INVALID, ARG_EMPTY = 0, 1, 2, 3, 4

SCHEME_K1, SCHEME_R1, SCHEME_ED25519 = 2, 3, 4


class Curve:
    def __init__(self, name, p, a, b, gx, gy, n):
        self.name, self.p, self.a, self.b, self.n = name, p, a, b, n
        self.g = (gx, gy)


P256 = Curve(
    "secp256r1",
    0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF,
    0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFC,
    0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
    0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
    0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5,
    0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
)
SECP256K1 = Curve(
    "secp256k1",
    0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F,
    0,
    7,
    0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
    0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8,
    0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141,
)
CURVES = {SCHEME_K1: SECP256K1, SCHEME_R1: P256}


# ---------------------------------------------------------------- group law
def on_curve(c: Curve, q) -> bool:
    x, y = q
    return 0 <= x < c.p and 0 <= y < c.p and (y * y - x * x * x - c.a * x - c.b) % c.p == 0


def _add(c: Curve, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % c.p == 0:
            return None
        lam = (3 * x1 * x1 + c.a) * pow(2 * y1, -1, c.p) % c.p
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, c.p) % c.p
    x3 = (lam * lam - x1 - x2) % c.p
    return (x3, (lam * (x1 - x3) - y1) % c.p)


def _mul(c: Curve, k: int, pt):
    r = None
    for bit in bin(k)[2:] if k > 0 else "":
        r = _add(c, r, r)
        if bit == "1":
            r = _add(c, r, pt)
    return r


# ---------------------------------------------------------------------- DER
def der_decode(sig: bytes):
    """BC 1.57 ``StdDSAEncoder.decode`` as a strict grammar.  Returns the signed
    integers (r, s) or None when BC would throw (-> SIG_MALFORMED)."""

    def read_len(buf, i):
        if i >= len(buf):
            return None
        b0 = buf[i]
        if b0 < 0x80:
            return b0, i + 1
        nb = b0 & 0x7F
        if nb == 0 or nb > 4 or i + 1 + nb > len(buf):  # indefinite / absurd
            return None
        v = int.from_bytes(buf[i + 1:i + 1 + nb], "big")
        if v < 0x80 or buf[i + 1] == 0:  # non-minimal long form
            return None
        return v, i + 1 + nb

    def read_int(buf, i, end):
        if i >= end or buf[i] != 0x02:
            return None
        t = read_len(buf, i + 1)
        if t is None:
            return None
        ln, j = t
        if ln == 0 or j + ln > end:
            return None
        body = buf[j:j + ln]
        if ln > 1 and ((body[0] == 0x00 and body[1] < 0x80) or (body[0] == 0xFF and body[1] >= 0x80)):
            return None
        return int.from_bytes(body, "big", signed=True), j + ln

    if len(sig) < 2 or sig[0] != 0x30:
        return None
    t = read_len(sig, 1)
    if t is None:
        return None
    ln, i = t
    if i + ln != len(sig):  # trailing bytes or truncated
        return None
    t = read_int(sig, i, len(sig))
    if t is None:
        return None
    r, i = t
    t = read_int(sig, i, len(sig))
    if t is None:
        return None
    s, i = t
    if i != len(sig):  # a third element
        return None
    return r, s


def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    raw = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(raw)]) + raw


def der_int(v: int) -> bytes:
    body = v.to_bytes((v.bit_length() + 8) // 8 if v >= 0 else ((v + 1).bit_length() + 8) // 8, "big", signed=True)
    return b"\x02" + _der_len(len(body)) + body


def der_encode(r: int, s: int) -> bytes:
    body = der_int(r) + der_int(s)
    return b"\x30" + _der_len(len(body)) + body


# -------------------------------------------------------------------- verify
def is_valid(scheme: int, q, sig: bytes, msg: bytes) -> int:
    """Verdict of ``Crypto.isValid`` for an ECDSA scheme; q = affine (x, y)."""
    c = CURVES[scheme]
    if not on_curve(c, q):
        return KEY_INVALID
    rs = der_decode(sig)
    if rs is None:
        return SIG_MALFORMED
    r, s = rs
    n = c.n
    if not (1 <= r < n and 1 <= s < n):
        return REJECT
    e = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    w = pow(s, -1, n)
    u1, u2 = e * w % n, r * w % n
    pt = _add(c, _mul(c, u1, c.g), _mul(c, u2, q))
    if pt is None:
        return REJECT
    return ACCEPT if pt[0] % n == r else REJECT


def do_verify(scheme: int, q, sig: bytes, msg: bytes) -> int:
    """``Crypto.doVerify`` wrapper order (Crypto.kt:472-483)."""
    if not on_curve(CURVES[scheme], q):
        return KEY_INVALID
    if len(sig) == 0 or len(msg) == 0:
        return ARG_EMPTY
    return is_valid(scheme, q, sig, msg)


# ------------------------------------------------------------------- signing
def pubkey(scheme: int, d: int):
    c = CURVES[scheme]
    return _mul(c, d, c.g)


def rfc6979_k(n: int, d: int, h1: bytes) -> int:
    """RFC 6979 §3.2 deterministic nonce for qlen = hlen = 256 (HMAC-SHA256)."""
    x = d.to_bytes(32, "big")
    h = (int.from_bytes(h1, "big") % n).to_bytes(32, "big")
    v, k = b"\x01" * 32, b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + x + h, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + x + h, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    while True:
        v = hmac.new(k, v, hashlib.sha256).digest()
        t = int.from_bytes(v, "big")
        if 1 <= t < n:
            return t
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()


def sign_rs(scheme: int, d: int, msg: bytes) -> tuple[int, int]:
    c = CURVES[scheme]
    h1 = hashlib.sha256(msg).digest()
    e = int.from_bytes(h1, "big")
    k = rfc6979_k(c.n, d, h1)
    r = _mul(c, k, c.g)[0] % c.n
    s = pow(k, -1, c.n) * (e + r * d) % c.n
    return r, s


def sign(scheme: int, d: int, msg: bytes) -> bytes:
    return der_encode(*sign_rs(scheme, d, msg))


def decode_spki_point(c: Curve, enc: bytes):
    """SEC1 point decoding of the key bytes inside an X.509 SPKI (host side of the
    boundary): 04||X||Y or 02/03||X.  Returns (x, y) or None."""
    if len(enc) == 65 and enc[0] == 4:
        return int.from_bytes(enc[1:33], "big"), int.from_bytes(enc[33:], "big")
    if len(enc) == 33 and enc[0] in (2, 3):
        x = int.from_bytes(enc[1:], "big")
        if x >= c.p:
            return None
        rhs = (x * x * x + c.a * x + c.b) % c.p
        y = pow(rhs, (c.p + 1) // 4, c.p)  # both primes are 3 mod 4
        if y * y % c.p != rhs:
            return None
        if (y & 1) != (enc[0] & 1):
            y = c.p - y
        return x, y
    return None
