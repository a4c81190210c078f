"""TEST INFRASTRUCTURE ONLY — pure-Python twin of the Ed25519 oracle.

Never imported by the product path (corda_amd/); only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() may use anything under oracle/.

Restates the verification semantics of ``net.i2p.crypto:eddsa:0.2.0`` as driven by
Corda's ``Crypto.isValid`` / ``Crypto.doVerify``
(/root/reference/core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:472-483,534-541)
for ``EDDSA_ED25519_SHA512`` (Crypto.kt:119-132).  The jar is not vendored in the
reference and no JVM exists here, so the algorithm is restated from SURVEY.md
Appendix A (rules A.1–A.9):

* A.2 key decode: y = low 255 bits (NOT reduced / range-checked), x from
  ``pow22523``; no root -> invalid key; x=0 with the sign bit set is accepted.
* A.3 no on-curve / order check at verify time.
* A.4 ``Abyte`` hashed is the canonical re-encoding of the decoded point.
* A.5 h = SHA-512(R || Abyte || M) mod L.
* A.6/A.7 S is not range-checked; it goes through ``slide()`` whose top carry is
  dropped, so the effective scalar is S or S - 2^256.
* A.8/A.9 R' = [S_eff]B + [h](-A) (exact group law), accepted iff enc(R') == R bytes.

Pure Python ints: a few ms per verify; meant for fixtures and small parity runs.
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# Verdict codes of the C ABI (include/cordagpu.h).
ACCEPT, REJECT, SIG_MALFORMED, KEY_INVALID, ARG_EMPTY = 0, 1, 2, 3, 4


class KeyInvalid(Exception):
    """The 32-byte key does not decode (i2p GroupElement ctor throws)."""


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


# ---------------------------------------------------------------- point ops
# Extended twisted-Edwards coordinates (X:Y:Z:T), a = -1.  The unified
# addition/doubling used here is complete on this curve (d non-square), so
# results are exact group elements for every decoded key, torsion included.

def _add(p1, p2):
    x1, y1, z1, t1 = p1
    x2, y2, z2, t2 = p2
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = 2 * D * t1 * t2 % P
    d = 2 * z1 * z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _neg(p):
    x, y, z, t = p
    return ((-x) % P, y, z, (-t) % P)


IDENTITY = (0, 1, 1, 0)
_BY = 4 * _inv(5) % P


def _recover_x(y: int, sign: int) -> int:
    xx = (y * y - 1) * _inv(D * y * y + 1) % P
    x = pow(xx, (P + 3) // 8, P)
    if (x * x - xx) % P != 0:
        x = x * SQRT_M1 % P
    if x & 1 != sign:
        x = P - x
    return x


_BX = _recover_x(_BY, 0)
BASE = (_BX, _BY, 1, _BX * _BY % P)


def scalarmult(pt, k: int):
    """[k]pt for k >= 0 by plain double-and-add (exact)."""
    q = IDENTITY
    for bit in bin(k)[2:] if k > 0 else "":
        q = _add(q, q)
        if bit == "1":
            q = _add(q, pt)
    return q


def encode_point(pt) -> bytes:
    x, y, z, _ = pt
    zi = _inv(z)
    x, y = x * zi % P, y * zi % P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def point_equal(p1, p2) -> bool:
    return (p1[0] * p2[2] - p2[0] * p1[2]) % P == 0 and (p1[1] * p2[2] - p2[1] * p1[2]) % P == 0


# ------------------------------------------------------------- i2p decode
def decode_point_i2p(b: bytes):
    """i2p ``GroupElement(curve, bytes)``: returns the affine point
    as extended coordinates.  Raises KeyInvalid when neither root works."""
    if len(b) != 32:
        raise KeyInvalid("public-key length is wrong")
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)  # top bit masked, not reduced
    sign = b[31] >> 7
    yy = y * y % P
    u = (yy - 1) % P
    v = (D * yy + 1) % P
    v3 = v * v % P * v % P
    x = v3 * u % P * pow(v3 * v3 % P * v % P * u % P, (P - 5) // 8, P) % P
    vxx = x * x % P * v % P
    if (vxx - u) % P != 0:
        if (vxx + u) % P != 0:
            raise KeyInvalid("not a valid GroupElement")
        x = x * SQRT_M1 % P
    if (x & 1) != sign:  # x = 0 with sign set stays 0 (no canonical check)
        x = (-x) % P
    y %= P
    return (x, y, 1, x * y % P)


def abyte(pk: bytes) -> bytes:
    """``EdDSAPublicKey.getAbyte()`` = canonical re-encoding of the decoded A (A.4)."""
    return encode_point(decode_point_i2p(pk))


# ------------------------------------------------------------------- slide
def slide(s: bytes) -> list[int]:
    """ref10/i2p ``slide()``: signed sliding-window digits in [-15, 15]; a carry
    rippling past bit 255 is silently dropped (A.7)."""
    r = [(s[i >> 3] >> (i & 7)) & 1 for i in range(256)]
    for i in range(256):
        if not r[i]:
            continue
        b = 1
        while b <= 6 and i + b < 256:
            if r[i + b]:
                if r[i] + (r[i + b] << b) <= 15:
                    r[i] += r[i + b] << b
                    r[i + b] = 0
                elif r[i] - (r[i + b] << b) >= -15:
                    r[i] -= r[i + b] << b
                    for k in range(i + b, 256):
                        if not r[k]:
                            r[k] = 1
                            break
                        r[k] = 0
                else:
                    break
            b += 1
    return r


def slide_value(s: bytes) -> int:
    """Integer the slide digits represent: S, or S - 2^256 when the carry fell off."""
    return sum(d << i for i, d in enumerate(slide(s)))


def sc_reduce(h64: bytes) -> int:
    return int.from_bytes(h64, "little") % L


# ------------------------------------------------------------------ verify
def is_valid(pk: bytes, sig: bytes, msg: bytes) -> int:
    """Verdict of ``Crypto.isValid(EDDSA_ED25519_SHA512, pk, sig, msg)``.

    Returns ACCEPT / REJECT, SIG_MALFORMED (EdDSAEngine throws SignatureException
    on a length != 64, A.1) or KEY_INVALID (the key object cannot be built)."""
    try:
        a = decode_point_i2p(pk)
    except KeyInvalid:
        return KEY_INVALID
    if len(sig) != 64:
        return SIG_MALFORMED
    ab = encode_point(a)
    h = sc_reduce(hashlib.sha512(sig[:32] + ab + msg).digest())
    s_eff = slide_value(sig[32:])
    sb = scalarmult(BASE, s_eff % L)  # B has order L: only S_eff mod L matters
    ha = scalarmult(_neg(a), h)       # h < L, exact integer multiple (torsion kept)
    r = _add(sb, ha)
    return ACCEPT if encode_point(r) == sig[:32] else REJECT


def do_verify(pk: bytes, sig: bytes, msg: bytes) -> int:
    """Verdict of ``Crypto.doVerify`` (Crypto.kt:472-483): empty sig / data throw
    IllegalArgumentException before the engine runs; ``false`` becomes
    SignatureException (REJECT here).  The key object exists before the call,
    so a key that cannot be decoded is reported first."""
    try:
        decode_point_i2p(pk)
    except KeyInvalid:
        return KEY_INVALID
    if len(sig) == 0 or len(msg) == 0:
        return ARG_EMPTY
    return is_valid(pk, sig, msg)


# ----------------------------------------------------------------- signing
def seed_to_keypair(seed: bytes):
    """RFC 8032 key expansion (= i2p ``EdDSAPrivateKeySpec(seed, spec)``)."""
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    pk = encode_point(scalarmult(BASE, a))
    return a, h[32:], pk


def sign(seed: bytes, msg: bytes) -> tuple[bytes, bytes]:
    """RFC 8032 deterministic Ed25519 signature; returns (pk, sig)."""
    a, prefix, pk = seed_to_keypair(seed)
    r = sc_reduce(hashlib.sha512(prefix + msg).digest())
    rb = encode_point(scalarmult(BASE, r))
    k = sc_reduce(hashlib.sha512(rb + pk + msg).digest())
    s = (r + k * a) % L
    return pk, rb + s.to_bytes(32, "little")


def entropy_seed(k: int) -> bytes:
    """Seed of Corda's ``entropyToKeyPair(BigInteger.valueOf(k))``
    (Crypto.kt:733-739): Java ``BigInteger.toByteArray()`` (big-endian, minimal
    two's complement) then ``copyOf(32)`` (zero-padded on the right)."""
    n = (k.bit_length() + 8) // 8 if k >= 0 else (k.bit_length() + 8) // 8
    raw = k.to_bytes(max(n, 1), "big", signed=True)
    return (raw + bytes(32))[:32]
