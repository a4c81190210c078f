"""Batch signature verification surface mirroring Corda's ``Crypto`` object.

Reference (Kerwong/corda @ 0.14):
  * ``Crypto.isValid(scheme, publicKey, signatureData, clearData)``
    core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:534-541
  * ``Crypto.doVerify(scheme, publicKey, signatureData, clearData)``
    Crypto.kt:472-483 (empty sig / data -> IllegalArgumentException; ``false`` ->
    SignatureException("Signature Verification failed!"))
  * schemes ``ECDSA_SECP256K1_SHA256`` (2), ``ECDSA_SECP256R1_SHA256`` (3),
    ``EDDSA_ED25519_SHA512`` (4) — Crypto.kt:91-132

``is_valid_batch`` returns one verdict code per element (what a loop of
``isValid`` would have returned / thrown); ``do_verify_batch`` raises exactly the
exception a ``for`` loop over ``doVerify`` would raise first (lowest failing
index), so callers such as ``checkSignaturesAreValid`` keep their semantics.
The work runs in libcordagpu's HIP kernels; this module only marshals buffers.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import numpy as np

from . import _lib
from ._lib import ACCEPT, ARG_EMPTY, KEY_INVALID, MODE_DO_VERIFY, MODE_IS_VALID, REJECT, SIG_MALFORMED, UNSUPPORTED


@dataclass(frozen=True)
class SignatureScheme:
    """Subset of ``net.corda.core.crypto.SignatureScheme`` (SignatureScheme.kt:22-32)."""

    scheme_number_id: int
    scheme_code_name: str
    signature_name: str


ECDSA_SECP256K1_SHA256 = SignatureScheme(2, "ECDSA_SECP256K1_SHA256", "SHA256withECDSA")
ECDSA_SECP256R1_SHA256 = SignatureScheme(3, "ECDSA_SECP256R1_SHA256", "SHA256withECDSA")
EDDSA_ED25519_SHA512 = SignatureScheme(4, "EDDSA_ED25519_SHA512", "NONEwithEdDSA")
SUPPORTED_SCHEMES = {s.scheme_code_name: s for s in (ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256,
                                                      EDDSA_ED25519_SHA512)}


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException raised by the reference (e.g. Crypto.kt:475-476)."""

    def __init__(self, msg: str, index: int | None = None):
        super().__init__(msg)
        self.index = index


class SignatureException(Exception):
    """java.security.SignatureException (Crypto.kt:481, or a malformed signature in the engine)."""

    def __init__(self, msg: str, index: int | None = None):
        super().__init__(msg)
        self.index = index


class InvalidKeyException(Exception):
    """java.security.InvalidKeyException: the public key cannot be used."""

    def __init__(self, msg: str, index: int | None = None):
        super().__init__(msg)
        self.index = index


def _scheme_id(s) -> int:
    if isinstance(s, SignatureScheme):
        return s.scheme_number_id
    if isinstance(s, str):
        if s not in SUPPORTED_SCHEMES:
            raise IllegalArgumentException(f"Unsupported key/algorithm for schemeCodeName: {s}")
        return SUPPORTED_SCHEMES[s].scheme_number_id
    return int(s)


KEY_BYTES = {ECDSA_SECP256K1_SHA256.scheme_number_id: 64, ECDSA_SECP256R1_SHA256.scheme_number_id: 64,
             EDDSA_ED25519_SHA512.scheme_number_id: 32}


def key_length_ok(scheme_id: int, key) -> bool:
    """The key bytes must be the scheme's wire form: 32-byte A for Ed25519 (i2p's
    EdDSAPublicKeySpec refuses any other length, so the key object cannot exist),
    64-byte X||Y for ECDSA (see corda_amd.keys for X.509 decoding).  Keys are never
    truncated or zero-padded into that form."""
    want = KEY_BYTES.get(scheme_id)
    return want is None or len(bytes(key)) == want


# OR-ed into the scheme id of an element whose key bytes are not the scheme's wire form
# (include/cordagpu.h CG_SCHEME_FLAG_KEY_INVALID): the key object cannot be constructed,
# so the library reports KEY_INVALID for it on every path (verify, prepared batches and
# their device bitmaps, shards, transactions) and never reads its rows.
SCHEME_FLAG_KEY_INVALID = 0x80


def pack_key_row(pk: np.ndarray, scheme: np.ndarray, i: int, key) -> bool:
    """Writes element i's key row (device schemes only — the rows of host-verified schemes
    such as RSA are never read by the device and may be any length).  A key of the wrong
    length flags the element KEY_INVALID and leaves its row zero.  Returns False for it."""
    sid = int(scheme[i])
    if sid not in KEY_BYTES:
        return True
    kb = bytes(key)
    if not key_length_ok(sid, kb):
        scheme[i] = sid | SCHEME_FLAG_KEY_INVALID
        return False
    pk[i, :len(kb)] = np.frombuffer(kb, dtype=np.uint8)
    return True


@dataclass
class PackedBatch:
    """Element-major host buffers in the C ABI's layout."""

    n: int
    scheme: np.ndarray
    pk: np.ndarray
    pk_stride: int
    sig: np.ndarray
    sig_stride: int
    sig_len: np.ndarray
    msg: np.ndarray
    msg_off: np.ndarray
    msg_len: np.ndarray
    # elements whose key bytes are not the scheme's wire form (flagged in `scheme` with
    # SCHEME_FLAG_KEY_INVALID: the library gives them KEY_INVALID); informational
    key_invalid: np.ndarray | None = None


def pack(schemes, public_keys: Sequence[bytes], signatures: Sequence[bytes], clear_data: Sequence[bytes]) -> PackedBatch:
    """Packs per-element byte strings.  ``public_keys``: Ed25519 32-byte A, ECDSA
    64-byte X||Y (see corda_amd.keys for X.509 decoding).  ``schemes`` may be a
    single scheme or one per element."""
    n = len(signatures)
    if not (len(public_keys) == n == len(clear_data)):
        raise IllegalArgumentException("public_keys, signatures and clear_data differ in length")
    if isinstance(schemes, (SignatureScheme, str, int)):
        scheme = np.full(n, _scheme_id(schemes), dtype=np.uint8)
    else:
        scheme = np.array([_scheme_id(s) for s in schemes], dtype=np.uint8)
    pk_stride = 64
    pk = np.zeros((max(n, 1), pk_stride), dtype=np.uint8)
    bad_keys = [i for i, k in enumerate(public_keys) if not pack_key_row(pk, scheme, i, k)]
    maxlen = max([len(s) for s in signatures] + [64])
    sig_stride = (maxlen + 3) // 4 * 4
    sig = np.zeros((max(n, 1), sig_stride), dtype=np.uint8)
    sig_len = np.zeros(max(n, 1), dtype=np.uint32)
    for i, s in enumerate(signatures):
        sb = bytes(s)
        sig[i, :len(sb)] = np.frombuffer(sb, dtype=np.uint8)
        sig_len[i] = len(sb)
    msg_len = np.array([len(m) for m in clear_data] + [0] * (n == 0), dtype=np.uint32)
    msg_off = np.zeros(max(n, 1), dtype=np.uint64)
    if n:
        msg_off[1:n] = np.cumsum(msg_len[:n - 1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(bytes(m) for m in clear_data) or b"\0", dtype=np.uint8).copy()
    return PackedBatch(n, scheme, pk, pk_stride, sig, sig_stride, sig_len, arena, msg_off, msg_len,
                       np.array(bad_keys, dtype=np.int64) if bad_keys else None)


def verify_packed(ctx: _lib.Context, b: PackedBatch, mode: int, bitmap: bool = False):
    verdict = np.empty(max(b.n, 1), dtype=np.uint8)
    bm = np.zeros(max((b.n + 31) // 32, 1), dtype=np.uint32) if bitmap else None
    ctx.check(ctx.lib.cg_verify_batch(ctx.h, b.n, mode, _lib.ptr(b.scheme), _lib.ptr(b.pk), b.pk_stride,
                                      _lib.ptr(b.sig), b.sig_stride, _lib.ptr(b.sig_len), _lib.ptr(b.msg),
                                      len(b.msg), _lib.ptr(b.msg_off), _lib.ptr(b.msg_len), _lib.ptr(verdict),
                                      _lib.ptr(bm)))
    return (verdict[:b.n], bm) if bitmap else verdict[:b.n]


# Schemes Crypto supports (Crypto.kt:176-183) that the device does not run: RSA_SHA256 (1),
# SPHINCS-256_SHA512 (5) and COMPOSITE (6) are verified by the host's own JCA path.
HOST_SCHEMES = {1: "RSA_SHA256", 5: "SPHINCS-256_SHA512", 6: "COMPOSITE"}


def _verify_mixed(ctx, schemes, public_keys, signatures, clear_data, mode, host_verify):
    """Device batch for schemes 2/3/4; elements of HOST_SCHEMES go to
    ``host_verify(scheme_id, key, signature, data, mode) -> verdict code`` (on the JVM:
    Crypto.isValid / doVerify under try/catch) and are merged back in index order, so
    first-failure-wins still holds.  Without a host_verifier such elements raise
    IllegalArgumentException — they are not silently reported UNSUPPORTED."""
    b = pack(schemes, public_keys, signatures, clear_data)
    host = np.flatnonzero(np.isin(b.scheme[:b.n], list(HOST_SCHEMES)))
    if host.size and host_verify is None:
        i = int(host[0])
        raise IllegalArgumentException(f"scheme {HOST_SCHEMES[int(b.scheme[i])]} is verified on the host JCA path: "
                                       "pass host_verify", i)
    v = verify_packed(ctx, b, mode)
    for i in host:
        i = int(i)
        v[i] = host_verify(int(b.scheme[i]), bytes(public_keys[i]), bytes(signatures[i]), bytes(clear_data[i]), mode)
    return v


def is_valid_batch(ctx: _lib.Context, schemes, public_keys, signatures, clear_data, host_verify=None) -> np.ndarray:
    """Per-element verdict codes of ``Crypto.isValid`` (ACCEPT=0 means ``true``,
    REJECT=1 ``false``; 2/3/5 mean isValid would have thrown)."""
    return _verify_mixed(ctx, schemes, public_keys, signatures, clear_data, MODE_IS_VALID, host_verify)


def raise_for_verdict(code: int, index: int):
    """The exception ``Crypto.doVerify`` throws for a non-ACCEPT verdict."""
    if code == REJECT:
        raise SignatureException("Signature Verification failed!", index)
    if code == SIG_MALFORMED:
        raise SignatureException("signature length is wrong / error decoding signature bytes.", index)
    if code == KEY_INVALID:
        raise InvalidKeyException("public key cannot be decoded", index)
    if code == ARG_EMPTY:
        raise IllegalArgumentException("Signature data is empty! / Clear data is empty, nothing to verify!", index)
    if code == UNSUPPORTED:
        raise IllegalArgumentException("Unsupported key/algorithm", index)


def do_verify_batch(ctx: _lib.Context, schemes, public_keys, signatures, clear_data, host_verify=None) -> bool:
    """``for i in range(n): Crypto.doVerify(...)``: returns True or raises the
    exception of the lowest failing index."""
    v = _verify_mixed(ctx, schemes, public_keys, signatures, clear_data, MODE_DO_VERIFY, host_verify)
    bad = np.flatnonzero(v != ACCEPT)
    if bad.size:
        i = int(bad[0])
        raise_for_verdict(int(v[i]), i)
    return True


class PreparedBatch:
    """A batch staged once in HBM (``cg_batch_create``) and verified on demand."""

    def __init__(self, ctx: _lib.Context, b: PackedBatch):
        self.ctx, self.n = ctx, b.n
        h = _lib.c_void_p()
        ctx.check(ctx.lib.cg_batch_create(ctx.h, b.n, _lib.ptr(b.scheme), _lib.ptr(b.pk), b.pk_stride,
                                          _lib.ptr(b.sig), b.sig_stride, _lib.ptr(b.sig_len), _lib.ptr(b.msg),
                                          len(b.msg), _lib.ptr(b.msg_off), _lib.ptr(b.msg_len),
                                          _lib.ctypes.byref(h)))
        self.h = h

    def verify(self, mode: int = MODE_IS_VALID, want_verdicts: bool = True, device_bitmap_ptr: int | None = None):
        verdict = np.empty(max(self.n, 1), dtype=np.uint8) if want_verdicts else None
        self.ctx.check(self.ctx.lib.cg_batch_verify(self.ctx.h, self.h, mode, _lib.ptr(verdict), None,
                                                    device_bitmap_ptr))
        return verdict[:self.n] if want_verdicts else None

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.cg_batch_destroy(self.ctx.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
