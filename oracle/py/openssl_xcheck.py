"""TEST INFRASTRUCTURE ONLY — OpenSSL 3 (libcrypto.so.3) as an independent
cross-check of the oracle on the semantic overlap with i2p / BouncyCastle:
valid signatures and plain corruptions.  OpenSSL is NOT the reference: it rejects
non-canonical S / points that i2p accepts, and its DER handling differs in corner
cases, so it is only consulted where both must agree.
"""
from __future__ import annotations

import ctypes
import ctypes.util

_c = None
EVP_PKEY_ED25519 = 1087
NID_secp256k1 = 714
NID_X9_62_prime256v1 = 415


def lib():
    global _c
    if _c is None:
        path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        c = ctypes.CDLL(path)
        c.EVP_PKEY_new_raw_public_key.restype = ctypes.c_void_p
        c.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        c.EVP_PKEY_new_raw_private_key.restype = ctypes.c_void_p
        c.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        c.EVP_MD_CTX_new.restype = ctypes.c_void_p
        c.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
        c.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
        c.EVP_DigestVerifyInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]
        c.EVP_DigestVerify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.c_size_t]
        c.EVP_DigestSignInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]
        c.EVP_DigestSign.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_char_p, ctypes.c_size_t]
        c.EC_KEY_new_by_curve_name.restype = ctypes.c_void_p
        c.EC_KEY_get0_group.restype = ctypes.c_void_p
        c.EC_KEY_get0_group.argtypes = [ctypes.c_void_p]
        c.EC_POINT_new.restype = ctypes.c_void_p
        c.EC_POINT_new.argtypes = [ctypes.c_void_p]
        c.EC_POINT_oct2point.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.c_void_p]
        c.EC_KEY_set_public_key.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        c.EC_POINT_free.argtypes = [ctypes.c_void_p]
        c.EC_KEY_free.argtypes = [ctypes.c_void_p]
        c.ECDSA_verify.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                   ctypes.c_void_p]
        _c = c
    return _c


def ed25519_verify(pk: bytes, sig: bytes, msg: bytes) -> bool:
    c = lib()
    key = c.EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, None, pk, 32)
    if not key:
        return False
    ctx = c.EVP_MD_CTX_new()
    try:
        if c.EVP_DigestVerifyInit(ctx, None, None, None, key) != 1:
            return False
        return c.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg)) == 1
    finally:
        c.EVP_MD_CTX_free(ctx)
        c.EVP_PKEY_free(key)


def ed25519_sign(seed: bytes, msg: bytes) -> bytes:
    c = lib()
    key = c.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    ctx = c.EVP_MD_CTX_new()
    try:
        assert c.EVP_DigestSignInit(ctx, None, None, None, key) == 1
        out = ctypes.create_string_buffer(64)
        ln = ctypes.c_size_t(64)
        assert c.EVP_DigestSign(ctx, out, ctypes.byref(ln), msg, len(msg)) == 1
        return out.raw[:ln.value]
    finally:
        c.EVP_MD_CTX_free(ctx)
        c.EVP_PKEY_free(key)


def ecdsa_verify(scheme: int, q_xy: bytes, sig_der: bytes, digest: bytes) -> bool:
    c = lib()
    nid = NID_secp256k1 if scheme == 2 else NID_X9_62_prime256v1
    key = c.EC_KEY_new_by_curve_name(nid)
    grp = c.EC_KEY_get0_group(key)
    pt = c.EC_POINT_new(grp)
    try:
        if c.EC_POINT_oct2point(grp, pt, b"\x04" + q_xy, 65, None) != 1:
            return False
        if c.EC_KEY_set_public_key(key, pt) != 1:
            return False
        return c.ECDSA_verify(0, digest, len(digest), sig_der, len(sig_der), key) == 1
    finally:
        c.EC_POINT_free(pt)
        c.EC_KEY_free(key)
