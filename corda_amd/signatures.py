"""Key- and signature-object entry points of Corda's crypto API over the batch engine
(SURVEY §8a row a6): the calls a JVM caller makes on a ``PublicKey``, a
``DigitalSignature.WithKey`` or a ``TransactionSignature`` instead of on ``Crypto``.

Reference (Kerwong/corda @ 0.14, core/src/main/kotlin/net/corda/core/crypto/):
  * ``PublicKey.verify(content, signature)`` = ``Crypto.doVerify(this, signature.bytes, content)``
    CryptoUtils.kt:49
  * ``PublicKey.isValid(content, signature)``: a ``CompositeKey`` throws
    ``IllegalStateException("Verification of CompositeKey signatures currently not supported.")``,
    otherwise ``Crypto.isValid(this, signature.bytes, content)``  CryptoUtils.kt:63-67
  * ``DigitalSignature.WithKey.verify / isValid(content)`` = ``by.verify / by.isValid``
    DigitalSignature.kt:24-46
  * ``TransactionSignature.verify()`` = ``Crypto.doVerify(metaData.publicKey, signatureData,
    metaData.bytes())``  TransactionSignature.kt:20
  * ``Crypto.doVerify(publicKey, transactionSignature)``  Crypto.kt:497-501: verifies with the
    *passed* key over ``metaData.bytes()``.  Line 499 constructs an IllegalArgumentException for a
    key that differs from ``metaData.publicKey`` but never throws it, so a mismatching key is not an
    error by itself (the signature simply has to verify under the passed key) — mirrored as is.
  * ``Crypto.isValid(publicKey, ...)``  Crypto.kt:518, 535-541: no empty-data check (unlike
    doVerify); an undecodable signature / key throws (SignatureException / InvalidKeyException).

Every function here is a loop of the reference call collapsed into one device batch
(``corda_amd.crypto``): it returns what the loop returns, or raises the exception the loop's
first throwing element raises.  ``MetaData.bytes()`` is the Kryo serialization of the
MetaData object (MetaData.kt:41); the engine never serializes, so a TransactionSignature here
carries those bytes as the JVM produced them.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import numpy as np

from . import _lib
from .crypto import (ACCEPT, REJECT, SignatureScheme, _scheme_id, _verify_mixed, do_verify_batch,
                     raise_for_verdict)

COMPOSITE_SCHEME_ID = 6  # Crypto.COMPOSITE_KEY (Crypto.kt:176-183); verified by CompositeSignature on the JVM


class IllegalStateException(RuntimeError):
    """java.lang.IllegalStateException (CryptoUtils.kt:65)."""

    def __init__(self, msg: str, index: int | None = None):
        super().__init__(msg)
        self.index = index


@dataclass(frozen=True)
class PublicKey:
    """A public key as the engine sees it: the scheme ``findSignatureScheme(key)`` resolves
    (Crypto.kt:228-236) and the key's wire bytes (Ed25519 A, 32 bytes; ECDSA X||Y, 64 bytes;
    for host-verified schemes whatever ``host_verify`` consumes)."""

    scheme: SignatureScheme | int | str
    encoded: bytes

    @property
    def scheme_id(self) -> int:
        return _scheme_id(self.scheme)

    @property
    def is_composite(self) -> bool:
        return self.scheme_id == COMPOSITE_SCHEME_ID


@dataclass(frozen=True)
class WithKey:
    """``DigitalSignature.WithKey(by, bits)`` (DigitalSignature.kt:16)."""

    by: PublicKey
    bytes: bytes


@dataclass(frozen=True)
class TransactionSignature:
    """``TransactionSignature(signatureData, metaData)`` (TransactionSignature.kt:10): the
    signature over ``MetaData.bytes()``; ``metadata_public_key`` is ``metaData.publicKey``."""

    signature_data: bytes
    metadata_bytes: bytes
    metadata_public_key: PublicKey


def _raise_first(v: np.ndarray, allowed=(ACCEPT,)):
    bad = np.flatnonzero(~np.isin(v, allowed))
    if bad.size:
        i = int(bad[0])
        raise_for_verdict(int(v[i]), i)


def _columns(keys: Sequence[PublicKey]):
    return [k.scheme_id for k in keys], [k.encoded for k in keys]


def public_key_verify_batch(ctx: _lib.Context, keys: Sequence[PublicKey], contents: Sequence[bytes],
                            signatures: Sequence[bytes], host_verify=None) -> bool:
    """``for i: keys[i].verify(contents[i], DigitalSignature(signatures[i]))`` (CryptoUtils.kt:49):
    True, or the exception of the lowest failing index (Crypto.doVerify's, incl. empty data)."""
    schemes, enc = _columns(keys)
    return do_verify_batch(ctx, schemes, enc, signatures, contents, host_verify)


def public_key_is_valid_batch(ctx: _lib.Context, keys: Sequence[PublicKey], contents: Sequence[bytes],
                              signatures: Sequence[bytes], host_verify=None) -> np.ndarray:
    """``[keys[i].isValid(contents[i], DigitalSignature(signatures[i])) for i]`` (CryptoUtils.kt:63-67):
    a bool per element, or the first exception the loop would meet — IllegalStateException for a
    CompositeKey, else Crypto.isValid's (SignatureException for an undecodable signature,
    InvalidKeyException for an unusable key, IllegalArgumentException for an unsupported scheme)."""
    n = len(keys)
    if not (len(contents) == n == len(signatures)):
        raise ValueError("keys, contents and signatures differ in length")
    composite = [i for i, k in enumerate(keys) if k.is_composite]
    stop = composite[0] if composite else n  # the loop never reaches elements past the first composite key
    schemes, enc = _columns(keys[:stop])
    v = _verify_mixed(ctx, schemes, enc, signatures[:stop], contents[:stop], _lib.MODE_IS_VALID, host_verify)
    _raise_first(v, (ACCEPT, REJECT))
    if composite:
        raise IllegalStateException("Verification of CompositeKey signatures currently not supported.", stop)
    return v == ACCEPT


def with_key_verify_batch(ctx: _lib.Context, sigs: Sequence[WithKey], contents: Sequence[bytes],
                          host_verify=None) -> bool:
    """``for i: sigs[i].verify(contents[i])`` (DigitalSignature.kt:24) = ``by.verify(content, this)``."""
    return public_key_verify_batch(ctx, [s.by for s in sigs], contents, [s.bytes for s in sigs], host_verify)


def with_key_is_valid_batch(ctx: _lib.Context, sigs: Sequence[WithKey], contents: Sequence[bytes],
                            host_verify=None) -> np.ndarray:
    """``[sigs[i].isValid(contents[i]) for i]`` (DigitalSignature.kt:46) = ``by.isValid(content, this)``."""
    return public_key_is_valid_batch(ctx, [s.by for s in sigs], contents, [s.bytes for s in sigs], host_verify)


def transaction_signatures_verify(ctx: _lib.Context, sigs: Sequence[TransactionSignature],
                                  host_verify=None) -> bool:
    """``for s in sigs: s.verify()`` (TransactionSignature.kt:20): each signature under its own
    ``metaData.publicKey`` over ``metaData.bytes()``."""
    return public_key_verify_batch(ctx, [s.metadata_public_key for s in sigs], [s.metadata_bytes for s in sigs],
                                   [s.signature_data for s in sigs], host_verify)


def do_verify_transaction_signatures(ctx: _lib.Context, keys: Sequence[PublicKey],
                                     sigs: Sequence[TransactionSignature], host_verify=None) -> bool:
    """``for i: Crypto.doVerify(keys[i], sigs[i])`` (Crypto.kt:497-501): verification under the
    passed key over ``metaData.bytes()``; a key different from ``metaData.publicKey`` is not
    rejected by itself (the reference builds that exception without throwing it)."""
    if len(keys) != len(sigs):
        raise ValueError("keys and sigs differ in length")
    return public_key_verify_batch(ctx, keys, [s.metadata_bytes for s in sigs], [s.signature_data for s in sigs],
                                   host_verify)
