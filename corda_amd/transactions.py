"""Batch transaction-id recompute and signed-transaction signature checking,
mirroring Corda's transaction layer (Kerwong/corda @ 0.14):

* ``WireTransaction.id`` = Merkle root of ``availableComponentHashes``
  (core/src/main/kotlin/net/corda/core/transactions/WireTransaction.kt:39,104;
  MerkleTransaction.kt:16-33,74-93; crypto/MerkleTree.kt:27-66)
* ``TransactionWithSignatures.checkSignaturesAreValid`` — every signature over
  ``id.bytes``, in order, the first failure throws
  (transactions/TransactionWithSignatures.kt:58-62; DigitalSignature.kt:25 ->
  Crypto.doVerify)

A transaction here is its serialized components (Kryo P2P no-refs bytes, produced
by the caller; the last one is the serialized PrivacySalt) + the raw 32-byte salt.
The hashing and verification run in libcordagpu (K5/K6 + K1-K3).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _lib
from .crypto import IllegalArgumentException, SignatureException, _scheme_id, raise_for_verdict


class MerkleTreeException(Exception):
    """net.corda.core.crypto.MerkleTreeException (MerkleTree.kt:29-30)."""


@dataclass
class WireTx:
    components: list[bytes]   # availableComponents order; last = serialized privacy salt
    salt: bytes               # PrivacySalt.bytes (32)


@dataclass
class SignedTx:
    wire: WireTx
    sigs: list[tuple] = field(default_factory=list)  # (scheme, public_key_bytes, signature_bytes)


def _pack_txs(txs: Sequence[WireTx]):
    comps = [c for t in txs for c in t.components]
    comp_len = np.array([len(c) for c in comps] or [0], dtype=np.uint32)
    comp_off = np.zeros(max(len(comps), 1), dtype=np.uint64)
    if len(comps) > 1:
        comp_off[1:len(comps)] = np.cumsum(comp_len[:len(comps) - 1], dtype=np.uint64)
    comp_start = np.zeros(len(txs) + 1, dtype=np.uint32)
    comp_start[1:] = np.cumsum([len(t.components) for t in txs])
    arena = np.frombuffer(b"".join(comps) or b"\0", dtype=np.uint8).copy()
    salts = np.frombuffer(b"".join(bytes(t.salt) for t in txs), dtype=np.uint8).copy()
    if any(len(t.salt) != 32 for t in txs):
        raise IllegalArgumentException("privacy salt must be 32 bytes")
    return arena, comp_off, comp_len, comp_start, salts


def tx_ids(ctx: _lib.Context, txs: Sequence[WireTx]) -> list[bytes]:
    """WireTransaction.id for each tx (raises MerkleTreeException if some tx has no
    component, like MerkleTree.getMerkleTree on an empty list)."""
    arena, off, ln, start, salts = _pack_txs(txs)
    ids = np.zeros(max(len(txs), 1) * 32, dtype=np.uint8)
    st = ctx.lib.cg_txid_batch(ctx.h, len(txs), _lib.ptr(arena), len(arena), _lib.ptr(off), _lib.ptr(ln),
                               _lib.ptr(start), _lib.ptr(salts), _lib.ptr(ids))
    if st == _lib.CG_E_MERKLE_EMPTY:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    ctx.check(st)
    return [bytes(ids[32 * i:32 * i + 32]) for i in range(len(txs))]


def check_signatures_batch(ctx: _lib.Context, stxs: Sequence[SignedTx], mode: int = _lib.MODE_DO_VERIFY):
    """Runs checkSignaturesAreValid for every tx in one device batch.
    Returns (first_bad[n_tx], verdicts[n_sig], ids): first_bad[t] = -1 when all of
    tx t's signatures verify, the index of the first failing signature otherwise,
    -2 for a tx without signatures, -3 for a tx without components."""
    arena, off, ln, start, salts = _pack_txs([s.wire for s in stxs])
    sig_start = np.zeros(len(stxs) + 1, dtype=np.uint32)
    sig_start[1:] = np.cumsum([len(s.sigs) for s in stxs])
    flat = [x for s in stxs for x in s.sigs]
    n_sig = len(flat)
    scheme = np.array([_scheme_id(x[0]) for x in flat] or [4], dtype=np.uint8)
    pk = np.zeros((max(n_sig, 1), 64), dtype=np.uint8)
    sig_stride = (max([len(x[2]) for x in flat] + [64]) + 3) // 4 * 4
    sig = np.zeros((max(n_sig, 1), sig_stride), dtype=np.uint8)
    sig_len = np.zeros(max(n_sig, 1), dtype=np.uint32)
    for i, (_, k, s) in enumerate(flat):
        pk[i, :len(k)] = np.frombuffer(bytes(k)[:64], dtype=np.uint8)
        sig[i, :len(s)] = np.frombuffer(bytes(s), dtype=np.uint8)
        sig_len[i] = len(s)
    first_bad = np.zeros(max(len(stxs), 1), dtype=np.int32)
    verdict = np.zeros(max(n_sig, 1), dtype=np.uint8)
    ids = np.zeros(max(len(stxs), 1) * 32, dtype=np.uint8)
    st = ctx.lib.cg_tx_verify_batch(ctx.h, mode, len(stxs), _lib.ptr(arena), len(arena), _lib.ptr(off), _lib.ptr(ln),
                                    _lib.ptr(start), _lib.ptr(salts), _lib.ptr(sig_start), _lib.ptr(scheme),
                                    _lib.ptr(pk), 64, _lib.ptr(sig), sig_stride, _lib.ptr(sig_len),
                                    _lib.ptr(first_bad), _lib.ptr(verdict), _lib.ptr(ids))
    if st not in (_lib.CG_OK, _lib.CG_E_MERKLE_EMPTY):
        ctx.check(st)
    return first_bad[:len(stxs)], verdict[:n_sig], [bytes(ids[32 * i:32 * i + 32]) for i in range(len(stxs))]


def check_signatures_are_valid(ctx: _lib.Context, stxs: Sequence[SignedTx]) -> None:
    """Loop of ``stx.checkSignaturesAreValid()`` over the batch: raises the exception
    the first failing transaction would raise (its first failing signature)."""
    first_bad, verdict, _ = check_signatures_batch(ctx, stxs)
    base = 0
    for t, s in enumerate(stxs):
        fb = int(first_bad[t])
        if fb == -3:
            raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
        if fb == -2:
            raise IllegalArgumentException("Tried to instantiate a SignedTransaction without any signatures ", t)
        if fb >= 0:
            code = int(verdict[base + fb])
            try:
                raise_for_verdict(code, base + fb)
            except SignatureException as e:
                e.tx_index, e.sig_index = t, fb
                raise
        base += len(s.sigs)
