"""Batch transaction-id recompute and signed-transaction signature checking,
mirroring Corda's transaction layer (Kerwong/corda @ 0.14):

* ``WireTransaction.id`` = Merkle root of ``availableComponentHashes``
  (core/src/main/kotlin/net/corda/core/transactions/WireTransaction.kt:39,104;
  MerkleTransaction.kt:16-33,74-93; crypto/MerkleTree.kt:27-66)
* ``FilteredTransaction.verify`` / ``PartialMerkleTree.verify`` — the non-validating
  notary's check (transactions/MerkleTransaction.kt:140-178,
  crypto/PartialMerkleTree.kt:44-156, NonValidatingNotaryFlow.kt:25-27)
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
from .crypto import IllegalArgumentException, SignatureException, _scheme_id, pack_key_row, raise_for_verdict


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


def _pack_sigs(stxs: Sequence[SignedTx]):
    sig_start = np.zeros(len(stxs) + 1, dtype=np.uint32)
    sig_start[1:] = np.cumsum([len(s.sigs) for s in stxs])
    flat = [x for s in stxs for x in s.sigs]
    n_sig = len(flat)
    scheme = np.array([_scheme_id(x[0]) for x in flat] or [4], dtype=np.uint8)
    pk = np.zeros((max(n_sig, 1), 64), dtype=np.uint8)
    sig_stride = (max([len(x[2]) for x in flat] + [64]) + 3) // 4 * 4
    sig = np.zeros((max(n_sig, 1), sig_stride), dtype=np.uint8)
    sig_len = np.zeros(max(n_sig, 1), dtype=np.uint32)
    for i, (sch, k, s) in enumerate(flat):
        # a wrong-length key is KEY_INVALID for that signature alone (flagged in its scheme
        # id), so the first failing signature in tx order still decides the exception
        pack_key_row(pk, scheme, i, k)
        sig[i, :len(s)] = np.frombuffer(bytes(s), dtype=np.uint8)
        sig_len[i] = len(s)
    return sig_start, scheme, pk, sig, sig_stride, sig_len, n_sig


def check_signatures_batch(ctx: _lib.Context, stxs: Sequence[SignedTx], mode: int = _lib.MODE_DO_VERIFY):
    """Runs checkSignaturesAreValid for every tx in one device batch.
    Returns (first_bad[n_tx], verdicts[n_sig], ids): first_bad[t] = -1 when all of
    tx t's signatures verify, the index of the first failing signature otherwise,
    -2 for a tx without signatures, -3 for a tx without components."""
    arena, off, ln, start, salts = _pack_txs([s.wire for s in stxs])
    sig_start, scheme, pk, sig, sig_stride, sig_len, n_sig = _pack_sigs(stxs)
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


class SignaturesMissingException(Exception):
    """SignedTransaction.SignaturesMissingException (SignedTransaction.kt): required keys
    neither fulfilled by the signatures' keys nor allowed to be missing."""

    def __init__(self, missing: list, tx_index: int):
        super().__init__(f"Missing signatures for {len(missing)} required key(s) on transaction {tx_index}")
        self.missing, self.tx_index = missing, tx_index


def verify_signatures_except_batch(ctx: _lib.Context, stxs: Sequence[SignedTx], required: Sequence[Sequence[object]],
                                   allowed_to_be_missing: Sequence[Sequence[object]] | None = None,
                                   mode: int = _lib.MODE_DO_VERIFY):
    """``stx.verifySignaturesExcept(*allowed)`` for every tx in ONE device call
    (cg_tx_verify_signatures_except; TransactionWithSignatures.kt:41-47): ids
    recomputed, every signature verified, then getMissingSignatures (:72-77) — each of
    the tx's ``requiredSigningKeys`` (plain key bytes or a composite.CompositeKey)
    evaluated with isFulfilledBy against the tx's signature keys, minus the allowed
    keys — with the verdicts kept on the device.

    Returns (status[n_tx], missing): status per tx as the _lib.TX_* codes (>= 0 = first
    failing signature); missing[t] = the required keys of tx t in the exception's set."""
    from .composite import _ident, _program
    arena, off, ln, start, salts = _pack_txs([s.wire for s in stxs])
    sig_start, scheme, pk, sig, sig_stride, sig_len, n_sig = _pack_sigs(stxs)
    allowed_to_be_missing = allowed_to_be_missing or [[] for _ in stxs]
    prog, prog_start, req_start, allowed = [], [0], [0], []
    for t, s in enumerate(stxs):
        index = {}
        for i, (_, k, _sig) in enumerate(s.sigs):
            index.setdefault(bytes(k), i)  # sigKeys = sigs.map { it.by }.toSet(): leaf -> a signature by it
        ok = {_ident(a) for a in allowed_to_be_missing[t]}
        for key in required[t]:
            _program(key, index, prog)
            prog_start.append(len(prog))
            allowed.append(1 if _ident(key) in ok else 0)
        req_start.append(len(prog_start) - 1)
    n_tx, n_req = len(stxs), len(allowed)
    status = np.zeros(max(n_tx, 1), dtype=np.int32)
    missing = np.zeros(max(n_req, 1), dtype=np.uint8)
    p = np.array(prog or [(0, 0, 0, 0)], dtype=np.int32)
    ps, rs = np.array(prog_start, dtype=np.uint32), np.array(req_start, dtype=np.uint32)
    al = np.array(allowed or [0], dtype=np.uint8)
    st = ctx.lib.cg_tx_verify_signatures_except(
        ctx.h, mode, n_tx, _lib.ptr(arena), len(arena), _lib.ptr(off), _lib.ptr(ln), _lib.ptr(start), _lib.ptr(salts),
        _lib.ptr(sig_start), _lib.ptr(scheme), _lib.ptr(pk), 64, _lib.ptr(sig), sig_stride, _lib.ptr(sig_len),
        _lib.ptr(rs), _lib.ptr(ps), _lib.ptr(p), _lib.ptr(al), _lib.ptr(status), _lib.ptr(missing), None)
    if st == _lib.CG_E_INVALID_ARGUMENT:
        raise IllegalArgumentException((ctx.lib.cg_last_error(ctx.h) or b"").decode())
    if st not in (_lib.CG_OK, _lib.CG_E_MERKLE_EMPTY):
        ctx.check(st)
    miss = [[required[t][r - req_start[t]] for r in range(req_start[t], req_start[t + 1]) if missing[r]]
            for t in range(n_tx)]
    return status[:n_tx], miss


def verify_signatures_except(ctx: _lib.Context, stxs: Sequence[SignedTx], required: Sequence[Sequence[object]],
                             allowed_to_be_missing: Sequence[Sequence[object]] | None = None) -> None:
    """Loop of ``stx.verifySignaturesExcept(*allowed)``: raises what the first failing
    tx would raise (SignatureException & co. for its first bad signature, else
    SignaturesMissingException)."""
    status, miss = verify_signatures_except_batch(ctx, stxs, required, allowed_to_be_missing)
    first_bad, verdict, _ = None, None, None
    for t, st in enumerate(status):
        st = int(st)
        if st == _lib.TX_OK:
            continue
        if st == _lib.TX_NO_COMPONENTS:
            raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
        if st == _lib.TX_NO_SIGNATURES:
            raise IllegalArgumentException("Tried to instantiate a SignedTransaction without any signatures ", t)
        if st == _lib.TX_SIGNATURES_MISSING:
            raise SignaturesMissingException(miss[t], t)
        if first_bad is None:  # the failing signature's verdict code decides the exception class
            first_bad, verdict, _ = check_signatures_batch(ctx, [stxs[t]])
        raise_for_verdict(int(verdict[st]), st)


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


# ---------------------------------------------------------------- filtered transactions
ZERO_HASH = bytes(32)


@dataclass(frozen=True)
class IncludedLeaf:
    """PartialMerkleTree.PartialTree.IncludedLeaf (PartialMerkleTree.kt:55)."""
    hash: bytes


@dataclass(frozen=True)
class Leaf:
    """PartialMerkleTree.PartialTree.Leaf (PartialMerkleTree.kt:56)."""
    hash: bytes


@dataclass(frozen=True)
class Node:
    """PartialMerkleTree.PartialTree.Node (PartialMerkleTree.kt:57)."""
    left: object
    right: object


class PartialMerkleTree:
    """net.corda.core.crypto.PartialMerkleTree (PartialMerkleTree.kt:44-157).  ``build``
    is the sender side (structural: it only reads the hashes the full MerkleTree already
    carries); verification of filtered transactions runs on the device
    (``verify_filtered_batch``)."""

    def __init__(self, root):
        self.root = root

    @staticmethod
    def build(merkle_root, include_hashes: Sequence[bytes]) -> "PartialMerkleTree":
        """PartialMerkleTree.build (PartialMerkleTree.kt:66-76).  ``merkle_root`` is a
        full MerkleTree: objects with ``hash`` and, for nodes, ``left``/``right``."""
        include = list(include_hashes)
        if ZERO_HASH in include:
            raise IllegalArgumentException("Zero hashes shouldn't be included in partial tree.")
        PartialMerkleTree._check_full(merkle_root)
        used: list[bytes] = []
        tree = PartialMerkleTree._build(merkle_root, include, used)[1]
        if len(include) != len(used):
            raise MerkleTreeException("Some of the provided hashes are not in the tree.")
        return PartialMerkleTree(tree)

    @staticmethod
    def _is_leaf(t) -> bool:
        return getattr(t, "left", None) is None

    @staticmethod
    def _check_full(tree, level: int = 0) -> int:  # PartialMerkleTree.kt:79-89
        if PartialMerkleTree._is_leaf(tree):
            return level
        l1 = PartialMerkleTree._check_full(tree.left, level + 1)
        l2 = PartialMerkleTree._check_full(tree.right, level + 1)
        if l1 != l2:
            raise MerkleTreeException("Got not full binary tree.")
        return l1

    @staticmethod
    def _build(root, include: list, used: list):  # PartialMerkleTree.kt:98-123
        if PartialMerkleTree._is_leaf(root):
            if root.hash in include:
                used.append(root.hash)
                return True, IncludedLeaf(root.hash)
            return False, Leaf(root.hash)
        lf, ln = PartialMerkleTree._build(root.left, include, used)
        rf, rn = PartialMerkleTree._build(root.right, include, used)
        if lf or rf:
            return True, Node(ln, rn)
        return False, Leaf(root.hash)

    @staticmethod
    def from_postorder(prog: Sequence[tuple[int, bytes]]) -> "PartialMerkleTree":
        """Inverse of ``postorder`` (e.g. for a tree received as a node program)."""
        st: list = []
        for kind, h in prog:
            if kind == 0:
                st.append(IncludedLeaf(bytes(h)))
            elif kind == 1:
                st.append(Leaf(bytes(h)))
            elif kind == 2 and len(st) >= 2:
                r = st.pop()
                st.append(Node(st.pop(), r))
            else:
                raise IllegalArgumentException("not a post-order partial tree program")
        if len(st) != 1:
            raise IllegalArgumentException("not a post-order partial tree program")
        return PartialMerkleTree(st[0])

    def postorder(self) -> list[tuple[int, bytes]]:
        """The node program cg_ftx_verify_batch takes: (kind, hash) in post-order, kind 0
        IncludedLeaf / 1 Leaf / 2 Node.  Iterative, so adversarially deep trees encode."""
        out, stack = [], [(self.root, False)]
        while stack:
            node, seen = stack.pop()
            if isinstance(node, IncludedLeaf):
                out.append((0, node.hash))
            elif isinstance(node, Leaf):
                out.append((1, node.hash))
            elif seen:
                out.append((2, ZERO_HASH))
            else:
                stack += [(node, True), (node.right, False), (node.left, False)]
        return out


@dataclass
class FilteredLeaves:
    """FilteredLeaves (MerkleTransaction.kt:140-170): the visible components, serialized
    (Kryo P2P no-refs bytes, availableComponents order), each with its nonce."""
    components: list[bytes]
    nonces: list[bytes]

    def __post_init__(self):
        if len(self.components) != len(self.nonces):  # MerkleTransaction.kt:153
            raise IllegalArgumentException("Each visible component should be accompanied by a nonce.")
        if any(len(n) != 32 for n in self.nonces):
            raise IllegalArgumentException("nonces are 32-byte SecureHashes")


@dataclass
class FilteredTransaction:
    """FilteredTransaction (MerkleTransaction.kt:179-209)."""
    root_hash: bytes
    filtered_leaves: FilteredLeaves
    partial_merkle_tree: PartialMerkleTree

    def verify(self, ctx: _lib.Context) -> bool:
        """FilteredTransaction.verify (MerkleTransaction.kt:173-178) on the device."""
        return verify_filtered(ctx, [self])[0]


def _pack_ftxs(ftxs: Sequence[FilteredTransaction]):
    comps = [c for f in ftxs for c in f.filtered_leaves.components]
    comp_len = np.array([len(c) for c in comps] or [0], dtype=np.uint32)
    comp_off = np.zeros(max(len(comps), 1), dtype=np.uint64)
    if len(comps) > 1:
        comp_off[1:len(comps)] = np.cumsum(comp_len[:len(comps) - 1], dtype=np.uint64)
    comp_start = np.zeros(len(ftxs) + 1, dtype=np.uint32)
    comp_start[1:] = np.cumsum([len(f.filtered_leaves.components) for f in ftxs])
    arena = np.frombuffer(b"".join(comps) or b"\0", dtype=np.uint8).copy()
    nonces = np.frombuffer(b"".join(n for f in ftxs for n in f.filtered_leaves.nonces) or bytes(32),
                           dtype=np.uint8).copy()
    progs = [f.partial_merkle_tree.postorder() for f in ftxs]
    node_start = np.zeros(len(ftxs) + 1, dtype=np.uint32)
    node_start[1:] = np.cumsum([len(p) for p in progs])
    node_kind = np.array([k for p in progs for k, _ in p] or [0], dtype=np.uint8)
    node_hash = np.frombuffer(b"".join(h for p in progs for _, h in p) or bytes(32), dtype=np.uint8).copy()
    if any(len(f.root_hash) != 32 for f in ftxs):
        raise IllegalArgumentException("rootHash must be a 32-byte SecureHash")
    roots = np.frombuffer(b"".join(f.root_hash for f in ftxs), dtype=np.uint8).copy()
    return arena, comp_off, comp_len, comp_start, nonces, node_start, node_kind, node_hash, roots


def verify_filtered_batch(ctx: _lib.Context, ftxs: Sequence[FilteredTransaction]) -> np.ndarray:
    """FilteredTransaction.verify for every tx in one device batch; per tx one of
    FTX_TRUE / FTX_FALSE / FTX_NO_LEAVES (verify() would throw MerkleTreeException) /
    FTX_MALFORMED."""
    if not ftxs:
        return np.zeros(0, dtype=np.uint8)
    a = _pack_ftxs(ftxs)
    out = np.zeros(len(ftxs), dtype=np.uint8)
    ctx.check(ctx.lib.cg_ftx_verify_batch(ctx.h, len(ftxs), _lib.ptr(a[0]), len(a[0]), *(_lib.ptr(x) for x in a[1:]),
                                          _lib.ptr(out)))
    return out


def verify_filtered(ctx: _lib.Context, ftxs: Sequence[FilteredTransaction]) -> list[bool]:
    """A loop of ``ftx.verify()``: raises MerkleTreeException where the first such tx
    would, returns the Boolean results otherwise."""
    res = verify_filtered_batch(ctx, ftxs)
    for t, r in enumerate(res):
        if r == _lib.FTX_NO_LEAVES:
            raise MerkleTreeException("Transaction without included leaves.")
        if r == _lib.FTX_MALFORMED:
            raise IllegalArgumentException(f"filtered transaction {t}: partial tree is not a single tree")
    return [bool(r == _lib.FTX_TRUE) for r in res]
