"""CompositeKey fulfilment over verification verdicts, mirroring
Corda's composite keys (Kerwong/corda @ 0.14):

* ``CompositeKey`` / ``Builder`` with the construction-time constraints
  (core/src/main/kotlin/net/corda/core/crypto/composite/CompositeKey.kt:35-85,
  139-144, 235-268) and ``check_validity`` (cycle detection, :87-122);
* ``is_fulfilled_by_batch`` — ``PublicKey.isFulfilledBy(keys)`` (CryptoUtils.kt:78-82,
  CompositeKey.kt:186-209) for many (key, signers) queries in one device batch;
* ``missing_signatures`` — ``TransactionWithSignatures.getMissingSignatures``
  (TransactionWithSignatures.kt:72-77);
* ``composite_verify_batch`` — the composite signature engine
  (composite/CompositeSignature.kt:77-85): fulfilled by the signers' keys and every
  component signature valid (verdicts from the signature kernels).

Keys are their encoded bytes (PublicKey equality).  The threshold-tree evaluation
runs in libcordagpu (``cg_composite_eval_batch``); this module only flattens trees
into op programs and resolves leaf keys to signature indices, as the JVM side would.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import _lib
from .crypto import IllegalArgumentException

INT_MAX = 2**31 - 1


class CompositeKey:
    """net.corda.core.crypto.composite.CompositeKey: a threshold over weighted children
    (plain keys as ``bytes`` or nested CompositeKeys)."""

    def __init__(self, threshold: int, children: Sequence[tuple[object, int]]):
        self.threshold = threshold
        self.children = list(children)
        self._check_constraints()

    def _check_constraints(self):  # CompositeKey.kt:73-85
        idents = [(_ident(n), w) for n, w in self.children]
        if len(idents) != len(set(idents)):
            raise IllegalArgumentException("CompositeKey with duplicated child nodes detected.")
        if len(self.children) <= 1:
            raise IllegalArgumentException("CompositeKey must consist of two or more child nodes.")
        if self.threshold <= 0:
            raise IllegalArgumentException(f"CompositeKey threshold is set to {self.threshold}, but it should be "
                                           "a positive integer.")
        total = 0
        for _, w in self.children:
            if w <= 0:
                raise IllegalArgumentException(f"Non-positive weight: {w} detected.")
            total += w
            if total > INT_MAX:
                raise IllegalArgumentException("integer overflow")  # exactAdd
        if self.threshold > total:
            raise IllegalArgumentException(f"CompositeKey threshold: {self.threshold} cannot be bigger than "
                                           f"aggregated weight of child nodes: {total}")

    def check_validity(self):
        """CompositeKey.checkValidity (:110-122): graph cycles over object identity, then
        the constraints of this node and its children."""
        def walk(node, path):
            for child, _ in node.children:
                if isinstance(child, CompositeKey):
                    if any(child is p for p in path):
                        raise IllegalArgumentException("Cycle detected for CompositeKey")
                    walk(child, path + [child])
        walk(self, [self])
        self._check_constraints()
        for child, _ in self.children:
            if isinstance(child, CompositeKey):
                child._check_constraints()

    @property
    def leaf_keys(self) -> set:
        out: set = set()
        for n, _ in self.children:
            out |= n.leaf_keys if isinstance(n, CompositeKey) else {n}
        return out

    def __eq__(self, other):
        return isinstance(other, CompositeKey) and _ident(self) == _ident(other)

    def __hash__(self):
        return hash(_ident(self))


def _ident(n):
    # NodeAndWeight equality (the children are kept sorted, so order is irrelevant)
    if isinstance(n, CompositeKey):
        return ("C", n.threshold, tuple(sorted((_ident(c), w) for c, w in n.children)))
    return ("K", bytes(n))


class Builder:
    """CompositeKey.Builder (CompositeKey.kt:235-268)."""

    def __init__(self):
        self._children: list[tuple[object, int]] = []

    def add_key(self, key, weight: int = 1) -> "Builder":
        if weight <= 0:  # NodeAndWeight init
            raise IllegalArgumentException(f"A non-positive weight was detected. Weight: {weight}")
        self._children.append((key, weight))
        return self

    def add_keys(self, *keys) -> "Builder":
        for k in keys:
            self.add_key(k)
        return self

    def build(self, threshold: int | None = None):
        n = len(self._children)
        if n > 1:
            return CompositeKey(sum(w for _, w in self._children) if threshold is None else threshold,
                                self._children)
        if n == 1:
            if threshold is not None and threshold != self._children[0][1]:
                raise IllegalArgumentException("Trying to build invalid CompositeKey, threshold value different "
                                               "than weight of single child node.")
            return self._children[0][0]
        raise IllegalArgumentException("Trying to build CompositeKey without child nodes.")


def _program(key, sig_index: dict, out: list):
    """Post-order ops (kind, arg, weight, threshold) of one key; leaves resolve to the
    index of a signature by that key, or -1."""
    if isinstance(key, CompositeKey):
        key.check_validity()  # isFulfilledBy validates first (CompositeKey.kt:206-207)
    stack = [(key, 1, False)]
    while stack:
        node, w, seen = stack.pop()
        if not isinstance(node, CompositeKey):
            out.append((_lib.COMPOSITE_LEAF, sig_index.get(bytes(node), -1), w, 0))
        elif seen:
            out.append((_lib.COMPOSITE_NODE, len(node.children), w, node.threshold))
        else:
            stack.append((node, w, True))
            stack += [(c, cw, False) for c, cw in reversed(node.children)]


def eval_batch(ctx: _lib.Context, queries: Sequence[tuple[object, Sequence[bytes]]],
               verdicts: np.ndarray | None = None) -> np.ndarray:
    """Device evaluation of (key, signer keys) queries.  ``verdicts`` (optional, one per
    signer in query order) are cg_verify_batch codes.  Returns per query
    fulfilled | all_valid << 1 (or COMPOSITE_INVALID)."""
    prog, prog_start, sig_start = [], [0], [0]
    for key, signers in queries:
        base = sig_start[-1]
        index = {}
        for i, k in enumerate(signers):
            index.setdefault(bytes(k), base + i)
        _program(key, index, prog)
        prog_start.append(len(prog))
        sig_start.append(base + len(signers))
    n = len(queries)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    if n == 0:
        return out[:0]
    p = np.array(prog or [(0, 0, 0, 0)], dtype=np.int32)
    ps = np.array(prog_start, dtype=np.uint32)
    ss = np.array(sig_start, dtype=np.uint32)
    v = None if verdicts is None else np.ascontiguousarray(verdicts, dtype=np.uint8)
    if v is not None and len(v) != sig_start[-1]:
        raise IllegalArgumentException("one verdict per signer is required")
    ctx.check(ctx.lib.cg_composite_eval_batch(ctx.h, n, _lib.ptr(ps), _lib.ptr(p), int(sig_start[-1]),
                                              _lib.ptr(ss), _lib.ptr(v), _lib.ptr(out)))
    return out[:n]


def is_fulfilled_by_batch(ctx: _lib.Context, queries: Sequence[tuple[object, Sequence[bytes]]]) -> list[bool]:
    """``key.isFulfilledBy(signerKeys)`` for every query."""
    return [bool(r & 1) for r in eval_batch(ctx, queries)]


def missing_signatures(ctx: _lib.Context, required_keys: Sequence[object], signer_keys: Sequence[bytes]) -> list:
    """TransactionWithSignatures.getMissingSignatures: the required keys (plain or
    composite) not fulfilled by the signers' keys."""
    res = eval_batch(ctx, [(k, signer_keys) for k in required_keys])
    return [k for k, r in zip(required_keys, res) if not r & 1]


def composite_verify_batch(ctx: _lib.Context, queries: Sequence[tuple[CompositeKey, Sequence[bytes]]],
                           verdicts: np.ndarray) -> list[bool]:
    """CompositeSignature engineVerify for each (composite key, component signers)
    query given the component signatures' verdicts: fulfilled and all valid."""
    return [r == 3 for r in eval_batch(ctx, queries, verdicts)]
