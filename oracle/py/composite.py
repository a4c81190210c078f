"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of Corda's CompositeKey
fulfilment, the step after signature verification:

* CompositeKey(threshold, children) with constraints checked at construction
  (/root/reference/core/src/main/kotlin/net/corda/core/crypto/composite/CompositeKey.kt:35-85)
  and ``checkValidity`` (cycle detection over object identity, :87-122);
* ``Builder.build`` (:235-268): one child -> that child (threshold must equal its
  weight), none -> IllegalArgumentException, default threshold = total weight;
* ``checkFulfilledBy`` (:186-196): weight of satisfied children >= threshold, a
  leaf is satisfied iff its key is among the signers' keys;
* ``PublicKey.isFulfilledBy`` (CryptoUtils.kt:78-82) for plain keys;
* the composite signature engine (CompositeSignature.kt:77-85): fulfilled by the
  signers' keys AND every component signature valid.

Keys are opaque ``bytes`` (the encoded PublicKey); equality is byte equality.
"""
from __future__ import annotations

INT_MAX = 2**31 - 1


class IllegalArgument(Exception):
    pass


class CompositeKey:
    def __init__(self, threshold: int, children: list[tuple[object, int]]):
        self.threshold = threshold
        self.children = list(children)
        self._check_constraints()

    def _total_weight(self) -> int:
        s = 0
        for _, w in self.children:
            if w <= 0:
                raise IllegalArgument(f"Non-positive weight: {w} detected.")
            s += w
            if s > INT_MAX:  # exactAdd
                raise IllegalArgument("integer overflow")
        return s

    def _check_constraints(self):  # CompositeKey.kt:73-85
        keys = [(_ident(n), w) for n, w in self.children]
        if len(keys) != len(set(keys)):
            raise IllegalArgument("CompositeKey with duplicated child nodes detected.")
        if len(self.children) <= 1:
            raise IllegalArgument("CompositeKey must consist of two or more child nodes.")
        if self.threshold <= 0:
            raise IllegalArgument("CompositeKey threshold must be positive")
        if self.threshold > self._total_weight():
            raise IllegalArgument("CompositeKey threshold cannot be bigger than aggregated weight")

    def check_validity(self):  # CompositeKey.kt:87-122
        def cycles(node, visited):
            for child, _ in node.children:
                if isinstance(child, CompositeKey):
                    if any(child is v for v in visited):
                        raise IllegalArgument("Cycle detected for CompositeKey")
                    cycles(child, visited + [child])
        cycles(self, [self])
        self._check_constraints()
        for child, _ in self.children:
            if isinstance(child, CompositeKey):
                child._check_constraints()

    def is_fulfilled_by(self, keys) -> bool:  # CompositeKey.kt:203-209
        self.check_validity()
        return self._check_fulfilled_by(set(keys))

    def _check_fulfilled_by(self, keys: set) -> bool:  # CompositeKey.kt:186-196
        total = 0
        for node, w in self.children:
            if isinstance(node, CompositeKey):
                total += w if node._check_fulfilled_by(keys) else 0
            else:
                total += w if node in keys else 0
        return total >= self.threshold

    @property
    def leaf_keys(self) -> set:
        out = set()
        for n, _ in self.children:
            out |= n.leaf_keys if isinstance(n, CompositeKey) else {n}
        return out


def _ident(n):
    """NodeAndWeight equality: leaves by bytes, composite children structurally."""
    if isinstance(n, CompositeKey):
        return ("C", n.threshold, tuple(sorted((_ident(c), w) for c, w in n.children)))
    return ("K", n)


class Builder:
    """CompositeKey.Builder (CompositeKey.kt:235-268)."""

    def __init__(self):
        self.children: list[tuple[object, int]] = []

    def add_key(self, key, weight: int = 1) -> "Builder":
        if weight <= 0:  # NodeAndWeight init
            raise IllegalArgument("A non-positive weight was detected.")
        self.children.append((key, weight))
        return self

    def add_keys(self, *keys) -> "Builder":
        for k in keys:
            self.add_key(k)
        return self

    def build(self, threshold: int | None = None):
        n = len(self.children)
        if n > 1:
            return CompositeKey(threshold if threshold is not None else sum(w for _, w in self.children),
                                self.children)
        if n == 1:
            if threshold is not None and threshold != self.children[0][1]:
                raise IllegalArgument("Trying to build invalid CompositeKey, threshold value different than "
                                      "weight of single child node.")
            return self.children[0][0]
        raise IllegalArgument("Trying to build CompositeKey without child nodes.")


def is_fulfilled_by(key, keys) -> bool:
    """PublicKey.isFulfilledBy (CryptoUtils.kt:78-82)."""
    if isinstance(key, CompositeKey):
        return key.is_fulfilled_by(keys)
    return key in set(keys)


def program(key, sig_index: dict) -> list[tuple[int, int, int, int]]:
    """The post-order op program of cg_composite_eval_batch: (0, signature index or
    -1, weight, 0) for a leaf, (1, n_children, weight, threshold) for a node; the
    root's weight is 1."""
    out = []

    def emit(node, weight):
        if isinstance(node, CompositeKey):
            for c, w in node.children:
                emit(c, w)
            out.append((1, len(node.children), weight, node.threshold))
        else:
            out.append((0, sig_index.get(node, -1), weight, 0))
    emit(key, 1)
    return out


def composite_verify(key, signer_keys, all_valid: bool) -> bool:
    """CompositeSignature engineVerify (CompositeSignature.kt:77-85)."""
    return is_fulfilled_by(key, signer_keys) and all_valid
