"""TEST INFRASTRUCTURE ONLY — pure-Python twin of the transaction-id oracle.

Restates Corda's WireTransaction id computation, fully specified in the reference:

* nonce_i = SHA256(salt(32) || BE32(i))
  (/root/reference/core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:33)
* leaf_i  = SHA256(ser_i || nonce_i) for every component but the salt,
  leaf_salt = SHA256(ser_salt)       (MerkleTransaction.kt:16-30)
* component order inputs, attachments, outputs, commands, notary?, timeWindow?,
  salt (MerkleTransaction.kt:74-87); i is the index in that flattened list.
* pad with 32 zero bytes to the next power of two (MerkleTree.kt:35-43), node =
  SHA256(left || right) (SecureHash.kt:25, MerkleTree.kt:50-66); a single leaf is
  its own root; an empty list throws MerkleTreeException (MerkleTree.kt:27-32).

``ser_i`` are the Kryo P2P no-refs bytes of each component; they are produced by
the host (out of scope), and reach the id engine as an opaque byte arena.
"""
from __future__ import annotations

import hashlib

ZERO_HASH = bytes(32)


class MerkleTreeException(Exception):
    pass


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def compute_nonce(salt: bytes, index: int) -> bytes:
    return sha256(salt + index.to_bytes(4, "big", signed=True))


def leaf_hash(ser: bytes, salt: bytes, index: int, is_salt: bool) -> bytes:
    if is_salt:
        return sha256(ser)
    return sha256(ser + compute_nonce(salt, index))


def _is_pow2(n: int) -> bool:
    return n & (n - 1) == 0


def merkle_root(leaves: list[bytes]) -> bytes:
    if not leaves:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    level = list(leaves)
    n = len(level)
    while not _is_pow2(n):
        level.append(ZERO_HASH)
        n += 1
    while len(level) > 1:
        level = [sha256(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
    return level[0]


def tx_id(components: list[bytes], salt: bytes) -> bytes:
    """components: serialized bytes in availableComponents order, the LAST one
    being the serialized privacy salt (ser_salt)."""
    leaves = [leaf_hash(c, salt, i, i == len(components) - 1) for i, c in enumerate(components)]
    return merkle_root(leaves)


# --------------------------------------------------------------------------
# Partial Merkle trees / FilteredTransaction.verify (non-validating notary).
# Restates /root/reference/core/src/main/kotlin/net/corda/core/crypto/MerkleTree.kt:27-66
# (the full tree with its node hashes), PartialMerkleTree.kt:60-155 (build, verify)
# and transactions/MerkleTransaction.kt:23-27,153,173-178 (FilteredLeaves hashes with
# the given nonces, FilteredTransaction.verify).

class MTLeaf:
    """MerkleTree.Leaf(hash)"""

    def __init__(self, h: bytes):
        self.hash = h


class MTNode:
    """MerkleTree.Node(hash, left, right)"""

    def __init__(self, h: bytes, left, right):
        self.hash, self.left, self.right = h, left, right


def get_merkle_tree(hashes: list[bytes]):
    """MerkleTree.getMerkleTree (MerkleTree.kt:27-66): pad with zero hashes to a power
    of two, build pairwise bottom-up."""
    if not hashes:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    level = list(hashes)
    while not _is_pow2(len(level)):
        level.append(ZERO_HASH)
    nodes = [MTLeaf(h) for h in level]
    while len(nodes) > 1:
        nodes = [MTNode(sha256(nodes[i].hash + nodes[i + 1].hash), nodes[i], nodes[i + 1])
                 for i in range(0, len(nodes), 2)]
    return nodes[0]


class PTIncluded:
    """PartialTree.IncludedLeaf(hash)"""

    def __init__(self, h: bytes):
        self.hash = h


class PTLeaf:
    """PartialTree.Leaf(hash)"""

    def __init__(self, h: bytes):
        self.hash = h


class PTNode:
    """PartialTree.Node(left, right)"""

    def __init__(self, left, right):
        self.left, self.right = left, right


def _check_full(tree, level=0) -> int:
    # PartialMerkleTree.kt:79-89
    if isinstance(tree, MTLeaf):
        return level
    l1 = _check_full(tree.left, level + 1)
    l2 = _check_full(tree.right, level + 1)
    if l1 != l2:
        raise MerkleTreeException("Got not full binary tree.")
    return l1


def _build_partial(root, include: list[bytes], used: list[bytes]):
    # PartialMerkleTree.kt:98-123
    if isinstance(root, MTLeaf):
        if root.hash in include:
            used.append(root.hash)
            return True, PTIncluded(root.hash)
        return False, PTLeaf(root.hash)
    lf, ln = _build_partial(root.left, include, used)
    rf, rn = _build_partial(root.right, include, used)
    if lf or rf:
        return True, PTNode(ln, rn)
    return False, PTLeaf(root.hash)


def pmt_build(merkle_root, include_hashes: list[bytes]):
    """PartialMerkleTree.build (PartialMerkleTree.kt:66-76). Raises ValueError for
    the require() (IllegalArgumentException), MerkleTreeException otherwise."""
    if ZERO_HASH in include_hashes:
        raise ValueError("Zero hashes shouldn't be included in partial tree.")
    _check_full(merkle_root)
    used: list[bytes] = []
    _, tree = _build_partial(merkle_root, include_hashes, used)
    if len(include_hashes) != len(used):
        raise MerkleTreeException("Some of the provided hashes are not in the tree.")
    return tree


def _pmt_root(node, used: list[bytes]) -> bytes:
    # PartialMerkleTree.kt:143-156
    if isinstance(node, PTIncluded):
        used.append(node.hash)
        return node.hash
    if isinstance(node, PTLeaf):
        return node.hash
    left = _pmt_root(node.left, used)
    right = _pmt_root(node.right, used)
    return sha256(left + right)


def pmt_verify(tree, merkle_root_hash: bytes, hashes_to_check: list[bytes]) -> bool:
    """PartialMerkleTree.verify (PartialMerkleTree.kt:130-137): groupBy equality is
    multiset equality."""
    used: list[bytes] = []
    root = _pmt_root(tree, used)
    if sorted(hashes_to_check) != sorted(used):
        return False
    return root == merkle_root_hash


def filtered_leaf_hash(ser: bytes, nonce: bytes) -> bytes:
    """serializedHash(x, nonce) (MerkleTransaction.kt:23-27) for a non-salt component."""
    return sha256(ser + nonce)


def ftx_verify(components: list[bytes], nonces: list[bytes], tree, root_hash: bytes) -> bool:
    """FilteredTransaction.verify (MerkleTransaction.kt:173-178)."""
    hashes = [filtered_leaf_hash(c, n) for c, n in zip(components, nonces)]
    if not hashes:
        raise MerkleTreeException("Transaction without included leaves.")
    return pmt_verify(tree, root_hash, hashes)


def pmt_postorder(tree) -> list[tuple[int, bytes]]:
    """The (kind, hash) node program of the batch ABI: 0 IncludedLeaf, 1 Leaf, 2 Node,
    post-order (iterative: adversarial trees may be deep)."""
    out, stack = [], [(tree, False)]
    while stack:
        node, seen = stack.pop()
        if isinstance(node, PTIncluded):
            out.append((0, node.hash))
        elif isinstance(node, PTLeaf):
            out.append((1, node.hash))
        elif seen:
            out.append((2, ZERO_HASH))
        else:
            stack.append((node, True))
            stack.append((node.right, False))
            stack.append((node.left, False))
    return out


def pmt_from_postorder(prog: list[tuple[int, bytes]]):
    """Inverse of pmt_postorder; None when the program is not exactly one tree."""
    st = []
    for kind, h in prog:
        if kind == 0:
            st.append(PTIncluded(h))
        elif kind == 1:
            st.append(PTLeaf(h))
        elif kind == 2 and len(st) >= 2:
            r = st.pop()
            st.append(PTNode(st.pop(), r))
        else:
            return None
    return st[0] if len(st) == 1 else None
