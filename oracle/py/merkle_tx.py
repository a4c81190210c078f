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
