"""Extract the reference's own Ed25519 artefacts as parity vectors.

Build-container only (reads /root/reference, which does not exist on the GPU box);
its output `ref_ed25519_vectors.json` is the committed fixture the tests read.

The reference holds no EdDSA certificate or key store, but two text files carry
Ed25519 material in Corda's wire forms:

* samples/irs-demo/src/main/resources/net/corda/irs/simulation/trade.json:3,25 —
  the two IRS parties' keys as `PublicKey.toBase58String()` (`EncodingUtils.kt:66-67`:
  Base58 of the Kryo serialisation);
* docs/source/tutorial-cordapp.rst:472-476,498-499 — a `run verifiedTransactions`
  dump: two signatures (`sigs:`, Base64 of the 64-byte R‖S) over the transaction id
  (`id:`, hex), and the command signers' keys (Base58, as above).

Kryo wire form of an Ed25519 key (`Ed25519PublicKeySerializer`, `Kryo.kt:330-340`):
the 8-byte header `corda\\0\\0\\1` (`SerializationScheme.kt:216`), the class-registration
varint, the reference marker 0x01, then `writeBytesWithLength(abyte)` = varint 0x20 and
the 32-byte A.  The dump's signatures are `TransactionSignature`-free `DigitalSignature`s
over `id.bytes` (`TransactionWithSignatures.checkSignaturesAreValid`,
`TransactionWithSignatures.kt:58-62`: `sig.verify(id.bytes)`).

What the rows pin, checked here at generation time with the C restatement, the Python
twin and OpenSSL (independent of both):
* the two trade.json keys are `entropyToKeyPair(1)` / `entropyToKeyPair(2)`
  (`Crypto.kt:733-739`) — seed derivation, RFC 8032 key expansion, point encoding;
* the two tutorial signatures verify under the two tutorial keys over the id bytes
  (and under no other key) — i2p decode of canonical keys (A.2/A.4), SHA-512 of
  R‖Abyte‖M (A.5), the double-scalar multiply and byte compare (A.8/A.9) on valid
  signatures with S < L.

Usage:  python tests/golden/make_ref_ed25519_vectors.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import base64
import ctypes
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, os.path.join(ROOT, "oracle", "py"))
import ed25519_i2p as ED  # noqa: E402
import openssl_xcheck as OSSL  # noqa: E402  (independent check at generation time)

TRADE = "samples/irs-demo/src/main/resources/net/corda/irs/simulation/trade.json"
TUTORIAL = "docs/source/tutorial-cordapp.rst"
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"
KRYO_HEADER = b"corda\x00\x00\x01"  # SerializationScheme.kt:216


def base58_decode(s: str) -> bytes:
    n = 0
    for c in s:
        n = n * 58 + B58.index(c)
    zeros = len(s) - len(s.lstrip("1"))
    return b"\x00" * zeros + (n.to_bytes((n.bit_length() + 7) // 8, "big") if n else b"")


def kryo_ed25519_key(wire: bytes) -> tuple[int, bytes]:
    """(class-registration byte, A) of a Kryo-serialised EdDSAPublicKey."""
    assert wire[:8] == KRYO_HEADER, wire[:8]
    assert len(wire) == 8 + 1 + 1 + 1 + 32, len(wire)
    cls, ref, ln = wire[8], wire[9], wire[10]
    assert cls < 0x80 and ref == 0x01 and ln == 32, (cls, ref, ln)
    return cls, wire[11:]


def scan_keys(reference: str, rel: str):
    out = []
    with open(os.path.join(reference, rel), encoding="utf-8") as f:
        for lineno, line in enumerate(f, 1):
            for m in re.finditer(r'"(8Kqd4[1-9A-HJ-NP-Za-km-z]{40,})"', line):
                out.append((f"{rel}:{lineno}", m.group(1)))
    return out


def scan_tutorial_sigs(reference: str):
    """The `sigs:` list and the `id:` that follows it in the verifiedTransactions dump."""
    with open(os.path.join(reference, TUTORIAL), encoding="utf-8") as f:
        lines = f.read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.strip() == "sigs:")
    sigs, i = [], start + 1
    while lines[i].strip().startswith("- "):
        sigs.append((f"{TUTORIAL}:{i + 1}", lines[i].strip()[2:].strip('"')))
        i += 1
    m = re.match(r'id: "([0-9A-F]{64})"', lines[i].strip())
    assert m, lines[i]
    return sigs, (f"{TUTORIAL}:{i + 1}", m.group(1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "ref_ed25519_vectors.json"))
    args = ap.parse_args()

    oracle = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    sz = ctypes.c_size_t
    oracle.oracle_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.c_int]

    def verdicts(pk, sig, msg):
        py = (ED.is_valid(pk, sig, msg), ED.do_verify(pk, sig, msg))
        c = tuple(oracle.oracle_ed25519_verify(pk, sig, len(sig), msg, len(msg), m) for m in (0, 1))
        assert py == c, (pk.hex(), sig.hex(), py, c)
        return py

    # entropyToKeyPair(k) public keys for the small k a sample would use (k < 256: the seed is
    # the minimal big-endian bytes zero-padded on the right, so k and 256·k share a seed)
    entropy = {ED.seed_to_keypair(ED.entropy_seed(k))[2]: k for k in range(0, 256)}
    keys, seen = [], set()
    for rel in (TRADE, TUTORIAL):
        for where, b58 in scan_keys(args.reference, rel):
            if b58 in seen:
                continue
            seen.add(b58)
            wire = base58_decode(b58)
            cls, a = kryo_ed25519_key(wire)
            ED.decode_point_i2p(a)  # a valid key: raises KeyInvalid otherwise
            assert ED.abyte(a) == a  # canonical encoding (Abyte re-encodes to itself)
            keys.append({"where": where, "base58": b58, "wire": wire.hex(), "kryo_class": cls, "a": a.hex(),
                         "entropy_k": entropy.get(a)})
    assert len(keys) == 4, len(keys)
    assert [k["entropy_k"] for k in keys if k["where"].startswith(TRADE)] == [1, 2]

    sig_lines, (id_where, id_hex) = scan_tutorial_sigs(args.reference)
    msg = bytes.fromhex(id_hex)
    sigs = []
    for where, b64 in sig_lines:
        sig = base64.b64decode(b64)
        assert len(sig) == 64
        signers = []
        for k in keys:
            a = bytes.fromhex(k["a"])
            v = verdicts(a, sig, msg)
            assert OSSL.ed25519_verify(a, sig, msg) == (v[0] == 0)
            if v == (0, 0):
                signers.append(k["a"])
            else:
                assert v == (1, 1), v
        assert len(signers) == 1, signers
        assert int.from_bytes(sig[32:], "little") < ED.L
        sigs.append({"where": where, "id_where": id_where, "a": signers[0], "msg": id_hex.lower(), "sig": sig.hex(),
                     "is_valid": 0, "do_verify": 0})
    assert len(sigs) == 2 and len({s["a"] for s in sigs}) == 2

    with open(args.out, "w") as f:
        json.dump({"generator": "tests/golden/make_ref_ed25519_vectors.py", "sources": [TRADE, TUTORIAL],
                   "keys": keys, "sigs": sigs}, f, indent=1)
        f.write("\n")
    print(f"{len(keys)} keys, {len(sigs)} signatures -> {args.out}")


if __name__ == "__main__":
    main()
