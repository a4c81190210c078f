"""Extract the reference's own ECDSA signatures as parity vectors.

Build-container only (reads /root/reference, which does not exist on the GPU box);
its output `ref_cert_vectors.json` is the committed fixture the tests read.

The reference ships X.509 certificates signed `ecdsa-with-SHA256` by BouncyCastle
(the dev CA chain its nodes use, `X509Utilities.kt` + `ContentSignerBuilder.kt`):

* config/dev/corda_dev_ca.cer                                 (PEM)
* node/src/main/resources/net/corda/node/internal/certificates/*.jks
* samples/{trader,attachment}-demo/src/main/resources/certificates/*.jks

A certificate's signature is `SHA256withECDSA` over the DER bytes of its
TBSCertificate, under the issuer's public key — exactly the `Crypto.isValid(scheme,
issuerKey, signature, tbs)` call of `Crypto.kt:534-541` for ECDSA_SECP256R1_SHA256 /
ECDSA_SECP256K1_SHA256 (`Crypto.kt:91-116`).  Each row is therefore (curve scheme id,
issuer Q as X‖Y, message = TBS bytes, DER signature).

Keystores are read as data: the JKS container is walked for certificate entries only
(trusted-cert entries and the certificate chains stored beside private-key entries).
Private-key blobs are skipped by length, never decrypted, never written.  The keyed
SHA-1 trailer is not checked (it needs the store password).  Certificates are paired
with their issuer by comparing the DER of the issuer Name with every candidate's
subject Name, narrowed by the Authority/Subject Key Identifier extensions; two roots
share the DN "Corda Node Root CA" with keys on different curves, and where the
identifiers leave two candidates OpenSSL (independent of the oracle) says which key
verifies — the other pairing is kept as a wrong-key row that must REJECT.

Usage:  python tests/golden/make_ref_cert_vectors.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import base64
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle", "py"))
import openssl_xcheck as OSSL  # noqa: E402  (independent check at generation time)

SOURCES = [
    "config/dev/corda_dev_ca.cer",
    "node/src/main/resources/net/corda/node/internal/certificates/cordadevcakeys.jks",
    "node/src/main/resources/net/corda/node/internal/certificates/cordatruststore.jks",
    "samples/trader-demo/src/main/resources/certificates/truststore.jks",
    "samples/trader-demo/src/main/resources/certificates/sslkeystore.jks",
    "samples/attachment-demo/src/main/resources/certificates/truststore.jks",
    "samples/attachment-demo/src/main/resources/certificates/sslkeystore.jks",
]

OID_EC_PUBLIC_KEY = "1.2.840.10045.2.1"
OID_ECDSA_SHA256 = "1.2.840.10045.4.3.2"
CURVE_SCHEME = {"1.3.132.0.10": 2,          # secp256k1 -> ECDSA_SECP256K1_SHA256 (Crypto.kt:92)
                "1.2.840.10045.3.1.7": 3}   # prime256v1 -> ECDSA_SECP256R1_SHA256 (Crypto.kt:106)


# ---------------------------------------------------------------- DER walking
def der_tlv(buf: bytes, pos: int):
    """(tag, header_len, content_start, content_end) of the TLV at pos (definite lengths)."""
    tag = buf[pos]
    ln = buf[pos + 1]
    hdr = 2
    if ln & 0x80:
        k = ln & 0x7F
        ln = int.from_bytes(buf[pos + 2:pos + 2 + k], "big")
        hdr += k
    return tag, hdr, pos + hdr, pos + hdr + ln


def der_children(buf: bytes, start: int, end: int):
    out, p = [], start
    while p < end:
        t, h, cs, ce = der_tlv(buf, p)
        out.append((t, p, cs, ce))
        p = ce
    return out


def oid_str(b: bytes) -> str:
    first = b[0]
    parts = [first // 40, first % 40]
    v = 0
    for c in b[1:]:
        v = (v << 7) | (c & 0x7F)
        if not c & 0x80:
            parts.append(v)
            v = 0
    return ".".join(map(str, parts))


def parse_cert(der: bytes) -> dict:
    """Certificate ::= SEQUENCE { tbsCertificate, signatureAlgorithm, signatureValue BIT STRING }."""
    t, _, cs, ce = der_tlv(der, 0)
    assert t == 0x30 and ce == len(der), "not one DER SEQUENCE"
    tbs, alg, sigv = der_children(der, cs, ce)
    tbs_bytes = der[tbs[1]:tbs[3]]
    alg_oid = oid_str(der[der_children(der, alg[2], alg[3])[0][2]:der_children(der, alg[2], alg[3])[0][3]])
    assert sigv[0] == 0x03 and der[sigv[2]] == 0, "signatureValue is not a whole-byte BIT STRING"
    signature = der[sigv[2] + 1:sigv[3]]
    f = der_children(der, tbs[2], tbs[3])
    i = 1 if f[0][0] == 0xA0 else 0           # [0] EXPLICIT version
    issuer, subject, spki = f[i + 2], f[i + 4], f[i + 5]
    ka, kbits = der_children(der, spki[2], spki[3])
    ka_oids = [oid_str(der[c[2]:c[3]]) for c in der_children(der, ka[2], ka[3]) if c[0] == 0x06]
    ski = aki = None
    if len(f) > i + 6 and f[-1][0] == 0xA3:       # [3] EXPLICIT Extensions
        exts = der_children(der, *der_children(der, f[-1][2], f[-1][3])[0][2:4])
        for e in exts:
            parts = der_children(der, e[2], e[3])
            eid, val = oid_str(der[parts[0][2]:parts[0][3]]), parts[-1]
            if eid == "2.5.29.14":                # SubjectKeyIdentifier ::= OCTET STRING
                inner = der_tlv(der, val[2])
                ski = der[inner[2]:inner[3]]
            elif eid == "2.5.29.35":              # AuthorityKeyIdentifier ::= SEQUENCE { [0] keyIdentifier .. }
                seq = der_tlv(der, val[2])
                for t, _, cs2, ce2 in der_children(der, seq[2], seq[3]):
                    if t == 0x80:
                        aki = der[cs2:ce2]
    key = None
    if ka_oids and ka_oids[0] == OID_EC_PUBLIC_KEY:
        pt = der[kbits[2] + 1:kbits[3]]
        assert pt[0] == 4 and len(pt) == 65, "EC key is not an uncompressed point"
        key = {"curve_oid": ka_oids[1], "q": pt[1:].hex()}
    return {"der": der, "tbs": tbs_bytes, "sig_alg": alg_oid, "signature": signature,
            "issuer": der[issuer[1]:issuer[3]], "subject": der[subject[1]:subject[3]], "key": key,
            "ski": ski, "aki": aki}


# ---------------------------------------------------------------- containers
def read_pem_certs(data: bytes):
    out, text = [], data.decode("ascii")
    for blk in text.split("-----BEGIN CERTIFICATE-----")[1:]:
        out.append(base64.b64decode(blk.split("-----END CERTIFICATE-----")[0]))
    return out


def read_jks_certs(data: bytes):
    """Certificates of a Java KeyStore (magic FEEDFEED, version 1/2).  Entry tag 1 =
    private key (u32-length protected blob, skipped unread, then a certificate chain),
    tag 2 = trusted certificate."""
    magic, version, count = struct.unpack_from(">III", data, 0)
    assert magic == 0xFEEDFEED and version in (1, 2), "not a JKS keystore"
    p, out = 12, []

    def utf():
        nonlocal p
        (n,) = struct.unpack_from(">H", data, p)
        s = data[p + 2:p + 2 + n].decode("utf-8", "replace")
        p += 2 + n
        return s

    def cert():
        nonlocal p
        ctype = utf() if version == 2 else "X.509"
        (n,) = struct.unpack_from(">I", data, p)
        c = data[p + 4:p + 4 + n]
        p += 4 + n
        assert ctype == "X.509"
        return c

    for _ in range(count):
        (tag,) = struct.unpack_from(">I", data, p)
        p += 4
        alias = utf()
        p += 8                                   # creation time
        if tag == 1:
            (n,) = struct.unpack_from(">I", data, p)
            p += 4 + n                           # protected private key: skipped, never decoded
            (chain,) = struct.unpack_from(">I", data, p)
            p += 4
            for _ in range(chain):
                out.append((alias, cert()))
        elif tag == 2:
            out.append((alias, cert()))
        else:
            raise ValueError(f"unknown JKS entry tag {tag}")
    return out


def collect(reference: str):
    certs = {}
    for rel in SOURCES:
        path = os.path.join(reference, rel)
        with open(path, "rb") as f:
            data = f.read()
        found = [("pem", c) for c in read_pem_certs(data)] if rel.endswith(".cer") else read_jks_certs(data)
        for alias, der in found:
            h = hashlib.sha256(der).hexdigest()
            certs.setdefault(h, {"cert": parse_cert(der), "sources": []})["sources"].append(f"{rel}#{alias}")
    return certs


def make_rows(certs):
    by_subject = {}
    for h, c in certs.items():
        by_subject.setdefault(c["cert"]["subject"], []).append(c["cert"])
    rows, skipped = [], []
    for h in sorted(certs):
        c = certs[h]["cert"]
        if c["sig_alg"] != OID_ECDSA_SHA256:
            skipped.append((certs[h]["sources"][0], f"signature algorithm {c['sig_alg']}"))
            continue
        issuers = [i for i in by_subject.get(c["issuer"], []) if i["key"] is not None]
        # several certificates share a DN (the node's dev root and config/dev's root are both
        # "Corda Node Root CA" with different keys): the key identifiers decide
        if c["aki"] is not None:
            issuers = [i for i in issuers if i["ski"] == c["aki"]]
        elif c["issuer"] == c["subject"]:
            issuers = [c]
        if not issuers:
            skipped.append((certs[h]["sources"][0], "issuer certificate not in the reference"))
            continue
        for iss in issuers:
            scheme = CURVE_SCHEME.get(iss["key"]["curve_oid"])
            if scheme is None:
                skipped.append((certs[h]["sources"][0], f"issuer curve {iss['key']['curve_oid']}"))
                continue
            # OpenSSL (independent of the oracle) decides a DN-ambiguous pairing: the issuer whose
            # key verifies is the real one; the other pairing is kept as a wrong-key row (REJECT)
            ok = OSSL.ecdsa_verify(scheme, bytes.fromhex(iss["key"]["q"]), c["signature"],
                                   hashlib.sha256(c["tbs"]).digest())
            rows.append({"cls": "ref_cert" if ok else "ref_cert_wrong_issuer", "scheme": scheme, "q": iss["key"]["q"], "msg": c["tbs"].hex(),
                         "sig": c["signature"].hex(), "cert_sha256": h,
                         "self_signed": c["issuer"] == c["subject"], "sources": certs[h]["sources"]})
    return rows, skipped


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "ref_cert_vectors.json"))
    a = ap.parse_args()
    rows, skipped = make_rows(collect(a.reference))
    # expected verdicts: the reference's signer produced certificates that chain (OpenSSL verifies each
    # against its issuer's key), so a true pairing is ACCEPT (0) under Crypto.isValid / doVerify; a
    # same-DN pairing with another curve's or another key's root is REJECT (1, well-formed DER, valid key)
    for r in rows:
        r["is_valid"] = r["do_verify"] = 0 if r["cls"] == "ref_cert" else 1
    assert sum(r["cls"] == "ref_cert" for r in rows) == len({r["cert_sha256"] for r in rows}), \
        "every certificate must pair with exactly one issuer that verifies it"
    with open(a.out, "w") as f:
        json.dump({"generator": "tests/golden/make_ref_cert_vectors.py", "sources": SOURCES,
                   "skipped": [list(s) for s in skipped], "rows": rows}, f, indent=1)
    print(f"{len(rows)} rows ({sum(r['scheme'] == 2 for r in rows)} secp256k1, "
          f"{sum(r['scheme'] == 3 for r in rows)} P-256), {len(skipped)} skipped -> {a.out}")
    for s in skipped:
        print("  skipped:", *s)


if __name__ == "__main__":
    sys.exit(main())
