"""GPU parity of the key- and signature-object entry points (corda_amd.signatures,
SURVEY §8a row a6): PublicKey.isValid / verify, DigitalSignature.WithKey, TransactionSignature.verify
and Crypto.doVerify(publicKey, transactionSignature), each a loop of the reference call collapsed
into one device batch.  Expected values come from the golden fixtures (verdict codes of the
restated i2p / BC verifiers, tests/golden/make_golden.py) — a loop over them decides what the
reference returns or throws."""
from __future__ import annotations

import numpy as np
import pytest

from corda_amd import crypto
from corda_amd import signatures as S
from corda_amd._lib import ACCEPT, REJECT

pytestmark = pytest.mark.gpu


def _rows(golden_ed25519, golden_ecdsa):
    rows = [(S.PublicKey(4, bytes.fromhex(e["pk"])), bytes.fromhex(e["sig"]), bytes.fromhex(e["msg"]), e)
            for e in golden_ed25519]
    rows += [(S.PublicKey(int(e["scheme"]), bytes.fromhex(e["q"])), bytes.fromhex(e["sig"]), bytes.fromhex(e["msg"]), e)
             for e in golden_ecdsa]
    return rows


def _loop_is_valid(rows):
    """What `for r in rows: r.key.isValid(msg, sig)` does: bools, or the first throwing index."""
    for i, (k, _, _, e) in enumerate(rows):
        if k.is_composite:
            return i, S.IllegalStateException
        if e["is_valid"] not in (ACCEPT, REJECT):
            return i, {2: crypto.SignatureException, 3: crypto.InvalidKeyException}.get(e["is_valid"],
                                                                                       crypto.IllegalArgumentException)
    return None, None


def test_public_key_is_valid_golden(gpu_ctx, golden_ed25519, golden_ecdsa):
    rows = _rows(golden_ed25519, golden_ecdsa)
    ok = [r for r in rows if r[3]["is_valid"] in (ACCEPT, REJECT)]
    got = S.public_key_is_valid_batch(gpu_ctx, [r[0] for r in ok], [r[2] for r in ok], [r[1] for r in ok])
    assert np.array_equal(got, np.array([r[3]["is_valid"] == ACCEPT for r in ok]))
    wk = S.with_key_is_valid_batch(gpu_ctx, [S.WithKey(r[0], r[1]) for r in ok], [r[2] for r in ok])
    assert np.array_equal(wk, got)
    # the full golden list, in order: the loop's first throwing element decides
    i, exc = _loop_is_valid(rows)
    with pytest.raises(exc) as ei:
        S.public_key_is_valid_batch(gpu_ctx, [r[0] for r in rows], [r[2] for r in rows], [r[1] for r in rows])
    assert ei.value.index == i
    # a CompositeKey ahead of every throwing element: IllegalStateException at its index
    comp = ok[:5] + [(S.PublicKey(6, b"\x01" * 40), b"s", b"m", {"is_valid": ACCEPT})] + rows
    with pytest.raises(S.IllegalStateException) as ei:
        S.public_key_is_valid_batch(gpu_ctx, [r[0] for r in comp], [r[2] for r in comp], [r[1] for r in comp])
    assert ei.value.index == 5


def test_public_key_verify_golden(gpu_ctx, golden_ed25519, golden_ecdsa):
    rows = _rows(golden_ed25519, golden_ecdsa)
    good = [r for r in rows if r[3]["do_verify"] == ACCEPT]
    assert S.public_key_verify_batch(gpu_ctx, [r[0] for r in good], [r[2] for r in good], [r[1] for r in good])
    assert S.with_key_verify_batch(gpu_ctx, [S.WithKey(r[0], r[1]) for r in good], [r[2] for r in good])
    bad_at = len(good) // 2
    mixed = good[:bad_at] + [next(r for r in rows if r[3]["do_verify"] == REJECT)] + good[bad_at:]
    with pytest.raises(crypto.SignatureException) as ei:
        S.public_key_verify_batch(gpu_ctx, [r[0] for r in mixed], [r[2] for r in mixed], [r[1] for r in mixed])
    assert ei.value.index == bad_at


def test_transaction_signatures(gpu_ctx, golden_ed25519, golden_ecdsa):
    """The golden message bytes stand in for MetaData.bytes() (the Kryo form the JVM produces)."""
    rows = [r for r in _rows(golden_ed25519, golden_ecdsa) if r[3]["do_verify"] == ACCEPT]
    ts = [S.TransactionSignature(r[1], r[2], r[0]) for r in rows]
    assert S.transaction_signatures_verify(gpu_ctx, ts)
    keys = [r[0] for r in rows]
    assert S.do_verify_transaction_signatures(gpu_ctx, keys, ts)
    # Crypto.kt:498-500: verification runs under the PASSED key.  A signature by key B over
    # metadata naming key A verifies when B is passed (the mismatch exception is never
    # thrown), and fails under A.
    a = next(i for i, r in enumerate(rows) if r[0].scheme_id == 4)
    b = next(i for i, r in enumerate(rows) if r[0].scheme_id == 4 and r[0].encoded != rows[a][0].encoded)
    crossed = S.TransactionSignature(rows[b][1], rows[b][2], rows[a][0])
    assert S.do_verify_transaction_signatures(gpu_ctx, [rows[b][0]], [crossed])
    with pytest.raises(crypto.SignatureException):
        S.transaction_signatures_verify(gpu_ctx, [crossed])
    with pytest.raises(crypto.SignatureException) as ei:
        S.do_verify_transaction_signatures(gpu_ctx, keys[:3] + [rows[a][0]], ts[:3] + [crossed])
    assert ei.value.index == 3
