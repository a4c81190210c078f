"""CompositeKey fulfilment: the oracle restatement against the
reference's CompositeKeyTests semantics, the product mirror's construction rules and
op programs (CPU), and the device evaluation against the fixtures (GPU)."""
from __future__ import annotations

import random

import numpy as np
import pytest

import composite as CK
from corda_amd import composite as C
from corda_amd.crypto import IllegalArgumentException

ALICE, BOB, CHARLIE, DAVE = (bytes([0x30 + i]) * 32 for i in range(4))


def test_oracle_like_reference_tests():
    # CompositeKeyTests.kt:45-82
    assert CK.is_fulfilled_by(ALICE, [ALICE]) and not CK.is_fulfilled_by(ALICE, [CHARLIE])
    a_or_b = CK.Builder().add_keys(ALICE, BOB).build(1)
    assert CK.is_fulfilled_by(a_or_b, [ALICE]) and CK.is_fulfilled_by(a_or_b, [BOB])
    assert not CK.is_fulfilled_by(a_or_b, [CHARLIE])
    a_and_b = CK.Builder().add_keys(ALICE, BOB).build()
    assert not CK.is_fulfilled_by(a_and_b, [ALICE]) and CK.is_fulfilled_by(a_and_b, [ALICE, BOB])
    ab_or_c = CK.Builder().add_keys(a_and_b, CHARLIE).build(1)
    assert CK.is_fulfilled_by(ab_or_c, [ALICE, BOB]) and CK.is_fulfilled_by(ab_or_c, [CHARLIE])
    # tree canonical form (:126-150): one child is the child; order does not matter
    assert CK.Builder().add_keys(ALICE).build() == ALICE
    n1, n2 = CK.Builder().add_keys(ALICE, BOB).build(1), CK.Builder().add_keys(ALICE, BOB).build(2)
    assert not CK.is_fulfilled_by(n2, [ALICE])
    t1 = CK.Builder().add_key(n1, 13).add_key(n2, 27).build()
    t2 = CK.Builder().add_key(n2, 27).add_key(n1, 13).build()
    assert CK._ident(t1) == CK._ident(t2)
    # composite signature verification (:156-174): 2-of-3 and a broken component
    two = CK.Builder().add_keys(ALICE, BOB, CHARLIE).build(2)
    assert not CK.composite_verify(two, [ALICE], True)
    assert CK.composite_verify(two, [ALICE, CHARLIE], True)
    assert not CK.composite_verify(two, [ALICE, BOB], False)


@pytest.mark.parametrize("mod", [CK, C])
def test_construction_constraints_like_reference(mod):
    """CompositeKeyTests.kt:176-215 — every case raises IllegalArgumentException."""
    exc = CK.IllegalArgument if mod is CK else IllegalArgumentException
    B = mod.Builder
    cases = [lambda: B().build(),                                              # no children
             lambda: B().add_key(ALICE, 0),                                     # zero weight
             lambda: B().add_key(ALICE).build(0),
             lambda: B().add_key(ALICE).build(-1),
             lambda: B().add_key(ALICE, 2).add_key(BOB, 2).build(5),            # threshold > total
             lambda: B().add_key(ALICE, 3).build(2),                            # single child, other threshold
             lambda: B().add_key(ALICE, 2**31 - 1).add_key(BOB, 2**31 - 1).build(),  # Int overflow
             lambda: B().add_keys(ALICE, BOB, ALICE).build(),                   # duplicate child
             lambda: B().add_keys(B().add_keys(ALICE, BOB).build(), B().add_keys(BOB, ALICE).build()).build()]
    for f in cases:
        with pytest.raises(exc):
            f()


def test_cycle_detection_like_reference():
    """CompositeKeyTests.kt:218-280: a cycle injected below key3 is found from every
    key above it, not from key2 / key1."""
    k1 = C.Builder().add_keys(ALICE, BOB).build()
    k2 = C.Builder().add_keys(ALICE, k1).build()
    k3 = C.Builder().add_keys(ALICE, k2).build()
    k4 = C.Builder().add_keys(ALICE, k3).build()
    k5 = C.Builder().add_keys(ALICE, k4).build()
    k6 = C.Builder().add_keys(ALICE, k5, k2).build()
    for k in (k1, k2, k3, k4, k5, k6):
        k.check_validity()
    k3.children = k3.children + [(k5, 1)]
    for k in (k3, k4, k5, k6):
        with pytest.raises(IllegalArgumentException):
            k.check_validity()
    k2.check_validity()
    k1.check_validity()


def test_mirror_programs_match_oracle():
    rnd = random.Random(4)
    keys = [bytes([i]) * 32 for i in range(20)]

    def tree(mod, depth, r):
        b = mod.Builder()
        for k in r.sample(keys, r.randint(2, 4)):
            b.add_key(tree(mod, depth - 1, r) if depth and r.random() < 0.3 else k, r.randint(1, 3))
        return b.build(r.randint(1, sum(w for _, w in (b.children if mod is CK else b._children))))
    for t in range(200):
        seed = rnd.random()
        ko, kp = tree(CK, 3, random.Random(seed)), tree(C, 3, random.Random(seed))
        signers = rnd.sample(keys, rnd.randint(0, 8))
        idx = {}
        for i, k in enumerate(signers):
            idx.setdefault(k, i)
        prog = []
        C._program(kp, idx, prog)
        assert prog == CK.program(ko, idx)


def _flat(rows):
    prog, ps, ss, vs = [], [0], [0], []
    for r in rows:
        base = ss[-1]
        prog += [[o[0], o[1] + base if o[0] == 0 and o[1] >= 0 else o[1], o[2], o[3]] for o in r["prog"]]
        ps.append(len(prog))
        ss.append(base + r["n_sig"])
        vs += r["verdicts"]
    return (np.array(prog or [[0, 0, 0, 0]], dtype=np.int32), np.array(ps, dtype=np.uint32),
            np.array(ss, dtype=np.uint32), np.array(vs or [0], dtype=np.uint8), ss[-1])


@pytest.mark.gpu
def test_composite_golden(gpu_ctx, golden_composite):
    from corda_amd._lib import ptr
    prog, ps, ss, vs, n_sig = _flat(golden_composite)
    out = np.zeros(len(golden_composite), dtype=np.uint8)
    gpu_ctx.check(gpu_ctx.lib.cg_composite_eval_batch(gpu_ctx.h, len(golden_composite), ptr(ps), ptr(prog), n_sig,
                                                      ptr(ss), ptr(vs), ptr(out)))
    assert out.tolist() == [r["out"] for r in golden_composite]


@pytest.mark.gpu
def test_composite_mirror_on_device(gpu_ctx):
    """isFulfilledBy / getMissingSignatures / composite signature verify through the
    mirror, against the oracle."""
    a_and_b = C.Builder().add_keys(ALICE, BOB).build()
    ab_or_c = C.Builder().add_keys(a_and_b, CHARLIE).build(1)
    two = C.Builder().add_keys(ALICE, BOB, CHARLIE).build(2)
    q = [(ALICE, [ALICE]), (ALICE, [CHARLIE]), (a_and_b, [ALICE]), (a_and_b, [BOB, ALICE]),
         (ab_or_c, [CHARLIE]), (ab_or_c, [ALICE]), (two, [ALICE, DAVE]), (two, [CHARLIE, BOB])]
    assert C.is_fulfilled_by_batch(gpu_ctx, q) == [True, False, False, True, True, False, False, True]
    assert C.missing_signatures(gpu_ctx, [ALICE, a_and_b, ab_or_c, DAVE], [ALICE, CHARLIE]) == [a_and_b, DAVE]
    qv = [(two, [ALICE, BOB]), (two, [ALICE, BOB]), (two, [ALICE])]
    assert C.composite_verify_batch(gpu_ctx, qv, np.array([0, 0, 0, 1, 0], dtype=np.uint8)) == [True, False, False]
