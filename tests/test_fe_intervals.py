"""Interval proof of the limb bounds of the Ed25519 field / group code.

cg_fe25519.h computes a product as ten chains of signed 32 x 32 -> 64-bit mads with
prescaled operands (19 g_j, 2 f_i, ...) that must stay within int32, column sums
that must stay within int64, and either rounding or floor carries (cg_ge25519.h
picks one per product).  Random inputs cannot show that the bounds hold for every
input, so this test runs an interval analysis over the exact operation sequences
of cg_ge25519.h / cg_ed25519.h — the decode (ge_frombytes_i2p), the lane and key
table builders, the B table builder, the balanced and key-reuse MSM loops as a
state machine over which operation produced the running p1p1 point — and checks
every prescale and every partial column sum for ALL limb values the preceding
operations can produce.  A product's output range depends only on its carry mode
(and, for limb 1, on the column bound), so the state machine reaches a fixed point
after a few rounds.

The model mirrors the C++ operation by operation; if cg_ge25519.h changes, this file
changes with it (the -DCG_CHECK_BOUNDS host build in test_native_host.py is the
empirical cross-check on real data).
"""
import itertools

W = [26 if k % 2 == 0 else 25 for k in range(10)]
P_LIMBS = [(1 << 26) - 19] + [(1 << w) - 1 for w in W[1:]]
I32 = (-(1 << 31), (1 << 31) - 1)
I64 = 1 << 63


def const(limbs):
    return [(v, v) for v in limbs]


def canon(x):
    """canonical limbs of an integer < 2^255 (constants d2, sqrt(-1), 1)"""
    out, s = [], 0
    for w in W:
        out.append((x >> s) & ((1 << w) - 1))
        s += w
    return const(out)


P = 2 ** 255 - 19
D = (-121665 * pow(121666, P - 2, P)) % P
D_L = canon(D)
D2 = canon(2 * D % P)
SQRTM1 = canon(pow(2, (P - 1) // 4, P))
ONE = canon(1)
ZERO = canon(0)
F_RANGE = [(0, (1 << w) - 1) for w in W]  # frombytes output (masked limbs)


def iv_add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def iv_neg(a):
    return (-a[1], -a[0])


def iv_mul(a, b):
    c = [a[0] * b[0], a[0] * b[1], a[1] * b[0], a[1] * b[1]]
    return (min(c), max(c))


def iv_union(a, b):
    return (min(a[0], b[0]), max(a[1], b[1]))


def fe_add(f, g):
    return [iv_add(a, b) for a, b in zip(f, g)]


def fe_sub(f, g):
    return [iv_add(a, iv_neg(b)) for a, b in zip(f, g)]


def fe_add_p(f, g):
    return [iv_add(iv_add(a, b), (-p, -p)) for a, b, p in zip(f, g, P_LIMBS)]


def fe_neg_p(f):
    return [iv_add((p, p), iv_neg(a)) for a, p in zip(f, P_LIMBS)]


def fe_select(f, g):
    return [iv_union(a, b) for a, b in zip(f, g)]


def fe_cneg(f):
    return [iv_union(a, iv_neg(a)) for a in f]


def fe_union(f, g):
    return fe_select(f, g)


class Checker:
    def __init__(self):
        self.max_col = 0
        self.max_g = 0
        self.max_f = 0
        self.n = 0

    def scale(self, iv, m, g_side, what):
        r = iv_mul(iv, (m, m))
        assert I32[0] <= r[0] and r[1] <= I32[1], f"{what}: prescale x{m} of {iv} leaves int32"
        mag = max(abs(iv[0]), abs(iv[1]))
        if g_side:
            self.max_g = max(self.max_g, mag)
        else:
            self.max_f = max(self.max_f, mag)
        return r

    def chain(self, terms_of, floor, what):
        """terms_of(k) -> list of term intervals of column k; returns output limbs"""
        self.n += 1
        c = (0, 0)
        r = []
        c9 = None
        for k in range(10):
            acc = c
            for t in terms_of(k):
                acc = iv_add(acc, t)
                m = max(abs(acc[0]), abs(acc[1]))
                self.max_col = max(self.max_col, m)
                assert m < I64, f"{what}: column {k} partial sum 2^{m.bit_length()} leaves int64"
            w = W[k]
            if floor:
                c = (acc[0] >> w, acc[1] >> w)
                r.append((0, (1 << w) - 1))
            else:
                h = 1 << (w - 1)
                c = ((acc[0] + h) >> w, (acc[1] + h) >> w)
                r.append((-h, h - 1))
        t0 = iv_add(r[0], iv_mul(c, (19, 19)))
        if floor:
            cc = (t0[0] >> 26, t0[1] >> 26)
            r[0] = (0, (1 << 26) - 1)
        else:
            cc = ((t0[0] + (1 << 25)) >> 26, (t0[1] + (1 << 25)) >> 26)
            r[0] = (-(1 << 25), (1 << 25) - 1)
        r[1] = iv_add(r[1], cc)
        for v in r:
            assert I32[0] <= v[0] and v[1] <= I32[1]
        return r

    def mul(self, f, g, floor, scale=1, what="mul"):
        fa = [self.scale(f[i], scale, False, what) for i in range(10)]
        f2 = [self.scale(f[i], 2 * scale, False, what) if i % 2 else fa[i] for i in range(10)]
        g19 = [self.scale(g[j], 19, True, what) for j in range(10)]

        def terms(k):
            out = []
            for i in range(10):
                j = (k - i) % 10
                a = f2[i] if j % 2 else fa[i]
                b = g19[j] if i + j >= 10 else g[j]
                out.append(iv_mul(a, b))
            return out
        return self.chain(terms, floor, what)

    def sq(self, f, floor, scale=1, what="sq"):
        f19 = {j: self.scale(f[j], 19, True, what) for j in range(5, 10)}
        fm = {}
        for i in range(10):
            fm[(i, 1)] = f[i]
            fm[(i, 2)] = self.scale(f[i], 2, False, what)
            if i % 2 or scale == 2:
                fm[(i, 4)] = self.scale(f[i], 4, False, what)
            if i % 2 and scale == 2:
                fm[(i, 8)] = self.scale(f[i], 8, False, what)

        def terms(k):
            out = []
            for i in range(10):
                for j in range(i, 10):
                    if (i + j) % 10 != k:
                        continue
                    m = (1 if i == j else 2) * (2 if (i % 2 and j % 2) else 1) * scale
                    b = f19[j] if i + j >= 10 else f[j]
                    out.append(iv_mul(fm[(i, m)], b))
            return out
        return self.chain(terms, floor, what)


# --- cg_ge25519.h, operation by operation ------------------------------------------

def to_p2(C, p):
    X, Y, Z, T = p
    return (C.mul(X, T, True, what="to_p2 X"), C.mul(Y, Z, True, what="to_p2 Y"), C.mul(Z, T, True, what="to_p2 Z"))


def to_p3(C, p, z_round=False):
    X, Y, Z, T = p
    return (C.mul(X, T, True, what="to_p3 X"), C.mul(Z, Y, True, what="to_p3 Y"),
            C.mul(Z, T, not z_round, what="to_p3 Z"), C.mul(X, Y, True, what="to_p3 T"))


def p3_to_cached(C, p):
    X, Y, Z, T = p
    return (fe_add_p(Y, X), fe_sub(Y, X), Z, C.mul(T, D2, True, what="p3_to_cached T2d"))


def p1p1_to_cached(C, p):
    X, Y, Z, T = p
    x3 = C.mul(X, T, True, what="to_cached x3")
    y3 = C.mul(Z, Y, True, what="to_cached y3")
    dx = C.mul(X, D2, True, what="to_cached dx")
    z3 = C.mul(Z, T, True, what="to_cached z3")
    t2d = C.mul(dx, Y, True, what="to_cached t2d")
    return (fe_add_p(y3, x3), fe_sub(y3, x3), z3, t2d)


def dbl(C, p2, add_ready):
    X, Y, Z = p2
    s = fe_add_p(X, Y)
    xx = C.sq(X, True, what="dbl XX")
    yy = C.sq(Y, True, what="dbl YY")
    zz2 = C.sq(Z, False, scale=2, what="dbl 2ZZ")
    ss = C.sq(s, True, what="dbl S^2")
    H = fe_add_p(yy, xx) if add_ready else fe_add(yy, xx)
    G = fe_sub(yy, xx)
    return (fe_sub(ss, H), H, G, fe_sub(zz2, G))


def add_cached(C, p3, q):
    X, Y, Z, T = p3
    YpX, YmX, Zq, T2d = q
    qa = fe_select(YpX, YmX)
    qb = fe_select(YmX, YpX)
    t2d = fe_cneg(T2d)
    a = fe_add(Y, X)
    b = fe_sub(Y, X)
    A = C.mul(a, qa, True, what="add A")
    B = C.mul(b, qb, True, what="add B")
    Cc = C.mul(t2d, T, True, what="add C")
    D2v = C.mul(Z, Zq, True, scale=2, what="add D2")
    return (fe_sub(A, B), fe_add_p(A, B), fe_add_p(D2v, Cc), fe_sub(D2v, Cc))


def madd(C, p3, q):
    X, Y, Z, T = p3
    ypx, ymx, xy2d = q
    qa = fe_select(ypx, ymx)
    qb = fe_select(ymx, ypx)
    xy = fe_cneg(xy2d)
    a = fe_add(Y, X)
    b = fe_sub(Y, X)
    A = C.mul(a, qa, True, what="madd A")
    B = C.mul(b, qb, True, what="madd B")
    Cc = C.mul(xy, T, False, what="madd C")
    D2v = fe_add(Z, Z)
    return (fe_sub(A, B), fe_add_p(A, B), fe_add(D2v, Cc), fe_sub(D2v, Cc))


def fe_reduce_range():
    """cg_fe25519.h fe_reduce output for inputs well inside int32 (B table entries)"""
    r = [(-(1 << (w - 1)), (1 << (w - 1)) - 1) for w in W]
    r[1] = (r[1][0] - 1, r[1][1] + 1)
    return r


def pow_chain(C, z):
    """fe_pow2_250_1 / fe_pow22523 / fe_invert: floor squarings and products of
    reduced values; the output range is that of one floor product."""
    a = C.sq(z, True, what="pow sq")
    a = C.sq(a, True, what="pow sq")
    m = C.mul(a, z, True, what="pow mul")
    m2 = C.mul(m, m, True, what="pow mul")
    return fe_union(m, m2)


def decode(C):
    """ge_frombytes_i2p(_pair): the p3 point it returns"""
    Y = F_RANGE
    u = C.sq(Y, True, what="decode u")
    v = C.mul(u, D_L, True, what="decode v")
    u = fe_sub(u, ONE)
    v = fe_add(v, ONE)
    v3 = C.mul(C.sq(v, True), v, True, what="decode v3")
    x = C.mul(C.mul(C.sq(v3, True), v, True), u, True, what="decode uv7")
    x = pow_chain(C, x)
    x = C.mul(C.mul(x, v3, True), u, True, what="decode x")
    vxx = C.mul(C.sq(x, True), v, True, what="decode vxx")
    for chk in (fe_sub(vxx, u), fe_add(vxx, u)):  # fe_iszero inputs
        assert all(abs(a) < 1 << 29 and abs(b) < 1 << 29 for a, b in chk)
    xi = C.mul(x, SQRTM1, True, what="decode x sqrt(-1)")
    x = fe_union(x, xi)
    X = fe_select(x, fe_neg_p(x))
    T = C.mul(X, Y, True, what="decode T")
    return (X, Y, ONE, T)


def negate_p3(p):
    X, Y, Z, T = p
    return (fe_neg_p(X), Y, Z, fe_neg_p(T))


IDENTITY_P1P1 = (ZERO, ONE, ONE, ONE)
IDENTITY_P3 = (ZERO, ONE, ONE, ZERO)
IDENTITY_CACHED = (ONE, ONE, ONE, ZERO)


def p3_union(a, b):
    return tuple(fe_union(x, y) for x, y in zip(a, b))


def lane_table(C, P3):
    """ed25519_build_table: entries 0..8 of a decoded point (or -A); returns the
    union of the entries' ranges"""
    c = p3_to_cached(C, P3)
    tab = p3_union(IDENTITY_CACHED, c)
    for _ in range(7):
        t = add_cached(C, P3, c)
        c = p1p1_to_cached(C, t)
        tab = p3_union(tab, c)
    return tab


def dbl64(C, P3):
    """ge_p3_dbl64 (the key-reuse path's per-key tables, the four-lane latency mode's
    high-half points): 63 x (p2_dbl<false> + to_p2) from the point's (X, Y, Z), then
    p2_dbl<true> + to_p3"""
    q = P3[:3]
    for _ in range(3):  # ranges settle after one round; iterate for the fixed point
        q = p3_union(q, to_p2(C, dbl(C, q, False)))
    return p3_union(P3, to_p3(C, dbl(C, q, True)))


def key_tables(C, P3):
    """ed25519_key_tables: -A, then ge_p3_dbl64 between the four tables"""
    P = negate_p3(P3)
    tab = lane_table(C, P)
    for _ in range(3):
        P = p3_union(P, dbl64(C, P))
        tab = p3_union(tab, lane_table(C, P))
    return tab


def btab_entry(C):
    """ed25519_btab_entry: left-to-right double-and-add of k * 2^(64 t) B; the entry
    itself is affine and passed through fe_reduce"""
    P = decode(C)
    for _ in range(3):
        P = p3_union(P, to_p3(C, dbl(C, P[:3], True)))
    pc = p3_to_cached(C, P)
    R = (ZERO, ONE, ONE, ZERO)
    for _ in range(3):
        R = p3_union(R, to_p3(C, dbl(C, R[:3], True)))
        R = p3_union(R, to_p3(C, add_cached(C, R, pc)))
    recip = pow_chain(C, R[2])
    ax = C.mul(R[0], recip, False, what="btab ax")
    ay = C.mul(R[1], recip, False, what="btab ay")
    xy2d = C.mul(C.mul(ax, ay, False), D2, False, what="btab xy2d")
    for v in (fe_add(ay, ax), fe_sub(ay, ax)):  # fe_reduce inputs
        assert all(abs(a) < 1 << 29 and abs(b) < 1 << 29 for a, b in v)
    return (fe_reduce_range(), fe_reduce_range(), xy2d)


def msm_states(C, tab_a, tab_r, btab, rounds=4):
    """The MSM loops (balanced and key-reuse) as transitions between the producers of
    the running p1p1 point t:
        ID    identity start
        DBL0  ge_p2_dbl<false>   (after ge_p1p1_to_p2 of DBL0/DBL1/ADD/MADD)
        DBL1  ge_p2_dbl<true>    (same inputs; the additions follow)
        ADD   ge_add_cached      (after ge_p1p1_to_p3 of ID/DBL1/ADD)
        MADD  ge_madd            (after ge_p1p1_to_p3<true> of ADD/MADD)"""
    st = {"ID": IDENTITY_P1P1}
    tab = p3_union(tab_a, tab_r)

    def union_of(names):
        vals = [st[n] for n in names if n in st]
        out = vals[0]
        for v in vals[1:]:
            out = p3_union(out, v)
        return out

    for _ in range(rounds):
        new = dict(st)
        src = union_of(["DBL0", "DBL1", "ADD", "MADD"]) if any(n in st for n in ("DBL0", "DBL1", "ADD", "MADD")) else None
        if src is not None:
            p2 = to_p2(C, src)
            new["DBL0"] = dbl(C, p2, False)
            new["DBL1"] = dbl(C, p2, True)
        new["ADD"] = p3_union(add_cached(C, to_p3(C, union_of(["ID", "DBL1", "ADD"])), tab),
                              add_cached(C, IDENTITY_P3, tab))  # first window: the constant identity
        if "ADD" in st:
            new["MADD"] = madd(C, to_p3(C, union_of(["ADD", "MADD"]), z_round=True), btab)
        for k, v in new.items():
            st[k] = p3_union(st[k], v) if k in st else v
    # the verdict: fe_iszero(X), fe_iszero(Y - T) of any final p1p1
    for v in st.values():
        for fe in (v[0], fe_sub(v[1], v[3])):
            assert all(abs(a) < 1 << 29 and abs(b) < 1 << 29 for a, b in fe)
    return st


def pair_combine(C, st):
    """ed25519_pair_combine (latency mode): each lane's partial sum — the output of its
    last addition (ADD or MADD: ed25519_msm_lane ends every window with one) — to p3,
    the partner's p3 to cached, one cached addition, the identity test."""
    src = p3_union(st["ADD"], st["MADD"])
    own = to_p3(C, src)
    s = add_cached(C, own, p3_to_cached(C, own))
    for fe in (s[0], fe_sub(s[1], s[3])):
        assert all(abs(a) < 1 << 29 and abs(b) < 1 << 29 for a, b in fe)


def lanes_combine(C, st, levels):
    """The four- / eight-lane combine: ed25519_lane_sum with lanes q ^ 1 (, q ^ 2) (each
    output, a cached addition's p1p1, is the next level's input), then
    ed25519_pair_combine; `levels` = the lane sums before it (1 or 2)."""
    src = p3_union(st["ADD"], st["MADD"])
    for _ in range(levels):
        own = to_p3(C, src)
        src = p3_union(src, add_cached(C, own, p3_to_cached(C, own)))
    own2 = to_p3(C, src)
    s = add_cached(C, own2, p3_to_cached(C, own2))
    for fe in (s[0], fe_sub(s[1], s[3])):
        assert all(abs(a) < 1 << 29 and abs(b) < 1 << 29 for a, b in fe)


def test_limb_bounds_hold_for_all_inputs():
    C = Checker()
    A = decode(C)
    R = decode(C)
    tab_a = lane_table(C, negate_p3(A))
    tab_r = lane_table(C, R)
    tab_k = key_tables(C, A)  # (covers 2^64 (-A) of the four-lane mode too)
    tab_r64 = lane_table(C, dbl64(C, R))  # (any 2^n R of the latency mode's parts: the same fixed point)
    btab = btab_entry(C)
    # the balanced and key-reuse loops; the latency mode's lanes (ed25519_msm_lane) run
    # a subset of the same transitions (no ADD -> ADD), so their states are covered too
    st = msm_states(C, p3_union(tab_a, tab_k), p3_union(tab_r, tab_r64), btab)
    pair_combine(C, st)
    lanes_combine(C, st, 1)
    lanes_combine(C, st, 2)
    # 19-scaled operands within int32 (|g| <= 113025455 = 1.684 * 2^26), f sides below
    # 2^28, columns below 2^62 (int64 has a factor 2 of headroom on top)
    assert C.max_g <= (2 ** 31 - 1) // 19
    assert C.max_f < 1 << 28
    assert C.max_col < 1 << 62, C.max_col.bit_length()
    assert C.n > 100


def test_checker_catches_an_uncorrected_sum():
    """Negative control: without the fe_add_p correction, the doubling's S = X + Y of
    two floor-reduced values overflows the 19 x prescale — the analysis must say so."""
    C = Checker()
    X = [(0, (1 << w) - 1) for w in W]
    try:
        C.sq(fe_add(X, X), True)
    except AssertionError as e:
        assert "leaves int32" in str(e)
    else:
        raise AssertionError("the uncorrected sum was not flagged")
    C.sq(fe_add_p(X, X), True)  # corrected: fine


def test_interval_arithmetic_matches_products():
    """The interval product / carry model against exact integer chains on random
    extreme limb vectors drawn from the analysed ranges."""
    import random
    rnd = random.Random(3)
    C = Checker()
    rng = [(-(1 << 26), 1 << 26) if k % 2 == 0 else (-(1 << 25), 1 << 25) for k in range(10)]
    out_f = C.mul(rng, rng, True)
    out_r = C.mul(rng, rng, False)
    for _ in range(300):
        f = [rnd.choice([lo, hi, rnd.randint(lo, hi)]) for lo, hi in rng]
        g = [rnd.choice([lo, hi, rnd.randint(lo, hi)]) for lo, hi in rng]
        for floor, out in ((True, out_f), (False, out_r)):
            limbs = _exact_mul(f, g, floor)
            for v, (lo, hi) in zip(limbs, out):
                assert lo <= v <= hi
            assert _value(limbs) % P == _value(f) * _value(g) % P


def _value(limbs):
    s, v = 0, 0
    for x, w in zip(limbs, W):
        v += x << s
        s += w
    return v


def _exact_mul(f, g, floor):
    cols = [0] * 10
    for i, j in itertools.product(range(10), range(10)):
        m = 2 if (i % 2 and j % 2) else 1
        cols[(i + j) % 10] += f[i] * g[j] * m * (19 if i + j >= 10 else 1)
    c, r = 0, []
    for k in range(10):
        a = cols[k] + c
        w = W[k]
        c = a >> w if floor else (a + (1 << (w - 1))) >> w
        r.append(a - (c << w))
    t0 = r[0] + 19 * c
    cc = t0 >> 26 if floor else (t0 + (1 << 25)) >> 26
    r[0] = t0 - (cc << 26)
    r[1] += cc
    return r
