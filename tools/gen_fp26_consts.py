"""Constants of the radix-2^26 Montgomery field (corda_amd/csrc/cg_fp26.h).

Prints, per curve, the canonical limbs of p, R mod p, R^2 mod p (R = 2^260), b R mod
p, -p^-1 mod 2^26 and (secp256k1) beta R mod p, as C initialisers.  Run:
    python tools/gen_fp26_consts.py
"""

M = (1 << 26) - 1
R = 1 << 260


def limbs(v):
    assert 0 <= v < (1 << 260)
    return [(v >> (26 * i)) & M for i in range(10)]


def words_le(ws):
    return sum(w << (32 * i) for i, w in enumerate(ws))


CURVES = {
    "CurveR1": dict(p=2**256 - 2**224 + 2**192 + 2**96 - 1,
                    b=0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B),
    "CurveK1": dict(p=2**256 - 2**32 - 977, b=7,
                    beta=words_le([0x719501EE, 0xC1396C28, 0x12F58995, 0x9CF04975,
                                   0xAC3434E9, 0x6E64479E, 0x657C0710, 0x7AE96A2B])),
}


def c_init(v):
    return "{" + ", ".join("0x%07X" % x for x in limbs(v)) + "}"


def main():
    for name, c in CURVES.items():
        p = c["p"]
        print(f"// {name}")
        print(f"p      {c_init(p)}")
        print(f"one    {c_init(R % p)}")
        print(f"r2     {c_init(R * R % p)}")
        print(f"b      {c_init(c['b'] * R % p)}")
        print(f"pinv   0x{(-pow(p, -1, 1 << 26)) % (1 << 26):07X}")
        if "beta" in c:
            print(f"beta   {c_init(c['beta'] * R % p)}")


if __name__ == "__main__":
    main()
