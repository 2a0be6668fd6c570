"""CPU checks of the algebra the wavefront-cooperative kernels use, restated per output coefficient exactly as the
device computes it (one coefficient per wave / per half), against the oracle's tower arithmetic
(oracle/bls_oracle.py).  The device kernels themselves are checked on the GPU (tests/test_gpu_percall.py); these
pin the rewritten formulas -- index maps, xi on wrap-around, the linear terms folded into products -- on every
CPU run.

  k_fe_wide (bls_fe_wide.hip): Fp12 product per w-coefficient, Granger-Scott cyclotomic squaring with the
      +-2 terms as products, Frobenius maps with the per-coefficient gamma tables, the hard-part schedule.
  k_miller_wide (bls_wide.hip): f^2 through the FSQ_TERMS table, f * sparse line (l0, l2, l3).
  k_msm_upairs (bls_msm.hip): the MSM's 64 bit-sums as Miller pairs (-2^b G1, U_b) in place of the weighted sum.
"""
import os
import random
import re

from oracle import bls_oracle as O

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
SRC = os.path.join(ROOT, "eth-consensus-specs_amd", "csrc")

P = O.P
XI = O.XI
add, sub, mul, muls, conj = O.f2_add, O.f2_sub, O.f2_mul, O.f2_muls, O.f2_conj


def xi(a):
    return mul(XI, a)


def rnd_f2(r):
    return (r.randrange(P), r.randrange(P))


def rnd_f12(r):
    return O.f12_from_coeffs([rnd_f2(r) for _ in range(6)])


def cyclotomic(r):
    """f^((p^6 - 1)(p^2 + 1)) for a random f: an element of the cyclotomic subgroup."""
    f = rnd_f12(r)
    t = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
    return O.f12_mul(O.f12_frobenius(O.f12_frobenius(t)), t)


# ---- k_fe_wide, per coefficient k ----------------------------------------------------------------------------
def fe_mul(a, b):
    """FeWide::mul: c_k = sum_{i <= k} a_i b_{k-i} + sum_{i > k} a_i (xi b_{k-i+6})."""
    out = []
    for k in range(6):
        acc = O.F2_ZERO
        for i in range(6):
            j = k - i if k - i >= 0 else k - i + 6
            bj = b[j] if i <= k else xi(b[j])
            acc = add(acc, mul(a[i], bj))
        out.append(acc)
    return out


def fe_cyc(a):
    """FeWide::cyc: a0' = a0 (3 a0 - 2) + (3 xi a3) a3,  a3' = a3 (6 a0 + 2),  a2' = a1 (3 a1) + (3 xi a4) a4 - 2 a2,
    a5' = a1 (6 a4) + 2 a5,  a4' = a2 (3 a2) + (3 xi a5) a5 - 2 a4,  a1' = (6 xi a2) a5 + 2 a1."""
    two, mtwo = (2, 0), (P - 2, 0)
    out = [None] * 6
    for k in range(6):
        m = 0 if k in (0, 3) else (1 if k in (2, 5) else 2)
        x, y = a[m], a[m + 3]
        if k == 0:
            v = add(mul(x, sub(muls(x, 3), two)), mul(muls(xi(y), 3), y))
        elif k == 3:
            v = mul(y, add(muls(x, 6), two))
        elif k in (2, 4):
            v = add(add(mul(x, muls(x, 3)), mul(muls(xi(y), 3), y)), mul(a[k], mtwo))
        elif k == 5:
            v = add(mul(x, muls(y, 6)), mul(a[5], two))
        else:
            v = add(mul(muls(xi(x), 6), y), mul(a[1], two))
        out[k] = v
    return out


GAMMA1 = [O.f2_pow(XI, k * (P - 1) // 6) for k in range(6)]
GAMMA2 = [mul(g, conj(g)) for g in GAMMA1]


def fe_frob1(a):
    return [mul(conj(a[k]), GAMMA1[k]) for k in range(6)]


def fe_frob2(a):
    return [mul(a[k], GAMMA2[k]) for k in range(6)]


def fe_conj(a):
    return [a[k] if k % 2 == 0 else O.f2_neg(a[k]) for k in range(6)]


def test_fe_wide_products_and_squaring():
    r = random.Random(0xFE01)
    for _ in range(3):
        a, b = rnd_f12(r), rnd_f12(r)
        assert fe_mul(O.f12_to_coeffs(a), O.f12_to_coeffs(b)) == O.f12_to_coeffs(O.f12_mul(a, b))
        t = cyclotomic(r)
        assert fe_cyc(O.f12_to_coeffs(t)) == O.f12_to_coeffs(O.f12_sqr(t))
        assert fe_frob1(O.f12_to_coeffs(a)) == O.f12_to_coeffs(O.f12_frobenius(a))
        assert fe_frob2(O.f12_to_coeffs(a)) == O.f12_to_coeffs(O.f12_frobenius(O.f12_frobenius(a)))
        assert all(g[1] == 0 for g in GAMMA2)  # gamma2_k real: one Fp constant in both halves


def test_fe_wide_hard_part_schedule():
    """The hard-part schedule of k_fe_wide (bls_fe.h fe_schedule's order) with the per-coefficient operations: the
    result is t^(3 (p^4 - p^2 + 1) / r), i.e. the cube of the oracle's hard part."""
    r = random.Random(0xFE02)
    t = O.f12_to_coeffs(cyclotomic(r))

    def powx(src):  # src^x = conj(src^|x|), x = -X_ABS
        acc = src
        for i in range(62, -1, -1):
            acc = fe_cyc(acc)
            if (O.X_ABS >> i) & 1:
                acc = fe_mul(acc, src)
        return fe_conj(acc)

    b1 = powx(t)
    a = fe_mul(fe_conj(t), b1)  # t^(x-1)
    a = fe_mul(powx(a), fe_conj(a))  # t^((x-1)^2)
    b = fe_mul(fe_frob1(a), powx(a))  # a^(x+p)
    c = fe_mul(fe_mul(powx(powx(b)), fe_frob2(b)), fe_conj(b))  # b^(x^2+p^2-1)
    res = fe_mul(c, fe_mul(fe_cyc(t), t))
    want = O.f12_pow(O.f12_from_coeffs(t), 3 * ((P**4 - P**2 + 1) // O.R))
    assert O.f12_from_coeffs(res) == want


# ---- k_miller_wide f accumulation -----------------------------------------------------------------------------
def fsq_terms():
    with open(os.path.join(SRC, "bls_wide.hip")) as fh:
        text = fh.read()
    body = text[text.index("FSQ_TERMS[6][4][4] = {"):]
    body = body[: body.index("};")]
    quads = [tuple(int(v) for v in q) for q in re.findall(r"\{(\d+), (\d+), (\d+), (\d+)\}", body)]
    assert len(quads) == 24
    return [quads[4 * k: 4 * k + 4] for k in range(6)]


def test_miller_wide_square_and_line():
    r = random.Random(0xFE03)
    terms = fsq_terms()
    for _ in range(3):
        fa = rnd_f12(r)
        f = O.f12_to_coeffs(fa)
        sq = []
        for k in range(6):
            acc = O.F2_ZERO
            for i, j, m, x in terms[k]:
                if not m:
                    continue
                v = muls(f[i], m)
                v = xi(v) if x else v
                acc = add(acc, mul(v, f[j]))
            sq.append(acc)
        assert sq == O.f12_to_coeffs(O.f12_sqr(fa))
        l0, l2, l3 = rnd_f2(r), rnd_f2(r), rnd_f2(r)
        fl = []
        for k in range(6):
            i2, i3 = (k + 4 if k < 2 else k - 2), (k + 3 if k < 3 else k - 3)
            acc = mul(f[k], l0)
            acc = add(acc, mul(xi(f[i2]) if k < 2 else f[i2], l2))
            acc = add(acc, mul(xi(f[i3]) if k < 3 else f[i3], l3))
            fl.append(acc)
        line = O.f12_from_coeffs([l0, O.F2_ZERO, l2, l3, O.F2_ZERO, O.F2_ZERO])
        assert fl == O.f12_to_coeffs(O.f12_mul(fa, line))


# ---- the MSM's bit-sum pairs (bls_msm.hip k_msm_upairs) ------------------------------------------------------
def test_msm_bit_sum_pairs_replace_the_weighted_sum():
    """fav_prepare no longer forms S = sum_b 2^b U_b: the 64 pairs (-2^b G1, U_b) join the batch's Miller loops,
    since prod_b e(-2^b G1, U_b) = e(-G1, sum_b 2^b U_b).  The -2^b G1 are comb entries 256 (b / 8) + 2^(b % 8)
    of the bisection's fixed-base table comb[256 w + d] = d 2^(8 w) (-G1) (bls_bisect.hip).  Checked here on a
    few nonzero bit-sums (identity U_b are skipped pairs) with the oracle's pairing."""
    g = O.hash_to_g2(b"msm bit sums")
    bits = {0: 5, 9: 11, 40: 3, 63: 7}  # b -> U_b = k G
    neg_g1 = O.g1_neg(O.G1_GEN)
    f = O.F12_ONE
    S = None
    for b, k in bits.items():
        comb_index = 256 * (b // 8) + (1 << (b % 8))
        w, d = divmod(comb_index, 256)
        assert d * (1 << (8 * w)) == 1 << b
        f = O.f12_mul(f, O.miller_loop(O.g1_mul(neg_g1, d << (8 * w)), O.g2_mul(g, k)))
        S = O.g2_add(S, O.g2_mul(g, k << b))
    f = O.f12_mul(f, O.miller_loop(O.G1_GEN, S))  # times e(G1, S): the product is 1 iff the decomposition holds
    assert O.final_exponentiation(f) == O.F12_ONE
