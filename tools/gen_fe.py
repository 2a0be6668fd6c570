#!/usr/bin/env python3
"""gen_fe -- phase tables of the lane-parallel final exponentiation (build tool).

Emits eth-consensus-specs_amd/csrc/bls_fe_tables.h for k_fe_check
(csrc/bls_fe.hip).  One 64-lane wave holds its Fp12 values in LDS slots (14
radix-2^29 digits, N form: digits 0..12 exact, value below a small multiple of
p) and advances them in *phases*; in one phase every active lane does one of

  PROD  dst = (sum x_t) * (sum y_t) / R      (<= 8 + 8 positive terms, one
                                              Montgomery product, R = 2^406)
  LIN   dst = sum c_t x_t + K p              (<= 16 terms, small signed
                                              coefficients, exact carry chain)

and a barrier separates phases.  Operations (Fp12 product, cyclotomic
squaring, Frobenius maps, conjugation, the pieces of the easy part) are lists
of phases whose slot references are relative to *banks* (A, B, D: the
operand and destination registers, 12 slots each) or absolute (products,
temporaries, constants), so one table serves every call of an operation.

Each lane's descriptor of a phase is NW = 17 u32 words:
  w[0]   dst ref (bits 0..9) | K (bits 10..19) | nx (20..24) | kind (30..31)
  w[1..16] terms, two 16-bit halves per word: ref (bits 0..9) | coef + 32 (10..15)
PROD terms are the nx terms of x, then those of y (coef 1).  A ref is
frame (bits 8..9: 0 absolute, 1 A, 2 B, 3 D) | index (bits 0..7).

The generator simulates every phase on integers (Montgomery semantics) and
tracks worst-case value bounds in units of p: product operands must satisfy
x y < p R (R / p ~ 2^25.3), positive operand sums must fit the u32 digit sums
(<= 8 N-form terms), and LIN offsets K p must cover the negative mass so the
carry chain ends non-negative.  tests/test_fe_tables.py runs the same
simulation against oracle/bls_oracle.py.  Standalone (no oracle import).
"""
from __future__ import annotations

import os
import random

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
RMONT = 1 << 406
RINV = pow(RMONT, -1, P)
X_ABS = 0xD201000000010000
NW = 17          # descriptor words per lane and phase
MAXT = 16        # terms per phase and lane
ABS_BASE = 128   # absolute refs address slots ABS_BASE + index
NBANK = 10       # register banks of 12 slots: slots 0 .. 119
PS, TS, CS = 0, 64, 128  # absolute regions (indices): products, temporaries, constants
ZERO = CS        # constant 0
R_OVER_P = RMONT / P

KIND = {"idle": 0, "prod": 1, "lin": 2, "inv": 3, "lin32": 4}
K32_C = 16  # LIN32 offset: 16 p, digits below the top raised by b 2^29 (b: the lane's subtracted terms)


def ref(frame, idx):
    fr = {"abs": 0, "A": 1, "B": 2, "D": 3}[frame]
    assert 0 <= idx < 256
    return (fr << 8) | idx


def P_(k):  # product slot
    return ref("abs", PS + k)


def T_(k):  # temporary slot
    return ref("abs", TS + k)


def C_(k):  # constant slot
    return ref("abs", CS + k)


def A(j):
    return ref("A", j)


def B(j):
    return ref("B", j)


def D(j):
    return ref("D", j)


# ------------------------------------------------------------------ constants --
def _f2mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _f2pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = _f2mul(r, a)
        a = _f2mul(a, a)
        e >>= 1
    return r


XI = (1, 1)
GAMMA1 = [_f2pow(XI, k * (P - 1) // 6) for k in range(6)]          # (c w^k)^p = conj(c) gamma1_k w^k
GAMMA2 = [_f2mul(GAMMA1[k], (GAMMA1[k][0], (-GAMMA1[k][1]) % P)) for k in range(6)]  # real
assert all(g[1] == 0 for g in GAMMA2)

# constant pool (field values, stored in Montgomery form): 0, 2, frobenius constants
CONSTS = [0, 2, 1]
G1RE, G1IM, G1DIFF = {}, {}, {}
for k in range(1, 6):
    G1RE[k] = len(CONSTS)
    CONSTS.append(GAMMA1[k][0])
    G1IM[k] = len(CONSTS)
    CONSTS.append(GAMMA1[k][1])
    G1DIFF[k] = len(CONSTS)
    CONSTS.append((GAMMA1[k][0] - GAMMA1[k][1]) % P)
G2C = {}
for k in range(1, 6):
    G2C[k] = len(CONSTS)
    CONSTS.append(GAMMA2[k][0])
assert len(CONSTS) <= 32
C_TWO, C_ONE = 1, 2


# w-basis coefficient k (Fp2) of an Fp12 <-> tower slots (j = 6 h + 2 kk + part): c_k = (h = k & 1, kk = k >> 1)
def wslot(k, part):
    return 6 * (k & 1) + 2 * (k >> 1) + part


# ------------------------------------------------------------------- builders --
class Phase:
    def __init__(self, kind, name):
        self.kind, self.name, self.lanes = kind, name, []

    def prod(self, dst, xs, ys):
        assert self.kind == "prod" and len(xs) + len(ys) <= MAXT and xs and ys
        self.lanes.append({"dst": dst, "x": list(xs), "y": list(ys)})

    def lin(self, dst, terms, K=None):
        assert self.kind in ("lin", "lin32")
        terms = [(r, c) for r, c in terms if c]
        assert 0 < len(terms) <= MAXT, (self.name, len(terms))
        self.lanes.append({"dst": dst, "t": terms, "K": K})


def fp2_prod_lanes(ph, dst0, a, b):
    """Karatsuba Fp2 product a * b (a, b: (re_terms, im_terms) lists of refs): products
    t0 = a.re b.re, t1 = a.im b.im, t2 = (a.re + a.im)(b.re + b.im) into dst0 .. dst0 + 2."""
    ph.prod(P_(dst0), a[0], b[0])
    ph.prod(P_(dst0 + 1), a[1], b[1])
    ph.prod(P_(dst0 + 2), a[0] + a[1], b[0] + b[1])


def fp2_from_prods(p0):
    """(re, im) of a Karatsuba Fp2 product as linear forms over product slots."""
    return ({P_(p0): 1, P_(p0 + 1): -1}, {P_(p0 + 2): 1, P_(p0): -1, P_(p0 + 1): -1})


def lf_add(*fs, coef=None):
    out = {}
    for i, f in enumerate(fs):
        c = 1 if coef is None else coef[i]
        for r, v in f.items():
            out[r] = out.get(r, 0) + c * v
    return {r: v for r, v in out.items() if v}


def lf_scale(f, c):
    return {r: v * c for r, v in f.items()}


def f2_xi(z):  # xi (re + im i) = (re - im) + (re + im) i
    return (lf_add(z[0], z[1], coef=[1, -1]), lf_add(z[0], z[1]))


def f2_add(*zs):
    return (lf_add(*[z[0] for z in zs]), lf_add(*[z[1] for z in zs]))


def f2_sub(a, b):
    return (lf_add(a[0], b[0], coef=[1, -1]), lf_add(a[1], b[1], coef=[1, -1]))


def f2_scale(z, c):
    return (lf_scale(z[0], c), lf_scale(z[1], c))


def fp6_prod_lanes(ph, p0, X, Y):
    """Karatsuba Fp6 product X * Y (X, Y: three Fp2 operands, each (re_terms, im_terms)); 18 products from
    p0.  Returns the three Fp2 coefficients as linear forms over the products."""
    pairs = [(X[0], Y[0]), (X[1], Y[1]), (X[2], Y[2]),
             ((X[1][0] + X[2][0], X[1][1] + X[2][1]), (Y[1][0] + Y[2][0], Y[1][1] + Y[2][1])),
             ((X[0][0] + X[1][0], X[0][1] + X[1][1]), (Y[0][0] + Y[1][0], Y[0][1] + Y[1][1])),
             ((X[0][0] + X[2][0], X[0][1] + X[2][1]), (Y[0][0] + Y[2][0], Y[0][1] + Y[2][1]))]
    V = []
    for i, (x, y) in enumerate(pairs):
        fp2_prod_lanes(ph, p0 + 3 * i, x, y)
        V.append(fp2_from_prods(p0 + 3 * i))
    v0, v1, v2, v12, v01, v02 = V
    c0 = f2_add(v0, f2_xi(f2_sub(f2_sub(v12, v1), v2)))
    c1 = f2_add(f2_sub(f2_sub(v01, v0), v1), f2_xi(v2))
    c2 = f2_add(f2_sub(f2_sub(v02, v0), v2), v1)
    return [c0, c1, c2]


def bank_fp6(bank, h):
    """The Fp6 half h of a bank as three Fp2 operands of single refs."""
    return [([bank(6 * h + 2 * k)], [bank(6 * h + 2 * k + 1)]) for k in range(3)]


def bank_fp6_sum(bank):
    return [([bank(2 * k), bank(6 + 2 * k)], [bank(2 * k + 1), bank(6 + 2 * k + 1)]) for k in range(3)]


def store_fp2_lin(ph, dst_re, dst_im, z):
    ph.lin(dst_re, list(z[0].items()))
    ph.lin(dst_im, list(z[1].items()))


# ------------------------------------------------------------------ operations --
def op_mul():
    """D = A * B (Fp12, Karatsuba over Fp6 over Fp2: 54 products), then two LIN phases."""
    pr = Phase("prod", "mul.prod")
    M0 = fp6_prod_lanes(pr, 0, bank_fp6(A, 0), bank_fp6(B, 0))
    M1 = fp6_prod_lanes(pr, 18, bank_fp6(A, 1), bank_fp6(B, 1))
    M2 = fp6_prod_lanes(pr, 36, bank_fp6_sum(A), bank_fp6_sum(B))
    l1 = Phase("lin", "mul.fp6")  # the three Fp6 products into temporaries 0..17
    for m, M in enumerate((M0, M1, M2)):
        for k in range(3):
            store_fp2_lin(l1, T_(6 * m + 2 * k), T_(6 * m + 2 * k + 1), M[k])
    l2 = Phase("lin", "mul.fp12")  # D.c0 = M0 + v M1, D.c1 = M2 - M0 - M1
    t = lambda m, k: ({T_(6 * m + 2 * k): 1}, {T_(6 * m + 2 * k + 1): 1})  # noqa: E731
    c0 = [f2_add(t(0, 0), f2_xi(t(1, 2))), f2_add(t(0, 1), t(1, 0)), f2_add(t(0, 2), t(1, 1))]
    c1 = [f2_sub(f2_sub(t(2, k), t(0, k)), t(1, k)) for k in range(3)]
    for k in range(3):
        store_fp2_lin(l2, D(2 * k), D(2 * k + 1), c0[k])
        store_fp2_lin(l2, D(6 + 2 * k), D(6 + 2 * k + 1), c1[k])
    return [pr, l1, l2]


def op_cyc():
    """D = A^2 for A in the cyclotomic subgroup (Granger-Scott, as zkcrypto's cyclotomic_square and
    tools/wavec.py cyc_sqr): for each pair (a, b) of Fp2 coefficients, (a + b y)^2 = (a^2 + xi b^2) + 2 a b y,
    and z' = 3 c -/+ 2 z.  Every product already carries its coefficient (3 a0^2 = (a0 + a0 + a0) a0,
    6 a0 a1 = (3 a0)(2 a1), 2 z = z * 2), so the LIN phase only adds and subtracts products (u32 digit sums,
    LIN32): 30 + 12 products, at most 6 terms per output."""
    z = {0: (0, 0), 4: (0, 1), 3: (0, 2), 2: (1, 0), 1: (1, 1), 5: (1, 2)}  # z name -> (h, k) of the tower

    def zs(n, part):
        h, k = z[n]
        return 6 * h + 2 * k + part

    pr = Phase("prod", "cyc.prod")
    n = [0]

    def prod(xs, ys):
        pr.prod(P_(n[0]), xs, ys)
        n[0] += 1
        return P_(n[0] - 1)

    out = {}
    for za, zb in ((0, 1), (2, 3), (4, 5)):
        a0, a1, b0, b1 = A(zs(za, 0)), A(zs(za, 1)), A(zs(zb, 0)), A(zs(zb, 1))
        # 3 (a^2 + xi b^2) = 3 (a0^2 - a1^2 + b0^2 - b1^2 - 2 b0 b1) + 3 (2 a0 a1 + b0^2 - b1^2 + 2 b0 b1) i
        sa0, sa1, sb0, sb1 = prod([a0] * 3, [a0]), prod([a1] * 3, [a1]), prod([b0] * 3, [b0]), prod([b1] * 3, [b1])
        sa01, sb01 = prod([a0] * 3, [a1] * 2), prod([b0] * 3, [b1] * 2)
        c0 = ({sa0: 1, sa1: -1, sb0: 1, sb1: -1, sb01: -1}, {sa01: 1, sb0: 1, sb1: -1, sb01: 1})
        # 3 (2 a b) = 6 (a0 b0 - a1 b1) + 6 (a0 b1 + a1 b0) i
        p00, p11, p01, p10 = (prod([a0] * 3, [b0] * 2), prod([a1] * 3, [b1] * 2), prod([a0] * 3, [b1] * 2),
                              prod([a1] * 3, [b0] * 2))
        c1 = ({p00: 1, p11: -1}, {p01: 1, p10: 1})
        out[(za, zb)] = (c0, c1)
    two_z = {}
    for zn in range(6):
        for part in range(2):
            two_z[(zn, part)] = prod([A(zs(zn, part))], [C_(C_TWO)])
    li = Phase("lin32", "cyc.lin")

    def emit(zn, f, sgn):
        for part in range(2):
            li.lin(D(zs(zn, part)), list(f[part].items()) + [(two_z[(zn, part)], sgn)])

    (c00, c01), (c10, c11), (c20, c21) = out[(0, 1)], out[(2, 3)], out[(4, 5)]
    emit(0, c00, -1)
    emit(1, c01, 1)
    emit(4, c10, -1)
    emit(5, c11, 1)
    emit(3, c20, -1)
    emit(2, f2_xi(c21), 1)  # 3 xi c1 + 2 z
    return [pr, li]


def op_conj():
    li = Phase("lin", "conj")
    for j in range(12):
        li.lin(D(j), [(A(j), 1 if j < 6 else -1)])
    return [li]


def op_frob1():
    """D = A^p: w-basis coefficient k -> conj(c_k) gamma1_k, conj(c) g = (c0 g0 + c1 g1, c0 g1 - c1 g0) by
    Karatsuba with (g0 - g1): t0 = c0 g0, t1 = c1 g1, t2 = (c0 + c1)(g0 - g1); re = t0 + t1, im = t0 - t1 - t2."""
    pr = Phase("prod", "frob1.prod")
    li = Phase("lin", "frob1.lin")
    for k in range(6):
        c0, c1 = A(wslot(k, 0)), A(wslot(k, 1))
        if k == 0:
            li.lin(D(wslot(0, 0)), [(c0, 1)])
            li.lin(D(wslot(0, 1)), [(c1, -1)])
            continue
        p = 3 * k
        pr.prod(P_(p), [c0], [C_(G1RE[k])])
        pr.prod(P_(p + 1), [c1], [C_(G1IM[k])])
        pr.prod(P_(p + 2), [c0, c1], [C_(G1DIFF[k])])
        li.lin(D(wslot(k, 0)), [(P_(p), 1), (P_(p + 1), 1)])
        li.lin(D(wslot(k, 1)), [(P_(p), 1), (P_(p + 1), -1), (P_(p + 2), -1)])
    return [pr, li]


def op_frob2():
    """D = A^(p^2): coefficient k times the real gamma2_k (one product per Fp, straight into D; k = 0 by the
    constant 1)."""
    pr = Phase("prod", "frob2.prod")
    for k in range(6):
        for part in range(2):
            pr.prod(D(wslot(k, part)), [A(wslot(k, part))], [C_(C_ONE if k == 0 else G2C[k])])
    return [pr]


def op_easy_front():
    """From f = a + b w in bank A: a^2, b^2, a b (54 products); N = a^2 - v b^2 -> temporaries 0..5,
    conj(f)^2 = (a^2 + v b^2) - 2 a b w -> bank D."""
    pr = Phase("prod", "easy.sq")
    Aa, Ab = bank_fp6(A, 0), bank_fp6(A, 1)
    a2 = fp6_prod_lanes(pr, 0, Aa, Aa)
    b2 = fp6_prod_lanes(pr, 18, Ab, Ab)
    ab = fp6_prod_lanes(pr, 36, Aa, Ab)
    l1 = Phase("lin", "easy.fp6")  # a^2 -> T 0..5, b^2 -> T 6..11, ab -> T 12..17
    for m, M in enumerate((a2, b2, ab)):
        for k in range(3):
            store_fp2_lin(l1, T_(6 * m + 2 * k), T_(6 * m + 2 * k + 1), M[k])
    t = lambda m, k: ({T_(6 * m + 2 * k): 1}, {T_(6 * m + 2 * k + 1): 1})  # noqa: E731
    vb2 = [f2_xi(t(1, 2)), t(1, 0), t(1, 1)]  # v b^2
    l2 = Phase("lin", "easy.split")
    for k in range(3):
        store_fp2_lin(l2, T_(20 + 2 * k), T_(20 + 2 * k + 1), f2_sub(t(0, k), vb2[k]))       # N
        store_fp2_lin(l2, D(2 * k), D(2 * k + 1), f2_add(t(0, k), vb2[k]))                  # conj(f)^2 .c0
        store_fp2_lin(l2, D(6 + 2 * k), D(6 + 2 * k + 1), f2_scale(t(2, k), -2))             # .c1
    return [pr, l1, l2]


def op_easy_inv():
    """N (Fp6, temporaries 20..25) -> N^-1 (temporaries 40..45), with one Fp inversion (kind INV, lane 0:
    temporary 34 -> 35)."""
    N = [([T_(20 + 2 * k)], [T_(21 + 2 * k)]) for k in range(3)]
    p1 = Phase("prod", "inv.p1")  # N0^2, N1^2, N2^2, N1 N2, N0 N1, N0 N2 (Karatsuba, 3 products each)
    pairs = [(N[0], N[0]), (N[1], N[1]), (N[2], N[2]), (N[1], N[2]), (N[0], N[1]), (N[0], N[2])]
    F = []
    for i, (x, y) in enumerate(pairs):
        fp2_prod_lanes(p1, 3 * i, x, y)
        F.append(fp2_from_prods(3 * i))
    n00, n11, n22, n12, n01, n02 = F
    c = [f2_sub(n00, f2_xi(n12)), f2_sub(f2_xi(n22), n01), f2_sub(n11, n02)]
    l1 = Phase("lin", "inv.l1")
    for k in range(3):
        store_fp2_lin(l1, T_(26 + 2 * k), T_(27 + 2 * k), c[k])
    C = [([T_(26 + 2 * k)], [T_(27 + 2 * k)]) for k in range(3)]
    p2 = Phase("prod", "inv.p2")  # det = N0 c0 + xi (N2 c1 + N1 c2)
    for i, (x, y) in enumerate(((N[0], C[0]), (N[2], C[1]), (N[1], C[2]))):
        fp2_prod_lanes(p2, 3 * i, x, y)
    d0, d1, d2 = (fp2_from_prods(3 * i) for i in range(3))
    det = f2_add(d0, f2_xi(f2_add(d1, d2)))
    l2 = Phase("lin", "inv.l2")
    store_fp2_lin(l2, T_(32), T_(33), det)
    p3 = Phase("prod", "inv.p3")  # |det|^2 = re^2 + im^2
    p3.prod(P_(0), [T_(32)], [T_(32)])
    p3.prod(P_(1), [T_(33)], [T_(33)])
    l3 = Phase("lin", "inv.l3")
    l3.lin(T_(34), [(P_(0), 1), (P_(1), 1)])
    inv = Phase("inv", "inv.fp")  # T35 = T34^-1 (lane 0)
    inv.lanes.append({"dst": T_(35), "src": T_(34)})
    p4 = Phase("prod", "inv.p4")  # det^-1 = (re, -im) / |det|^2
    p4.prod(P_(0), [T_(32)], [T_(35)])
    p4.prod(P_(1), [T_(33)], [T_(35)])
    l4 = Phase("lin", "inv.l4")
    l4.lin(T_(36), [(P_(0), 1)])
    l4.lin(T_(37), [(P_(1), -1)])
    p5 = Phase("prod", "inv.p5")  # N^-1 = c det^-1
    di = ([T_(36)], [T_(37)])
    for k in range(3):
        fp2_prod_lanes(p5, 3 * k, C[k], di)
    l5 = Phase("lin", "inv.l5")
    for k in range(3):
        store_fp2_lin(l5, T_(40 + 2 * k), T_(41 + 2 * k), fp2_from_prods(3 * k))
    return [p1, l1, p2, l2, p3, l3, inv, p4, l4, p5, l5]


def op_easy_back():
    """D = A * N^-1 (A: conj(f)^2 in a bank, N^-1 in temporaries 40..45): two Fp6 products."""
    pr = Phase("prod", "easyb.prod")
    Ni = [([T_(40 + 2 * k)], [T_(41 + 2 * k)]) for k in range(3)]
    M0 = fp6_prod_lanes(pr, 0, bank_fp6(A, 0), Ni)
    M1 = fp6_prod_lanes(pr, 18, bank_fp6(A, 1), Ni)
    li = Phase("lin", "easyb.lin")
    for h, M in enumerate((M0, M1)):
        for k in range(3):
            store_fp2_lin(li, D(6 * h + 2 * k), D(6 * h + 2 * k + 1), M[k])
    return [pr, li]


OPS = {"MUL": op_mul, "CYC": op_cyc, "CONJ": op_conj, "FROB1": op_frob1, "FROB2": op_frob2,
       "EASY_FRONT": op_easy_front, "EASY_INV": op_easy_inv, "EASY_BACK": op_easy_back}


# ------------------------------------------------------------------ simulation --
class Sim:
    """Integer model of the LDS slots: value (Montgomery representation, exact integer, not reduced) and a
    worst-case bound in units of p."""

    def __init__(self, grow=False):
        self.val, self.bnd = {}, {}
        self.grow = grow  # first pass: raise each LIN lane's K to cover its negative mass

    def addr(self, r, banks):
        fr, ix = r >> 8, r & 0xFF
        return ABS_BASE + ix if fr == 0 else banks[fr] * 12 + ix

    def get(self, r, banks):
        a = self.addr(r, banks)
        if a == ABS_BASE + ZERO:
            return 0, 0.0
        return self.val[a], self.bnd[a]

    def set(self, r, banks, v, b):
        a = self.addr(r, banks)
        self.val[a], self.bnd[a] = v, b

    def run(self, ph: Phase, banks):
        out = []
        for ln in ph.lanes:
            if ph.kind == "prod":
                xs = [self.get(r, banks) for r in ln["x"]]
                ys = [self.get(r, banks) for r in ln["y"]]
                assert len(xs) <= 8 and len(ys) <= 8, ph.name  # u32 digit sums of N-form terms
                X, Y = sum(v for v, _ in xs), sum(v for v, _ in ys)
                bx, by = sum(b for _, b in xs), sum(b for _, b in ys)
                assert bx * by < R_OVER_P / 4, (ph.name, bx, by)  # x y < p R with margin
                # Montgomery product of the exact values: a result below 2p, congruent to X Y / R
                out.append((ln["dst"], X * Y * RINV % P, 2.0))
            elif ph.kind == "lin32":  # u32 digit sums: coefficients +-1, N-form terms, offset 16 p borrowed by 4
                v, npos, nneg, pos, neg = K32_C * P, 0, 0, 0.0, 0.0
                for r, c in ln["t"]:
                    x, b = self.get(r, banks)
                    assert c in (1, -1), ph.name
                    v += c * x
                    if c > 0:
                        npos, pos = npos + 1, pos + b
                    else:
                        nneg, neg = nneg + 1, neg + b
                # digits: 2^29 per N-form term; the offset (16 p, every digit below the top raised by b 2^29,
                # b = the lane's number of subtracted terms) has digits in [b 2^29, (b + 1) 2^29); its top digit
                # 16 * 13 - b covers the subtrahends' top digits (13.0021 per p of value)
                b = nneg
                assert npos + b + 1 <= 8 and neg * 13.01 + nneg <= 13 * K32_C - b, (ph.name, npos, nneg)
                assert v >= 0
                ln["K"] = b
                out.append((ln["dst"], v, pos + K32_C))
            elif ph.kind == "lin":
                v, pos, neg = 0, 0.0, 0.0
                for r, c in ln["t"]:
                    x, b = self.get(r, banks)
                    v += c * x
                    if c > 0:
                        pos += c * b
                    else:
                        neg += -c * b
                need = int(neg) + 2
                if self.grow:
                    ln["K"] = max(ln["K"] or 0, need)
                K = ln["K"]
                assert K is not None and K >= neg + 1 and K < 1024, (ph.name, K, neg)
                v += K * P
                assert v >= 0
                out.append((ln["dst"], v, pos + K))
            else:  # inv
                x, b = self.get(ln["src"], banks)
                m = x * RINV % P  # field element
                out.append((ln["dst"], pow(m, -1, P) * RMONT % P if m else 0, 1.0))
        for dst, v, b in out:
            self.set(dst, banks, v, b)


BANKS_OF = {}


def build_ops():
    return {name: fn() for name, fn in OPS.items()}


def sim_op(sim, phases, a, b, d):
    banks = {1: a, 2: b, 3: d}
    for ph in phases:
        sim.run(ph, banks)


def load_f12(sim, bank, coeffs_mont):
    for j, v in enumerate(coeffs_mont):
        sim.val[bank * 12 + j] = v
        sim.bnd[bank * 12 + j] = 1.0


def init_consts(sim):
    for i, c in enumerate(CONSTS):
        sim.val[ABS_BASE + CS + i] = c * RMONT % P
        sim.bnd[ABS_BASE + CS + i] = 1.0


# the device schedule of k_fe_check: (op, a, b, d) on banks; POWX expands to its squarings/products
def xabs_bits():
    return [(X_ABS >> i) & 1 for i in range(62, -1, -1)]


def schedule():
    s = [("EASY_FRONT", 0, 0, 2), ("EASY_INV", 0, 0, 0), ("EASY_BACK", 2, 0, 0),
         ("FROB2", 0, 0, 1), ("MUL", 1, 0, 0)]
    # hard part (bls_wave_kernels.hip k_final_check_vm order): result e^3 in bank 1

    def powx(src, dst):  # dst = src^x = conj(src^|x|) (cyclotomic: the inverse is the conjugate)
        out, acc = [], src
        for bit in xabs_bits():  # the 63 bits after the leading one
            out.append(("CYC", acc, 0, dst))
            acc = dst
            if bit:
                out.append(("MUL", dst, src, dst))
        out.append(("CONJ", dst, 0, dst))
        return out

    s += powx(0, 1)                       # R1 = t^x
    s += [("CONJ", 0, 0, 3), ("MUL", 3, 1, 2)]   # R2 = a = t^(x-1)
    s += powx(2, 1)                       # R1 = a^x
    s += [("CONJ", 2, 0, 3), ("MUL", 1, 3, 2)]   # R2 = a^(x-1) = t^((x-1)^2)
    s += powx(2, 1)                       # R1 = a^x
    s += [("FROB1", 2, 0, 3), ("MUL", 3, 1, 3)]  # R3 = b = a^(x+p)
    s += powx(3, 1)                       # R1 = b^x
    s += powx(1, 4)                       # R4 = b^(x^2)
    s += [("FROB2", 3, 0, 5), ("MUL", 4, 5, 1)]  # R1 = b^(x^2 + p^2)
    s += [("CONJ", 3, 0, 4), ("MUL", 1, 4, 1)]   # R1 = c = b^(x^2 + p^2 - 1)
    s += [("CYC", 0, 0, 5), ("MUL", 5, 0, 5)]    # R5 = t^3
    s += [("MUL", 1, 5, 1)]                      # R1 = c t^3 = t^(3 h)
    return s


def check_schedule(ops, seed=5):
    """Two passes of the whole device schedule (partial product of 8 inputs first): the first sets every LIN
    offset K, the second asserts every bound with those K.  Returns the second pass's simulator."""
    for grow in (True, False):
        sim = Sim(grow)
        init_consts(sim)
        rng = random.Random(seed)
        load_f12(sim, 0, [rng.randrange(P) * RMONT % P for _ in range(12)])
        for _ in range(7):  # the product of up to 8 partials: bank 0 *= bank 1
            load_f12(sim, 1, [rng.randrange(P) * RMONT % P for _ in range(12)])
            sim_op(sim, ops["MUL"], 0, 1, 0)
        for name, a, b, d in schedule():
            sim_op(sim, ops[name], a, b, d)
    return sim


# --------------------------------------------------------------------- emission --
def encode(ph: Phase):
    """64 lanes x NW words; PROD x terms at positions [0, nx), y terms at [nx, nx + ny) (phase-uniform nx, ny);
    unused positions (and idle lanes) hold the zero constant with coefficient 0."""
    nx, ny = nterms(ph)
    pad = C_(0) | (32 << 10)  # the zero constant, coefficient 0 (LIN) / + 0 (PROD)
    rows = []
    for lane in range(64):
        w = [0] * NW
        slots = [pad] * MAXT
        if lane < len(ph.lanes):
            ln = ph.lanes[lane]
            if ph.kind == "prod":
                for t, r in enumerate(ln["x"]):
                    slots[t] = r | (33 << 10)
                for t, r in enumerate(ln["y"]):
                    slots[nx + t] = r | (33 << 10)
                w[0] = ln["dst"] | (KIND["prod"] << 29)
            elif ph.kind in ("lin", "lin32"):
                for t, (r, c) in enumerate(ln["t"]):
                    assert -32 <= c < 32 and r < 1024
                    slots[t] = r | ((c + 32) << 10)
                w[0] = ln["dst"] | (ln["K"] << 10) | (KIND[ph.kind] << 29)
            else:
                slots[0] = ln["src"] | (33 << 10)
                w[0] = ln["dst"] | (KIND["inv"] << 29)
        for t in range(MAXT):
            w[1 + t // 2] |= slots[t] << (16 * (t % 2))
        rows.append(w)
    return rows


def nterms(ph: Phase):
    if ph.kind == "prod":
        return max(len(l["x"]) for l in ph.lanes), max(len(l["y"]) for l in ph.lanes)
    if ph.kind in ("lin", "lin32"):
        return max(len(l["t"]) for l in ph.lanes), 0
    return 1, 0


def digits(x):
    return [(x >> (29 * i)) & ((1 << 29) - 1) for i in range(14)]


def emit(path):
    ops = build_ops()
    check_schedule(ops)
    lines = ["// GENERATED by tools/gen_fe.py -- do not edit.",
             "// Phase tables of the lane-parallel final exponentiation (bls_fe.hip): per phase 64 lanes x "
             f"{NW} words.",
             "#pragma once", "#include <stdint.h>", "", "namespace bls {", "",
             f"constexpr int FE_NW = {NW};", f"constexpr int FE_ABS_BASE = {ABS_BASE};",
             f"constexpr int FE_NBANK = {NBANK};", f"constexpr int FE_NSLOT = {ABS_BASE + CS + 32};",
             f"constexpr int FE_NCONST = {len(CONSTS)};", f"constexpr int FE_CS = {CS};",
             f"constexpr int FE_K32_C = {K32_C};",
             "static constexpr uint32_t FE_K32[14] = {" + ", ".join(f"0x{d:08x}u" for d in digits(K32_C * P)) + "};",
             ""]
    # constants in digit form (Montgomery representation, canonical)
    cl = []
    for c in CONSTS:
        cl.append("{" + ", ".join(f"0x{d:08x}u" for d in digits(c * RMONT % P)) + "}")
    lines.append(f"static constexpr uint32_t FE_CONSTS[{len(CONSTS)}][14] = {{\n  " + ",\n  ".join(cl) + "};")
    lines.append("")
    table, index = [], []
    for name, phases in ops.items():
        for i, ph in enumerate(phases):
            nx, ny = nterms(ph)
            index.append((name, i, len(table) // (64 * NW), ph.kind, nx, ny, ph.name))
            for row in encode(ph):
                table += row
    lines.append(f"// {len(index)} phases")
    for name, i, off, kind, nx, ny, pname in index:
        lines.append(f"constexpr int FE_PH_{name}_{i} = {off};  // {pname}: {kind}, terms {nx}/{ny}")
    lines.append("")
    for name, i, off, kind, nx, ny, pname in index:
        lines.append(f"constexpr int FE_KIND_{name}_{i} = {KIND[kind]}, FE_NT_{name}_{i} = {nx}, "
                     f"FE_NY_{name}_{i} = {ny};")
    lines.append("")
    lines.append(f"static constexpr uint32_t FE_DESC[{len(table)}] = {{")
    for k in range(0, len(table), 8):
        lines.append("  " + ", ".join(f"0x{v:08x}u" for v in table[k:k + 8]) + ",")
    lines.append("};")
    lines.append("")
    lines.append("}  // namespace bls")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return index


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    idx = emit(os.path.join(root, "eth-consensus-specs_amd", "csrc", "bls_fe_tables.h"))
    for row in idx:
        print(row)
