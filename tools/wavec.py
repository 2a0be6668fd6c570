#!/usr/bin/env python3
"""wavec -- compile extension-field / curve formulas into wave programs (build tool).

A *wave program* is a straight-line program over Fp whose only non-linear
operation is the Montgomery product.  The formulas (Fp12 multiplication,
cyclotomic squaring runs, Miller-loop steps, complete projective point
arithmetic on E1 / E2, ...) are written once below against a symbolic Fp;
tracing them yields a DAG of products whose operands are small-integer
linear combinations of earlier values.  Products are levelled (ASAP) so
every product of a level is independent: on the device a 64-lane workgroup
executes one level per step for G items at once (bls_vm.h), lane work
index k -> (op j = k / G, item g = k % G).

Op kinds (2 bits in the destination word):
  0 lin  dest = reduce(sum c_t x_t)
  1 mul  dest = (sum a_t x_t) * (sum b_t y_t)      (Montgomery product)
  2 sel  dest = pred[g] & 1 ? reduce(A) : reduce(B)
  3 lut  dest = slot[frame][ix + pred[g] * stride]  (per-item table lookup)

Frames: frame k < 15 of a program is a contiguous run of per-item Fp slots
whose base the kernel passes at run time; the program's last frame is its
private scratch.  Frame 15 is the global constant pool (WP_CONST_POOL),
shared by all items and loaded into LDS once per workgroup.

Output: eth-consensus-specs_amd/csrc/bls_waveprog.h (constant tables).
This module is standalone (no oracle import); tests/test_wavec.py checks the
traced formulas numerically against the oracle with a Python model of the
device interpreter.
"""
from __future__ import annotations

import os
from collections import defaultdict

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
X_ABS = 0xD201000000010000
CONST_FRAME = 15
KIND = {"lin": 0, "mul": 1, "sel": 2, "lut": 3}

# --------------------------------------------------------------------------
# symbolic Fp: a linear form over "atoms"
# --------------------------------------------------------------------------


class Ctx:
    def __init__(self):
        self.atoms = []  # ('in', fr, ix) | ('const', v) | ('prod', fa, fb) | ('lin', f) | ('sel', fa, fb) | ('lut', fr, ix, stride)
        self.consts = {}

    def atom(self, desc):
        self.atoms.append(desc)
        return len(self.atoms) - 1


class V:
    __slots__ = ("c", "f")

    def __init__(self, c, f):
        self.c = c
        self.f = {k: v for k, v in f.items() if v}

    def __add__(self, o):
        f = dict(self.f)
        for k, v in o.f.items():
            f[k] = f.get(k, 0) + v
        return V(self.c, f)

    def __sub__(self, o):
        f = dict(self.f)
        for k, v in o.f.items():
            f[k] = f.get(k, 0) - v
        return V(self.c, f)

    def __neg__(self):
        return V(self.c, {k: -v for k, v in self.f.items()})

    def smul(self, k: int):
        return V(self.c, {a: v * k for a, v in self.f.items()})

    def __mul__(self, o):
        if isinstance(o, int):
            return self.smul(o)
        if not self.f or not o.f:
            return V(self.c, {})
        a = self.c.atom(("prod", dict(self.f), dict(o.f)))
        return V(self.c, {a: 1})

    __rmul__ = smul

    def is_zero(self):
        return not self.f


def inp(c, frame, idx):
    return V(c, {c.atom(("in", frame, idx)): 1})


def const(c, value):
    value %= P
    if value == 0:
        return V(c, {})
    if value not in c.consts:
        c.consts[value] = c.atom(("const", value))
    return V(c, {c.consts[value]: 1})


def zero(c):
    return V(c, {})


def mat(v: V) -> V:
    """Materialise a linear form as a reduced slot value (a 'lin' op)."""
    if len(v.f) == 1 and list(v.f.values())[0] == 1:
        return v
    return V(v.c, {v.c.atom(("lin", dict(v.f))): 1})


def mat12(a):
    co = [mat(x) for x in a.coeffs()]
    w = [F2(co[2 * k], co[2 * k + 1]) for k in range(6)]
    return F12(F6(w[0], w[2], w[4]), F6(w[1], w[3], w[5]))


def sel(c, a: V, b: V) -> V:
    """pred ? a : b  (per item)."""
    return V(c, {c.atom(("sel", dict(a.f), dict(b.f))): 1})


def lut(c, frame, idx, stride) -> V:
    return V(c, {c.atom(("lut", frame, idx, stride)): 1})


# --------------------------------------------------------------------------
# tower formulas (same algorithms as bls_tower.h / bls_pairing.h)
# --------------------------------------------------------------------------


class F2:
    def __init__(self, a, b):
        self.a, self.b = a, b

    def __add__(s, o):
        return F2(s.a + o.a, s.b + o.b)

    def __sub__(s, o):
        return F2(s.a - o.a, s.b - o.b)

    def __neg__(s):
        return F2(-s.a, -s.b)

    def smul(s, k):
        return F2(s.a.smul(k), s.b.smul(k))

    def __mul__(s, o):
        if isinstance(o, int):
            return s.smul(o)
        if isinstance(o, V):  # Fp2 x Fp
            return F2(s.a * o, s.b * o)
        if s.b.is_zero() and o.b.is_zero():
            return F2(s.a * o.a, s.b)
        if o.b.is_zero():
            return F2(s.a * o.a, s.b * o.a)
        if s.b.is_zero():
            return F2(o.a * s.a, o.b * s.a)
        if o.a.is_zero():  # (a + b i)(d i) = -b d + a d i
            return F2(-(s.b * o.b), s.a * o.b)
        t0 = s.a * o.a
        t1 = s.b * o.b
        t2 = (s.a + s.b) * (o.a + o.b)
        return F2(t0 - t1, t2 - t0 - t1)

    def sqr(s):
        t0 = (s.a + s.b) * (s.a - s.b)
        t1 = s.a * s.b
        return F2(t0, t1.smul(2))

    def mul_xi(s):
        return F2(s.a - s.b, s.a + s.b)

    def conj(s):
        return F2(s.a, -s.b)

    def is_zero(s):
        return s.a.is_zero() and s.b.is_zero()


def f2c(c, v):
    """Fp2 constant from a (c0, c1) tuple of ints."""
    return F2(const(c, v[0]), const(c, v[1]))


class F6:
    def __init__(self, c0, c1, c2):
        self.c = (c0, c1, c2)

    def __add__(s, o):
        return F6(*(x + y for x, y in zip(s.c, o.c)))

    def __sub__(s, o):
        return F6(*(x - y for x, y in zip(s.c, o.c)))

    def __neg__(s):
        return F6(*(-x for x in s.c))

    def smul(s, k):
        return F6(*(x.smul(k) for x in s.c))

    def __mul__(s, o):
        a0, a1, a2 = s.c
        b0, b1, b2 = o.c
        t0, t1, t2 = a0 * b0, a1 * b1, a2 * b2
        c0 = ((a1 + a2) * (b1 + b2) - t1 - t2).mul_xi() + t0
        c1 = (a0 + a1) * (b0 + b1) - t0 - t1 + t2.mul_xi()
        c2 = (a0 + a2) * (b0 + b2) - t0 - t2 + t1
        return F6(c0, c1, c2)

    def sqr(s):  # Chung-Hasan SQR2
        a0, a1, a2 = s.c
        s0 = a0.sqr()
        s1 = (a0 * a1).smul(2)
        s2 = (a0 - a1 + a2).sqr()
        s3 = (a1 * a2).smul(2)
        s4 = a2.sqr()
        return F6(s0 + s3.mul_xi(), s1 + s4.mul_xi(), s1 + s2 + s3 - s0 - s4)

    def mul_v(s):
        return F6(s.c[2].mul_xi(), s.c[0], s.c[1])

    def mul_f2(s, k):
        return F6(*(x * k for x in s.c))

    def mul_01(s, b0, b1):
        a0, a1, a2 = s.c
        t0, t1 = a0 * b0, a1 * b1
        return F6(t0 + (a2 * b1).mul_xi(), (a0 + a1) * (b0 + b1) - t0 - t1, t1 + a2 * b0)

    def mul_1(s, b1):
        a0, a1, a2 = s.c
        return F6((a2 * b1).mul_xi(), a0 * b1, a1 * b1)


class F12:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def __mul__(s, o):
        t0 = s.c0 * o.c0
        t1 = s.c1 * o.c1
        c1 = (s.c0 + s.c1) * (o.c0 + o.c1) - t0 - t1
        return F12(t0 + t1.mul_v(), c1)

    def sqr(s):
        t = s.c0 * s.c1
        c0 = (s.c0 + s.c1) * (s.c0 + s.c1.mul_v()) - t - t.mul_v()
        return F12(c0, t.smul(2))

    def cyc_sqr(s):
        """Granger-Scott squaring, valid in the cyclotomic subgroup: 6 Fp2 products."""
        z0, z4, z3 = s.c0.c
        z2, z1, z5 = s.c1.c

        def fp4_sqr(a, b):  # (a + b y)^2, y^2 = xi
            t = a * b
            return (a + b) * (a + b.mul_xi()) - t - t.mul_xi(), t.smul(2)

        t0, t1 = fp4_sqr(z0, z1)
        t2, t3 = fp4_sqr(z2, z3)
        t4, t5 = fp4_sqr(z4, z5)
        z0 = t0.smul(3) - z0.smul(2)
        z1 = t1.smul(3) + z1.smul(2)
        z2 = t5.mul_xi().smul(3) + z2.smul(2)
        z3 = t4.smul(3) - z3.smul(2)
        z4 = t2.smul(3) - z4.smul(2)
        z5 = t3.smul(3) + z5.smul(2)
        return F12(F6(z0, z4, z3), F6(z2, z1, z5))

    def conj(s):
        return F12(s.c0, -s.c1)

    def mul_line(s, l0, l2, l3):
        t0 = s.c0.mul_01(l0, l2)
        t1 = s.c1.mul_1(l3)
        x = (s.c0 + s.c1).mul_01(l0, l2 + l3)
        return F12(t0 + t1.mul_v(), x - t0 - t1)

    def coeffs(s):
        # w-basis order c0..c5 -> Fp list (c0.a, c0.b, c1.a, ...)
        w = [s.c0.c[0], s.c1.c[0], s.c0.c[1], s.c1.c[1], s.c0.c[2], s.c1.c[2]]
        out = []
        for x in w:
            out += [x.a, x.b]
        return out


def f12_from_frame(c, frame):
    v = [inp(c, frame, i) for i in range(12)]
    w = [F2(v[2 * k], v[2 * k + 1]) for k in range(6)]
    return F12(F6(w[0], w[2], w[4]), F6(w[1], w[3], w[5]))


def f2_from_frame(c, frame, off):
    return F2(inp(c, frame, off), inp(c, frame, off + 1))


# --------------------------------------------------------------------------
# field constants (computed here so the tool stays standalone)
# --------------------------------------------------------------------------


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


def _f2inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * n % P, (-a[1]) * n % P)


XI = (1, 1)
PSI_CX = _f2inv(_f2pow(XI, (P - 1) // 3))
PSI_CY = _f2inv(_f2pow(XI, (P - 1) // 2))
GAMMA1 = [_f2pow(XI, k * (P - 1) // 6) for k in range(6)]
GAMMA2 = [_f2mul(_f2pow(XI, k * (P - 1) // 6), _f2pow(XI, k * (P - 1) // 6 * P)) for k in range(6)]
B2_3 = (12, 12)  # 3 * b for E2: b = 4(1 + i)
B1_3 = 12        # 3 * b for E1: b = 4
# 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3), coefficients c0 + c1 i
ISO_XNUM = [
    (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    (0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO_XDEN = [
    (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    (0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    (1, 0),
]
ISO_YNUM = [
    (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
     0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    (0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO_YDEN = [
    (0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    (0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    (1, 0),
]

# --------------------------------------------------------------------------
# complete projective point arithmetic on y^2 = x^3 + b (a = 0):
# Renes-Costello-Batina 2016, algorithms 7 (add), 8 (mixed add), 9 (double).
# Exception-free: the identity is (0 : 1 : 0) and every input is handled, so
# a wave program needs no branches.  Works over Fp (E1) and Fp2 (E2); b3 =
# 3b enters only linearly (12 and 12(1+i)).
# --------------------------------------------------------------------------


def _mulb3(t, b3):
    if isinstance(t, F2):  # 12(1+i) * (a + b i) = 12(a - b) + 12(a + b) i
        return F2((t.a - t.b).smul(b3[0]), (t.a + t.b).smul(b3[0]))
    return t.smul(b3)


def rcb_add(P1, P2, b3):
    X1, Y1, Z1 = P1
    X2, Y2, Z2 = P2
    t0, t1, t2 = X1 * X2, Y1 * Y2, Z1 * Z2
    t3 = (X1 + Y1) * (X2 + Y2) - t0 - t1
    t4 = (Y1 + Z1) * (Y2 + Z2) - t1 - t2
    y3 = (X1 + Z1) * (X2 + Z2) - t0 - t2
    t0 = t0.smul(3)
    t2 = _mulb3(t2, b3)
    z3 = t1 + t2
    t1 = t1 - t2
    y3 = _mulb3(y3, b3)
    X3 = t3 * t1 - t4 * y3
    Y3 = t1 * z3 + y3 * t0
    Z3 = z3 * t4 + t0 * t3
    return (X3, Y3, Z3)


def rcb_add_aff(P1, Q, b3):
    """P1 projective + Q affine (Q must not be the identity)."""
    X1, Y1, Z1 = P1
    X2, Y2 = Q
    t0, t1 = X1 * X2, Y1 * Y2
    t3 = (X1 + Y1) * (X2 + Y2) - t0 - t1
    t4 = Y2 * Z1 + Y1
    y3 = X2 * Z1 + X1
    t0 = t0.smul(3)
    t2 = _mulb3(Z1, b3)
    z3 = t1 + t2
    t1 = t1 - t2
    y3 = _mulb3(y3, b3)
    X3 = t3 * t1 - t4 * y3
    Y3 = t1 * z3 + y3 * t0
    Z3 = z3 * t4 + t0 * t3
    return (X3, Y3, Z3)


def rcb_dbl(P1, b3):
    X, Y, Z = P1
    t0 = Y.sqr() if isinstance(Y, F2) else Y * Y
    t1 = Y * Z
    t2 = _mulb3(Z.sqr() if isinstance(Z, F2) else Z * Z, b3)
    u = X * Y
    z8 = t0.smul(8)
    X3a = t2 * z8
    Z3 = t1 * z8
    w = t0 - t2.smul(3)
    Y3 = w * (t0 + t2) + X3a
    X3 = (w * u).smul(2)
    return (X3, Y3, Z3)


def pt_from_frame(c, frame, off, ext):
    if ext:
        return tuple(f2_from_frame(c, frame, off + 2 * k) for k in range(3))
    return tuple(inp(c, frame, off + k) for k in range(3))


def pt_out(pt):
    out = []
    for v in pt:
        out += [v.a, v.b] if isinstance(v, F2) else [v]
    return out


def g2_psi_proj(c, pt):
    X, Y, Z = pt
    return (X.conj() * f2c(c, PSI_CX), Y.conj() * f2c(c, PSI_CY), Z.conj())


def g2_psi2_proj(c, pt):
    cx = _f2mul(PSI_CX, (PSI_CX[0], (-PSI_CX[1]) % P))
    cy = _f2mul(PSI_CY, (PSI_CY[0], (-PSI_CY[1]) % P))
    X, Y, Z = pt
    return (X * f2c(c, cx), Y * f2c(c, cy), Z)


def neg_pt(pt):
    return (pt[0], -pt[1], pt[2])


def xabs_runs():
    """Square-and-multiply schedule of |x| after the leading bit: list of
    (doublings, add_after)."""
    runs, k = [], 0
    for i in range(62, -1, -1):
        k += 1
        if (X_ABS >> i) & 1:
            runs.append((k, True))
            k = 0
    if k:
        runs.append((k, False))
    return runs


# --------------------------------------------------------------------------
# programs
# --------------------------------------------------------------------------


def prog_fp12_mul(c):
    a = f12_from_frame(c, 0)
    b = f12_from_frame(c, 1)
    return {2: (a * b).coeffs()}


def prog_fp12_sqr(c):
    a = f12_from_frame(c, 0)
    return {1: a.sqr().coeffs()}


CYC_MAT = 1


def make_cyc_run(k, mul):
    """frame 0: a, frame 1: base (multiplier), frame 2: out = a^(2^k) [* base]."""

    def prog(c):
        a = f12_from_frame(c, 0)
        for j in range(k):
            a = a.cyc_sqr()
            # materialise every CYC_MAT squarings (and before the product):
            # in between, the next squaring's operands are short linear
            # forms of the previous products
            if (j + 1 < k and (j + 1) % CYC_MAT == 0) or (j + 1 == k and mul):
                a = mat12(a)
        if mul:
            a = a * f12_from_frame(c, 1)
        return {2: a.coeffs()}

    return prog


def prog_fp12_frob(n):
    """frame 0: a, frame 1: out = a^(p^n): w-basis coefficient k becomes
    conj^n(c_k) * xi^(k (p^n - 1) / 6)."""

    def prog(c):
        v = [inp(c, 0, i) for i in range(12)]
        out = []
        for k in range(6):
            x = F2(v[2 * k], v[2 * k + 1])
            if n % 2 == 1:
                x = x.conj()
            g = _f2pow(XI, k * (P ** n - 1) // 6)
            if g != (1, 0):
                x = x * f2c(c, g)
            out += [x.a, x.b]
        return {1: out}

    return prog


def _ml_line_dbl(c, T, nxP, yP):
    X, Y, Z = T
    A = X.sqr()
    B = Y.sqr()
    C = B.sqr()
    D = ((X + B).sqr() - A - C).smul(2)
    E = A.smul(3)
    Fv = E.sqr()
    ZZ = Z.sqr()
    l0 = E * X - B.smul(2)
    l2 = (E * ZZ) * nxP
    z3 = (Y + Z).sqr() - B - ZZ
    l3 = (z3 * ZZ) * yP
    x3 = Fv - D.smul(2)
    y3 = E * (D - x3) - C.smul(8)
    return (x3, y3, z3), (l0, l2, l3)


def _ml_line_add(c, T, xQ, yQ, nxP, yP):
    X, Y, Z = T
    z1z1 = Z.sqr()
    u2 = xQ * z1z1
    s2 = (yQ * Z) * z1z1
    h = u2 - X
    hh = h.sqr()
    i = hh.smul(4)
    j = h * i
    r = (s2 - Y).smul(2)
    v = X * i
    x3 = r.sqr() - j - v.smul(2)
    y3 = r * (v - x3) - (Y * j).smul(2)
    z3 = (Z + h).sqr() - z1z1 - hh
    l0 = r * xQ - yQ * z3
    l2 = r * nxP
    l3 = z3 * yP
    return (x3, y3, z3), (l0, l2, l3)


def _pair_frames(c):
    # frame 0: f (12 Fp); frame 1: T (X,Y,Z as 6 Fp); frame 2: P: (-xP, yP); frame 3: Q: (xQ, yQ) 4 Fp
    f = f12_from_frame(c, 0)
    T = (f2_from_frame(c, 1, 0), f2_from_frame(c, 1, 2), f2_from_frame(c, 1, 4))
    nxP, yP = inp(c, 2, 0), inp(c, 2, 1)
    xQ, yQ = f2_from_frame(c, 3, 0), f2_from_frame(c, 3, 2)
    return f, T, nxP, yP, xQ, yQ


def _t_out(T):
    out = []
    for x in T:
        out += [x.a, x.b]
    return out


def prog_ml_dbl(c):
    """f <- f^2 * l_{T,T}(P); T <- 2T."""
    f, T, nxP, yP, xQ, yQ = _pair_frames(c)
    T2, (l0, l2, l3) = _ml_line_dbl(c, T, nxP, yP)
    f2 = f.sqr().mul_line(l0, l2, l3)
    return {0: f2.coeffs(), 1: _t_out(T2)}


def prog_ml_dbl_first(c):
    """First step (f = 1): f <- l_{T,T}(P); T <- 2T."""
    f, T, nxP, yP, xQ, yQ = _pair_frames(c)
    T2, (l0, l2, l3) = _ml_line_dbl(c, T, nxP, yP)
    z = zero(c)
    Z2 = F2(z, z)
    line = F12(F6(l0, l2, Z2), F6(Z2, l3, Z2))
    return {0: line.coeffs(), 1: _t_out(T2)}


def make_ml_shared(K, step):
    """K pairs sharing one Miller accumulator f.  frame 0: f (12); frame
    1 + 3k, 2 + 3k, 3 + 3k: T_k (6), P_k = (-xP, yP) (2), Q_k (4).
    step 'dbl':   f <- f^2 * prod_k l_{T_k,T_k}(P_k),  T_k <- 2 T_k
    step 'first': f <- prod_k l_{T_k,T_k}(P_k)  (f = 1 before)
    step 'add':   f <- f * prod_k l_{T_k,Q_k}(P_k),   T_k <- T_k + Q_k"""

    def prog(c):
        f = f12_from_frame(c, 0)
        outs = {}
        lines = []
        for k in range(K):
            T = (f2_from_frame(c, 1 + 3 * k, 0), f2_from_frame(c, 1 + 3 * k, 2), f2_from_frame(c, 1 + 3 * k, 4))
            nxP, yP = inp(c, 2 + 3 * k, 0), inp(c, 2 + 3 * k, 1)
            xQ, yQ = f2_from_frame(c, 3 + 3 * k, 0), f2_from_frame(c, 3 + 3 * k, 2)
            if step == "add":
                T2, ln = _ml_line_add(c, T, xQ, yQ, nxP, yP)
            else:
                T2, ln = _ml_line_dbl(c, T, nxP, yP)
            outs[1 + 3 * k] = _t_out(T2)
            lines.append(ln)
        if step == "first":
            z = zero(c)
            Z2 = F2(z, z)
            l0, l2, l3 = lines[0]
            acc = F12(F6(l0, l2, Z2), F6(Z2, l3, Z2))
            rest = lines[1:]
        else:
            acc = f.sqr() if step == "dbl" else f
            rest = lines
        for l0, l2, l3 in rest:
            acc = acc.mul_line(l0, l2, l3)
        outs[0] = acc.coeffs()
        return outs

    return prog


def prog_ml_add(c):
    """f <- f * l_{T,Q}(P); T <- T + Q."""
    f, T, nxP, yP, xQ, yQ = _pair_frames(c)
    T2, (l0, l2, l3) = _ml_line_add(c, T, xQ, yQ, nxP, yP)
    return {0: f.mul_line(l0, l2, l3).coeffs(), 1: _t_out(T2)}


# ---- curve programs (projective, complete) -------------------------------


def make_xmul_run(ext, k, add):
    """frame 0: R (projective), frame 1: base (projective), frame 2: out = [2^k] R (+ base)."""
    b3 = B2_3 if ext else B1_3

    def prog(c):
        R = pt_from_frame(c, 0, 0, ext)
        for _ in range(k):
            R = rcb_dbl(R, b3)
        if add:
            R = rcb_add(R, pt_from_frame(c, 1, 0, ext), b3)
        return {2: pt_out(R)}

    return prog


def make_pt_add(ext):
    """frame 0: A, frame 1: B, frame 2: out = A + B (projective)."""
    b3 = B2_3 if ext else B1_3

    def prog(c):
        return {2: pt_out(rcb_add(pt_from_frame(c, 0, 0, ext), pt_from_frame(c, 1, 0, ext), b3))}

    return prog


def make_dbl_add_sel(ext):
    """Double-and-always-add step with a per-item select:
    frame 0: R (projective, updated in place), frame 1: Q (affine x, y);
    R <- pred ? 2R + Q : 2R."""
    b3 = B2_3 if ext else B1_3

    def prog(c):
        R = pt_from_frame(c, 0, 0, ext)
        if ext:
            Q = (f2_from_frame(c, 1, 0), f2_from_frame(c, 1, 2))
        else:
            Q = (inp(c, 1, 0), inp(c, 1, 1))
        D = rcb_dbl(R, b3)
        S = rcb_add_aff(D, Q, b3)
        outs = [sel(c, s, d) for s, d in zip(pt_out(S), pt_out(D))]
        return {0: outs}

    return prog


def prog_g2_aff_to_proj_psi_check(c):
    """Subgroup check inputs/outputs for sigma: frame 0: sigma affine (x, y);
    frame 1: M = [|x|] sigma (projective).  Output frame 2: the three values
    X_psi Z_M - X_M Z_psi, Y_psi Z_M + Y_M Z_psi (Fp2 each) and Z_M; sigma
    is in G2 iff psi(sigma) == -M, i.e. the first two are zero and Z_M != 0."""
    S = (f2_from_frame(c, 0, 0), f2_from_frame(c, 0, 2), F2(const(c, 1), zero(c)))
    Xp, Yp, Zp = g2_psi_proj(c, S)
    M = pt_from_frame(c, 1, 0, True)
    dx = Xp * M[2] - M[0] * Zp
    dy = Yp * M[2] + M[1] * Zp
    return {2: [dx.a, dx.b, dy.a, dy.b, M[2].a, M[2].b]}


def prog_iso_pair(c):
    """3-isogeny of the two SSWU outputs and their sum on E2.
    frame 0: (x0, y0, x1, y1) affine on E2' (8 Fp); frame 1: out projective
    Q = iso(P0) + iso(P1) (6 Fp)."""
    pts = []
    for k in range(2):
        x, y = f2_from_frame(c, 0, 4 * k), f2_from_frame(c, 0, 4 * k + 2)
        xx = x.sqr()
        xxx = xx * x

        def poly(coefs, has_x3_one=False):
            acc = f2c(c, coefs[0])
            terms = [x, xx, xxx]
            for j in range(1, len(coefs)):
                if coefs[j] == (1, 0):
                    acc = acc + terms[j - 1]
                elif coefs[j] != (0, 0):
                    acc = acc + terms[j - 1] * f2c(c, coefs[j])
            return acc

        xnum, xden, ynum, yden = poly(ISO_XNUM), poly(ISO_XDEN), poly(ISO_YNUM), poly(ISO_YDEN)
        # (xnum/xden, y ynum/yden) -> projective (xnum yden : y ynum xden : xden yden)
        pts.append((xnum * yden, (y * ynum) * xden, xden * yden))
    z0, z1 = pts[0][2], pts[1][2]
    return {1: pt_out(rcb_add(pts[0], pts[1], B2_3)), 2: [z0.a, z0.b, z1.a, z1.b]}


def prog_clear_pre(c):
    """Cofactor clearing, part 1 (Budroni-Pintore).  frame 0: P; frame 1:
    M1 = [|x|] P.  Outputs frame 2: A = t1 + psi(P) where t1 = -M1 (the
    input of the second [|x|] multiplication) and frame 3: C = psi^2(2P) -
    psi(P) - t1 - P  (so h_eff P = C - [|x|] A)."""
    Pp = pt_from_frame(c, 0, 0, True)
    M1 = pt_from_frame(c, 1, 0, True)
    t1 = neg_pt(M1)
    t2 = g2_psi_proj(c, Pp)
    t3 = g2_psi2_proj(c, rcb_dbl(Pp, B2_3))
    A = rcb_add(t1, t2, B2_3)
    Cc = rcb_add(rcb_add(t3, neg_pt(t2), B2_3), rcb_add(M1, neg_pt(Pp), B2_3), B2_3)
    return {2: pt_out(A), 3: pt_out(Cc)}


def prog_clear_post(c):
    """frame 0: C, frame 1: M2 = [|x|] A; out frame 2: C - M2."""
    return {2: pt_out(rcb_add(pt_from_frame(c, 0, 0, True), neg_pt(pt_from_frame(c, 1, 0, True)), B2_3))}


def prog_proj_to_aff2(c):
    """frame 0: projective (X, Y, Z) over Fp2, frame 1: zi = 1/Z (Fp2);
    out frame 2: (x, y) affine."""
    X, Y, Z = pt_from_frame(c, 0, 0, True)
    zi = f2_from_frame(c, 1, 0)
    x, y = X * zi, Y * zi
    return {2: [x.a, x.b, y.a, y.b]}


def prog_proj_to_aff1(c):
    X, Y, Z = pt_from_frame(c, 0, 0, False)
    zi = inp(c, 1, 0)
    return {2: [X * zi, Y * zi]}


def prog_fp2_norm(c):
    """frame 0: a (Fp2); out frame 1: a0^2 + a1^2 (Fp)."""
    a = f2_from_frame(c, 0, 0)
    return {1: [a.a * a.a + a.b * a.b]}


def prog_fp2_inv_finish(c):
    """frame 0: a (Fp2), frame 1: n = 1/norm(a); out frame 2: a^-1 = conj(a) n."""
    a = f2_from_frame(c, 0, 0)
    n = inp(c, 1, 0)
    return {2: [a.a * n, -(a.b * n)]}


def make_sig_step(mode):
    """One bit step of the two per-item signature-side chains of an FAV item:
      frame 0: sigma affine (x, y)          frame 1: apk projective (X : Y : Z)
      frame 2: M (projective, [|x|] sigma chain)
      frame 3: R (G1 projective, r * apk)
    R <- pred ? 2R + apk : 2R (pred = bit of the item's RLC scalar);
    M <- 2M (mode 1), 2M + sigma (mode 2), unchanged (mode 0, the leading
    bit).  sum r_i sigma_i is a batch MSM (bls_msm.hip)."""

    def prog(c):
        sig = (f2_from_frame(c, 0, 0), f2_from_frame(c, 0, 2))
        apk = pt_from_frame(c, 1, 0, False)  # projective: no inversion after the gather
        out = {}
        if mode:
            M = rcb_dbl(pt_from_frame(c, 2, 0, True), B2_3)
            if mode == 2:
                M = rcb_add_aff(M, sig, B2_3)
            out[2] = pt_out(M)
        R = pt_from_frame(c, 3, 0, False)
        D = rcb_dbl(R, B1_3)
        A = rcb_add(D, apk, B1_3)
        out[3] = [sel(c, a, d) for a, d in zip(pt_out(A), pt_out(D))]
        return out

    return prog


def prog_g2_add_aff_sel(c):
    """MSM bucket step: frame 0: R (projective), frame 1: Q (affine);
    R <- pred ? R + Q : R."""
    R = pt_from_frame(c, 0, 0, True)
    Q = (f2_from_frame(c, 1, 0), f2_from_frame(c, 1, 2))
    S = rcb_add_aff(R, Q, B2_3)
    return {0: [sel(c, a, b) for a, b in zip(pt_out(S), pt_out(R))]}


def prog_runsum(c):
    """MSM window reduction step: frame 0: T, frame 1: S, frame 2: B (all
    projective); T <- T + B, S <- S + T  (visiting buckets d = 255 .. 1 gives
    S = sum d B_d)."""
    T = rcb_add(pt_from_frame(c, 0, 0, True), pt_from_frame(c, 2, 0, True), B2_3)
    S = rcb_add(pt_from_frame(c, 1, 0, True), T, B2_3)
    return {0: pt_out(T), 1: pt_out(S)}


def prog_g2_proj_to_jac(c):
    """frame 0: (X : Y : Z) homogeneous; out frame 1: Jacobian (X Z, Y Z^2, Z)."""
    X, Y, Z = pt_from_frame(c, 0, 0, True)
    return {1: pt_out((X * Z, Y * Z.sqr(), Z))}


X_RUNS = xabs_runs()

PROGRAMS = {
    # name: (builder, frame sizes (excluding scratch))
    "FP12_MUL": (prog_fp12_mul, [12, 12, 12], {2: 0}),
    "FP12_SQR": (prog_fp12_sqr, [12, 12]),
    "FP12_FROB1": (prog_fp12_frob(1), [12, 12]),
    "FP12_FROB2": (prog_fp12_frob(2), [12, 12]),
    "ML_DBL": (prog_ml_dbl, [12, 6, 2, 4]),
    "ML_DBL_FIRST": (prog_ml_dbl_first, [12, 6, 2, 4]),
    "ML_ADD": (prog_ml_add, [12, 6, 2, 4]),
    **{f"ML{_K}_{_st.upper()}": (make_ml_shared(_K, _st), [12] + [6, 2, 4] * _K)
       for _K in (2,) for _st in ("dbl", "first", "add")},
    "G2_ADD": (make_pt_add(True), [6, 6, 6]),
    "G1_ADD": (make_pt_add(False), [3, 3, 3]),
    "G1_DAS": (make_dbl_add_sel(False), [3, 2]),
    "G2_DAS": (make_dbl_add_sel(True), [6, 4]),
    "G2_SUBCHK": (prog_g2_aff_to_proj_psi_check, [4, 6, 6]),
    "ISO_PAIR": (prog_iso_pair, [8, 6, 4]),
    "CLEAR_PRE": (prog_clear_pre, [6, 6, 6, 6]),
    "CLEAR_POST": (prog_clear_post, [6, 6, 6]),
    "G2_TOAFF": (prog_proj_to_aff2, [6, 2, 4]),
    "G1_TOAFF": (prog_proj_to_aff1, [3, 1, 2]),
    "FP2_NORM": (prog_fp2_norm, [2, 1]),
    "FP2_INVFIN": (prog_fp2_inv_finish, [2, 1, 2]),
    "SIG_STEP0": (make_sig_step(0), [4, 3, 6, 3]),
    "SIG_STEP1": (make_sig_step(1), [4, 3, 6, 3]),
    "SIG_STEP2": (make_sig_step(2), [4, 3, 6, 3]),
    "G2_ADDAFF_SEL": (prog_g2_add_aff_sel, [6, 4]),
    "RUNSUM": (prog_runsum, [6, 6, 6]),
    "G2X_8A": (make_xmul_run(True, 8, True), [6, 6, 6], {2: 0}),
    **{f"G2P_{k}": (make_xmul_run(True, k, True), [6, 6, 6]) for k in (1, 2, 4, 8, 16, 32)},
    "G2_PROJ2JAC": (prog_g2_proj_to_jac, [6, 6]),
}
for _k, _add in X_RUNS:
    # the output frame may alias the running value (in-place runs)
    PROGRAMS[f"CYC_{_k}{'M' if _add else ''}"] = (make_cyc_run(_k, _add), [12, 12, 12], {2: 0})
    PROGRAMS[f"G2X_{_k}{'A' if _add else ''}"] = (make_xmul_run(True, _k, _add), [6, 6, 6], {2: 0})

# --------------------------------------------------------------------------
# compiler: level scheduling, slot assignment, table emission
# --------------------------------------------------------------------------
MAX_TERMS = 12  # per operand (after splitting)
MAX_COEF = 127
MAX_MAG = 190  # sum of |coefficients| per accumulated form (the 256 p offset bounds it)
SPLIT = 12  # linear combinations longer than this are summed as a tree of partial sums
CONST_POOL: dict = {}  # canonical value -> pool index (shared by all programs)


def _pool_index(v):
    if v not in CONST_POOL:
        CONST_POOL[v] = len(CONST_POOL)
    return CONST_POOL[v]


def compile_program(name, builder, frames, alias=None, schedule="asap"):
    alias = alias or {}

    def canon(key):
        return (alias.get(key[0], key[0]), key[1])

    c = Ctx()
    outputs = builder(c)  # {frame: [V...]}
    scratch_frame = len(frames)
    assert scratch_frame < CONST_FRAME
    out_list = [(fr, i, v.f) for fr, vs in outputs.items() for i, v in enumerate(vs)]

    def deps(a):
        d = c.atoms[a]
        if d[0] in ("prod", "sel"):
            return list(d[1]) + list(d[2])
        if d[0] == "lin":
            return list(d[1])
        return []

    need = set()
    stack = [a for _, _, f in out_list for a in f]
    while stack:
        a = stack.pop()
        if a in need:
            continue
        need.add(a)
        stack += deps(a)

    def chunked(items):
        chunks, cur, mag = [], [], 0
        for a, k in items:
            if cur and (len(cur) >= SPLIT or mag + abs(k) > MAX_MAG):
                chunks.append(dict(cur))
                cur, mag = [], 0
            cur.append((a, k))
            mag += abs(k)
        if cur:
            chunks.append(dict(cur))
        return chunks

    def shrink(form):
        items = sorted(form.items())
        while len(items) > SPLIT or sum(abs(k) for _, k in items) > MAX_MAG:
            chunks = chunked(items)
            items = []
            for ch in chunks:
                if len(ch) == 1:
                    items += list(ch.items())
                else:
                    a = c.atom(("lin", ch))
                    need.add(a)
                    items.append((a, 1))
        return dict(items)

    for a in sorted(a for a in need if c.atoms[a][0] in ("prod", "sel", "lin")):
        if c.atoms[a][0] == "lin":
            c.atoms[a] = ("lin", shrink(c.atoms[a][1]))
        else:
            k, fa, fb = c.atoms[a]
            c.atoms[a] = (k, shrink(fa), shrink(fb))
    out_list = [(fr, i, shrink(f)) for fr, i, f in out_list]

    level = {}

    def lvl(a):
        if a not in level:
            if c.atoms[a][0] in ("in", "const"):
                level[a] = 0
            else:
                level[a] = 1 + max([lvl(x) for x in deps(a)] or [0])
        return level[a]

    work = [a for a in need if c.atoms[a][0] in ("prod", "lin", "sel", "lut")]
    for a in work:
        lvl(a)
    if schedule.startswith("list:"):
        # list scheduling with at most W ops per level (W = 64 / G fills one
        # pass of a G-item workgroup): ready ops by decreasing height (longest
        # path to the end of the program), so narrow dependency-bound levels
        # are padded with work that the ASAP levelling put in wide levels
        W = int(schedule.split(":")[1])
        users = defaultdict(list)
        for a in work:
            for s_ in deps(a):
                users[s_].append(a)
        height = {}
        for a in sorted(work, key=lambda a: -level[a]):
            height[a] = 1 + max([height[u] for u in users.get(a, ())] or [0])
        placed = {}
        rem = set(work)
        L = 0
        while rem:
            L += 1
            ready = [a for a in rem
                     if all(c.atoms[d][0] in ("in", "const") or placed.get(d, L) < L for d in deps(a))]
            ready.sort(key=lambda a: (-height[a], a))
            for a in ready[:W]:
                placed[a] = L
                rem.discard(a)
        level.update(placed)
    if schedule == "alap":
        # as late as possible (within the ASAP depth): an op moves to one level
        # before its earliest consumer, so values live shorter (fewer LDS slots)
        depth_ = max([level[a] for a in work] or [0])
        users = defaultdict(list)
        for a in work:
            for s_ in deps(a):
                users[s_].append(a)
        out_of = defaultdict(list)
        for fr, i, f in out_list:
            for s_ in f:
                out_of[s_].append((fr, i))
        for a in sorted(work, key=lambda a: -level[a]):
            lim = depth_ if out_of.get(a) else depth_ + 1
            if users.get(a):
                lim = min(lim, min(level[u] for u in users[a]) - 1)
            if lim > level[a]:
                level[a] = lim
    # last level at which each input slot is read
    last_read = defaultdict(int)
    for a in work:
        d = c.atoms[a]
        srcs = deps(a)
        for s in srcs:
            if c.atoms[s][0] == "in":
                key = canon((c.atoms[s][1], c.atoms[s][2]))
                last_read[key] = max(last_read[key], level[a])
        if d[0] == "lut":
            for j in range(16):
                key = canon((d[1], d[2] + j * d[3]))
                last_read[key] = max(last_read[key], level[a])
    slot = {}
    for a in need:
        d = c.atoms[a]
        if d[0] == "in":
            slot[a] = (d[1], d[2])
        elif d[0] == "const":
            slot[a] = (CONST_FRAME, _pool_index(d[1]))
    # outputs: direct write of an op result when safe, else a lin item
    out_items = []
    direct = {}
    for fr, i, f in out_list:
        key = (fr, i)
        ck = canon(key)
        if len(f) == 1:
            (a, k), = f.items()
            if k == 1 and c.atoms[a][0] in ("prod", "sel", "lut") and a not in direct \
                    and last_read.get(ck, 0) < level[a] and key not in direct.values():
                direct[a] = key
                continue
        lvl_o = 1 + max([lvl(a) for a in f] or [0])
        lvl_o = max(lvl_o, last_read.get(ck, 0) + 1)
        out_items.append((lvl_o, key, f))
    for a, key in direct.items():
        slot[a] = key
    # scratch slots by liveness: a slot is reused once every reader of its
    # previous value ran at an earlier level (reads and writes of one level
    # may interleave across the passes of a multi-item level)
    last_use = defaultdict(int)
    for a in work:
        for s_ in deps(a):
            last_use[s_] = max(last_use[s_], level[a])
    for lv_o, _, f in out_items:
        for s_ in f:
            last_use[s_] = max(last_use[s_], lv_o)
    occupied = []  # [last_use_level, slot]
    for a in sorted(work, key=lambda a: (level[a], a)):
        if a in slot:
            continue
        for ent in occupied:
            if ent[0] < level[a]:
                slot[a] = (scratch_frame, ent[1])
                ent[0] = last_use[a]
                break
        else:
            slot[a] = (scratch_frame, len(occupied))
            occupied.append([last_use[a], len(occupied)])
    scratch_size = len(occupied)

    def terms(form):
        ts = []
        for a, k in sorted(form.items()):
            if k == 0:
                continue
            assert -MAX_COEF <= k <= MAX_COEF, (name, k)
            fr, ix = slot[a]
            ts.append((fr, ix, k))
        assert len(ts) <= MAX_TERMS, (name, len(ts))
        return ts

    by_level = defaultdict(list)
    for a in work:
        d = c.atoms[a]
        if d[0] == "prod":
            by_level[level[a]].append(("mul", slot[a], terms(d[1]), terms(d[2])))
        elif d[0] == "sel":
            by_level[level[a]].append(("sel", slot[a], terms(d[1]), terms(d[2])))
        elif d[0] == "lut":
            by_level[level[a]].append(("lut", slot[a], [(d[1], d[2], d[3])], []))
        else:
            by_level[level[a]].append(("lin", slot[a], terms(d[1]), []))
    for lv, key, f in out_items:
        by_level[lv].append(("lin", key, terms(f), []))
    order = {"mul": 0, "sel": 1, "lut": 2, "lin": 3}
    levels = []
    for L in sorted(by_level):
        its = by_level[L]
        its.sort(key=lambda t: (order[t[0]], -(len(t[2]) + len(t[3]))))
        levels.append(its)
    # hazard check: every write of an input-frame slot happens at a level
    # after the last read of that slot's input value
    writes = {}
    for L in sorted(by_level):
        for kind, dst, a, b in by_level[L]:
            assert dst not in writes or dst[0] == scratch_frame, (name, dst)
            writes[dst] = L
            if dst[0] != scratch_frame:
                assert last_read.get(canon(dst), -1) < L, (name, dst, L)
    nprod = sum(1 for a in work if c.atoms[a][0] == "prod")
    return {"name": name, "frames": frames + [scratch_size], "levels": levels, "nprod": nprod,
            "written": sorted(outputs) + [scratch_frame],
            "depth": max([level[a] for a in work] or [0])}


# --------------------------------------------------------------------------
# binding: a program instance places its frames at fixed slot offsets of the
# item region, so table words carry absolute slot indices.
#   term word: [31:24] coef + 128 (lut: stride + 128) | [23] const pool | [22:0] slot
#   dest word: [31:30] kind | [29:26] na | [25:22] nb | [21:0] slot
# --------------------------------------------------------------------------
LAYOUT = {}      # layout name -> {"stride": n, "consts": {...}} (emitted as C++ constants)
INSTANCES = []   # (instance name, program name, frame bases, scratch base)


def layout(name, **slots):
    # Odd item strides: LDS slots are 80 B (Fd, bls_field_types.h), so slot s
    # starts at bank group (5 s) mod 16 of a ds_read_b128; with an odd stride
    # the same slot of up to 16 items of one workgroup lands in 16 different
    # groups (an even stride put items in the same group: 2-16-way conflicts).
    if "STRIDE" in slots and slots["STRIDE"] % 2 == 0:
        slots = dict(slots, STRIDE=slots["STRIDE"] + 1)
    LAYOUT[name] = slots


def instance(iname, prog, bases, scratch):
    INSTANCES.append((iname, prog, list(bases), scratch))


def bind(p, bases, scratch, alias):
    nfr = len(p["frames"]) - 1
    assert len(bases) == nfr, (p["name"], bases)
    sizes = p["frames"][:-1]
    rng_ = [(bases[i], bases[i] + sizes[i]) for i in range(nfr)] + [(scratch, scratch + p["frames"][-1])]
    for i in range(nfr + 1):
        for j in range(i + 1, nfr + 1):
            (a0, a1), (b0, b1) = rng_[i], rng_[j]
            if a0 < b1 and b0 < a1 and (i in p["written"] or j in p["written"]):
                # overlap with a written frame: only a declared alias with identical placement
                ok = (alias.get(i) == j or alias.get(j) == i) and a0 == b0
                assert ok, (p["name"], "frames", i, j, "overlap", bases, scratch)

    def slot_of(fr, ix):
        if fr == CONST_FRAME:
            return (1 << 23) | ix
        b = scratch if fr == nfr else bases[fr]
        return b + ix

    levels = []
    for items in p["levels"]:
        bl = []
        for kind, (fr, ix), a, b in items:
            # dest word: kind | own operand widths (na, nb: 4 bits each) | slot
            assert slot_of(fr, ix) < (1 << 22)
            d = (KIND[kind] << 30) | (len(a) << 26) | (len(b) << 22) | slot_of(fr, ix)
            if kind == "lut":
                (tf, ti, ts), = a
                ta = [((ts + 128) << 24) | slot_of(tf, ti)]
            else:
                ta = [((k + 128) << 24) | slot_of(f, i) for f, i, k in a]
            tb = [((k + 128) << 24) | slot_of(f, i) for f, i, k in b]
            bl.append((d, ta, tb))
        levels.append(bl)
    return levels


def emit(progs, path):
    by_name = {p["name"]: p for p in progs}
    out = ["// GENERATED by tools/wavec.py -- do not edit.",
           "// Wave program instances: levels of independent Montgomery products / linear ops",
           "// whose operands are small-integer linear combinations of slots (see bls_vm.h).",
           "#pragma once", "#include <stdint.h>", "", "namespace bls {", ""]
    for lname, vals in LAYOUT.items():
        for k, v in vals.items():
            out.append(f"static constexpr int WL_{lname}_{k} = {v};")
    out.append("")
    for p in progs:
        out.append(f"static constexpr int WP_{p['name']}_SCRATCH = {p['frames'][-1]};")
    out.append("")
    for iname, pname, bases, scratch in INSTANCES:
        p = by_name[pname]
        lv_desc, tbl = [], []
        for items in bind(p, bases, scratch, PROGRAMS[pname][2] if len(PROGRAMS[pname]) > 2 else {}):
            na = max(len(a) for _, a, _ in items)
            nb = max(len(b) for _, _, b in items)
            base = len(tbl)
            for d, ta, tb in items:
                tbl.append(d)
                tbl += ta + [0] * (na - len(ta)) + tb + [0] * (nb - len(tb))
            lv_desc.append((len(items), na, nb, base))
        out.append(f"// {iname} = {pname} at frames {bases}, scratch {scratch}: {p['nprod']} products, "
                   f"{len(lv_desc)} levels")
        out.append(f"static constexpr uint32_t WP_{iname}_TERMS[{len(tbl)}] = {{{', '.join(str(x) for x in tbl)}}};")
        out.append(f"static constexpr uint32_t WP_{iname}_LEVELS[{len(lv_desc)}][4] = {{"
                   + ", ".join("{%d, %d, %d, %d}" % d for d in lv_desc) + "};")
        out.append(f"static constexpr int WP_{iname}_NLEVELS = {len(lv_desc)};")
        out.append("")
    pool = sorted(CONST_POOL.items(), key=lambda kv: kv[1])
    rows = []
    for v, _ in pool:  # Montgomery form (R = 2^406) as 14 radix-2^29 digits + 2 pad words
        m = v * (1 << 406) % P
        rows.append("{{" + ", ".join("0x%08xu" % ((m >> (29 * i)) & 0x1FFFFFFF) for i in range(14)) + ", 0u, 0u}}")
    out.append(f"static constexpr int WP_NCONST = {len(pool)};")
    out.append("struct WpConst { uint32_t d[16]; };")
    out.append(f"static constexpr WpConst WP_CONST_POOL[{max(1, len(pool))}] = {{{', '.join(rows or ['{{0}}'])}}};")
    out.append("")
    out.append("}  // namespace bls")
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")


def define_instances(progs):
    """Slot layouts of the device kernels and the program instances they run."""
    LAYOUT.clear()
    INSTANCES.clear()
    sc = {p["name"]: p["frames"][-1] for p in progs}
    # Miller loop item region: f | T | P (-x, y) | Q | scratch
    ml_s = max(sc["ML_DBL"], sc["ML_ADD"], sc["ML_DBL_FIRST"])
    layout("ML", F=0, T=12, P=18, Q=20, S=24, STRIDE=24 + ml_s)
    for nm in ("ML_DBL", "ML_ADD", "ML_DBL_FIRST"):
        instance(nm, nm, [0, 12, 18, 20], 24)
    # shared-accumulator Miller loop, K = 2 pairs: f | (T, P, Q) x K | scratch
    m2s = max(sc["ML2_DBL"], sc["ML2_FIRST"], sc["ML2_ADD"])
    layout("M2", F=0, PAIR=12, PSTRIDE=12, S=36, STRIDE=36 + m2s)
    for st_ in ("DBL", "FIRST", "ADD"):
        instance(f"M2_{st_}", f"ML2_{st_}", [0, 12, 18, 20, 24, 30, 32], 36)
    # chunked Fp12 product: acc | in | scratch
    layout("CH", STRIDE=24 + sc["FP12_MUL"])
    instance("CH_MUL", "FP12_MUL", [0, 12, 0], 24)
    # final exponentiation: registers R0..R6 (12 slots each) | scratch
    cyc = [n for n in sc if n.startswith("CYC_")]
    fe_s = max([sc["FP12_MUL"], sc["FP12_FROB1"], sc["FP12_FROB2"]] + [sc[n] for n in cyc])
    layout("FE", NREG=7, S=84, STRIDE=84 + fe_s)
    R = lambda k: 12 * k  # noqa: E731
    for d, a, b in ((0, 0, 1), (0, 2, 1), (2, 2, 1), (2, 1, 3), (3, 3, 1), (1, 1, 4), (1, 1, 5)):
        instance(f"FE_MUL_{d}{a}{b}", "FP12_MUL", [R(a), R(b), R(d)], 84)
    instance("FE_FROB2_10", "FP12_FROB2", [R(0), R(1)], 84)
    instance("FE_FROB2_43", "FP12_FROB2", [R(3), R(4)], 84)
    instance("FE_FROB1_32", "FP12_FROB1", [R(2), R(3)], 84)
    for i, (k, add) in enumerate(X_RUNS):  # pow_x: R1 = R2^|x|
        nm = f"CYC_{k}{'M' if add else ''}"
        cur = R(2) if i == 0 else R(1)
        instance(f"FE_POWX_{i}", nm, [cur, R(2), R(1)], 84)
    instance("FE_CUBE", "CYC_1M", [R(0), R(0), R(5)], 84)
    # hash_to_G2 phases (k_h2c_iso / _pre / _post): SSWU points | Q | M | A | C | H | izs | scratch
    H = dict(U=0, Q=8, M=14, A=20, C=26, H=32, IZ=38, S=42)
    hs = max(sc["ISO_PAIR"], sc["CLEAR_PRE"], sc["CLEAR_POST"])
    layout("HC", STRIDE=H["S"] + hs, **H)
    instance("HC_ISO", "ISO_PAIR", [H["U"], H["Q"], H["IZ"]], H["S"])
    # [|x|] chains of cofactor clearing as their own kernel (k_g2x_chain):
    # base | M | scratch only, so several more items share an LDS budget
    xs = max(sc[n] for n in sc if n.startswith("G2X_"))
    layout("XC", B=0, M=6, S=12, STRIDE=12 + xs)
    for i, (k, add) in enumerate(X_RUNS):  # M = [|x|] B
        instance(f"XC_{i}", f"G2X_{k}{'A' if add else ''}", [0 if i == 0 else 6, 0, 6], 12)
    instance("HC_PRE", "CLEAR_PRE", [H["Q"], H["M"], H["A"], H["C"]], H["S"])
    instance("HC_POST", "CLEAR_POST", [H["C"], H["M"], H["H"]], H["S"])
    # signature side: sigma | apk | M | R | D (subgroup check) | scratch
    G = dict(SIG=0, APK=4, M=7, R=13, D=16, SC=22)
    gs = max(sc["SIG_STEP0"], sc["SIG_STEP1"], sc["SIG_STEP2"], sc["G2_SUBCHK"])
    layout("SG", STRIDE=G["SC"] + gs, **G)
    for m in range(3):
        instance(f"SG_STEP{m}", f"SIG_STEP{m}", [G["SIG"], G["APK"], G["M"], G["R"]], G["SC"])
    instance("SG_SUBCHK", "G2_SUBCHK", [G["SIG"], G["M"], G["D"]], G["SC"])
    # MSM bucket accumulation: R | Q | scratch
    layout("MB", R=0, Q=6, S=10, STRIDE=10 + sc["G2_ADDAFF_SEL"])
    instance("MB_ADD", "G2_ADDAFF_SEL", [0, 6], 10)
    # MSM trees: pairwise sums out = A + B, and weighted pairs out = A + [2^k] B
    layout("MT", A=0, B=6, O=12, S=18, STRIDE=18 + max(sc["G2_ADD"], *[sc[f"G2P_{k}"] for k in (1, 2, 4, 8, 16, 32)]))
    instance("MT_ADD", "G2_ADD", [0, 6, 12], 18)
    for k in (1, 2, 4, 8, 16, 32):
        instance(f"MT_P{k}", f"G2P_{k}", [6, 0, 12], 18)  # R = B doubled k times, + base A
    # final affine conversion: P | N | NI | ZI | XY | scratch
    layout("MA", P=0, N=6, NI=7, ZI=8, XY=10, S=14,
           STRIDE=14 + max(sc["FP2_NORM"], sc["FP2_INVFIN"], sc["G2_TOAFF"]))
    instance("MA_NORM", "FP2_NORM", [4, 6], 14)
    instance("MA_INVFIN", "FP2_INVFIN", [4, 7, 8], 14)
    instance("MA_TOAFF", "G2_TOAFF", [0, 8, 10], 14)


def compile_all():
    CONST_POOL.clear()
    progs = []
    for n, spec in PROGRAMS.items():
        # as-soon-as-possible vs as-late-as-possible levelling: keep whichever
        # needs fewer scratch slots (shorter item stride, more items per LDS)
        a = compile_program(n, *spec, schedule="asap")
        b = compile_program(n, *spec, schedule="alap")
        progs.append(b if b["frames"][-1] < a["frames"][-1] else a)
    define_instances(progs)
    return progs


if __name__ == "__main__":
    progs = compile_all()
    for p in progs:
        sizes = [len(items) for items in p["levels"]]
        print(f"{p['name']:14s} products={p['nprod']:4d} depth={p['depth']:3d} levels={len(p['levels']):3d} "
              f"scratch={p['frames'][-1]:4d} sizes={sizes if len(sizes) < 12 else sizes[:12] + ['...']}")
    print("const pool:", len(CONST_POOL))
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "eth-consensus-specs_amd", "csrc",
                       "bls_waveprog.h")
    emit(progs, dst)
    print("wrote", os.path.normpath(dst))
