#!/usr/bin/env python3
"""wavec -- compile extension-field formulas into wave programs (build tool).

A *wave program* is a straight-line program over Fp whose only non-linear
operation is the Montgomery product.  The formulas (Fp12 multiplication,
the Miller-loop doubling step, ...) are written once below against a
symbolic Fp; tracing them yields a DAG of products whose operands are
small-integer linear combinations of earlier values.  Products are then
levelled (ASAP) so every product of a level is independent: on the device a
64-lane wave executes one level per step, lane j computing product j
(bls_wave.h).  The Fp12 product that costs one lane 54 sequential
multiplications therefore costs the wave one multiplication of latency.

Output: eth-consensus-specs_amd/csrc/bls_waveprog.h (constant tables).
Each program addresses slots through *frames*: frame k of a program is a
contiguous run of Fp slots whose base the kernel passes at run time; the
last frame is the program's private scratch (one slot per product plus the
output temporaries).

This module is standalone (no oracle import); tests/test_wavec.py checks the
traced formulas numerically against the oracle.
"""
from __future__ import annotations

import os
from collections import defaultdict

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB

# --------------------------------------------------------------------------
# symbolic Fp: a linear form over "atoms" (inputs or products)
# --------------------------------------------------------------------------


class Ctx:
    def __init__(self):
        self.atoms = []  # ('in', frame, idx) | ('prod', a_form, b_form) | ('const', value)
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
        a = self.c.atom(("prod", dict(self.f), dict(o.f)))
        return V(self.c, {a: 1})

    __rmul__ = smul

    def is_zero(self):
        return not self.f


def inp(c, frame, idx):
    return V(c, {c.atom(("in", frame, idx)): 1})


def const(c, value):
    value %= P
    if value not in c.consts:
        c.consts[value] = c.atom(("const", value))
    return V(c, {c.consts[value]: 1})


def zero(c):
    return V(c, {})


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
        if isinstance(o, V):  # Fp2 x Fp
            return F2(s.a * o, s.b * o)
        if s.b.is_zero() and o.b.is_zero():
            return F2(s.a * o.a, s.b)
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

    def mul_v(s):
        return F6(s.c[2].mul_xi(), s.c[0], s.c[1])

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
# programs
# --------------------------------------------------------------------------


def prog_fp12_mul(c):
    a = f12_from_frame(c, 0)
    b = f12_from_frame(c, 1)
    return {2: (a * b).coeffs()}


def prog_fp12_sqr(c):
    a = f12_from_frame(c, 0)
    return {1: a.sqr().coeffs()}


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


def prog_ml_add(c):
    """f <- f * l_{T,Q}(P); T <- T + Q."""
    f, T, nxP, yP, xQ, yQ = _pair_frames(c)
    T2, (l0, l2, l3) = _ml_line_add(c, T, xQ, yQ, nxP, yP)
    return {0: f.mul_line(l0, l2, l3).coeffs(), 1: _t_out(T2)}


PROGRAMS = {
    # name: (builder, frame sizes (excluding scratch))
    "FP12_MUL": (prog_fp12_mul, [12, 12, 12]),
    "FP12_SQR": (prog_fp12_sqr, [12, 12]),
    "ML_DBL": (prog_ml_dbl, [12, 6, 2, 4]),
    "ML_DBL_FIRST": (prog_ml_dbl_first, [12, 6, 2, 4]),
    "ML_ADD": (prog_ml_add, [12, 6, 2, 4]),
}

# --------------------------------------------------------------------------
# compiler: level scheduling, slot assignment, table emission
# --------------------------------------------------------------------------
LANES = 64
MAX_TERMS = 40  # per operand (padded); asserted
MAX_COEF = 31


SPLIT = 8  # linear combinations longer than this are summed as a tree of partial sums


def compile_program(name, builder, frames):
    c = Ctx()
    outputs = builder(c)  # {frame: [V...]}
    nframes = len(frames)
    scratch_frame = nframes
    out_list = [(fr, i, v) for fr, vs in outputs.items() for i, v in enumerate(vs)]

    # atoms reachable from the outputs
    need = set()
    stack = [a for _, _, v in out_list for a in v.f]
    while stack:
        a = stack.pop()
        if a in need:
            continue
        need.add(a)
        d = c.atoms[a]
        if d[0] == "prod":
            stack += list(d[1]) + list(d[2])

    # split long linear forms into partial-sum atoms ('lin', form)
    def shrink(form):
        items = sorted(form.items())
        while len(items) > SPLIT:
            chunks = [dict(items[k:k + SPLIT]) for k in range(0, len(items), SPLIT)]
            items = []
            for ch in chunks:
                if len(ch) == 1:
                    items += list(ch.items())
                else:
                    a = c.atom(("lin", ch))
                    need.add(a)
                    items.append((a, 1))
        return dict(items)

    prods = sorted(a for a in need if c.atoms[a][0] == "prod")
    for a in prods:
        _, fa, fb = c.atoms[a]
        c.atoms[a] = ("prod", shrink(fa), shrink(fb))
    out_list = [(fr, i, shrink(v.f)) for fr, i, v in out_list]

    level = {}

    def deps(a):
        d = c.atoms[a]
        if d[0] == "prod":
            return list(d[1]) + list(d[2])
        if d[0] == "lin":
            return list(d[1])
        return []

    def lvl(a):
        if a not in level:
            ds = deps(a)
            level[a] = 0 if c.atoms[a][0] in ("in", "const") else 1 + max([lvl(x) for x in ds] or [0])
        return level[a]

    work = [a for a in need if c.atoms[a][0] in ("prod", "lin")]
    for a in work:
        lvl(a)
    depth = max([level[a] for a in work] or [0])
    out_level = 1 + max([depth] + [max([level[a] for a in f] or [0]) for _, _, f in out_list])
    consts = sorted(a for a in need if c.atoms[a][0] == "const")
    slot = {}
    for a in need:
        d = c.atoms[a]
        if d[0] == "in":
            slot[a] = (d[1], d[2])
    sidx = 0
    for a in consts:
        slot[a] = (scratch_frame, sidx)
        sidx += 1
    for a in sorted(work, key=lambda a: (level[a], a)):
        slot[a] = (scratch_frame, sidx)
        sidx += 1
    scratch_size = sidx

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
        else:
            by_level[level[a]].append(("lin", slot[a], terms(d[1]), []))
    for fr, i, f in out_list:  # outputs last: every read of an input frame happens before
        by_level[out_level].append(("lin", (fr, i), terms(f), []))
    levels = []
    for L in sorted(by_level):
        its = by_level[L]
        its.sort(key=lambda t: t[0] != "mul")  # products first (lanes 0..)
        for k in range(0, len(its), LANES):
            levels.append(its[k:k + LANES])
    nprod = sum(1 for a in work if c.atoms[a][0] == "prod")
    return {"name": name, "frames": frames + [scratch_size], "levels": levels,
            "consts": [(slot[a][1], c.atoms[a][1]) for a in consts],
            "nprod": nprod, "depth": depth}


def pack_term(fr, ix, k):
    # 32 bits: frame (4) | index (12) | coef + 128 (8); 0 means "no term"
    assert 0 <= fr < 16 and 0 <= ix < 4096 and -MAX_COEF <= k <= MAX_COEF and k != 0
    return (fr << 20) | (ix << 8) | (k + 128)


def emit(progs, path):
    out = ["// GENERATED by tools/wavec.py -- do not edit.",
           "// Wave programs: levels of independent Montgomery products whose operands are",
           "// small-integer linear combinations of slots (see bls_wave.h).",
           "#pragma once", "#include <stdint.h>", "", "namespace bls {", ""]
    for p in progs:
        nm = p["name"]
        lv_desc = []
        tbl = []
        for items in p["levels"]:
            na = max(len(a) for _, _, a, _ in items)
            nb = max(len(b) for _, _, _, b in items)
            stride = 1 + na + nb
            base = len(tbl)
            for kind, (fr, ix), a, b in items:
                tbl.append((1 << 31 if kind == "mul" else 0) | (fr << 20) | (ix << 8))  # destination word
                ta = [pack_term(*t) for t in a] + [0] * (na - len(a))
                tb = [pack_term(*t) for t in b] + [0] * (nb - len(b))
                tbl += ta + tb
            lv_desc.append((0, len(items), na, nb, base))
        out.append(f"// {nm}: frames {p['frames']} (last = scratch), {p['nprod']} products, depth {p['depth']}, "
                   f"{len(p['levels'])} levels")
        out.append(f"static constexpr uint32_t WP_{nm}_TERMS[{len(tbl)}] = {{{', '.join(str(x) for x in tbl)}}};")
        out.append(f"static constexpr uint32_t WP_{nm}_LEVELS[{len(lv_desc)}][5] = {{"
                   + ", ".join("{%d, %d, %d, %d, %d}" % d for d in lv_desc) + "};")
        out.append(f"static constexpr int WP_{nm}_NLEVELS = {len(lv_desc)};")
        out.append(f"static constexpr int WP_{nm}_SCRATCH = {p['frames'][-1]};")
        cs = p["consts"]
        out.append(f"static constexpr int WP_{nm}_NCONST = {len(cs)};")
        if cs:
            out.append(f"static constexpr uint32_t WP_{nm}_CONSTS[{len(cs)}][13] = {{"
                       + ", ".join("{%d, %s}" % (ix, ", ".join("0x%08xu" % ((v * (1 << 406) % P) >> (32 * i) & 0xFFFFFFFF)
                                                             for i in range(12))) for ix, v in cs) + "};")
        out.append("")
    out.append("}  // namespace bls")
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")


def compile_all():
    return [compile_program(n, b, fr) for n, (b, fr) in PROGRAMS.items()]


if __name__ == "__main__":
    progs = compile_all()
    for p in progs:
        sizes = [len(items) for items in p["levels"]]
        print(f"{p['name']:14s} products={p['nprod']:4d} depth={p['depth']:2d} levels={len(p['levels'])} sizes={sizes} "
              f"scratch={p['frames'][-1]}")
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "eth-consensus-specs_amd", "csrc",
                       "bls_waveprog.h")
    emit(progs, dst)
    print("wrote", os.path.normpath(dst))
