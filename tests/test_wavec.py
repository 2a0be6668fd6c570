"""The wave programs (tools/wavec.py -> bls_waveprog.h) evaluated by a Python
model of the device interpreter (bls_vm.h) against the oracle: CPU-side
proof that the traced formulas, the level schedule and the slot allocation
are right."""
import os
import random
import sys

import pytest

from oracle import bls_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import wavec  # noqa: E402

PROGS = {p["name"]: p for p in wavec.compile_all()}
POOL = [v for v, _ in sorted(wavec.CONST_POOL.items(), key=lambda kv: kv[1])]
rng = random.Random(7)


def run(prog, frames, pred=0):
    """frames: list of lists of canonical ints (one per program frame, scratch
    excluded).  Mirrors vm_run for one item: every op of a level reads its
    operands before any op of the level writes."""
    fr = [list(f) for f in frames] + [[0] * prog["frames"][-1]]

    def get(f, i):
        return POOL[i] if f == wavec.CONST_FRAME else fr[f][i]

    def lin(ts):
        return sum(k * get(f, i) for f, i, k in ts) % O.P

    for items in prog["levels"]:
        vals = []
        for kind, (dfr, dix), a, b in items:
            if kind == "mul":
                v = lin(a) * lin(b) % O.P
            elif kind == "sel":
                v = lin(a) if pred & 1 else lin(b)
            elif kind == "lut":
                (f, i, s), = a
                v = get(f, i + pred * s)
            else:
                v = lin(a)
            vals.append(((dfr, dix), v))
        for (dfr, dix), v in vals:
            fr[dfr][dix] = v
    return fr


def f12_list(f):
    out = []
    for c in O.f12_to_coeffs(f):
        out += [c[0], c[1]]
    return out


def list_f12(v):
    return O.f12_from_coeffs([(v[2 * k], v[2 * k + 1]) for k in range(6)])


def rf12():
    return O.f12_from_coeffs([(rng.randrange(O.P), rng.randrange(O.P)) for _ in range(6)])


def cyclotomic(f):
    t = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
    return O.f12_mul(O.f12_frobenius(O.f12_frobenius(t)), t)


def g2_proj(pt, z=None):
    """affine oracle point -> projective Fp list with a random Z."""
    if pt is None:
        return [0, 0, 1, 0, 0, 0]
    z = z or (rng.randrange(1, O.P), rng.randrange(O.P))
    x, y = O.f2_mul(pt[0], z), O.f2_mul(pt[1], z)
    return [x[0], x[1], y[0], y[1], z[0], z[1]]


def g2_aff(v):
    z = (v[4], v[5])
    if z == (0, 0):
        return None
    zi = O.f2_inv(z)
    return (O.f2_mul((v[0], v[1]), zi), O.f2_mul((v[2], v[3]), zi))


def g1_proj(pt):
    if pt is None:
        return [0, 1, 0]
    z = rng.randrange(1, O.P)
    return [pt[0] * z % O.P, pt[1] * z % O.P, z]


def g1_aff(v):
    if v[2] == 0:
        return None
    zi = pow(v[2], -1, O.P)
    return (v[0] * zi % O.P, v[1] * zi % O.P)


def rand_e2_point():
    """A point of E2 outside G2 (the image of SSWU + isogeny)."""
    u = (rng.randrange(O.P), rng.randrange(O.P))
    return O.iso_map(O.map_to_curve_sswu(u))


def test_fp12_mul_sqr_frob_programs():
    for _ in range(3):
        a, b = rf12(), rf12()
        fr = run(PROGS["FP12_MUL"], [f12_list(a), f12_list(b), [0] * 12])
        assert list_f12(fr[2]) == O.f12_mul(a, b)
        fr = run(PROGS["FP12_SQR"], [f12_list(a), [0] * 12])
        assert list_f12(fr[1]) == O.f12_sqr(a)
        fr = run(PROGS["FP12_FROB1"], [f12_list(a), [0] * 12])
        assert list_f12(fr[1]) == O.f12_frobenius(a)
        fr = run(PROGS["FP12_FROB2"], [f12_list(a), [0] * 12])
        assert list_f12(fr[1]) == O.f12_frobenius(O.f12_frobenius(a))


def test_cyclotomic_runs_compose_pow_x():
    a = cyclotomic(rf12())
    base = f12_list(a)
    cur = base
    for k, add in wavec.X_RUNS:
        name = f"CYC_{k}{'M' if add else ''}"
        cur = run(PROGS[name], [cur, base, [0] * 12])[2]
    assert list_f12(cur) == O.f12_pow(a, O.X_ABS)


def test_level_descriptors_are_sane():
    for p in PROGS.values():
        for items in p["levels"]:
            assert len(items) >= 1
            for kind, dst, a, b in items:
                assert len(a) <= wavec.MAX_TERMS and len(b) <= wavec.MAX_TERMS


@pytest.mark.parametrize("k1,k2", [(3, 5), (0x1234567, 0x7654321)])
def test_miller_loop_program_sequence(k1, k2):
    P1 = O.g1_mul(O.G1_GEN, k1)
    Q2 = O.g2_mul(O.G2_GEN, k2)
    f = [0] * 12
    T = [Q2[0][0], Q2[0][1], Q2[1][0], Q2[1][1], 1, 0]
    Pf = [(-P1[0]) % O.P, P1[1]]
    Qf = [Q2[0][0], Q2[0][1], Q2[1][0], Q2[1][1]]
    fr = [f, T, Pf, Qf]
    fr = run(PROGS["ML_DBL_FIRST"], fr)[:4]
    if (O.X_ABS >> 62) & 1:
        fr = run(PROGS["ML_ADD"], fr)[:4]
    for b in range(61, -1, -1):
        fr = run(PROGS["ML_DBL"], fr)[:4]
        if (O.X_ABS >> b) & 1:
            fr = run(PROGS["ML_ADD"], fr)[:4]
    ml = O.f12_conj(list_f12(fr[0]))
    assert O.final_exponentiation(ml) == O.pairing(P1, Q2)


def test_complete_g2_arithmetic():
    p, q = rand_e2_point(), rand_e2_point()
    fr = run(PROGS["G2_ADD"], [g2_proj(p), g2_proj(q), [0] * 6])
    assert g2_aff(fr[2]) == O.g2_add(p, q)
    # exceptional inputs handled without branches: P + P, P + (-P), O + P
    fr = run(PROGS["G2_ADD"], [g2_proj(p), g2_proj(p), [0] * 6])
    assert g2_aff(fr[2]) == O.g2_add(p, p)
    fr = run(PROGS["G2_ADD"], [g2_proj(p), g2_proj(O.g2_neg(p)), [0] * 6])
    assert g2_aff(fr[2]) is None
    fr = run(PROGS["G2_ADD"], [g2_proj(None), g2_proj(q), [0] * 6])
    assert g2_aff(fr[2]) == q


def test_g2_xmul_runs_compose_xabs():
    p = rand_e2_point()
    base = g2_proj(p)
    cur = base
    for k, add in wavec.X_RUNS:
        cur = run(PROGS[f"G2X_{k}{'A' if add else ''}"], [cur, base, [0] * 6])[2]
    assert g2_aff(cur) == O.g2_mul(p, O.X_ABS)


@pytest.mark.parametrize("ext", [False, True])
def test_double_and_always_add_select(ext):
    k = rng.getrandbits(64) | 1
    if ext:
        p = O.g2_mul(O.G2_GEN, rng.randrange(1, O.R))
        R = g2_proj(None)
        q = [p[0][0], p[0][1], p[1][0], p[1][1]]
        name, aff, mul = "G2_DAS", g2_aff, O.g2_mul
    else:
        p = O.g1_mul(O.G1_GEN, rng.randrange(1, O.R))
        R = g1_proj(None)
        q = [p[0], p[1]]
        name, aff, mul = "G1_DAS", g1_aff, O.g1_mul
    for b in range(63, -1, -1):
        R = run(PROGS[name], [R, q], pred=(k >> b) & 1)[0]
    assert aff(R) == mul(p, k)


def test_g1_add_program():
    a = O.g1_mul(O.G1_GEN, 11)
    b = O.g1_mul(O.G1_GEN, 31)
    fr = run(PROGS["G1_ADD"], [g1_proj(a), g1_proj(b), [0] * 3])
    assert g1_aff(fr[2]) == O.g1_mul(O.G1_GEN, 42)


def test_g2_subgroup_check_program():
    def check(pt):
        base = g2_proj(pt, z=(1, 0))
        cur = base
        for k, add in wavec.X_RUNS:
            cur = run(PROGS[f"G2X_{k}{'A' if add else ''}"], [cur, base, [0] * 6])[2]
        out = run(PROGS["G2_SUBCHK"], [base[:4], cur, [0] * 6])[2]
        return out[:4] == [0, 0, 0, 0] and out[4:6] != [0, 0]

    assert check(O.g2_mul(O.G2_GEN, 0x5EED))
    assert not check(rand_e2_point())


def test_iso_and_cofactor_programs_match_hash_to_g2():
    msg = b"wave programs"
    u0, u1 = O.hash_to_field_fp2(msg, 2, O.DST_POP)
    p0, p1 = O.map_to_curve_sswu(u0), O.map_to_curve_sswu(u1)
    frame0 = [p0[0][0], p0[0][1], p0[1][0], p0[1][1], p1[0][0], p1[0][1], p1[1][0], p1[1][1]]
    q = run(PROGS["ISO_PAIR"], [frame0, [0] * 6, [0] * 4])[1]
    assert g2_aff(q) == O.g2_add(O.iso_map(p0), O.iso_map(p1))

    def xmul(v):
        cur = v
        for k, add in wavec.X_RUNS:
            cur = run(PROGS[f"G2X_{k}{'A' if add else ''}"], [cur, v, [0] * 6])[2]
        return cur

    m1 = xmul(q)
    fr = run(PROGS["CLEAR_PRE"], [q, m1, [0] * 6, [0] * 6])
    A, C = fr[2], fr[3]
    m2 = xmul(A)
    h = run(PROGS["CLEAR_POST"], [C, m2, [0] * 6])[2]
    # affine via the inversion programs
    z = (h[4], h[5])
    n = run(PROGS["FP2_NORM"], [list(z), [0]])[1][0]
    zi = run(PROGS["FP2_INVFIN"], [list(z), [pow(n, -1, O.P)], [0, 0]])[2]
    xy = run(PROGS["G2_TOAFF"], [h, zi, [0] * 4])[2]
    assert ((xy[0], xy[1]), (xy[2], xy[3])) == O.hash_to_g2(msg)


def test_g1_to_affine_program():
    p = O.g1_mul(O.G1_GEN, 77)
    v = g1_proj(p)
    xy = run(PROGS["G1_TOAFF"], [v, [pow(v[2], -1, O.P)], [0, 0]])[2]
    assert tuple(xy) == p


def test_signature_step_programs():
    """64 steps of SIG_STEP{0,1,2}: M = [|x|] sigma, R = r apk."""
    sig = O.g2_mul(O.G2_GEN, 0x1234_5678_9ABC)
    apk = O.g1_mul(O.G1_GEN, 0xDEADBEEF)
    r = rng.getrandbits(64) | (1 << 63)
    fr = [[sig[0][0], sig[0][1], sig[1][0], sig[1][1]], g1_proj(apk),
          [sig[0][0], sig[0][1], sig[1][0], sig[1][1], 1, 0], g1_proj(None)]
    for b in range(63, -1, -1):
        mode = 0 if b == 63 else (2 if (O.X_ABS >> b) & 1 else 1)
        fr = run(PROGS[f"SIG_STEP{mode}"], fr, pred=(r >> b) & 1)[:4]
    assert g2_aff(fr[2]) == O.g2_mul(sig, O.X_ABS)
    assert g1_aff(fr[3]) == O.g1_mul(apk, r)
    out = run(PROGS["G2_SUBCHK"], [fr[0], fr[2], [0] * 6])[2]
    assert out[:4] == [0, 0, 0, 0] and out[4:6] != [0, 0]


def test_msm_programs_pippenger():
    """Bucket accumulation (G2_ADDAFF_SEL), window running sums (RUNSUM) and
    the 2^8 Horner steps (G2X_8A) compute sum r_i sigma_i for 8-bit windows."""
    pts = [O.g2_mul(O.G2_GEN, 1000 + 17 * i) for i in range(5)]
    rs = [rng.getrandbits(64) for _ in pts]
    rs[0] = 0x0101010101010101  # repeated digits share buckets
    windows = []
    for w in range(8):
        buckets = {}
        for p_, r in zip(pts, rs):
            d = (r >> (8 * w)) & 0xFF
            if d:
                buckets.setdefault(d, []).append(p_)
        T, S = g2_proj(None), g2_proj(None)
        for d in range(255, 0, -1):
            B = g2_proj(None)
            for q in buckets.get(d, []):
                B = run(PROGS["G2_ADDAFF_SEL"], [B, [q[0][0], q[0][1], q[1][0], q[1][1]]], pred=1)[0]
            B = run(PROGS["G2_ADDAFF_SEL"], [B, [1, 2, 3, 4]], pred=0)[0]  # skipped step
            T, S = run(PROGS["RUNSUM"], [T, S, B])[:2]
        windows.append(S)
    W = windows[7]
    for w in range(6, -1, -1):
        W = run(PROGS["G2X_8A"], [W, windows[w], [0] * 6])[2]
    expect = None
    for p_, r in zip(pts, rs):
        expect = O.g2_add(expect, O.g2_mul(p_, r))
    assert g2_aff(W) == expect


@pytest.mark.parametrize("dummy", [False, True])
def test_shared_accumulator_miller_loop(dummy):
    """ML2_{FIRST,DBL,ADD}: two pairs share f; a pair with P = (0, 0) only
    contributes Fp2 factors, which the final exponentiation removes."""
    P1, Q1 = O.g1_mul(O.G1_GEN, 0x1111), O.g2_mul(O.G2_GEN, 0x2222)
    P2, Q2 = O.g1_mul(O.G1_GEN, 0x3333), O.g2_mul(O.G2_GEN, 0x4444)

    def pair_frames(P, Q):
        T = [Q[0][0], Q[0][1], Q[1][0], Q[1][1], 1, 0]
        Pf = [0, 0] if P is None else [(-P[0]) % O.P, P[1]]
        return [T, Pf, [Q[0][0], Q[0][1], Q[1][0], Q[1][1]]]

    fr = [[0] * 12] + pair_frames(P1, Q1) + pair_frames(None if dummy else P2, Q2)
    fr = run(PROGS["ML2_FIRST"], fr)[:7]
    if (O.X_ABS >> 62) & 1:
        fr = run(PROGS["ML2_ADD"], fr)[:7]
    for b in range(61, -1, -1):
        fr = run(PROGS["ML2_DBL"], fr)[:7]
        if (O.X_ABS >> b) & 1:
            fr = run(PROGS["ML2_ADD"], fr)[:7]
    got = O.final_exponentiation(O.f12_conj(list_f12(fr[0])))
    expect = O.pairing(P1, Q1) if dummy else O.f12_mul(O.pairing(P1, Q1), O.pairing(P2, Q2))
    assert got == expect
