"""The wave programs (tools/wavec.py -> bls_waveprog.h) evaluated by a Python
model of the device interpreter (bls_wave.h) against the oracle: CPU-side
proof that the traced formulas and the level schedule are right."""
import os
import random
import sys

import pytest

from oracle import bls_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import wavec  # noqa: E402

PROGS = {p["name"]: p for p in wavec.compile_all()}
rng = random.Random(7)
MONT = 1 << 384
RINV = pow(MONT, -1, O.P)


def run(prog, frames):
    """frames: list of lists of ints (canonical values); scratch appended. Mirrors wave_run."""
    fr = [list(f) for f in frames] + [[0] * prog["frames"][-1]]
    # Montgomery domain is transparent for lincombs; model products as a*b (canonical)
    for ix, v in prog["consts"]:
        fr[-1][ix] = v % O.P
    for items in prog["levels"]:
        assert len(items) <= 64
        vals = []
        for kind, (dfr, dix), a, b in items:
            va = sum(k * fr[f][i] for f, i, k in a) % O.P
            if kind == "mul":
                vb = sum(k * fr[f][i] for f, i, k in b) % O.P
                va = va * vb % O.P
            vals.append(((dfr, dix), va))
        for (dfr, dix), v in vals:  # all reads of a level precede its writes
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


def test_fp12_mul_and_sqr_programs():
    for _ in range(3):
        a, b = rf12(), rf12()
        fr = run(PROGS["FP12_MUL"], [f12_list(a), f12_list(b), [0] * 12])
        assert list_f12(fr[2]) == O.f12_mul(a, b)
        fr = run(PROGS["FP12_SQR"], [f12_list(a), [0] * 12])
        assert list_f12(fr[1]) == O.f12_sqr(a)


def test_level_widths_fit_a_wave():
    for p in PROGS.values():
        for items in p["levels"]:
            assert 1 <= len(items) <= 64


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
