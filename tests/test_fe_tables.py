"""tools/gen_fe.py (the phase tables of the lane-parallel final exponentiation, bls_fe.hip) against the
oracle: every operation's phases run on exact integers with the generator's own simulator (Montgomery
semantics, value-bound checks) and the results are compared with oracle/bls_oracle.py tower arithmetic; the
whole device schedule gives FE(f)^3 (the hard part's (x-1)^2 (x+p)(x^2+p^2-1) + 3 = 3 (p^4-p^2+1)/r)."""
import os
import random
import sys

import pytest

from oracle import bls_oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import gen_fe as G  # noqa: E402

RM = G.RMONT % G.P


def _rand12(rng):
    return tuple(tuple((rng.randrange(O.P), rng.randrange(O.P)) for _ in range(3)) for _ in range(2))


def _flat(f):  # tower order j = 6 h + 2 k + part
    return [f[h][k][part] for h in range(2) for k in range(3) for part in range(2)]


def _unflat(v):
    return tuple(tuple((v[6 * h + 2 * k], v[6 * h + 2 * k + 1]) for k in range(3)) for h in range(2))


@pytest.fixture(scope="module")
def ops():
    ops = G.build_ops()
    G.check_schedule(ops)  # sets every LIN offset and asserts the bounds
    return ops


def _sim_with(bank_vals):
    sim = G.Sim()
    G.init_consts(sim)
    for bank, f in bank_vals.items():
        G.load_f12(sim, bank, [x * RM % O.P for x in _flat(f)])
    return sim


def _read(sim, bank):
    return _unflat([sim.val[bank * 12 + j] * G.RINV % O.P for j in range(12)])


def _cyclotomic(rng):
    f = _rand12(rng)
    t = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
    return O.f12_mul(O.f12_frobenius(O.f12_frobenius(t)), t)


def test_mul(ops):
    rng = random.Random(1)
    for _ in range(3):
        a, b = _rand12(rng), _rand12(rng)
        sim = _sim_with({0: a, 1: b})
        G.sim_op(sim, ops["MUL"], 0, 1, 2)
        assert _read(sim, 2) == O.f12_mul(a, b)
        G.sim_op(sim, ops["MUL"], 0, 1, 0)  # destination aliasing an operand
        assert _read(sim, 0) == O.f12_mul(a, b)


def test_cyclotomic_square(ops):
    rng = random.Random(2)
    g = _cyclotomic(rng)
    sim = _sim_with({3: g})
    G.sim_op(sim, ops["CYC"], 3, 0, 3)
    assert _read(sim, 3) == O.f12_mul(g, g)


def test_conj_frobenius(ops):
    rng = random.Random(3)
    a = _rand12(rng)
    sim = _sim_with({0: a})
    G.sim_op(sim, ops["CONJ"], 0, 0, 1)
    G.sim_op(sim, ops["FROB1"], 0, 0, 2)
    G.sim_op(sim, ops["FROB2"], 0, 0, 3)
    assert _read(sim, 1) == O.f12_conj(a)
    assert _read(sim, 2) == O.f12_frobenius(a)
    assert _read(sim, 3) == O.f12_frobenius(O.f12_frobenius(a))


def test_easy_part(ops):
    rng = random.Random(4)
    f = _rand12(rng)
    sim = _sim_with({0: f})
    for name, a, b, d in G.schedule()[:3]:
        G.sim_op(sim, ops[name], a, b, d)
    assert _read(sim, 0) == O.f12_mul(O.f12_conj(f), O.f12_inv(f))


def test_full_schedule_is_fe_cubed(ops):
    rng = random.Random(6)
    f = _rand12(rng)
    sim = _sim_with({0: f})
    for name, a, b, d in G.schedule():
        G.sim_op(sim, ops[name], a, b, d)
    fe = O.final_exponentiation(f)
    assert _read(sim, 1) == O.f12_mul(O.f12_mul(fe, fe), fe)
