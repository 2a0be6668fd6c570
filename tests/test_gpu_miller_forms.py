"""GPU parity of the Miller-loop forms of the batch path (bls_test_miller_forms): the split kernels (the G2 lines of
k_miller_lines2 + the f accumulation of k_miller_acc4q, two, four or eight pairs per f, and k_miller_acc4l: four
pairs per f with each step's lines multiplied together before they meet f; k_miller_acc8: one pair per f on eight
lanes), the fused kernel
(k_miller_fused: lines formed in LDS by a line wave, one or two pairs per f) and the wave-program kernel of
bls_multi_pairing -- the final exponentiation of each form's product must be the same GT element, and equal the
oracle's pairing product (oracle/bls_oracle.py).  Pair counts are chosen off every multiple the kernels group by
(32 / 64 pairs per fused workgroup, 2 / 4 / 8 pairs per f, 16 f per wave), with identity pairs among them."""
import ctypes
import random

import pytest

from oracle import bls_oracle as O

pytestmark = pytest.mark.gpu

FORMS = ("split G=2", "fused G=2", "fused G=1", "split G=4", "wave program", "split G=8", "split G=4 lines first",
         "split G=1 eight lanes")


def _gt_bytes(f):
    return b"".join(c[0].to_bytes(48, "big") + c[1].to_bytes(48, "big") for c in O.f12_to_coeffs(f))


def _pairs(n, seed, identities=()):
    r = random.Random(seed)
    g1 = O.G1_GEN
    g2 = O.hash_to_g2(b"miller forms %d" % seed)
    ps, qs = [], []
    for i in range(n):
        a, b = r.randrange(1, 1 << 40), r.randrange(1, 1 << 40)
        ps.append(None if i in identities else O.g1_mul(g1, a))
        qs.append(O.g2_mul(g2, b))
    return ps, qs


def _forms(ps, qs):
    from bls_mi355x import _native

    ctx = _native.context()
    g1 = b"".join(O.g1_compress(p) for p in ps)
    g2 = b"".join(O.g2_compress(q) for q in qs)
    out = ctypes.create_string_buffer(len(FORMS) * 576)
    assert ctx.check(ctx.lib.bls_test_miller_forms(ctx.h, g1, g2, len(ps), out)) == 1
    return [out.raw[576 * k: 576 * k + 576] for k in range(len(FORMS))]


@pytest.mark.parametrize("n,ids", [(5, (2,)), (37, (0, 36)), (131, (64, 65, 130)), (13, (4, 5, 6, 7, 9, 10))])
def test_miller_forms_agree_with_the_oracle(n, ids):
    ps, qs = _pairs(n, 1000 + n, ids)
    got = _forms(ps, qs)
    for k in range(1, len(FORMS)):
        assert got[k] == got[0], FORMS[k]
    if n <= 5:  # the oracle's pairing product (slow in Python: small n only)
        f = O.F12_ONE
        for p, q in zip(ps, qs):
            if p is not None:
                f = O.f12_mul(f, O.miller_loop(p, q))
        assert got[0] == _gt_bytes(O.final_exponentiation(f))


def test_miller_forms_full_workgroups():
    """700 pairs: eleven fused G=2 workgroups (the last one short), 22 G=1 workgroups, partial waves of f."""
    ps, qs = _pairs(700, 77, identities=(0, 1, 63, 64, 699))
    got = _forms(ps, qs)
    assert all(g == got[0] for g in got), [FORMS[k] for k in range(len(FORMS)) if got[k] != got[0]]
