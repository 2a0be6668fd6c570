"""GPU parity of the curve objects behind the reference's fastest_bls helpers
(E/utils/bls.py:224-392, arkworks G1Point / G2Point / GT): decoding with and
without subgroup checks, add / neg / multiply / multi_exp in G1 and G2,
multi_pairing / pairing_check, and the spec call shapes
(process_sync_aggregate's complement subtraction,
specs/altair/beacon-chain.md:592-596; verify_kzg_proof's pairing check,
specs/deneb/polynomial-commitments.md:402-409).  Expected values come from the
Python oracle (oracle/bls_oracle.py) and the trusted setup fixture."""
import json
import os

import pytest

from oracle import bls_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def shim():
    from bls_mi355x import bls

    bls.use_mi355x()
    bls.bls_active = True
    return bls


@pytest.fixture(scope="module")
def setup():
    with open(os.path.join(HERE, "golden", "trusted_setup.json")) as fh:
        return json.load(fh)


def _gt_bytes(f):
    return b"".join(c[0].to_bytes(48, "big") + c[1].to_bytes(48, "big") for c in O.f12_to_coeffs(f))


def _non_subgroup_g1():
    """A point of E1(Fp) outside G1 (the cofactor is not 1): the first x >= 1 with x^3 + 4 a square."""
    x = 1
    while True:
        y = O.fp_sqrt((x ** 3 + 4) % O.P)
        if y is not None:
            pt = (x, y)
            if not O.g1_in_subgroup(pt):
                return pt
        x += 1


def _non_subgroup_g2():
    x = 1
    while True:
        X = (x, 1)
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(X), X), O.B2))
        if y is not None:
            pt = (X, y)
            if not O.g2_in_subgroup(pt):
                return pt
        x += 1


def test_g1_add_neg_mul_against_oracle(shim):
    from bls_mi355x.curve import G1Point, Scalar

    a, b = O.g1_mul(O.G1_GEN, 12345), O.g1_mul(O.G1_GEN, 678)
    A, Bp = shim.bytes48_to_G1(O.g1_compress(a)), shim.bytes48_to_G1(O.g1_compress(b))
    assert shim.G1_to_bytes48(shim.add(A, Bp)) == O.g1_compress(O.g1_add(a, b))
    assert shim.G1_to_bytes48(shim.neg(A)) == O.g1_compress(O.g1_neg(a))
    assert shim.G1_to_bytes48(shim.add(A, shim.neg(A))) == O.g1_compress(None)        # P + (-P) = O
    assert shim.G1_to_bytes48(shim.add(A, A)) == O.g1_compress(O.g1_mul(a, 2))        # doubling branch
    assert shim.G1_to_bytes48(shim.add(A, shim.Z1())) == O.g1_compress(a)
    assert shim.neg(shim.Z1()) == shim.Z1()
    k = 0x1234567890ABCDEF1234567890ABCDEF1234567890ABCDEF1234567890ABCDEF % O.R
    assert shim.G1_to_bytes48(shim.multiply(A, k)) == O.g1_compress(O.g1_mul(a, k))
    assert shim.G1_to_bytes48(shim.multiply(A, -3)) == O.g1_compress(O.g1_mul(a, O.R - 3))
    assert shim.multiply(A, 0) == shim.Z1() and shim.multiply(shim.Z1(), 5) == shim.Z1()
    assert (A * Scalar(7)) == (Scalar(7) * A) == shim.multiply(A, 7)
    assert shim.G1() == G1Point() and shim.G1_to_bytes48(shim.G1()) == O.g1_compress(O.G1_GEN)


def test_g2_add_neg_mul_against_oracle(shim):
    a, b = O.g2_mul(O.G2_GEN, 999), O.g2_mul(O.G2_GEN, 31337)
    A, Bp = shim.bytes96_to_G2(O.g2_compress(a)), shim.bytes96_to_G2(O.g2_compress(b))
    assert shim.G2_to_bytes96(shim.add(A, Bp)) == O.g2_compress(O.g2_add(a, b))
    assert shim.G2_to_bytes96(shim.neg(A)) == O.g2_compress(O.g2_neg(a))
    assert shim.add(A, shim.neg(A)) == shim.Z2()
    assert shim.G2_to_bytes96(shim.add(A, A)) == O.g2_compress(O.g2_mul(a, 2))
    k = 0xFEDCBA9876543210 ** 3 % O.R
    assert shim.G2_to_bytes96(shim.multiply(A, k)) == O.g2_compress(O.g2_mul(a, k))
    assert shim.G2_to_bytes96(shim.G2()) == O.g2_compress(O.G2_GEN)


def test_decode_checked_vs_unchecked(shim):
    """bytes48_to_G1 / bytes96_to_G2 skip the subgroup check (E/utils/bls.py:367-392) but reject invalid
    encodings; from_compressed_bytes checks the subgroup."""
    from bls_mi355x.curve import G1Point, G2Point

    p1, p2 = _non_subgroup_g1(), _non_subgroup_g2()
    e1, e2 = O.g1_compress(p1), O.g2_compress(p2)
    assert shim.G1_to_bytes48(shim.bytes48_to_G1(e1)) == e1
    assert shim.G2_to_bytes96(shim.bytes96_to_G2(e2)) == e2
    with pytest.raises(ValueError):
        G1Point.from_compressed_bytes(e1)
    with pytest.raises(ValueError):
        G2Point.from_compressed_bytes(e2)
    # arithmetic on a non-subgroup point still follows the group law of E1 / E2
    assert shim.G1_to_bytes48(shim.add(shim.bytes48_to_G1(e1), shim.G1())) == O.g1_compress(O.g1_add(p1, O.G1_GEN))
    assert shim.G2_to_bytes96(shim.multiply(shim.bytes96_to_G2(e2), 5)) == O.g2_compress(O.g2_mul(p2, 5))
    for bad in (bytes(48), b"\x40" + bytes(47), b"\xc0\x10" + bytes(46), b"\x9a" + b"\xff" * 47):
        with pytest.raises(ValueError):
            shim.bytes48_to_G1(bad)
    with pytest.raises(ValueError):
        shim.bytes96_to_G2(bytes(96))
    assert shim.bytes48_to_G1(b"\xc0" + bytes(47)) == shim.Z1()


def test_multi_exp_against_oracle(shim, setup):
    from bls_mi355x.curve import G1Point, G2Point, Scalar

    g1 = [bytes.fromhex(h[2:]) for h in setup["g1_lagrange"][:37]]
    ks = [(7 ** (i + 3) + i) % O.R for i in range(37)]
    ks[5] = 0
    pts = [shim.bytes48_to_G1(b) for b in g1]
    pts[9] = shim.Z1()
    want = None
    for i, (b, k) in enumerate(zip(g1, ks)):
        if i != 9:
            want = O.g1_add(want, O.g1_mul(O.g1_decompress(b), k))
    assert shim.G1_to_bytes48(shim.multi_exp(pts, ks)) == O.g1_compress(want)
    assert shim.multi_exp(pts, [Scalar(k) for k in ks]) == shim.multi_exp(pts, ks)
    # Lagrange basis sums to the generator: sum of all 4096 with unit scalars
    allp = [shim.bytes48_to_G1(bytes.fromhex(h[2:])) for h in setup["g1_lagrange"]]
    assert shim.multi_exp(allp, [1] * len(allp)) == G1Point()
    g2 = [bytes.fromhex(h[2:]) for h in setup["g2_monomial"][:5]]
    want2 = None
    for i, b in enumerate(g2):
        want2 = O.g2_add(want2, O.g2_mul(O.g2_decompress(b), i + 2))
    got2 = shim.multi_exp([shim.bytes96_to_G2(b) for b in g2], list(range(2, 7)))
    assert isinstance(got2, G2Point) and shim.G2_to_bytes96(got2) == O.g2_compress(want2)
    with pytest.raises(Exception):
        shim.multi_exp([], [])
    # unchecked: a non-subgroup point is accepted (arkworks multiexp_unchecked)
    ns = shim.bytes48_to_G1(O.g1_compress(_non_subgroup_g1()))
    assert shim.multi_exp([ns], [1]) == ns


def test_multi_pairing_and_gt(shim, setup):
    from bls_mi355x.curve import GT, G1Point, G2Point

    a, b = 11, 23
    P, Q = O.g1_mul(O.G1_GEN, a), O.g2_mul(O.G2_GEN, b)
    e = GT.pairing(shim.bytes48_to_G1(O.g1_compress(P)), shim.bytes96_to_G2(O.g2_compress(Q)))
    assert e.to_bytes() == _gt_bytes(O.pairing(P, Q))
    g = GT.pairing(G1Point(), G2Point())
    assert e == GT.pairing(G1Point() * (a * b), G2Point())                 # bilinearity
    assert g * g == GT.pairing(G1Point() * 2, G2Point())
    assert GT.multi_pairing([G1Point(), G1Point().identity()], [G2Point(), G2Point()]) == g
    assert GT.multi_pairing([], []) == GT.one()
    # pairing_check shape of verify_kzg_proof_impl: e(P - [y]G1, -G2) e(proof, [s - z]G2) == 1 with
    # commitment = [f(s)], proof = [q(s)], f(s) - y = q(s)(s - z); setup monomials give [s^i]
    s1 = shim.bytes48_to_G1(bytes.fromhex(setup["g1_monomial"][1][2:]))   # [s]G1
    s2 = shim.bytes96_to_G2(bytes.fromhex(setup["g2_monomial"][1][2:]))   # [s]G2
    z, y = 5, 7
    # f(X) = X + (y - z): f(z) = y, q = 1; commitment = [s] + [y - z]G1, proof = G1
    commitment = shim.add(s1, shim.multiply(shim.G1(), y - z))
    X_minus_z = shim.add(s2, shim.multiply(shim.G2(), -z))
    P_minus_y = shim.add(commitment, shim.multiply(shim.G1(), -y))
    assert shim.pairing_check([[P_minus_y, shim.neg(shim.G2())], [shim.G1(), X_minus_z]]) is True
    assert shim.pairing_check([[P_minus_y, shim.neg(shim.G2())], [shim.multiply(shim.G1(), 2), X_minus_z]]) is False


def test_sync_aggregate_complement(shim):
    """process_sync_aggregate (specs/altair/beacon-chain.md:582-596): the participants' aggregate key as the
    committee aggregate minus the non-participants' aggregate, then FastAggregateVerify with it."""
    sks = [i + 101 for i in range(16)]
    pks = [O.SkToPk(k) for k in sks]
    agg = shim.AggregatePKs(pks)
    non = [0, 3, 7]
    nonpart = shim.AggregatePKs([pks[i] for i in non])
    part = shim.G1_to_bytes48(shim.add(shim.bytes48_to_G1(agg), shim.neg(shim.bytes48_to_G1(nonpart))))
    assert part == O.AggregatePKs([pks[i] for i in range(16) if i not in non])
    m = b"\x42" * 32
    sig = O.Sign(sum(sks[i] for i in range(16) if i not in non) % O.R, m)
    assert shim.eth_fast_aggregate_verify([part], m, sig) is True
    assert shim.eth_fast_aggregate_verify([agg], m, sig) is False
