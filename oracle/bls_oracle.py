"""BLS12-381 CPU oracle -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the MI355X backend.  It must only be
imported by ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of ``bench.py``; the product path (``eth-consensus-specs_amd/``) never
imports, links or calls anything under ``oracle/``.

It is a plain, deliberately un-optimised restatement (Python big integers) of
the algorithms the reference reaches through third-party wheels
(``milagro_bls_binding==1.9.0``, ``py_arkworks_bls12381==0.3.8``,
``py_ecc==8.0.0``, pinned at reference ``pyproject.toml:19-21``; none of them
is vendored under ``/root/reference`` nor importable in this container):

* ciphersuite ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`` (IETF BLS
  draft-04) -- reference ``specs/phase0/beacon-chain.md:688-703``;
* hash-to-curve per RFC 9380 (expand_message_xmd SHA-256 §5.3.1,
  hash_to_field §5.2, simplified SWU §6.6.2, 3-isogeny App. E.3,
  clear_cofactor via h_eff §8.8.2);
* ZCash compressed point encoding with the py_ecc / milagro edge semantics
  (``E/utils/bls.py:141-221,395-397``; decode rules: SURVEY.md §8(a));
* a textbook optimal-ate Miller loop evaluated on the untwisted curve over
  Fp12 (affine, one Fp12 inversion per step) and the final exponentiation
  (p^12-1)/r = (p^6-1)(p^2+1)(p^4-p^2+1)/r.

``E/`` = ``tests/core/pyspec/eth2spec/`` of the reference.

Pinning (what proves this oracle right, see tests/test_oracle.py):
* the staking-deposit-cli Verify known answer
  (``E/test/capella/block_processing/test_process_bls_to_execution_change.py:257-288``);
* KZG trusted-setup points (``presets/mainnet/trusted_setups/trusted_setup_4096.json``):
  decode/subgroup, sum of Lagrange basis = G1, bilinearity;
* SkToPk(1) == g1_monomial[0] (``E/test/helpers/keys.py:4``);
* the 20 ``altair/bls`` reference-test verdicts (``E/test/altair/bls/*.py``).
"""

from __future__ import annotations

import hashlib

# ---------------------------------------------------------------------------
# Parameters (SURVEY.md §8 "Shared facts")
# ---------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # the BLS parameter is x = -X_ABS
X = -X_ABS

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"  # beacon-chain.md:692-693

# ---------------------------------------------------------------------------
# Fp2 = Fp[i]/(i^2+1), elements are tuples (c0, c1) = c0 + c1*i
# ---------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (1, 1)  # the sextic non-residue 1+i


def f2(c0: int, c1: int = 0):
    return (c0 % P, c1 % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, k: int):
    return (a[0] * k % P, a[1] * k % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    if n == 0:
        raise ZeroDivisionError("Fp2 inverse of zero")
    ni = pow(n, -1, P)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def f2_pow(a, e: int):
    r = F2_ONE
    b = a
    while e > 0:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


# ---------------------------------------------------------------------------
# Fp square roots
# ---------------------------------------------------------------------------
def fp_is_square(a: int) -> bool:
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sqrt(a: int):
    """Some square root of a in Fp (p = 3 mod 4), or None."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def f2_is_square(a) -> bool:
    # a is a square in Fp2 iff its norm a0^2 + a1^2 is a square in Fp.
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """Some square root of a in Fp2, or None (norm method)."""
    a0, a1 = a
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0)  # (s*i)^2 = -s^2 = a0
        return (0, s) if s is not None else None
    n = fp_sqrt(a0 * a0 + a1 * a1)
    if n is None:
        return None
    inv2 = pow(2, -1, P)
    t = (a0 + n) * inv2 % P
    x0 = fp_sqrt(t)
    if x0 is None:
        t = (a0 - n) * inv2 % P
        x0 = fp_sqrt(t)
        if x0 is None:
            return None
    x1 = a1 * pow(2 * x0, -1, P) % P
    cand = (x0, x1)
    return cand if f2_sqr(cand) == (a0 % P, a1 % P) else None


# ---------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
# ---------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    c0 = f2_add(f2_mul(a0, b0), f2_mul(XI, f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul(XI, f2_mul(a2, b2)))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a1, b1)), f2_mul(a2, b0))
    return (c0, c1, c2)


def f6_mul_v(a):
    """a * v."""
    return (f2_mul(XI, a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul(XI, f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul(XI, f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    det = f2_add(f2_mul(a0, t0), f2_mul(XI, f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(det)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


def f12_add(a, b):
    return (f6_add(a[0], b[0]), f6_add(a[1], b[1]))


def f12_sub(a, b):
    return (f6_sub(a[0], b[0]), f6_sub(a[1], b[1]))


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    """a^(p^6): (a0 + a1 w) -> (a0 - a1 w)."""
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    d = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    di = f6_inv(d)
    return (f6_mul(a0, di), f6_neg(f6_mul(a1, di)))


def f12_pow(a, e: int):
    r = F12_ONE
    b = a
    while e > 0:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_from_f2(c, k: int):
    """The Fp12 element c * w^k for c in Fp2, 0 <= k < 6."""
    coeffs = [F2_ZERO] * 6
    coeffs[k] = c
    return f12_from_coeffs(coeffs)


def f12_from_coeffs(c):
    """From the w-basis coefficients c[0..5] (w^2 = v): a0 = c0 + c2 v + c4 v^2, a1 = c1 + c3 v + c5 v^2."""
    return ((c[0], c[2], c[4]), (c[1], c[3], c[5]))


def f12_to_coeffs(a):
    (c0, c2, c4), (c1, c3, c5) = a
    return [c0, c1, c2, c3, c4, c5]


# Frobenius: (c w^k)^p = conj(c) * gamma_k * w^k with gamma_k = xi^(k(p-1)/6).
_GAMMA1 = [f2_pow(XI, k * (P - 1) // 6) for k in range(6)]


def f12_frobenius(a):
    c = f12_to_coeffs(a)
    return f12_from_coeffs([f2_mul(f2_conj(c[k]), _GAMMA1[k]) for k in range(6)])


_HARD_EXP = (P**4 - P**2 + 1) // R
assert (P**4 - P**2 + 1) % R == 0


def final_exponentiation(f):
    """f^((p^12-1)/r), easy part with conj/inverse/Frobenius, hard part by plain exponentiation."""
    f1 = f12_mul(f12_conj(f), f12_inv(f))  # f^(p^6 - 1)
    f2_ = f12_mul(f12_frobenius(f12_frobenius(f1)), f1)  # ^(p^2 + 1)
    return f12_pow(f2_, _HARD_EXP)


# ---------------------------------------------------------------------------
# Curves.  Affine points are tuples (x, y); None is the point at infinity.
# E1: y^2 = x^3 + 4 over Fp;  E2: y^2 = x^3 + 4(1+i) over Fp2.
# ---------------------------------------------------------------------------
B1 = 4
B2 = (4, 4)


def g1_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g1_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_mul(pt, k: int):
    if k < 0:
        return g1_mul(g1_neg(pt), -k)
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = g1_add(acc, add)
        add = g1_add(add, add)
        k >>= 1
    return acc


def g2_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_neg(pt):
    return None if pt is None else (pt[0], f2_neg(pt[1]))


def g2_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if f2_add(y1, y2) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


def g2_mul(pt, k: int):
    if k < 0:
        return g2_mul(g2_neg(pt), -k)
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = g2_add(acc, add)
        add = g2_add(add, add)
        k >>= 1
    return acc


def g1_in_subgroup(pt) -> bool:
    return g1_mul(pt, R) is None


def g2_in_subgroup(pt) -> bool:
    return g2_mul(pt, R) is None


# psi = untwist-Frobenius-twist endomorphism on E2 (used to cross-check h_eff)
_PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
_PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    return (f2_mul(f2_conj(pt[0]), _PSI_CX), f2_mul(f2_conj(pt[1]), _PSI_CY))


# ---------------------------------------------------------------------------
# Serialisation (ZCash format; py_ecc pubkey_to_G1 / signature_to_G2 rules)
# ---------------------------------------------------------------------------
_POW2_381 = 1 << 381
_HALF_P = (P - 1) // 2


class DecodeError(ValueError):
    pass


def g1_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    v = x | (1 << 383) | ((1 << 381) if y > _HALF_P else 0)
    return v.to_bytes(48, "big")


def g1_decompress(data: bytes):
    """Decode 48 bytes -> affine point or None (infinity); raises DecodeError."""
    if len(data) != 48:
        raise DecodeError("G1 encoding must be 48 bytes")
    z = int.from_bytes(data, "big")
    c_flag = (z >> 383) & 1
    b_flag = (z >> 382) & 1
    a_flag = (z >> 381) & 1
    if not c_flag:
        raise DecodeError("c_flag must be 1")
    x = z % _POW2_381
    is_inf = x == 0
    if b_flag != is_inf:
        raise DecodeError("b_flag inconsistent with x == 0")
    if is_inf:
        if a_flag:
            raise DecodeError("infinity with a_flag")
        return None
    if x >= P:
        raise DecodeError("x >= p")
    y = fp_sqrt(x * x * x + B1)
    if y is None:
        raise DecodeError("not on curve")
    if (y > _HALF_P) != bool(a_flag):
        y = P - y
    return (x, y)


def _f2_lexicographically_largest(y) -> bool:
    y0, y1 = y
    if y1 != 0:
        return y1 > _HALF_P
    return y0 > _HALF_P


def g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    (x0, x1), y = pt
    z1 = x1 | (1 << 383) | ((1 << 381) if _f2_lexicographically_largest(y) else 0)
    return z1.to_bytes(48, "big") + x0.to_bytes(48, "big")


def g2_decompress(data: bytes):
    if len(data) != 96:
        raise DecodeError("G2 encoding must be 96 bytes")
    z1 = int.from_bytes(data[:48], "big")
    z2 = int.from_bytes(data[48:], "big")
    c_flag = (z1 >> 383) & 1
    b_flag = (z1 >> 382) & 1
    a_flag = (z1 >> 381) & 1
    if not c_flag:
        raise DecodeError("c_flag must be 1")
    x1 = z1 % _POW2_381
    is_inf = x1 == 0 and z2 == 0
    if b_flag != is_inf:
        raise DecodeError("b_flag inconsistent with x == 0")
    if is_inf:
        if a_flag:
            raise DecodeError("infinity with a_flag")
        return None
    if x1 >= P or z2 >= P:
        raise DecodeError("x >= p")
    x = (z2, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("not on curve")
    if _f2_lexicographically_largest(y) != bool(a_flag):
        y = f2_neg(y)
    return (x, y)


# Generators: g1_monomial[0] / g2_monomial[0] of the reference trusted setup
G1_GEN = g1_decompress(
    bytes.fromhex(
        "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"
    )
)
G2_GEN = g2_decompress(
    bytes.fromhex(
        "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
        "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8"
    )
)

# ---------------------------------------------------------------------------
# Pairing: textbook optimal ate on E(Fp12)
# ---------------------------------------------------------------------------
_W = f12_from_f2(F2_ONE, 1)
_W_INV = f12_inv(_W)
_W_INV2 = f12_mul(_W_INV, _W_INV)
_W_INV3 = f12_mul(_W_INV2, _W_INV)


def _fp_to_12(a: int):
    return f12_from_f2((a % P, 0), 0)


def untwist(q):
    """E2 (the M-type sextic twist) -> E(Fp12): (x, y) -> (x w^-2, y w^-3)."""
    return (f12_mul(f12_from_f2(q[0], 0), _W_INV2), f12_mul(f12_from_f2(q[1], 0), _W_INV3))


def miller_loop(p1, q2):
    """f_{x,Q}(P) (x < 0 handled by conjugation); 1 if either point is infinity."""
    if p1 is None or q2 is None:
        return F12_ONE
    xp, yp = _fp_to_12(p1[0]), _fp_to_12(p1[1])
    qx, qy = untwist(q2)
    tx, ty = qx, qy
    f = F12_ONE
    for bit in bin(X_ABS)[3:]:
        # tangent at T
        lam = f12_mul(f12_mul(_fp_to_12(3), f12_sqr(tx)), f12_inv(f12_add(ty, ty)))
        line = f12_sub(f12_sub(yp, ty), f12_mul(lam, f12_sub(xp, tx)))
        f = f12_mul(f12_sqr(f), line)
        nx = f12_sub(f12_sqr(lam), f12_add(tx, tx))
        ty = f12_sub(f12_mul(lam, f12_sub(tx, nx)), ty)
        tx = nx
        if bit == "1":
            lam = f12_mul(f12_sub(qy, ty), f12_inv(f12_sub(qx, tx)))
            line = f12_sub(f12_sub(yp, ty), f12_mul(lam, f12_sub(xp, tx)))
            f = f12_mul(f, line)
            nx = f12_sub(f12_sub(f12_sqr(lam), tx), qx)
            ty = f12_sub(f12_mul(lam, f12_sub(tx, nx)), ty)
            tx = nx
    return f12_conj(f)


def pairing(p1, q2):
    return final_exponentiation(miller_loop(p1, q2))


def pairing_product_is_one(pairs) -> bool:
    f = F12_ONE
    for p1, q2 in pairs:
        f = f12_mul(f, miller_loop(p1, q2))
    return final_exponentiation(f) == F12_ONE


# ---------------------------------------------------------------------------
# Hash to G2 (RFC 9380, suite BLS12381G2_XMD:SHA-256_SSWU_RO_)
# ---------------------------------------------------------------------------
def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    if len(dst) > 255:
        raise ValueError("DST too long")
    ell = (len_in_bytes + 31) // 32
    if ell > 255:
        raise ValueError("len_in_bytes too large")
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(64) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, count: int, dst: bytes):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = [int.from_bytes(ub[L * (2 * i + j): L * (2 * i + j + 1)], "big") % P for j in range(2)]
        out.append((e[0], e[1]))
    return out


# Simplified SWU on E2': y^2 = x^3 + A'x + B'
SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = f2(-2, -1)


def f2_sgn0(a) -> int:
    sign_0 = a[0] & 1
    zero_0 = a[0] == 0
    sign_1 = a[1] & 1
    return sign_0 | (zero_0 & sign_1)


def map_to_curve_sswu(u):
    """RFC 9380 §6.6.2 straight-line description, output on E2'."""
    z_u2 = f2_mul(SSWU_Z, f2_sqr(u))
    den = f2_add(f2_sqr(z_u2), z_u2)  # Z^2 u^4 + Z u^2
    if den == F2_ZERO:
        x1 = f2_mul(SSWU_B, f2_inv(f2_mul(SSWU_Z, SSWU_A)))
    else:
        tv1 = f2_inv(den)
        x1 = f2_mul(f2_mul(f2_neg(SSWU_B), f2_inv(SSWU_A)), f2_add(F2_ONE, tv1))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(SSWU_A, x1)), SSWU_B)
    x2 = f2_mul(z_u2, x1)
    gx2 = f2_add(f2_add(f2_mul(f2_sqr(x2), x2), f2_mul(SSWU_A, x2)), SSWU_B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x, y = x2, f2_sqrt(gx2)
    assert y is not None
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def _k(c0, c1=0):
    return (c0 % P, c1 % P)


# 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3)
ISO_XNUM = [
    _k(0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
       0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    _k(0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    _k(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
       0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    _k(0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO_XDEN = [
    _k(0, -72),
    _k(12, -12),
    _k(1, 0),
]
ISO_YNUM = [
    _k(0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
       0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    _k(0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    _k(0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
       0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    _k(0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO_YDEN = [
    _k(-432, -432),
    _k(0, -216),
    _k(18, -18),
    _k(1, 0),
]


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso_map(pt):
    if pt is None:
        return None
    x, y = pt
    xd = _poly(ISO_XDEN, x)
    yd = _poly(ISO_YDEN, x)
    if xd == F2_ZERO or yd == F2_ZERO:
        return None
    xo = f2_mul(_poly(ISO_XNUM, x), f2_inv(xd))
    yo = f2_mul(y, f2_mul(_poly(ISO_YNUM, x), f2_inv(yd)))
    return (xo, yo)


H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551


def clear_cofactor_g2(pt):
    return g2_mul(pt, H_EFF_G2)


def clear_cofactor_g2_psi(pt):
    """Budroni-Pintore: [x^2-x-1]P + [x-1]psi(P) + psi^2(2P) (RFC 9380 App. G.3); cross-check only."""
    t1 = g2_mul(pt, X * X - X - 1)
    t2 = g2_mul(g2_psi(pt), X - 1)
    t3 = g2_psi(g2_psi(g2_add(pt, pt)))
    return g2_add(g2_add(t1, t2), t3)


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, 2, dst)
    q0 = iso_map(map_to_curve_sswu(u0))
    q1 = iso_map(map_to_curve_sswu(u1))
    return clear_cofactor_g2(g2_add(q0, q1))


# ---------------------------------------------------------------------------
# BLS POP ciphersuite with the reference's wrapper semantics
# ---------------------------------------------------------------------------
def _sk_int(sk) -> int:
    k = int.from_bytes(sk, "big") if isinstance(sk, (bytes, bytearray)) else int(sk)
    if not 0 < k < R:
        raise ValueError("secret key out of range")
    return k


def SkToPk(sk) -> bytes:
    return g1_compress(g1_mul(G1_GEN, _sk_int(sk)))


def Sign(sk, message: bytes) -> bytes:
    return g2_compress(g2_mul(hash_to_g2(message), _sk_int(sk)))


def KeyValidate(pk: bytes) -> bool:
    try:
        pt = g1_decompress(bytes(pk))
    except DecodeError:
        return False
    return pt is not None and g1_in_subgroup(pt)


def _decode_sig(sig: bytes):
    """Signature decode + subgroup check (raises DecodeError)."""
    pt = g2_decompress(bytes(sig))
    if not g2_in_subgroup(pt):
        raise DecodeError("signature not in G2")
    return pt


def _core_verify(pk_pt, message: bytes, sig: bytes) -> bool:
    try:
        s = _decode_sig(sig)
    except DecodeError:
        return False
    return pairing_product_is_one([(pk_pt, hash_to_g2(message)), (g1_neg(G1_GEN), s)])


def Verify(pk: bytes, message: bytes, sig: bytes) -> bool:
    if not KeyValidate(pk):
        return False
    return _core_verify(g1_decompress(bytes(pk)), message, sig)


def _aggregate_pk_points(pks):
    agg = None
    for pk in pks:
        if not KeyValidate(pk):
            raise DecodeError("invalid pubkey")
        agg = g1_add(agg, g1_decompress(bytes(pk)))
    return agg


def AggregatePKs(pks) -> bytes:
    """milagro ``_AggregatePKs`` under ``use_fastest`` (E/utils/bls.py:202-213): raises on empty / invalid."""
    pks = list(pks)
    if len(pks) == 0:
        raise DecodeError("no pubkeys")
    return g1_compress(_aggregate_pk_points(pks))


def FastAggregateVerify(pks, message: bytes, sig: bytes) -> bool:
    pks = list(pks)
    if len(pks) == 0:
        return False
    try:
        agg = _aggregate_pk_points(pks)
    except DecodeError:
        return False
    if agg is None:  # KeyValidate(aggregate) fails on the identity
        return False
    return _core_verify(agg, message, sig)


def AggregateVerify(pks, messages, sig: bytes) -> bool:
    pks = list(pks)
    messages = list(messages)
    if len(pks) == 0 or len(pks) != len(messages):
        return False
    if not all(KeyValidate(pk) for pk in pks):
        return False
    try:
        s = _decode_sig(sig)
    except DecodeError:
        return False
    pairs = [(g1_decompress(bytes(pk)), hash_to_g2(m)) for pk, m in zip(pks, messages)]
    pairs.append((g1_neg(G1_GEN), s))
    return pairing_product_is_one(pairs)


def Aggregate(sigs) -> bytes:
    sigs = list(sigs)
    if len(sigs) == 0:
        raise DecodeError("no signatures")
    agg = None
    for s in sigs:
        agg = g2_add(agg, _decode_sig(s))
    return g2_compress(agg)


G2_POINT_AT_INFINITY = bytes([0xC0]) + bytes(95)


def eth_fast_aggregate_verify(pks, message: bytes, sig: bytes) -> bool:
    """specs/altair/bls.md:58-67."""
    pks = list(pks)
    if len(pks) == 0 and bytes(sig) == G2_POINT_AT_INFINITY:
        return True
    return FastAggregateVerify(pks, message, sig)
