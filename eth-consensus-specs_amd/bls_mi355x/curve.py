"""Curve objects of the MI355X backend: ``G1Point``, ``G2Point``, ``GT`` and
``Scalar``, the roles ``fastest_bls.G1/G2/GT/Scalar`` play in the reference
(``py_arkworks_bls12381`` classes bound at E/utils/bls.py:3-8,57-61, with
E = tests/core/pyspec/eth2spec).  They back the reference's curve helpers --
``add`` / ``multiply`` / ``multi_exp`` / ``neg`` / ``Z1`` / ``Z2`` / ``G1`` /
``G2`` / ``G1_to_bytes48`` / ``G2_to_bytes96`` / ``bytes48_to_G1`` /
``bytes96_to_G2`` / ``pairing_check`` (E/utils/bls.py:224-392) -- that
``process_sync_aggregate`` (specs/altair/beacon-chain.md:592-596) and the KZG
functions (specs/deneb/polynomial-commitments.md) call.

A point object holds its compressed encoding (48 / 96 bytes).  A valid
compressed encoding is unique per point (flags are exact, x < p, one sign
bit), so equality and hashing are byte comparisons.  All group arithmetic
(decoding, addition, scalar multiplication, multi-exponentiation, pairings)
runs on the GPU through the C ABI (``bls_point_*``, ``bls_multi_exp``,
``bls_multi_pairing``; include/blsmi355x.h); there is no CPU fallback.
``Scalar`` is an element of the scalar field F_r with Python-int arithmetic,
as the reference's ``py_ecc_Scalar`` (E/utils/bls.py:35-54).
"""
from __future__ import annotations

import ctypes

from . import _native

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001  # BLS_MODULUS

G1_GENERATOR = bytes.fromhex(
    "97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G2_GENERATOR = bytes.fromhex(
    "93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
    "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")
G1_IDENTITY = b"\xc0" + bytes(47)
G2_IDENTITY = b"\xc0" + bytes(95)
GT_ONE = bytes(47) + b"\x01" + bytes(528)


def _ctx():
    return _native.context()


class Scalar:
    """Element of F_r (r = BLS_MODULUS); ints are reduced mod r on construction."""

    __slots__ = ("n",)

    def __init__(self, value=0):
        self.n = int(value) % R

    @staticmethod
    def _v(x) -> int:
        return x.n if isinstance(x, Scalar) else int(x) % R

    def _new(self, v: int):
        return type(self)(v)

    def __int__(self):
        return self.n

    __index__ = __int__

    def __add__(self, o):
        return self._new(self.n + self._v(o))

    __radd__ = __add__

    def __sub__(self, o):
        return self._new(self.n - self._v(o))

    def __rsub__(self, o):
        return self._new(self._v(o) - self.n)

    def __mul__(self, o):
        if isinstance(o, (G1Point, G2Point)):
            return o * self
        return self._new(self.n * self._v(o))

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self * type(self)(self._v(o)).inverse()

    def __rtruediv__(self, o):
        return type(self)(self._v(o)) * self.inverse()

    def __neg__(self):
        return self._new(-self.n)

    def __pow__(self, e):
        return self._new(pow(self.n, int(e), R))

    def pow(self, e):
        return self ** int(e)

    def inverse(self):
        if self.n == 0:
            raise ZeroDivisionError("inverse of zero in F_r")
        return self._new(pow(self.n, -1, R))

    def square(self):
        return self._new(self.n * self.n)

    def is_zero(self) -> bool:
        return self.n == 0

    def __eq__(self, o):
        if isinstance(o, Scalar):
            return self.n == o.n
        if isinstance(o, int):
            return self.n == o % R
        return NotImplemented

    def __ne__(self, o):
        r = self.__eq__(o)
        return r if r is NotImplemented else not r

    def __lt__(self, o):
        return self.n < self._v(o)

    def __hash__(self):
        return hash(self.n)

    def __repr__(self):
        return f"{type(self).__name__}({self.n})"

    def to_le_bytes(self) -> bytes:
        return self.n.to_bytes(32, "little")

    def to_be_bytes(self) -> bytes:
        return self.n.to_bytes(32, "big")

    @classmethod
    def from_le_bytes(cls, b: bytes):
        return cls(int.from_bytes(bytes(b), "little"))


def _k32(s) -> bytes:
    return (s.n if isinstance(s, Scalar) else int(s) % R).to_bytes(32, "big")


class _Point:
    GROUP = 0
    WIDTH = 0
    GEN = b""
    IDENTITY = b""

    __slots__ = ("_b",)

    def __init__(self, _encoding: bytes | None = None):
        """``G1Point()`` / ``G2Point()`` is the generator (arkworks convention)."""
        self._b = self.GEN if _encoding is None else _encoding

    @classmethod
    def _wrap(cls, b: bytes):
        p = cls.__new__(cls)
        p._b = bytes(b)
        return p

    @classmethod
    def identity(cls):
        return cls._wrap(cls.IDENTITY)

    @classmethod
    def _decode(cls, data, subgroup: int):
        b = bytes(data)
        if len(b) != cls.WIDTH:
            raise ValueError(f"expected {cls.WIDTH} bytes, got {len(b)}")
        c = _ctx()
        if c.check(c.lib.bls_point_decode(c.h, cls.GROUP, b, 1, subgroup, None)) != 1:
            raise ValueError("invalid compressed point encoding" + (" or not in the subgroup" if subgroup else ""))
        return cls._wrap(b)

    @classmethod
    def from_compressed_bytes_unchecked(cls, data):
        """Decode without the subgroup check (E/utils/bls.py:367-392); raises on invalid encodings."""
        return cls._decode(data, 0)

    @classmethod
    def from_compressed_bytes(cls, data):
        """Decode with the subgroup check."""
        return cls._decode(data, 1)

    def to_compressed_bytes(self) -> bytes:
        return self._b

    def __bytes__(self):
        return self._b

    def __add__(self, other):
        if type(other) is not type(self):
            return NotImplemented
        c = _ctx()
        out = ctypes.create_string_buffer(self.WIDTH)
        if c.check(c.lib.bls_point_add(c.h, self.GROUP, self._b, other._b, out)) != 1:
            raise ValueError("invalid point encoding")
        return self._wrap(out.raw)

    def __neg__(self):
        c = _ctx()
        out = ctypes.create_string_buffer(self.WIDTH)
        if c.check(c.lib.bls_point_neg(c.h, self.GROUP, self._b, out)) != 1:
            raise ValueError("invalid point encoding")
        return self._wrap(out.raw)

    def __sub__(self, other):
        return self + (-other)

    def __mul__(self, scalar):
        if not isinstance(scalar, (Scalar, int)):
            return NotImplemented
        c = _ctx()
        out = ctypes.create_string_buffer(self.WIDTH)
        if c.check(c.lib.bls_point_mul(c.h, self.GROUP, self._b, _k32(scalar), out)) != 1:
            raise ValueError("invalid point encoding")
        return self._wrap(out.raw)

    __rmul__ = __mul__

    def __eq__(self, other):
        if type(other) is not type(self):
            return NotImplemented
        return self._b == other._b

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __hash__(self):
        return hash((self.GROUP, self._b))

    def __repr__(self):
        return f"{type(self).__name__}({self._b.hex()})"

    @classmethod
    def multiexp_unchecked(cls, points, scalars):
        """sum_i [k_i] P_i without subgroup checks (E/utils/bls.py:273-282); raises on empty input."""
        return cls._multiexp(points, scalars, 0)

    @classmethod
    def multiexp(cls, points, scalars):
        return cls._multiexp(points, scalars, 1)

    @classmethod
    def _multiexp(cls, points, scalars, subgroup: int):
        pts = list(points)
        ks = list(scalars)
        if not pts or not ks:
            raise ValueError("Cannot call multi_exp with zero points or zero scalars")
        if len(pts) != len(ks):
            raise ValueError("one scalar per point")
        if any(type(p) is not cls for p in pts):
            raise TypeError(f"multiexp over {cls.__name__} needs {cls.__name__} points")
        c = _ctx()
        out = ctypes.create_string_buffer(cls.WIDTH)
        rc = c.check(c.lib.bls_multi_exp(c.h, cls.GROUP, b"".join(p._b for p in pts), b"".join(_k32(k) for k in ks),
                                         len(pts), subgroup, out))
        if rc != 1:
            raise ValueError("invalid point encoding")
        return cls._wrap(out.raw)


class G1Point(_Point):
    GROUP, WIDTH, GEN, IDENTITY = 1, 48, G1_GENERATOR, G1_IDENTITY
    __slots__ = ()


class G2Point(_Point):
    GROUP, WIDTH, GEN, IDENTITY = 2, 96, G2_GENERATOR, G2_IDENTITY
    __slots__ = ()


class GT:
    """Target-group element (576 bytes: six Fp2 coefficients, big-endian; include/blsmi355x.h)."""

    __slots__ = ("_b",)

    def __init__(self, _encoding: bytes = GT_ONE):
        self._b = bytes(_encoding)

    @classmethod
    def one(cls):
        return cls(GT_ONE)

    @classmethod
    def _pairing(cls, g1s, g2s, subgroup: int):
        g1s, g2s = list(g1s), list(g2s)
        if len(g1s) != len(g2s):
            raise ValueError("need as many G1 as G2 points")
        if any(not isinstance(p, G1Point) for p in g1s) or any(not isinstance(q, G2Point) for q in g2s):
            raise TypeError("multi_pairing takes G1Point and G2Point lists")
        c = _ctx()
        out = ctypes.create_string_buffer(576)
        rc = c.check(c.lib.bls_multi_pairing(c.h, b"".join(p._b for p in g1s), b"".join(q._b for q in g2s), len(g1s),
                                             subgroup, out))
        if rc != 1:
            raise ValueError("invalid point encoding")
        return cls(out.raw)

    @classmethod
    def multi_pairing(cls, g1s, g2s):
        """prod_i e(P_i, Q_i) (one shared final exponentiation), as arkworks GT.multi_pairing."""
        return cls._pairing(g1s, g2s, 0)

    @classmethod
    def pairing(cls, g1: G1Point, g2: G2Point):
        return cls._pairing([g1], [g2], 0)

    def __mul__(self, other):
        if not isinstance(other, GT):
            return NotImplemented
        c = _ctx()
        out = ctypes.create_string_buffer(576)
        c.check(c.lib.bls_gt_mul(c.h, self._b, other._b, out))
        return GT(out.raw)

    def to_bytes(self) -> bytes:
        return self._b

    def __eq__(self, other):
        if not isinstance(other, GT):
            return NotImplemented
        return self._b == other._b

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __hash__(self):
        return hash(self._b)


def pairing_product_is_one(g1s, g2s) -> bool:
    """GT.multi_pairing(g1s, g2s) == GT.one() in one device call (no GT bytes cross the boundary)."""
    g1s, g2s = list(g1s), list(g2s)
    if len(g1s) != len(g2s):
        raise ValueError("need as many G1 as G2 points")
    c = _ctx()
    return c.check(c.lib.bls_pairing_check_ex(c.h, b"".join(bytes(p) for p in g1s), b"".join(bytes(q) for q in g2s),
                                              len(g1s), 0)) == 1
