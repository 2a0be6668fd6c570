"""Drop-in mirror of ``eth2spec.utils.bls`` (reference
tests/core/pyspec/eth2spec/utils/bls.py, cited below as ``bls.py:LINE``).

Same module-level switch (``bls_active``, ``bls``, ``Scalar``, ``use_*``),
same ``fastest_bls`` backend class, same ``only_with_bls`` stub values, same
exception-to-False mapping for the verify family, the same raising behaviour
for Aggregate / AggregatePKs / Sign / SkToPk, and the same curve helpers
(``pairing_check`` / ``add`` / ``multiply`` / ``multi_exp`` / ``neg`` / ``Z1``
/ ``Z2`` / ``G1`` / ``G2`` / ``G1_to_bytes48`` / ``G2_to_bytes96`` /
``bytes48_to_G1`` / ``bytes96_to_G2``) with the same
``bls == fastest_bls`` branch structure.

``fastest_bls`` here is the MI355X backend: its signature attributes are
``mi355x_bls``'s (milagro's role at bls.py:62-68) and its curve classes are
``curve.G1Point`` / ``G2Point`` / ``GT`` / ``Scalar`` (arkworks' role at
bls.py:58-61), so every helper branch the reference takes under
``use_fastest()`` is taken here too and runs on the GPU.  ``use_mi355x()``
(the default) is ``use_fastest()``.  The reference's own backends (milagro,
arkworks, py_ecc) are selectable only when their wheels are importable.
"""
from __future__ import annotations

from . import curve as _curve
from .backend import mi355x_bls


class fastest_bls:  # noqa: N801 -- bls.py:57-68
    G1 = _curve.G1Point
    G2 = _curve.G2Point
    Scalar = _curve.Scalar
    GT = _curve.GT
    _AggregatePKs = mi355x_bls._AggregatePKs
    Sign = mi355x_bls.Sign
    Verify = mi355x_bls.Verify
    Aggregate = mi355x_bls.Aggregate
    AggregateVerify = mi355x_bls.AggregateVerify
    FastAggregateVerify = mi355x_bls.FastAggregateVerify
    SkToPk = mi355x_bls.SkToPk


# bls.py:72 -- flag to make BLS active or not (tests only)
bls_active = True

# bls.py:74-76 -- default to fastest_bls
bls = fastest_bls
Scalar = fastest_bls.Scalar

STUB_SIGNATURE = b"\x11" * 96  # bls.py:78
STUB_PUBKEY = b"\x22" * 48  # bls.py:79
G2_POINT_AT_INFINITY = b"\xc0" + b"\x00" * 95  # bls.py:80
# bls.py:81 STUB_COORDINATES = signature_to_G2(G2_POINT_AT_INFINITY): the G2 identity
STUB_COORDINATES = _curve.G2Point.identity()

# sigsets.deferred(): when set, verify calls whose result flows straight into an ``assert`` are recorded here
# (and return True); every other verify call runs at once (sigsets.py).
_collector = None

# the reference backends, bound by use_milagro / use_arkworks / use_py_ecc when their wheels are importable
milagro_bls = None
arkworks_bls = None
py_ecc_bls = None


def use_fastest():  # bls.py:114-121
    global bls, Scalar
    bls = fastest_bls
    Scalar = fastest_bls.Scalar


def use_mi355x():
    """The MI355X backend for signatures and curve objects (= use_fastest(); new switch, cf. bls.py:84-121)."""
    use_fastest()


def _import_reference(modname: str):
    import importlib

    try:
        return importlib.import_module(modname)
    except ImportError as e:  # the reference wheels are not vendored
        raise ImportError(f"{modname} is not installed; only use_fastest() / use_mi355x() are available") from e


def use_milagro():  # bls.py:84-91
    global bls, Scalar, milagro_bls
    milagro_bls = _import_reference("milagro_bls_binding")
    bls = milagro_bls
    Scalar = _curve.Scalar  # py_ecc_Scalar's role: F_r with int arithmetic


def use_arkworks():  # bls.py:94-101
    global bls, Scalar, arkworks_bls
    arkworks_bls = _import_reference("py_arkworks_bls12381")
    bls = arkworks_bls
    Scalar = arkworks_bls.Scalar


def use_py_ecc():  # bls.py:104-111
    global bls, Scalar, py_ecc_bls
    py_ecc_bls = _import_reference("py_ecc.bls").G2ProofOfPossession
    bls = py_ecc_bls
    Scalar = _curve.Scalar


def only_with_bls(alt_return=None):  # bls.py:124-138
    def runner(fn):
        def entry(*args, **kw):
            if bls_active:
                return fn(*args, **kw)
            return alt_return

        # the wrapper's frame carries the wrapped function's name, so sigsets.result_is_asserted matches it to
        # the spec's call (``bls.Verify(...)`` calls a function named Verify)
        entry.__code__ = entry.__code__.replace(co_name=fn.__name__)
        entry.__name__ = entry.__qualname__ = fn.__name__
        return entry

    return runner


def _defer(kind: str, *args) -> bool:
    """Inside sigsets.deferred(): record the call if its result is only ever asserted (sigsets.py)."""
    return _collector is not None and _collector.try_defer(kind, args)


@only_with_bls(alt_return=True)
def Verify(PK, message, signature):  # bls.py:141-151
    if _defer("verify", PK, message, signature):
        return True
    try:
        result = bls.Verify(PK, message, signature)
    except Exception:
        result = False
    return bool(result)


@only_with_bls(alt_return=True)
def AggregateVerify(pubkeys, messages, signature):  # bls.py:154-164
    if _defer("av", pubkeys, messages, signature):
        return True
    try:
        result = bls.AggregateVerify(list(pubkeys), list(messages), signature)
    except Exception:
        result = False
    return bool(result)


@only_with_bls(alt_return=True)
def FastAggregateVerify(pubkeys, message, signature):  # bls.py:167-177
    if _defer("fav", pubkeys, message, signature):
        return True
    try:
        result = bls.FastAggregateVerify(list(pubkeys), message, signature)
    except Exception:
        result = False
    return bool(result)


@only_with_bls(alt_return=STUB_SIGNATURE)
def Aggregate(signatures):  # bls.py:180-184 (errors propagate)
    return bls.Aggregate(list(signatures))


@only_with_bls(alt_return=STUB_SIGNATURE)
def Sign(SK, message):  # bls.py:187-194 -- SK is an int, as in the spec
    if bls is py_ecc_bls and bls is not None:
        return bls.Sign(SK, message)
    return bls.Sign(int(SK).to_bytes(32, "big"), message)


@only_with_bls(alt_return=STUB_COORDINATES)
def signature_to_G2(signature):  # bls.py:197-199
    return bytes96_to_G2(signature)


@only_with_bls(alt_return=STUB_PUBKEY)
def AggregatePKs(pubkeys):  # bls.py:202-213 (fastest: _AggregatePKs KeyValidates each key, raises on failure)
    if bls is py_ecc_bls and bls is not None:
        assert all(bls.KeyValidate(pubkey) for pubkey in pubkeys)
    return bls._AggregatePKs(list(pubkeys))


@only_with_bls(alt_return=STUB_SIGNATURE)
def SkToPk(SK):  # bls.py:216-221
    if bls is py_ecc_bls and bls is not None:
        return bls.SkToPk(SK)
    return bls.SkToPk(int(SK).to_bytes(32, "big"))


# ---- curve helpers (bls.py:224-392) -------------------------------------------
def _fastest() -> bool:
    return bls == fastest_bls


def _need_fastest(name: str):
    if not _fastest():
        raise NotImplementedError(f"{name}: only the fastest_bls curve objects are available in this build")


def pairing_check(values):  # bls.py:224-236
    _need_fastest("pairing_check")
    p_q_1, p_q_2 = values
    g1s = [p_q_1[0], p_q_2[0]]
    g2s = [p_q_1[1], p_q_2[1]]
    return fastest_bls.GT.multi_pairing(g1s, g2s) == fastest_bls.GT.one()


def add(lhs, rhs):  # bls.py:239-246
    _need_fastest("add")
    return lhs + rhs


def multiply(point, scalar):  # bls.py:249-259
    _need_fastest("multiply")
    if not isinstance(scalar, fastest_bls.Scalar):
        return point * fastest_bls.Scalar(int(scalar))
    return point * scalar


def multi_exp(points, scalars):  # bls.py:262-296
    if not points or not scalars:
        raise Exception("Cannot call multi_exp with zero points or zero scalars")
    _need_fastest("multi_exp")
    if not isinstance(scalars[0], fastest_bls.Scalar):
        scalars = [fastest_bls.Scalar(int(s)) for s in scalars]
    if isinstance(points[0], fastest_bls.G1):
        return fastest_bls.G1.multiexp_unchecked(points, scalars)
    elif isinstance(points[0], fastest_bls.G2):
        return fastest_bls.G2.multiexp_unchecked(points, scalars)
    raise Exception("Invalid point type")


def neg(point):  # bls.py:299-306
    _need_fastest("neg")
    return -point


def Z1():  # bls.py:309-315
    _need_fastest("Z1")
    return fastest_bls.G1.identity()


def Z2():  # bls.py:318-324
    _need_fastest("Z2")
    return fastest_bls.G2.identity()


def G1():  # bls.py:327-333
    _need_fastest("G1")
    return fastest_bls.G1()


def G2():  # bls.py:336-342
    _need_fastest("G2")
    return fastest_bls.G2()


def G1_to_bytes48(point):  # bls.py:345-353
    _need_fastest("G1_to_bytes48")
    return bytes(point.to_compressed_bytes())


def G2_to_bytes96(point):  # bls.py:356-364
    _need_fastest("G2_to_bytes96")
    return bytes(point.to_compressed_bytes())


def bytes48_to_G1(bytes48):  # bls.py:367-378 (no subgroup check; invalid encodings raise)
    _need_fastest("bytes48_to_G1")
    return fastest_bls.G1.from_compressed_bytes_unchecked(bytes48)


def bytes96_to_G2(bytes96):  # bls.py:381-392
    _need_fastest("bytes96_to_G2")
    return fastest_bls.G2.from_compressed_bytes_unchecked(bytes96)


@only_with_bls(alt_return=True)
def KeyValidate(pubkey):  # bls.py:395-397 (py_ecc KeyValidate semantics, on the GPU)
    return mi355x_bls.KeyValidate(pubkey)


# --- spec-level helpers the generated specs call (specs/altair/bls.md) ---
def eth_aggregate_pubkeys(pubkeys):
    """specs/altair/bls.md:36-52, replaced by bls.AggregatePKs in pysetup/constants.py:31-34."""
    return AggregatePKs(pubkeys)


def eth_fast_aggregate_verify(pubkeys, message, signature):
    """specs/altair/bls.md:58-67."""
    if len(pubkeys) == 0 and bytes(signature) == G2_POINT_AT_INFINITY:
        return True
    return FastAggregateVerify(pubkeys, message, signature)
