"""Drop-in mirror of ``eth2spec.utils.bls`` (reference
tests/core/pyspec/eth2spec/utils/bls.py, cited below as ``bls.py:LINE``).

Same module-level switch (``bls_active``, ``bls``, ``use_*``), same
``only_with_bls`` stub values, same exception-to-False mapping for the verify
family and the same raising behaviour for Aggregate / AggregatePKs / Sign /
SkToPk.  ``use_mi355x()`` (the default here) routes every call to the
MI355X backend; the reference's own backends (milagro, arkworks, py_ecc)
are selectable only when those wheels are importable.
"""
from __future__ import annotations

from .backend import mi355x_bls

# bls.py:72 -- flag to make BLS active or not (tests only)
bls_active = True

# bls.py:74-76 -- the current backend
bls = mi355x_bls

STUB_SIGNATURE = b"\x11" * 96  # bls.py:78
STUB_PUBKEY = b"\x22" * 48  # bls.py:79
G2_POINT_AT_INFINITY = b"\xc0" + b"\x00" * 95  # bls.py:80
# bls.py:81 STUB_COORDINATES = signature_to_G2(G2_POINT_AT_INFINITY): the identity
STUB_COORDINATES = None

# sigsets.deferred(): when set, the verify family records its arguments here and returns True
# (the collector checks them all in device batches at the end of the block).
_collector = None


def use_mi355x():
    """Route every BLS call to the MI355X backend (new switch, cf. bls.py:84-121)."""
    global bls
    bls = mi355x_bls


def _use_reference(modname: str, attr: str | None = None):
    import importlib

    global bls
    try:
        mod = importlib.import_module(modname)
    except ImportError as e:  # the reference wheels are not vendored
        raise ImportError(f"{modname} is not installed; only use_mi355x() is available") from e
    bls = getattr(mod, attr) if attr else mod


def use_milagro():  # bls.py:84-91
    _use_reference("milagro_bls_binding")


def use_arkworks():  # bls.py:94-101
    _use_reference("py_arkworks_bls12381")


def use_py_ecc():  # bls.py:104-111
    _use_reference("py_ecc.bls", "G2ProofOfPossession")


def use_fastest():  # bls.py:114-121 -- on this backend the fastest is the GPU
    use_mi355x()


def only_with_bls(alt_return=None):  # bls.py:124-138
    def runner(fn):
        def entry(*args, **kw):
            if bls_active:
                return fn(*args, **kw)
            return alt_return

        return entry

    return runner


@only_with_bls(alt_return=True)
def Verify(PK, message, signature):  # bls.py:141-151
    if _collector is not None:
        _collector.add_verify(PK, message, signature)
        return True
    try:
        result = bls.Verify(PK, message, signature)
    except Exception:
        result = False
    return bool(result)


@only_with_bls(alt_return=True)
def AggregateVerify(pubkeys, messages, signature):  # bls.py:154-164
    if _collector is not None:
        _collector.add_aggregate_verify(pubkeys, messages, signature)
        return True
    try:
        result = bls.AggregateVerify(list(pubkeys), list(messages), signature)
    except Exception:
        result = False
    return bool(result)


@only_with_bls(alt_return=True)
def FastAggregateVerify(pubkeys, message, signature):  # bls.py:167-177
    if _collector is not None:
        _collector.add_fast_aggregate_verify(pubkeys, message, signature)
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
    return bls.Sign(int(SK).to_bytes(32, "big"), message)


@only_with_bls(alt_return=STUB_PUBKEY)
def AggregatePKs(pubkeys):  # bls.py:202-213 (milagro checks KeyValidate internally)
    return bls._AggregatePKs(list(pubkeys))


@only_with_bls(alt_return=STUB_SIGNATURE)
def SkToPk(SK):  # bls.py:216-221
    return bls.SkToPk(int(SK).to_bytes(32, "big"))


@only_with_bls(alt_return=True)
def KeyValidate(pubkey):  # bls.py:395-397
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
