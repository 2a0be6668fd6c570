"""CPU-side checks of the product boundary: the C-ABI library loads, exports
every symbol include/blsmi355x.h declares, and the shim's host logic
(argument validation, stubs, raising vs False) behaves like the reference
wrappers -- without any compute call (no GPU here)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "blsmi355x.h")


def _declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(bls_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from bls_mi355x import _native
    lib = _native.load_library()
    names = _declared()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    assert set(_native.EXPORTS) == set(names)


def test_no_gpu_means_loud_failure(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from bls_mi355x import _native
    with pytest.raises(_native.NativeUnavailable):
        _native.Context(0)


def test_stub_mode_and_argument_checks():
    from bls_mi355x import bls
    bls.bls_active = False
    try:
        assert bls.Verify(b"x", b"y", b"z") is True
        assert bls.FastAggregateVerify([], b"", b"") is True
        assert bls.AggregateVerify([], [], b"") is True
        assert bls.Aggregate([]) == bls.STUB_SIGNATURE
        assert bls.Sign(5, b"m") == bls.STUB_SIGNATURE
        assert bls.SkToPk(5) == bls.STUB_SIGNATURE
        assert bls.AggregatePKs([b"x"]) == bls.STUB_PUBKEY
        assert bls.KeyValidate(b"") is True
    finally:
        bls.bls_active = True
    # malformed lengths are rejected in the shim before any device call
    from bls_mi355x.backend import mi355x_bls as M
    assert M.Verify(b"\x00" * 47, b"", b"\x00" * 96) is False
    assert M.FastAggregateVerify([], b"", b"\xc0" + bytes(95)) is False
    assert M.AggregateVerify([b"\x00" * 48], [], b"\x00" * 96) is False
    with pytest.raises(ValueError):
        M.Aggregate([])
    with pytest.raises(ValueError):
        M._AggregatePKs([])
    # spec-level special case (specs/altair/bls.md:64-65) needs no device
    assert bls.eth_fast_aggregate_verify([], b"\x00" * 32, bls.G2_POINT_AT_INFINITY) is True


def test_reference_backend_switches_raise_without_wheels():
    from bls_mi355x import bls
    for fn in (bls.use_milagro, bls.use_arkworks, bls.use_py_ecc):
        with pytest.raises(ImportError):
            fn()
    bls.use_fastest()
    assert bls.bls is bls.mi355x_bls
