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
    assert bls.bls is bls.fastest_bls


def test_fastest_bls_contract():
    """E/utils/bls.py:57-76: the default backend is fastest_bls; its signature attributes are the MI355X
    backend's (milagro's role) and its curve classes are the MI355X curve objects (arkworks' role), so every
    `bls == arkworks_bls or bls == fastest_bls` helper branch of the reference (:225, :244, ... :390) holds."""
    from bls_mi355x import bls, curve
    from bls_mi355x.backend import mi355x_bls

    bls.use_mi355x()
    assert bls.bls == bls.fastest_bls and bls.Scalar is curve.Scalar
    for name in ("Sign", "Verify", "Aggregate", "AggregateVerify", "FastAggregateVerify", "SkToPk", "_AggregatePKs"):
        assert getattr(bls.fastest_bls, name) is getattr(mi355x_bls, name), name
    assert (bls.fastest_bls.G1, bls.fastest_bls.G2, bls.fastest_bls.GT) == (curve.G1Point, curve.G2Point, curve.GT)


def test_helpers_take_the_fastest_branch(monkeypatch):
    """add / neg / multiply / multi_exp / pairing_check / Z1 / G1 dispatch to the curve objects (no device call:
    the point operations are replaced by recorders)."""
    from bls_mi355x import bls, curve

    bls.use_mi355x()
    seen = []
    monkeypatch.setattr(curve._Point, "__add__", lambda a, b: seen.append("add") or a)
    monkeypatch.setattr(curve._Point, "__neg__", lambda a: seen.append("neg") or a)
    monkeypatch.setattr(curve._Point, "__mul__", lambda a, k: seen.append(("mul", type(k).__name__, int(k))) or a)
    monkeypatch.setattr(curve.G1Point, "multiexp_unchecked",
                        classmethod(lambda cls, p, k: seen.append(("msm", len(p), type(k[0]).__name__)) or p[0]))
    monkeypatch.setattr(curve.GT, "multi_pairing", classmethod(lambda cls, a, b: seen.append(("pair", len(a))) or cls.one()))
    g = bls.G1()
    assert g.to_compressed_bytes() == curve.G1_GENERATOR and bls.Z1().to_compressed_bytes() == curve.G1_IDENTITY
    assert bls.G1_to_bytes48(bls.add(g, bls.neg(g))) == curve.G1_GENERATOR
    bls.multiply(g, 5)
    bls.multiply(g, curve.Scalar(-1))
    bls.multi_exp([g, g], [1, 2])
    assert bls.pairing_check([[g, bls.G2()], [g, bls.neg(bls.G2())]]) is True
    assert seen == ["neg", "add", ("mul", "Scalar", 5), ("mul", "Scalar", curve.R - 1), ("msm", 2, "Scalar"), "neg",
                    ("pair", 2)]
    with pytest.raises(Exception, match="zero points"):
        bls.multi_exp([], [])


def test_scalar_field_arithmetic():
    from bls_mi355x.curve import R, Scalar

    class BLSFieldElement(Scalar):  # pysetup/spec_builders/deneb.py:17-18
        pass

    a, b = BLSFieldElement(7), BLSFieldElement(R + 3)
    assert int(b) == 3 and isinstance(a + b, BLSFieldElement)
    assert int(a - b) == 4 and int(b - a) == R - 4 and int(-a) == R - 7
    assert int(a * b) == 21 and int(a / b) == 7 * pow(3, -1, R) % R
    assert a.pow(BLSFieldElement(3)) == BLSFieldElement(343) and int(a.inverse() * a) == 1
    assert a == 7 and a != b and hash(a) == hash(Scalar(7))
    with pytest.raises(ZeroDivisionError):
        BLSFieldElement(0).inverse()


def test_rlc_seed_fails_closed(tmp_path):
    """a short read of the entropy source must fail the batch call (BLS_E_DEVICE), never
    continue with a predictable RLC seed (bls_capi.hip bls_host_seed; host only, no device)."""
    import ctypes

    from bls_mi355x import _native
    lib = _native.load_library()
    buf = ctypes.create_string_buffer(32)
    short = tmp_path / "short"
    short.write_bytes(b"\x11" * 16)
    try:
        for src, want in ((str(tmp_path / "missing"), _native.BLS_E_DEVICE), ("/dev/null", _native.BLS_E_DEVICE),
                          (str(short), _native.BLS_E_DEVICE)):
            assert lib.bls_set_entropy_source(src.encode()) == 0
            assert lib.bls_host_seed(buf) == want, src
            assert buf.raw == bytes(32)
        assert lib.bls_set_entropy_source(b"x" * 300) == _native.BLS_E_ARG
    finally:
        assert lib.bls_set_entropy_source(b"/dev/urandom") == 0
    seeds = set()
    for _ in range(4):
        assert lib.bls_host_seed(buf) == 0
        seeds.add(buf.raw)
    assert len(seeds) == 4


def test_integration_patch_imports_without_wheels(monkeypatch):
    """the reference-side patch of INTEGRATION.md §1 must import where milagro, arkworks and
    py_ecc are absent (the MI355X box).  Executes the two python blocks of §1 -- the guarded imports replacing
    E/utils/bls.py:1-53 and the use_mi355x switch -- with those wheels made unimportable, between them the
    fastest_bls class as the patch describes it (E/utils/bls.py:57-68 with mi355x_bls for milagro_bls)."""
    import builtins
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "INTEGRATION.md")) as fh:
        text = fh.read()
    sec = text[text.index("## 1."):text.index("## 2.")]
    blocks = re.findall(r"```python\n(.*?)```", sec, re.S)
    assert len(blocks) == 3  # (a) guarded imports, (b) the switch, then the conftest choice
    monkeypatch.setenv("BLSMI355X_HOME", os.path.join(root, "eth-consensus-specs_amd"))
    real_import = builtins.__import__

    def no_wheels(name, *a, **kw):
        if name.split(".")[0] in ("milagro_bls_binding", "py_arkworks_bls12381", "py_ecc"):
            raise ImportError(f"No module named {name!r}")
        return real_import(name, *a, **kw)

    monkeypatch.setattr(builtins, "__import__", no_wheels)
    monkeypatch.setattr(sys, "path", list(sys.path))
    ns = {"__name__": "eth2spec_utils_bls_patched"}
    exec(compile(blocks[0], "<INTEGRATION §1a>", "exec"), ns)
    assert ns["milagro_bls"] is None and ns["arkworks_bls"] is None and ns["py_ecc_bls"] is None
    assert ns["BLS_MODULUS"] == 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    fastest = ("class fastest_bls:\n" + "".join(
        f"    {n} = {v}\n" for n, v in (("G1", "arkworks_G1"), ("G2", "arkworks_G2"), ("Scalar", "arkworks_Scalar"),
                                       ("GT", "arkworks_GT"))) + "".join(
        f"    {n} = mi355x_bls.{n}\n" for n in ("_AggregatePKs", "Sign", "Verify", "Aggregate", "AggregateVerify",
                                               "FastAggregateVerify", "SkToPk")) + "bls = fastest_bls\n")
    exec(compile(fastest, "<E/utils/bls.py:57-76>", "exec"), ns)
    exec(compile(blocks[1], "<INTEGRATION §1b>", "exec"), ns)
    from bls_mi355x import curve
    from bls_mi355x.backend import mi355x_bls

    assert callable(ns["use_mi355x"]) and ns["bls"] is ns["fastest_bls"]
    assert ns["bls"].FastAggregateVerify is mi355x_bls.FastAggregateVerify
    assert ns["arkworks_G1"] is curve.G1Point and ns["Scalar"] is curve.Scalar
    assert ns["py_ecc_Scalar"](5).inverse() * 5 == 1
