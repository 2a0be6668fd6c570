"""Host logic of the deferred signature-set collector (bls_mi355x/sigsets.py):
recording through the shim, routing of each set, stub mode and exception
handling -- no device call (the batch executors are replaced by fakes that
record what they were asked)."""
import linecache

import numpy as np
import pytest


def compile_spec(src: str, name: str) -> dict:
    """Compile spec-shaped source the way the generated pyspec modules exist -- with readable source lines
    (linecache, as a module file provides them): sigsets.result_is_asserted reads the caller's source."""
    linecache.cache[name] = (len(src), None, src.splitlines(True), name)
    ns = {}
    exec(compile(src, name, "exec"), ns)
    return ns


class FakeRegistry:
    def __init__(self, keys):
        self.map = {k: i for i, k in enumerate(keys)}

    def indices(self, pubkeys):
        try:
            return np.array([self.map[bytes(k)] for k in pubkeys], dtype=np.uint32)
        except KeyError:
            return None


def _pk(i):
    return bytes([0x80 | (i & 0x1f)]) + i.to_bytes(47, "big")


@pytest.fixture
def fakes(monkeypatch):
    from bls_mi355x import batch, sigsets

    calls = {}

    def fav(idx, offs, msgs, sigs, ctx=None):
        calls["fav"] = (np.asarray(idx).tolist(), np.asarray(offs).tolist(), len(msgs) // 32, len(sigs) // 96)
        return np.ones(len(offs) - 1, dtype=bool)

    def av(pks, msgs, sigs, ctx=None):
        calls["av"] = [len(p) for p in pks]
        return np.array([len(p) == len(m) for p, m in zip(pks, msgs)])

    monkeypatch.setattr(batch, "fast_aggregate_verify_batch", fav)
    monkeypatch.setattr(batch, "aggregate_verify_batch", av)
    return sigsets, calls


def test_routing(fakes):
    sigsets, calls = fakes
    keys = [_pk(i) for i in range(8)]
    s = sigsets.SignatureSets(FakeRegistry(keys))
    m32, sig = b"\x01" * 32, b"\x02" * 96
    s.add_fast_aggregate_verify(keys[:3], m32, sig)           # 0 indexed
    s.add_verify(keys[5], m32, sig)                           # 1 indexed (FAV with one key)
    s.add_fast_aggregate_verify_indexed([7, 6], m32, sig)     # 2 indexed
    s.add_verify(_pk(100), m32, sig)                          # 3 av (not resident)
    s.add_verify(keys[0], b"short", sig)                      # 4 av (not a 32-byte root)
    s.add_aggregate_verify(keys[:2], [m32, m32], sig)         # 5 av
    s.add_aggregate_verify(keys[:2], [m32], sig)              # 6 av, length mismatch -> False
    s.add_fast_aggregate_verify(None, m32, sig)               # 7 malformed -> False
    s.add_fast_aggregate_verify([], m32, sig)                 # 8 single (empty -> per-call path)
    indexed, av, single = s.plan()
    assert [i for i, _ in indexed] == [0, 1, 2]
    assert [x.tolist() for _, x in indexed] == [[0, 1, 2], [5], [7, 6]]
    assert av == [3, 4, 5, 6] and single == [8]


# Spec-shaped call sites, compiled from source like the generated spec modules (pytest rewrites the asserts
# of test modules, so these must not be defined in this file's own code).
SPEC_SRC = """
def _process_randao(shim, pk, m, sig):  # specs/phase0/beacon-chain.md:1893
    assert shim.Verify(pk, m, sig)


def _is_valid_indexed_attestation(shim, pks, m, sig):  # :776-790
    return shim.FastAggregateVerify(pks, m, sig)


def _process_attestation(shim, pks, m, sig):  # :2005
    assert _is_valid_indexed_attestation(shim, pks, m, sig)


def _process_av(shim, pks, msgs, sig):
    assert shim.AggregateVerify(pks, msgs, sig), "aggregate verify"


def _process_sync_aggregate(shim, pks, m, sig):  # specs/altair/beacon-chain.md:608
    assert shim.eth_fast_aggregate_verify(pks, m, sig)


def _apply_deposit(shim, pk, m, sig, applied):  # specs/phase0/beacon-chain.md:2055
    if shim.Verify(pk, m, sig):
        applied.append(pk)


def _compare(shim, pk, m, sig):
    return shim.Verify(pk, m, sig) is False
"""
_spec = compile_spec(SPEC_SRC, "<generated spec>")
_process_randao = _spec["_process_randao"]
_process_attestation = _spec["_process_attestation"]
_process_av = _spec["_process_av"]
_process_sync_aggregate = _spec["_process_sync_aggregate"]
_apply_deposit = _spec["_apply_deposit"]
_compare = _spec["_compare"]


def test_deferred_records_and_checks(fakes, monkeypatch):
    sigsets, calls = fakes
    from bls_mi355x import bls as shim
    from bls_mi355x.backend import mi355x_bls

    monkeypatch.setattr(mi355x_bls, "FastAggregateVerify", staticmethod(lambda pks, m, s: False))
    keys = [_pk(i) for i in range(4)]
    shim.bls_active = True
    with sigsets.deferred(FakeRegistry(keys), check=False) as col:
        _process_attestation(shim, keys, b"\x03" * 32, b"\x04" * 96)
        _process_randao(shim, keys[1], b"\x03" * 32, b"\x04" * 96)
        _process_av(shim, keys[:1], [b"m"], b"\x04" * 96)
        _process_sync_aggregate(shim, [], b"\x03" * 32, b"\xc0" + bytes(95))  # special case: no set
    assert shim._collector is None
    assert len(col) == 3 and col.results == [True, True, True] and col.eager == 0
    assert calls["fav"] == ([0, 1, 2, 3, 1], [0, 4, 5], 2, 2)
    assert calls["av"] == [1]
    with pytest.raises(AssertionError, match="set 0"):
        with sigsets.deferred(None):
            _process_attestation(shim, [_pk(50)], b"\x03" * 32, b"\x04" * 96)  # per-call path -> False
    assert shim._collector is None


def test_deferred_branching_site_gets_the_real_verdict(fakes, monkeypatch):
    """apply_deposit branches on Verify: an invalid proof of possession skips the deposit and the block stays
    valid (test_process_deposit.py:255-287), so inside deferred() that call runs at once."""
    sigsets, _ = fakes
    from bls_mi355x import bls as shim
    from bls_mi355x.backend import mi355x_bls

    seen = []
    monkeypatch.setattr(mi355x_bls, "Verify", staticmethod(lambda pk, m, s: seen.append(pk) or pk == _pk(1)))
    monkeypatch.setattr(shim.fastest_bls, "Verify", mi355x_bls.Verify)
    applied = []
    with sigsets.deferred(FakeRegistry([_pk(1)])) as col:  # no AssertionError at exit
        _apply_deposit(shim, _pk(2), b"\x05" * 32, b"\x06" * 96, applied)  # invalid PoP: skipped
        _apply_deposit(shim, _pk(1), b"\x05" * 32, b"\x06" * 96, applied)  # valid: applied
        assert _compare(shim, _pk(2), b"\x05" * 32, b"\x06" * 96)  # a comparison is not an assert
    assert applied == [_pk(1)] and seen == [_pk(2), _pk(1), _pk(2)]
    assert len(col) == 0 and col.eager == 3 and col.results == []


def test_deferred_is_interpreter_independent(fakes, monkeypatch):
    """the assert-site analysis reads source, not bytecode, so the reference's supported
    interpreters (pyproject.toml:10, >=3.10 <3.14) all batch the asserted calls (nothing keyed on the version)."""
    sigsets, calls = fakes
    from bls_mi355x import bls as shim

    keys = [_pk(i) for i in range(2)]
    shim.bls_active = True
    for ver in ((3, 11, 9, "final", 0), (3, 12, 0, "final", 0), (3, 13, 1, "final", 0)):
        monkeypatch.setattr(sigsets.sys, "version_info", ver)
        with sigsets.deferred(FakeRegistry(keys), check=False) as col:
            _process_attestation(shim, keys, b"\x03" * 32, b"\x04" * 96)
            _process_attestation(shim, keys, b"\x03" * 32, b"\x04" * 96)
        assert len(col) == 2 and col.eager == 0 and col.results == [True, True]
    assert not hasattr(sigsets.SignatureSets(None), "version_fallback")


def test_deferred_without_source_runs_at_once(fakes, monkeypatch):
    """A caller whose source cannot be read (no file, not in linecache) gets the real verdict at once."""
    sigsets, _ = fakes
    from bls_mi355x import bls as shim
    from bls_mi355x.backend import mi355x_bls

    monkeypatch.setattr(mi355x_bls, "FastAggregateVerify", staticmethod(lambda pks, m, s: True))
    monkeypatch.setattr(shim.fastest_bls, "FastAggregateVerify", mi355x_bls.FastAggregateVerify)
    ns = {}
    exec(compile("def f(shim, k):\n    assert shim.FastAggregateVerify(k, b'\\x03' * 32, b'\\x04' * 96)\n",
                 "<no source>", "exec"), ns)
    shim.bls_active = True
    with sigsets.deferred(FakeRegistry([_pk(0)]), check=False) as col:
        ns["f"](shim, [_pk(0)])
    assert len(col) == 0 and col.eager == 1


PATTERNS_SRC = """
import sys
from bls_mi355x.sigsets import result_is_asserted


def probe():
    return result_is_asserted(sys._getframe(1), "probe")


def asserted():
    assert probe()


def asserted_msg():
    assert probe(), "message"


def returned():
    return probe()


def through_return():
    assert returned()


def negated():
    assert not probe()


def branched():
    if probe():
        return True
    return False


def stored():
    x = probe()
    return x


def via_map():
    assert not any(map(lambda _: probe(), [0]))


def via_sorted():
    assert not sorted([probe()])[0]


def nested_arg(f):
    assert f(probe())


def in_conditional(c):
    assert (probe() if c else False) or True


def multi_line_assert():
    assert probe(
    ), (
        "message"
    )


def multi_line_return():
    return (
        probe()
    )


def through_multi_line():
    assert multi_line_return()


def same_line_mixed():
    assert probe() or not probe()


def in_lambda():
    assert not (lambda: probe())()


def in_comprehension():
    assert not [probe() for _ in [0]][0]
"""


def test_result_is_asserted_patterns():
    ns = compile_spec(PATTERNS_SRC, "<patterns>")
    ns["asserted"]()
    ns["asserted_msg"]()
    ns["through_return"]()
    ns["negated"]()  # `assert not f()`: f must see False (deferring would return True and fail the assert)
    assert ns["branched"]() is False and ns["stored"]() is False and ns["returned"]() is False
    ns["via_map"]()  # C-level callers (map / any) in between: the call runs at once (False here)
    ns["via_sorted"]()
    ns["nested_arg"](lambda v: v is False)  # probe() is an argument of f, not the asserted call
    ns["in_conditional"](True)
    ns["multi_line_assert"]()
    ns["through_multi_line"]()
    ns["same_line_mixed"]()  # one of the line's calls is negated: neither is deferred
    ns["in_lambda"]()
    ns["in_comprehension"]()


def test_wrong_lengths_are_false_not_errors(fakes):
    sigsets, calls = fakes
    s = sigsets.SignatureSets(FakeRegistry([_pk(0)]))
    s.add_verify(b"\x01" * 47, b"\x02" * 32, b"\x03" * 96)          # short key
    s.add_aggregate_verify([b"\x01" * 49], [b"m"], b"\x03" * 96)     # long key
    s.add_fast_aggregate_verify([_pk(0)], b"\x02" * 32, b"\x03" * 95)  # short signature
    assert all(x.malformed for x in s.sets)
    assert s.verify() == [False, False, False]


def test_deferred_restores_on_exception(fakes):
    sigsets, _ = fakes
    from bls_mi355x import bls as shim

    with pytest.raises(RuntimeError):
        with sigsets.deferred(None):
            raise RuntimeError("state transition failed")
    assert shim._collector is None


def test_stub_mode_records_nothing(fakes):
    sigsets, _ = fakes
    from bls_mi355x import bls as shim

    shim.bls_active = False
    try:
        with sigsets.deferred(None) as col:
            assert shim.FastAggregateVerify([b"x"], b"m", b"s") is True
        assert len(col) == 0 and col.results == []
    finally:
        shim.bls_active = True
