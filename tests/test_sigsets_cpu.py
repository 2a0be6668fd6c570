"""Host logic of the deferred signature-set collector (bls_mi355x/sigsets.py):
recording through the shim, routing of each set, stub mode and exception
handling -- no device call (the batch executors are replaced by fakes that
record what they were asked)."""
import numpy as np
import pytest


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


def test_deferred_records_and_checks(fakes, monkeypatch):
    sigsets, calls = fakes
    from bls_mi355x import bls as shim
    from bls_mi355x.backend import mi355x_bls

    monkeypatch.setattr(mi355x_bls, "FastAggregateVerify", staticmethod(lambda pks, m, s: False))
    keys = [_pk(i) for i in range(4)]
    shim.bls_active = True
    with sigsets.deferred(FakeRegistry(keys), check=False) as col:
        assert shim.FastAggregateVerify(keys, b"\x03" * 32, b"\x04" * 96) is True
        assert shim.Verify(keys[1], b"\x03" * 32, b"\x04" * 96) is True
        assert shim.AggregateVerify(keys[:1], [b"m"], b"\x04" * 96) is True
        assert shim.eth_fast_aggregate_verify([], b"\x03" * 32, b"\xc0" + bytes(95)) is True
    assert shim._collector is None
    assert len(col) == 3 and col.results == [True, True, True]
    assert calls["fav"] == ([0, 1, 2, 3, 1], [0, 4, 5], 2, 2)
    assert calls["av"] == [1]
    with pytest.raises(AssertionError, match="set 0"):
        with sigsets.deferred(None):
            shim.FastAggregateVerify([_pk(50)], b"\x03" * 32, b"\x04" * 96)  # per-call path -> False
    assert shim._collector is None


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
