"""The BASELINE.json configurations at full size on one MI355X (SURVEY.md
§8(d)): C2 sync-committee FastAggregateVerify (10,000 x 512 on a 2^20
registry, k in {0, 1, 8} bad items), C3 epoch replay (2,048 x 512 over a
permutation of 2^20; one message per (slot, committee), and the post-Electra
variant with one message per slot), C4 gossip (one 125,000-Verify shard of
the 10^6 firehose), C5 AggregateVerify with N = 8,192 distinct messages and
adversarial 1,024 x 512 FAV batches with every bad kind of §8(d) at
k in {1, 8, 64}.

Verdicts are checked against the construction (every item is valid unless
the test made it bad) and sampled items against the C oracle
(oracle/bls_oracle.c) through their compressed keys -- the edge cases
follow test_eth_fast_aggregate_verify.py:38-151 (infinity / zero / tampered
signatures, infinity and 0x40 pubkeys)."""
import hashlib

import numpy as np
import pytest

from oracle import bls_oracle as O
from oracle import bls_oracle_c as OC

pytestmark = pytest.mark.gpu

REG_N = 1 << 20
G1_INF = b"\xc0" + bytes(47)
PK_0x40 = b"\x40" + bytes(47)
IDX_INF, IDX_0x40 = REG_N, REG_N + 1  # appended invalid registry entries


@pytest.fixture(scope="module")
def batch():
    from bls_mi355x import batch as b
    return b


@pytest.fixture(scope="module")
def reg(batch):
    """2^20 keys sk_i = i + 1 generated on the device, then two invalid deposits appended (decoded and
    KeyValidated on the device like any registry key): G1 infinity and a 0x40-flag encoding."""
    r = batch.Registry()
    pks = r.generate(REG_N, first_sk=1, want_bytes=True)
    valid = r.append(G1_INF + PK_0x40)
    assert valid.tolist() == [0, 0] and len(r) == REG_N + 2
    return pks + G1_INF + PK_0x40


def _pk(reg, i):
    return reg[48 * int(i): 48 * int(i) + 48]


def _committees(B, n, seed):
    """B committees of n distinct registry indices (seeded permutations of the registry, never straddling)."""
    rng = np.random.default_rng(seed)
    per = REG_N // n
    out = [rng.permutation(REG_N).astype(np.uint32)[: per * n].reshape(per, n) for _ in range((B + per - 1) // per)]
    return np.concatenate(out)[:B]


def _sign(batch, idx2d, msgs):
    agg = (idx2d.astype(np.int64) + 1).sum(axis=1)
    return bytearray(batch.sign_batch(b"".join((int(a) % O.R).to_bytes(32, "big") for a in agg), b"".join(msgs)))


def _msgs(tag, B):
    return [hashlib.sha256(tag + j.to_bytes(8, "little")).digest() for j in range(B)]


def _corrupt(sigs, j, kind, B):
    if kind == "wrong_msg":  # a valid G2 point for another message: only the pairing check catches it
        sigs[96 * j: 96 * j + 96] = sigs[96 * ((j + 1) % B): 96 * ((j + 1) % B) + 96]
    elif kind == "inf_sig":
        sigs[96 * j: 96 * j + 96] = b"\xc0" + bytes(95)
    elif kind == "zero_sig":
        sigs[96 * j: 96 * j + 96] = bytes(96)
    elif kind == "ff_tail":  # test_eth_fast_aggregate_verify.py:104
        sigs[96 * j + 92: 96 * j + 96] = b"\xff" * 4
    else:
        raise AssertionError(kind)


def _oracle_check(reg, idx2d, msgs, sigs, items, expect):
    for j in items:
        pkl = [_pk(reg, x) for x in idx2d[j]]
        assert OC.FastAggregateVerify(pkl, msgs[j], bytes(sigs[96 * j: 96 * j + 96])) == bool(expect[j]), j


@pytest.mark.parametrize("k", [0, 1, 8])
def test_c2_sync_committee_full(batch, reg, k):
    """C2: 10,000 FastAggregateVerify x 512 distinct keys of the 2^20 registry, k bad items."""
    B, n = 10000, 512
    idx2d = _committees(B, n, seed=1000 + k)
    msgs = _msgs(b"c2" + bytes([k]), B)
    sigs = _sign(batch, idx2d, msgs)
    rng = np.random.default_rng(2000 + k)
    bad = sorted(rng.choice(B - 1, size=k, replace=False).tolist())
    kinds = ["wrong_msg", "ff_tail", "wrong_msg", "inf_sig", "wrong_msg", "zero_sig", "wrong_msg", "ff_tail"]
    for t, j in enumerate(bad):
        _corrupt(sigs, j, kinds[t], B)
    offs = np.arange(B + 1, dtype=np.uint64) * n
    out = batch.fast_aggregate_verify_batch(idx2d.reshape(-1), offs, b"".join(msgs), bytes(sigs))
    expect = np.ones(B, dtype=bool)
    expect[bad] = False
    assert (out == expect).all(), np.nonzero(out != expect)
    checks, rounds = batch.fallback_stats()
    assert (checks, rounds) == (0, 0) if k == 0 else rounds >= 2
    good = next(j for j in range(B) if expect[j])
    _oracle_check(reg, idx2d, msgs, sigs, (bad[:2] if bad else []) + [good, B - 1], expect)


@pytest.mark.parametrize("shared", [False, True])
def test_c3_epoch_replay_full(batch, reg, shared):
    """C3: a seeded permutation of 2^20 split into 32 slots x 64 committees of 512 -> 2,048 FAV in one RLC
    batch; one message per (slot, committee), or per slot (post-Electra: 32 messages)."""
    slots, per_slot, n = 32, 64, 512
    B = slots * per_slot
    perm = np.random.default_rng(77).permutation(REG_N).astype(np.uint32)
    idx2d = perm[: B * n].reshape(B, n)
    if shared:
        slot_msgs = _msgs(b"c3-slot", slots)
        msgs = [slot_msgs[j // per_slot] for j in range(B)]
    else:
        msgs = _msgs(b"c3", B)
    sigs = _sign(batch, idx2d, msgs)
    bad = [5, 1500]
    _corrupt(sigs, 5, "wrong_msg", B)
    _corrupt(sigs, 1500, "ff_tail", B)
    offs = np.arange(B + 1, dtype=np.uint64) * n
    out = batch.fast_aggregate_verify_batch(idx2d.reshape(-1), offs, b"".join(msgs), bytes(sigs))
    expect = np.ones(B, dtype=bool)
    expect[bad] = False
    if shared:  # 5 carries committee 6's signature of the same slot message: still a wrong aggregate key
        assert msgs[5] == msgs[6]
    assert (out == expect).all(), np.nonzero(out != expect)
    _oracle_check(reg, idx2d, msgs, sigs, [5, 6, B - 1], expect)


def test_c4_gossip_shard_full(batch, reg):
    """C4: one shard (125,000 = 10^6 / 8) of single-signature Verify with distinct messages, pk_i = registry[i]."""
    B = 125000
    idx = np.arange(B, dtype=np.uint32)
    msgs = _msgs(b"c4", B)
    sigs = bytearray(batch.sign_batch(b"".join(int(i + 1).to_bytes(32, "big") for i in range(B)), b"".join(msgs)))
    bad = [17, 4096, 99999, B - 1]
    _corrupt(sigs, 17, "wrong_msg", B)
    _corrupt(sigs, 4096, "inf_sig", B)
    _corrupt(sigs, 99999, "zero_sig", B)
    _corrupt(sigs, B - 1, "ff_tail", B)
    idx[123] = IDX_INF  # an invalid (infinity) registry key
    bad.append(123)
    out = batch.verify_batch(idx, b"".join(msgs), bytes(sigs))
    expect = np.ones(B, dtype=bool)
    expect[bad] = False
    assert (out == expect).all(), np.nonzero(out != expect)
    for j in (17, 18, 123, 64000):
        assert OC.Verify(_pk(reg, idx[j]), msgs[j], bytes(sigs[96 * j: 96 * j + 96])) == bool(expect[j]), j


def test_c5_aggregate_verify_8192(batch):
    """C5: AggregateVerify with N = 8,192 distinct messages through the drop-in API (one call)."""
    from bls_mi355x import bls as shim

    shim.use_mi355x()
    shim.bls_active = True
    N = 8192
    sks = [(104729 * (i + 1)) % O.R for i in range(N)]
    pks = batch.sk_to_pk_batch(b"".join(k.to_bytes(32, "big") for k in sks))
    pkl = [pks[48 * i: 48 * i + 48] for i in range(N)]
    msgs = _msgs(b"c5av", N)
    sigs = batch.sign_batch(b"".join(k.to_bytes(32, "big") for k in sks), b"".join(msgs))
    agg = shim.Aggregate([sigs[96 * i: 96 * i + 96] for i in range(N)])
    assert shim.AggregateVerify(pkl, msgs, agg) is True
    swapped = msgs[:]
    swapped[100], swapped[8000] = swapped[8000], swapped[100]
    assert shim.AggregateVerify(pkl, swapped, agg) is False
    assert shim.AggregateVerify(pkl[:-1], msgs[:-1], agg) is False
    assert shim.AggregateVerify(pkl, msgs, b"\xc0" + bytes(95)) is False
    # the C oracle on a prefix: same key / message / signature bytes
    assert OC.SkToPk(sks[0]) == pkl[0] and OC.Sign(sks[1], msgs[1]) == sigs[96:192]
    agg128 = OC.Aggregate([sigs[96 * i: 96 * i + 96] for i in range(128)])
    assert shim.AggregateVerify(pkl[:128], msgs[:128], agg128) is OC.AggregateVerify(pkl[:128], msgs[:128], agg128)


KINDS = ["wrong_msg", "inf_sig", "zero_sig", "ff_tail", "g1_inf_pk", "pk_0x40"]


@pytest.mark.parametrize("k", [1, 8, 64])
def test_c5_adversarial_1024x512(batch, reg, k):
    """C5 adversarial batches: 1,024 FAV x 512 keys with k bad entries of every §8(d) kind at seeded positions;
    the bisection must isolate exactly those items."""
    B, n = 1024, 512
    rng = np.random.default_rng(300 + k)
    bad = sorted(rng.choice(B, size=k, replace=False).tolist())
    kinds = {j: KINDS[t % len(KINDS)] for t, j in enumerate(bad)}
    idx2d = _committees(B, n, seed=400 + k)
    msgs = _msgs(b"c5adv" + bytes([k]), B)
    sigs = _sign(batch, idx2d, msgs)
    for j in bad:
        if kinds[j] == "g1_inf_pk":
            idx2d[j, 7] = IDX_INF
        elif kinds[j] == "pk_0x40":
            idx2d[j, 0] = IDX_0x40
        else:
            _corrupt(sigs, j, kinds[j], B)
    offs = np.arange(B + 1, dtype=np.uint64) * n
    out = batch.fast_aggregate_verify_batch(idx2d.reshape(-1), offs, b"".join(msgs), bytes(sigs))
    expect = np.ones(B, dtype=bool)
    expect[bad] = False
    assert (out == expect).all(), np.nonzero(out != expect)
    checks, rounds = batch.fallback_stats()
    if any(kinds[j] == "wrong_msg" for j in bad):
        assert rounds >= 2 and checks < B  # bisection, cheaper than one check per item
    good = next(j for j in range(B) if expect[j])
    _oracle_check(reg, idx2d, msgs, sigs, [bad[0], good], expect)
