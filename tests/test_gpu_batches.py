"""GPU parity of the batch configs of SURVEY.md §8(d): adversarial FAV
batches (C5, bisection fallback), gossip Verify batches (C4), epoch-shaped FAV
batches (C3) and AggregateVerify with many distinct messages (C5), checked
against verdicts known by construction and the C oracle (oracle/bls_oracle.c).
Requires an MI355X."""
import hashlib
import os

import numpy as np
import pytest

from oracle import bls_oracle as O
from oracle import bls_oracle_c as OC

pytestmark = pytest.mark.gpu

N_REG = 1 << 14
G1_INF = b"\xc0" + bytes(47)
BAD_PK_0x40 = b"\x40" + bytes(47)


@pytest.fixture(scope="module")
def batch():
    from bls_mi355x import batch as b
    return b


@pytest.fixture(scope="module")
def registry(batch):
    """Registry sk_i = i + 1 (N_REG keys) with two invalid entries: G1 infinity
    at index 1 and a 0x40-flag encoding at index 2."""
    reg = batch.Registry()
    pks = bytearray(reg.generate(N_REG, first_sk=1, want_bytes=True))
    pks[48:96] = G1_INF
    pks[96:144] = BAD_PK_0x40
    valid = reg.load(bytes(pks))
    assert not valid[1] and not valid[2] and valid.sum() == N_REG - 2
    return bytes(pks)


def _make_batch(batch, B, n, seed, bad_pk_items=()):
    """B committees of n distinct valid registry keys (>= 3); item j signs
    SHA256(seed||j) with the sum of its secret keys."""
    rng = np.random.default_rng(seed)
    idx = np.stack([rng.choice(np.arange(3, N_REG), size=n, replace=False) for _ in range(B)]).astype(np.uint32)
    for j, k in bad_pk_items:
        idx[j, 0] = k
    offs = np.arange(B + 1, dtype=np.uint64) * n
    msgs = [hashlib.sha256(seed.to_bytes(8, "little") + j.to_bytes(8, "little")).digest() for j in range(B)]
    agg = [int(a) % O.R for a in (idx.astype(np.int64) + 1).sum(axis=1)]
    sigs = bytearray(batch.sign_batch(b"".join(int(a).to_bytes(32, "big") for a in agg), b"".join(msgs)))
    return idx.reshape(-1), offs, msgs, sigs


def _corrupt(sigs, msgs, j, kind, B):
    if kind == "wrong_msg":  # a valid G2 point for another message: only the pairing check catches it
        k = (j + 1) % B
        sigs[96 * j: 96 * j + 96] = sigs[96 * k: 96 * k + 96]
    elif kind == "inf_sig":
        sigs[96 * j: 96 * j + 96] = b"\xc0" + bytes(95)
    elif kind == "zero_sig":
        sigs[96 * j: 96 * j + 96] = bytes(96)
    elif kind == "ff_tail":
        sigs[96 * j + 92: 96 * j + 96] = b"\xff" * 4
    else:
        raise AssertionError(kind)


KINDS = ["wrong_msg", "inf_sig", "zero_sig", "ff_tail", "g1_inf_pk", "pk_0x40"]


@pytest.mark.parametrize("k", [1, 8, 64])
def test_adversarial_fav_batch_bisection(batch, registry, k):
    """1024 FAV (n = 64) with k bad entries of every SURVEY §8(d) C5 kind at
    seeded positions; bisection must isolate exactly those items."""
    B, n = 1024, 64
    rng = np.random.default_rng(100 + k)
    bad = sorted(rng.choice(B, size=k, replace=False).tolist())
    kinds = {j: KINDS[t % len(KINDS)] for t, j in enumerate(bad)}
    pk_bad = [(j, 1 if kinds[j] == "g1_inf_pk" else 2) for j in bad if kinds[j] in ("g1_inf_pk", "pk_0x40")]
    idx, offs, msgs, sigs = _make_batch(batch, B, n, seed=200 + k, bad_pk_items=pk_bad)
    for j in bad:
        if kinds[j] not in ("g1_inf_pk", "pk_0x40"):
            _corrupt(sigs, msgs, j, kinds[j], B)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    expect = np.ones(B, dtype=bool)
    expect[bad] = False
    assert (out == expect).all(), np.nonzero(out != expect)
    checks, rounds = batch.fallback_stats()
    n_wrong = sum(1 for j in bad if kinds[j] == "wrong_msg")
    assert n_wrong > 0 and rounds >= 2  # a valid-point forgery forces the bisection
    assert checks < B                    # ... which costs fewer checks than one per item
    # C oracle on a few items (a bad one and a good one), through the compressed keys
    good = next(j for j in range(B) if j not in bad)
    for j in (bad[0], good):
        pkl = [registry[48 * int(x): 48 * int(x) + 48] for x in idx[n * j: n * j + n]]
        assert OC.FastAggregateVerify(pkl, msgs[j], bytes(sigs[96 * j: 96 * j + 96])) == bool(expect[j])


def test_fav_batch_all_valid_has_no_fallback(batch, registry):
    idx, offs, msgs, sigs = _make_batch(batch, 300, 16, seed=5)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    assert out.all()
    assert batch.fallback_stats() == (0, 0)


def test_fav_batch_every_item_bad(batch, registry):
    """Worst case for bisection: every item is a wrong-message forgery."""
    B = 40
    idx, offs, msgs, sigs = _make_batch(batch, B, 8, seed=6)
    rolled = sigs[96:] + sigs[:96]
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(rolled))
    assert not out.any()


def test_fav_batch_after_bisection_hashes_its_own_messages(batch, registry):
    """A host-buffer batch right after a bisected one: its hash must wait for its own message copy (it once forked
    from the bisection's event, recorded before that copy, and could hash the previous batch's messages)."""
    for r in range(3):
        idx, offs, msgs, sigs = _make_batch(batch, 64, 4, seed=60 + r)
        out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs[96:] + sigs[:96]))
        assert not out.any()
        idx, offs, msgs, sigs = _make_batch(batch, 2048, 4, seed=70 + r)
        out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
        assert out.all(), np.nonzero(~out)


def test_epoch_shaped_fav_batch(batch, registry):
    """C3 shape at reduced size: a seeded permutation of the registry split into
    slots x committees, one distinct message per (slot, committee)."""
    slots, per_slot, n = 8, 16, 96
    perm = np.random.default_rng(77).permutation(np.arange(3, N_REG))[: slots * per_slot * n].astype(np.uint32)
    B = slots * per_slot
    offs = np.arange(B + 1, dtype=np.uint64) * n
    msgs = [hashlib.sha256(b"epoch" + j.to_bytes(4, "little")).digest() for j in range(B)]
    agg = [int(a) % O.R for a in (perm.reshape(B, n).astype(np.int64) + 1).sum(axis=1)]
    sigs = batch.sign_batch(b"".join(int(a).to_bytes(32, "big") for a in agg), b"".join(msgs))
    out = batch.fast_aggregate_verify_batch(perm, offs, b"".join(msgs), sigs)
    assert out.all()


def test_gossip_verify_batch(batch, registry):
    """C4 at reduced size: B single-key Verify calls against the registry."""
    B = 2000
    rng = np.random.default_rng(9)
    idx = rng.integers(3, N_REG, size=B).astype(np.uint32)
    idx[17] = 1  # G1-infinity registry entry
    msgs = [hashlib.sha256(b"gossip" + j.to_bytes(4, "little")).digest() for j in range(B)]
    sigs = bytearray(batch.sign_batch(b"".join(int(k + 1).to_bytes(32, "big") for k in idx), b"".join(msgs)))
    sigs[96 * 5: 96 * 6] = sigs[96 * 6: 96 * 7]
    sigs[96 * 1500: 96 * 1501] = b"\xc0" + bytes(95)
    out = batch.verify_batch(idx, b"".join(msgs), bytes(sigs))
    expect = np.ones(B, dtype=bool)
    expect[[5, 17, 1500]] = False
    assert (out == expect).all(), np.nonzero(out != expect)
    for j in (5, 6, 17):
        pk = registry[48 * int(idx[j]): 48 * int(idx[j]) + 48]
        assert OC.Verify(pk, msgs[j], bytes(sigs[96 * j: 96 * j + 96])) == bool(expect[j])


@pytest.mark.parametrize("N", [128, 1024])
def test_aggregate_verify_many_messages(N):
    """C5: AggregateVerify with N distinct messages through the drop-in API."""
    from bls_mi355x import batch as b
    from bls_mi355x import bls as shim

    shim.use_mi355x()
    shim.bls_active = True
    sks = [(7919 * (i + 1)) % O.R for i in range(N)]
    pks = b.sk_to_pk_batch(b"".join(k.to_bytes(32, "big") for k in sks))
    pkl = [pks[48 * i: 48 * i + 48] for i in range(N)]
    msgs = [hashlib.sha256(b"av" + i.to_bytes(4, "little")).digest() for i in range(N)]
    sigs = b.sign_batch(b"".join(k.to_bytes(32, "big") for k in sks), b"".join(msgs))
    agg = shim.Aggregate([sigs[96 * i: 96 * i + 96] for i in range(N)])
    assert agg == OC.Aggregate([sigs[96 * i: 96 * i + 96] for i in range(N)])
    assert shim.AggregateVerify(pkl, msgs, agg) is True
    swapped = msgs[:]
    swapped[0], swapped[1] = swapped[1], swapped[0]
    assert shim.AggregateVerify(pkl, swapped, agg) is False
    assert OC.AggregateVerify(pkl[:128], msgs[:128], agg) is (N == 128)


def _e2_point(x0):
    """a point of E2(Fp2) with x = (x0, 1), any order"""
    x = x0
    while True:
        X = (x, 1)
        y = O.f2_sqrt(O.f2_add(O.f2_mul(O.f2_sqr(X), X), O.B2))
        if y is not None:
            return (X, y)
        x += 1


H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5


def _small_order_e2(q):
    """a point of E2 of order q for q = 13 or 23 (q^2 divides the G2 cofactor and E2's q-part has exponent q, so the
    multiplier drops every factor q; None is the identity in the oracle)"""
    x = 1
    while True:
        Q = O.g2_mul(_e2_point(x), H2 * O.R // (q * q))
        if Q is not None:
            assert O.g2_mul(Q, q) is None
            return Q
        x += 1


def test_fav_batch_signatures_outside_g2(batch, registry):
    """Signatures that decode to points of E2 outside G2 (the subgroup check): a random E2
    point, and points of order 13 and 23 -- the small-order ones make the incomplete Jacobian [|x|] chain of
    k_sig_lane2 hit its exceptional additions, which must reject.  Verdicts against the construction and the
    C oracle, through the batch path and the per-call path."""
    from bls_mi355x import bls as shim
    shim.use_mi355x()
    shim.bls_active = True
    B, n = 6, 16
    idx, offs, msgs, sigs = _make_batch(batch, B, n, seed=0xB2)
    bad = {1: _e2_point(3), 2: _small_order_e2(13), 4: _small_order_e2(23)}
    for j, pt in bad.items():
        assert not O.g2_in_subgroup(pt)
        sigs[96 * j: 96 * j + 96] = O.g2_compress(pt)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    expect = [j not in bad for j in range(B)]
    assert out.tolist() == expect
    idx2 = idx.reshape(B, n)
    for j in range(B):
        pks = [registry[48 * int(k): 48 * int(k) + 48] for k in idx2[j]]
        sig = bytes(sigs[96 * j: 96 * j + 96])
        assert OC.FastAggregateVerify(pks, msgs[j], sig) is expect[j]
        assert shim.FastAggregateVerify(pks, msgs[j], sig) is expect[j]


def test_h2c_fallback_routing_forced(batch, registry):
    """items of a batch forced onto k_h2c_fallback (bls_test_force_h2c_fallback, as if the
    lane SSWU had returned `rare` or a chain addition had been exceptional) get the reference-path H(m), which
    overwrites the lane kernels' output: the points equal the C oracle's hash_to_G2, and FAV / per-call Verify /
    AggregateVerify verdicts through the same routing match the construction."""
    import ctypes

    from bls_mi355x import _native
    from bls_mi355x.backend import mi355x_bls as M

    ctx = _native.context()
    n = 70  # past one 64-lane workgroup of the fallback's stride loop
    msgs = [hashlib.sha256(b"forced-fallback" + j.to_bytes(4, "little")).digest() for j in range(n)]
    forced = {0, 5, 63, 64, 69}
    mask = bytes(1 if j in forced else 0 for j in range(n))
    # the hook refuses without the process's opt-in (tests/conftest.py sets it)
    saved = os.environ.pop("BLSMI355X_TEST_HOOKS", None)
    try:
        assert ctx.lib.bls_test_force_h2c_fallback(ctx.h, mask, n) == -2  # BLS_E_ARG
    finally:
        os.environ["BLSMI355X_TEST_HOOKS"] = saved or "1"
    ctx.check(ctx.lib.bls_test_force_h2c_fallback(ctx.h, mask, n))
    try:
        out = ctypes.create_string_buffer(96 * n)
        ctx.check(ctx.lib.bls_test_hash_to_g2_batch(ctx.h, b"".join(msgs), n, out))
        for j in sorted(forced) + [1, 2, 62, 65]:
            assert out.raw[96 * j: 96 * j + 96] == OC.hash_to_g2(msgs[j]), j
        # a FAV batch whose forced items include valid and invalid ones
        B, k = n, 16
        idx, offs, bmsgs, sigs = _make_batch(batch, B, k, seed=0xFB)
        bad = {5: "wrong_msg", 64: "wrong_msg", 7: "wrong_msg"}
        for j, kind in bad.items():
            _corrupt(sigs, bmsgs, j, kind, B)
        got = batch.fast_aggregate_verify_batch(idx, offs, b"".join(bmsgs), bytes(sigs))
        expect = np.array([j not in bad for j in range(B)])
        assert (got == expect).all(), np.nonzero(got != expect)
        # per-call Verify and AggregateVerify (n = 1 and 3 messages) through the same routing
        pk, m = OC.SkToPk(11), msgs[0]
        assert M.Verify(pk, m, OC.Sign(11, m)) is True
        assert M.Verify(pk, m, OC.Sign(12, m)) is False
        pks = [OC.SkToPk(k) for k in (21, 22, 23)]
        agg = OC.Aggregate([OC.Sign(k, msgs[i]) for i, k in enumerate((21, 22, 23))])
        assert M.AggregateVerify(pks, msgs[:3], agg) is True
        assert M.AggregateVerify(pks, [msgs[0], msgs[2], msgs[1]], agg) is False
    finally:
        ctx.check(ctx.lib.bls_test_force_h2c_fallback(ctx.h, None, 0))
    # cleared: the lane path again, same points
    out2 = ctypes.create_string_buffer(96 * n)
    ctx.check(ctx.lib.bls_test_hash_to_g2_batch(ctx.h, b"".join(msgs), n, out2))
    assert out2.raw == out.raw


def test_resident_batch_chunked(batch, registry):
    """a ResidentFavBatch split into chunks (one FAV job per chunk, the C4 firehose's shape) with fewer
    jobs in flight than chunks: bad items in several chunks including the last item of the last chunk; every
    pass fails its batch check, and the stitched verdicts equal the unchunked batch's and the construction."""
    B, k, chunks = 512, 8, 4
    idx, offs, msgs, sigs = _make_batch(batch, B, k, seed=0xC4)
    bad = {3: "wrong_msg", 130: "inf_sig", 300: "zero_sig", B - 1: "wrong_msg"}
    for j, kind in bad.items():
        _corrupt(sigs, msgs, j, kind, B)
    expect = np.array([j not in bad for j in range(B)])
    rbc = batch.ResidentFavBatch(idx, offs, b"".join(msgs), bytes(sigs), chunks=chunks)
    rb1 = batch.ResidentFavBatch(idx, offs, b"".join(msgs), bytes(sigs))
    try:
        oks = rbc.run_pipelined([bytes([s]) * 32 for s in range(3)], depth=2)
        assert oks == [False] * 3
        vc = rbc.verdicts()
        assert rb1.run_pipelined([b"\x07" * 32], depth=1) == [False]
        assert (vc == rb1.verdicts()).all() and (vc == expect).all(), np.nonzero(vc != expect)
        # a clean chunked batch passes every pass
        idx2, offs2, msgs2, sigs2 = _make_batch(batch, B, k, seed=0xC5)
        rb2 = batch.ResidentFavBatch(idx2, offs2, b"".join(msgs2), bytes(sigs2), chunks=chunks)
        try:
            assert rb2.run_pipelined([b"\x01" * 32, b"\x02" * 32], depth=3) == [True, True]
            assert rb2.verdicts().all()
        finally:
            rb2.free()
    finally:
        rbc.free()
        rb1.free()


@pytest.mark.parametrize("B", [1, 2, 5])
def test_fav_small_batch_msm_identities(batch, registry, B):
    """Batches of 1, 2 and 5 items: most of the MSM's 64 bit-sums U_b are the identity (only the bits the few RLC
    scalars set), so most of the 64 pairs (-2^b G1, U_b) the MSM adds to the batch's Miller loops (k_msm_upairs)
    are skipped identities; a wrong or mis-skipped pair would fail the batch check and show as fallback work."""
    idx, offs, msgs, sigs = _make_batch(batch, B, 8, seed=40 + B)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    assert out.all()
    assert batch.fallback_stats() == (0, 0)
