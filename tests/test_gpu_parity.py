"""GPU parity: libblsmi355x.so (through the drop-in shim and the batch API)
against the golden fixtures and the CPU oracle.  Requires an MI355X."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from oracle import bls_oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as fh:
        return json.load(fh)


def hb(s):
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


@pytest.fixture(scope="module")
def B():
    from bls_mi355x import bls as shim
    shim.use_mi355x()
    shim.bls_active = True
    return shim


@pytest.fixture(scope="module")
def batch():
    from bls_mi355x import batch as b
    return b


def test_native_library_is_loaded(B):
    from bls_mi355x import _native
    ctx = _native.context()
    name, cus = ctx.device_info()
    assert "gfx950" in name and cus > 0


@pytest.mark.parametrize("case", _load("altair_bls.json"), ids=lambda c: c["case"])
def test_altair_bls_reference_vectors(B, case):
    if case["handler"] == "eth_aggregate_pubkeys":
        pks = [hb(p) for p in case["input"]]
        if case["output"] is None:
            with pytest.raises(Exception):
                B.eth_aggregate_pubkeys(pks)
        else:
            assert B.eth_aggregate_pubkeys(pks) == hb(case["output"])
    else:
        i = case["input"]
        got = B.eth_fast_aggregate_verify([hb(p) for p in i["pubkeys"]], hb(i["message"]), hb(i["signature"]))
        assert got == case["output"]


FORMATS = _load("bls_formats.json")


@pytest.mark.parametrize("case", FORMATS["sign"], ids=lambda c: c["input"]["privkey"][:10] + c["input"]["message"][:6])
def test_sign(B, case):
    sk = int.from_bytes(hb(case["input"]["privkey"]), "big")
    if case["output"] is None:
        with pytest.raises(Exception):
            B.Sign(sk, hb(case["input"]["message"]))
    else:
        assert B.Sign(sk, hb(case["input"]["message"])) == hb(case["output"])


@pytest.mark.parametrize("case", FORMATS["sk_to_pk"])
def test_sk_to_pk(B, case):
    assert B.SkToPk(int.from_bytes(hb(case["input"]), "big")) == hb(case["output"])


@pytest.mark.parametrize("case", FORMATS["verify"])
def test_verify(B, case):
    i = case["input"]
    assert B.Verify(hb(i["pubkey"]), hb(i["message"]), hb(i["signature"])) == case["output"]


@pytest.mark.parametrize("case", FORMATS["aggregate"])
def test_aggregate(B, case):
    sigs = [hb(s) for s in case["input"]]
    if case["output"] is None:
        with pytest.raises(Exception):
            B.Aggregate(sigs)
    else:
        assert B.Aggregate(sigs) == hb(case["output"])


@pytest.mark.parametrize("case", FORMATS["fast_aggregate_verify"])
def test_fast_aggregate_verify(B, case):
    i = case["input"]
    assert B.FastAggregateVerify([hb(p) for p in i["pubkeys"]], hb(i["message"]), hb(i["signature"])) == case["output"]


@pytest.mark.parametrize("case", FORMATS["aggregate_verify"])
def test_aggregate_verify(B, case):
    i = case["input"]
    got = B.AggregateVerify([hb(p) for p in i["pubkeys"]], [hb(m) for m in i["messages"]], hb(i["signature"]))
    assert got == case["output"]


@pytest.mark.parametrize("case", FORMATS["key_validate"])
def test_key_validate(B, case):
    assert B.KeyValidate(hb(case["input"])) == case["output"]


@pytest.mark.parametrize("case", _load("hash_to_g2.json"), ids=lambda c: c["msg"][:12] + c["dst"][:4])
def test_hash_to_g2(case):
    from bls_mi355x.backend import mi355x_bls
    assert mi355x_bls.hash_to_G2(hb(case["msg"]), case["dst"].encode()) == hb(case["output"])


def test_hash_to_g2_rfc9380_vectors():
    """The device hash_to_G2 (the per-call wide kernel) against RFC 9380 Appendix
    J.10.1's published points (tests/golden/rfc9380_hash_to_g2.json, QUUX DST): the raw hash bytes pinned to public
    vectors, not only to the oracle."""
    from bls_mi355x.backend import mi355x_bls

    g = _load("rfc9380_hash_to_g2.json")
    dst = g["dst"].encode()
    for v in g["vectors"]:
        pt = ((int(v["x"][0], 16), int(v["x"][1], 16)), (int(v["y"][0], 16), int(v["y"][1], 16)))
        assert mi355x_bls.hash_to_G2(v["msg"].encode(), dst) == O.g2_compress(pt), v["msg"]
    # (the FAV batch's lane kernels hash 32-byte signing roots under the POP DST; tests/test_gpu_percall.py::
    # test_h2c_wide_matches_oracle ties them to the wide kernel checked here)


def test_deposit_cli_known_answer(B):
    ka = _load("known_answers.json")
    for key in ("deposit_cli", "deposit_cli_flipped"):
        c = ka[key]
        assert B.Verify(hb(c["pubkey"]), hb(c["signing_root"]), hb(c["signature"])) == c["output"]


def test_stub_mode(B):
    B.bls_active = False
    try:
        assert B.Verify(b"", b"", b"") is True
        assert B.Sign(1, b"") == B.STUB_SIGNATURE
        assert B.AggregatePKs([]) == B.STUB_PUBKEY
    finally:
        B.bls_active = True


def test_trusted_setup_lagrange_sum_is_generator(B, batch):
    ts = _load("trusted_setup.json")
    lag = [hb(p) for p in ts["g1_lagrange"]]
    reg = batch.Registry()
    valid = reg.load(b"".join(lag))
    assert valid.all() and len(reg) == 4096
    # sum of the Lagrange basis is the generator (4096-key add tree)
    assert B.AggregatePKs(lag) == hb(ts["g1_monomial"][0])
    # every G2 setup point decodes and is in G2
    for q in ts["g2_monomial"][:8]:
        assert B.Aggregate([hb(q)]) == hb(q)


# ---------------------------------------------------------------- batches --
def _synthetic(n_reg, committees, seed=7, bad=()):
    """Registry sk_i = i+1; aggregate j signs SHA256(seed||j) with sum of its sks."""
    from bls_mi355x import batch as b
    rng = np.random.default_rng(seed)
    sks = b"".join((i + 1).to_bytes(32, "big") for i in range(n_reg))
    pks = b.sk_to_pk_batch(sks)
    idx, lens, msgs, agg_sks = [], [], [], []
    for j, size in enumerate(committees):
        c = rng.choice(n_reg, size=size, replace=False) if size else np.zeros(0, dtype=np.int64)
        idx.extend(int(x) for x in c)
        lens.append(size)
        msgs.append(hashlib.sha256(seed.to_bytes(8, "little") + j.to_bytes(8, "little")).digest())
        agg_sks.append(sum(int(x) + 1 for x in c) % O.R)
    sign_sks = b"".join((k if k else 1).to_bytes(32, "big") for k in agg_sks)
    sigs = bytearray(b.sign_batch(sign_sks, b"".join(msgs)))
    return pks, np.array(idx, dtype=np.uint32), b.offsets_from_lengths(lens), msgs, sigs


def test_sk_to_pk_and_sign_batch_match_oracle(batch):
    sks = [1, 2, 3, 0xDEADBEEF, O.R - 1]
    pks = batch.sk_to_pk_batch(b"".join(k.to_bytes(32, "big") for k in sks))
    for i, k in enumerate(sks):
        assert pks[48 * i: 48 * i + 48] == O.SkToPk(k)
    msgs = [bytes([i]) * 32 for i in range(len(sks))]
    sigs = batch.sign_batch(b"".join(k.to_bytes(32, "big") for k in sks), b"".join(msgs))
    for i, k in enumerate(sks[:2]):
        assert sigs[96 * i: 96 * i + 96] == O.Sign(k, msgs[i])


def test_fav_batch_all_valid(batch):
    committees = [1, 2, 3, 64, 65, 128, 200, 7]
    pks, idx, offs, msgs, sigs = _synthetic(512, committees)
    reg = batch.Registry()
    assert reg.load(pks).all()
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    assert out.all()
    # oracle cross-check of two items end to end
    for j in (0, 3):
        lo, hi = int(offs[j]), int(offs[j + 1])
        pkl = [pks[48 * int(k): 48 * int(k) + 48] for k in idx[lo:hi]]
        assert O.FastAggregateVerify(pkl, msgs[j], bytes(sigs[96 * j: 96 * j + 96]))


def test_fav_batch_adversarial(batch):
    committees = [16] * 24 + [0]
    pks, idx, offs, msgs, sigs = _synthetic(256, committees, seed=11)
    pks = bytearray(pks)
    # registry entry 5 replaced by a non-subgroup point -> KeyValidate fails
    x = 1
    while True:
        y = O.fp_sqrt(x ** 3 + 4)
        if y is not None and not O.g1_in_subgroup((x, y)):
            break
        x += 1
    pks[48 * 5: 48 * 6] = O.g1_compress((x, y))
    reg = batch.Registry()
    valid = reg.load(bytes(pks))
    assert valid.sum() == 255 and not valid[5]
    expect = np.ones(len(committees), dtype=bool)
    expect[-1] = False  # empty committee -> FastAggregateVerify([]) is False
    for j in range(len(committees) - 1):
        lo, hi = int(offs[j]), int(offs[j + 1])
        if 5 in idx[lo:hi]:
            expect[j] = False
    sigs[96 * 1: 96 * 2] = sigs[96 * 2: 96 * 3]              # valid point, wrong message: forces the fallback
    sigs[96 * 3: 96 * 4] = b"\xc0" + bytes(95)               # infinity signature
    sigs[96 * 4: 96 * 5] = bytes(96)                         # undecodable
    sigs[96 * 6 + 92: 96 * 7] = b"\xff" * 4                  # tampered tail
    q = O.iso_map(O.map_to_curve_sswu((5, 7)))               # on E2, outside G2: decodes, fails the subgroup check
    assert not O.g2_in_subgroup(q)
    sigs[96 * 8: 96 * 9] = O.g2_compress(q)
    expect[[1, 3, 4, 6, 8]] = False
    m = b"".join(msgs[:-1]) + msgs[-1]
    out = batch.fast_aggregate_verify_batch(idx, offs, m, bytes(sigs))
    assert (out == expect).all(), (out, expect)


@pytest.mark.parametrize("n_items", [1, 7, 33])
def test_fav_batch_odd_sizes_all_valid(batch, n_items):
    """Odd batch sizes exercise the padded pair of the 2-pair Miller groups."""
    pks, idx, offs, msgs, sigs = _synthetic(128, [3 + (j % 5) for j in range(n_items)], seed=21 + n_items)
    batch.Registry().load(pks)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    assert out.all()


def test_fav_batch_only_non_subgroup_signature_invalid(batch):
    """One decodable non-G2 signature in an otherwise valid batch: the batch
    check fails and the per-item re-check must flag exactly that item."""
    pks, idx, offs, msgs, sigs = _synthetic(128, [4] * 9, seed=31)
    batch.Registry().load(pks)
    q = O.iso_map(O.map_to_curve_sswu((11, 13)))
    assert not O.g2_in_subgroup(q)
    sigs[96 * 4: 96 * 5] = O.g2_compress(q)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    assert list(out) == [True] * 4 + [False] + [True] * 4


def test_fav_batch_out_of_range_index(batch):
    pks, idx, offs, msgs, sigs = _synthetic(64, [4, 4], seed=3)
    batch.Registry().load(pks)
    idx = idx.copy()
    idx[0] = 1000
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    assert list(out) == [False, True]


def test_verify_batch_indexed(batch):
    n = 40
    pks, idx, offs, msgs, sigs = _synthetic(n, [1] * n, seed=5)
    batch.Registry().load(pks)
    sigs[0:96] = sigs[96:192]
    out = batch.verify_batch(idx, b"".join(msgs), bytes(sigs))
    assert not out[0] and out[1:].all()


def test_resident_batch_partials(batch):
    pks, idx, offs, msgs, sigs = _synthetic(128, [8] * 10, seed=9)
    batch.Registry().load(pks)
    rb = batch.ResidentFavBatch(idx, offs, b"".join(msgs), bytes(sigs))
    p1 = rb.partial(b"\x01" * 32)
    # two shards' partials combine multiplicatively (here: the same shard twice)
    assert rb.check_partials(p1) and rb.check_partials(p1 + p1)
    rb.finish(True)
    assert rb.verdicts().all()
    rb.free()


def test_resident_batch_pipelined(batch):
    """bls_fav_job_*: consecutive passes with two batches in flight give the same verdicts as the
    one-at-a-time path, valid and with an invalid item (bisection inside a job)."""
    pks, idx, offs, msgs, sigs = _synthetic(128, [8] * 10, seed=11)
    batch.Registry().load(pks)
    good = batch.ResidentFavBatch(idx, offs, b"".join(msgs), bytes(sigs))
    assert good.run_pipelined([bytes([k]) * 32 for k in range(1, 6)]) == [True] * 5
    assert good.verdicts().all() and good.last_job == 4 % batch.FAV_JOBS
    bad_sigs = bytearray(sigs)
    bad_sigs[96 * 3:96 * 4] = sigs[96 * 4:96 * 5]
    bad = batch.ResidentFavBatch(idx, offs, b"".join(msgs), bytes(bad_sigs))
    assert bad.run_pipelined([bytes([k]) * 32 for k in range(1, 5)]) == [False] * 4
    v = bad.verdicts()
    assert not v[3] and v.sum() == 9 and bad.last_job == 3 % batch.FAV_JOBS
    # a job's own partial and an exchange that returns two shards' partials
    assert good.run_pipelined([b"\x07" * 32, b"\x08" * 32], exchange=lambda p: p + p) == [True, True]
    good.free()
    bad.free()


def test_percall_between_job_partial_and_finish(B, batch):
    """A per-call Verify / FastAggregateVerify on job 0 while a job-0 FAV batch sits between its partial and
    finish steps must not touch that batch's state: the bisection reads r_i apk_i back (the
    per-call pair points used to share the batch's slot, so items 0 and 1 came back invalid)."""
    pks, idx, offs, msgs, sigs = _synthetic(128, [8] * 10, seed=13)
    batch.Registry().load(pks)
    sigs[96 * 3: 96 * 4] = sigs[96 * 4: 96 * 5]  # item 3 invalid: the finish step bisects
    rb = batch.ResidentFavBatch(idx, offs, b"".join(msgs), bytes(sigs))
    rb.submit(0, b"\x09" * 32)
    ok = rb.job_check(0, rb.job_partial(0))
    assert ok is False
    m = b"\x12" * 32
    assert B.Verify(O.SkToPk(7), m, O.Sign(7, m)) is True
    assert B.FastAggregateVerify([O.SkToPk(5), O.SkToPk(6)], m, O.Sign(11, m)) is True
    rb.job_finish(0, ok)
    v = rb.verdicts()
    assert list(v) == [True] * 3 + [False] + [True] * 6
    rb.free()
