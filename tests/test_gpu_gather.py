"""The registry gather of FAV batches (E/utils/bls.py:167-177 aggregates the pubkeys before its pairing check)
against the construction: the complete-formula kernel (k_fav_gather_q, the default) and the affine kernel
(csrc/bls_gather_aff.hip, BLS_GATHER=affine, read per batch; one lane per aggregate from 4,096 aggregates up) on
the same batches, including the exceptional pairs the affine formulas cannot add -- a duplicate index (P + P) and a
key beside its negation (P + (-P)), which reach its redo path -- committees larger than one chunk (1,500 keys), and
the identity aggregate {P, -P}."""
import hashlib
import os
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
REG = 1 << 14


def _neg(pk48: bytes) -> bytes:
    return bytes([pk48[0] ^ 0x20]) + pk48[1:]  # the sign flag: -P has the other y


def _case(seed: int, B: int, sizes):
    """B committees (sizes cycled) over a 2^14 registry + the negations of keys 0..63 appended at REG .. REG + 63;
    committee 0 repeats a key, committee 1 holds a key and its negation (both at level 0 of the affine tree when
    the committee has >= 32 keys), committee 2 is only {P, -P} (the identity: invalid)."""
    rng = np.random.default_rng(seed)
    idx, lens, sks = [], [], []
    for b in range(B):
        n = sizes[b % len(sizes)]
        c = rng.choice(REG, size=n, replace=False).astype(np.int64)
        if b == 0 and n >= 2:
            c[1] = c[0]
        if b == 1 and n >= 2:
            c[0], c[1] = 5, REG + 5
        if b == 2:
            c = np.array([7, REG + 7], dtype=np.int64)
        sk = sum((int(k) + 1) if k < REG else -(int(k) - REG + 1) for k in c) % R
        idx.append(c.astype(np.uint32))
        lens.append(len(c))
        sks.append(sk)
    msgs = [hashlib.sha256(b"gather" + seed.to_bytes(4, "little") + j.to_bytes(4, "little")).digest() for j in range(B)]
    return idx, lens, sks, msgs


def _run(B, sizes, seed):
    from bls_mi355x import _native, batch

    ctx = _native.context()
    reg = batch.Registry(ctx)
    pks = reg.generate(REG, first_sk=1, want_bytes=True)
    assert reg.append(b"".join(_neg(pks[48 * i: 48 * i + 48]) for i in range(64))).all()
    idx, lens, sks, msgs = _case(seed, B, sizes)
    good = [sk != 0 for sk in sks]
    sigs = bytearray(batch.sign_batch(b"".join((sk or 1).to_bytes(32, "big") for sk in sks), b"".join(msgs), ctx=ctx))
    expect = np.array(good, dtype=bool)
    # item 3: the signature of another message (only the pairing check catches it)
    sigs[96 * 3: 96 * 4] = sigs[96 * 4: 96 * 5]
    expect[3] = False
    offs = batch.offsets_from_lengths(lens)
    flat = np.concatenate(idx)
    out = batch.fast_aggregate_verify_batch(flat, offs, b"".join(msgs), bytes(sigs), ctx=ctx)
    rb = batch.ResidentFavBatch(flat, offs, b"".join(msgs), bytes(sigs), ctx=ctx)
    oks = rb.run_pipelined([os.urandom(32) for _ in range(2)])
    v = rb.verdicts()
    rb.free()
    return out, v, oks, expect


@pytest.mark.parametrize("mode", ["affine", "complete"])
@pytest.mark.parametrize("B,sizes", [(4096, [64, 40, 33, 512, 31, 2, 1]), (1100, [128, 700, 1, 96, 63]),
                                     (4100, [1500])])
def test_gather_exceptional_pairs(B, sizes, mode, monkeypatch):
    monkeypatch.setenv("BLS_GATHER", mode)
    out, v, oks, expect = _run(B, sizes, seed=B)
    assert expect[0] and expect[1] and not expect[2] and not expect[3]
    assert (out == expect).all(), np.nonzero(out != expect)
    assert (v == expect).all() and oks == [False, False]


def test_gather_aff_matches_complete_kernel(monkeypatch):
    """One batch through both kernels: identical verdicts (two bad items: the identity aggregate, a wrong message)."""
    res = {}
    for mode in ("affine", "complete"):
        monkeypatch.setenv("BLS_GATHER", mode)
        out, v, oks, e = _run(4096, [64, 40, 33, 512, 31, 2, 1], 7)
        res[mode] = (out.tolist(), v.tolist())
    assert res["affine"] == res["complete"] and res["affine"][0].count(False) == 2
