"""Electra-size and phase0-maximum aggregates against the C oracle.

`is_valid_indexed_attestation` (specs/phase0/beacon-chain.md:776-790) hands FastAggregateVerify up to
MAX_VALIDATORS_PER_COMMITTEE = 2,048 keys in phase0 and up to 64 x 2,048 = 131,072 keys from Electra on
(MAX_VALIDATORS_PER_COMMITTEE * MAX_COMMITTEES_PER_SLOT, specs/electra/beacon-chain.md:365).  The C2/C3
configs stop at 512, so these cases exercise the long per-lane addition chains of the registry gather
(2,048 chained additions per lane at 131,072 keys) and the large-n per-call key validation:

  * batch path (registry-resident, bls_fav_batch_indexed): one ragged batch with two 131,072-key
    aggregates (one valid, one carrying another item's signature), 2,048- and 2,047-key committees, a
    1-key and a 3-key aggregate, and an ff-tail signature; verdicts against the construction and against
    oracle/bls_oracle.c's per-call (mode 0) FastAggregateVerify over the same affine registry keys;
  * per-call drop-in path (bls_fast_aggregate_verify on compressed keys) at 2,048 and 131,072 keys,
    against OC.FastAggregateVerify on the compressed keys (2,048) and the resident oracle (131,072).
"""
import hashlib

import numpy as np
import pytest

from oracle import bls_oracle as O
from oracle import bls_oracle_c as OC

pytestmark = pytest.mark.gpu

BIG = 64 * 2048  # 131,072
REG_N = (1 << 17) + 8192  # room for 131,072 distinct indices


@pytest.fixture(scope="module")
def env():
    from bls_mi355x import batch
    from bls_mi355x import bls as shim

    shim.use_mi355x()
    shim.bls_active = True
    r = batch.Registry()
    pks = r.generate(REG_N, first_sk=1, want_bytes=True)
    reg96 = OC.registry_generate(1, REG_N)  # the oracle's affine copy of the same keys (sk_i = i + 1)
    return batch, shim, pks, reg96


def _msgs(tag, B):
    return [hashlib.sha256(tag + j.to_bytes(8, "little")).digest() for j in range(B)]


def _items():
    rng = np.random.default_rng(0xE1EC)
    sizes = [BIG, BIG, 2048, 2047, 1, 3, 2048]
    return sizes, [np.sort(rng.choice(REG_N, size=n, replace=False)).astype(np.uint32) for n in sizes]


def _sign(batch, items, msgs):
    agg = [int((it.astype(np.int64) + 1).sum()) % O.R for it in items]
    return bytearray(batch.sign_batch(b"".join(a.to_bytes(32, "big") for a in agg), b"".join(msgs)))


def test_electra_batch_131072_and_2048(env):
    batch, _, _, reg96 = env
    sizes, items = _items()
    B = len(items)
    msgs = _msgs(b"electra", B)
    sigs = _sign(batch, items, msgs)
    sigs[96 * 1: 96 * 2] = sigs[0:96]  # item 1: item 0's signature (a valid point, wrong key set and message)
    sigs[96 * 6 + 92: 96 * 7] = b"\xff" * 4  # item 6: ff tail (test_eth_fast_aggregate_verify.py:104)
    idx = np.concatenate(items)
    offs = batch.offsets_from_lengths(sizes)
    out = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs))
    expect = np.array([True, False, True, True, True, True, False])
    assert (out == expect).all(), (out, expect)
    ref = OC.fav_batch_resident(reg96, idx, offs, b"".join(msgs), bytes(sigs), b"\x5e" * 32, 0, 8)
    assert ref == expect.tolist()


def test_electra_percall_2048_and_131072(env):
    batch, shim, pks, reg96 = env
    sizes, items = _items()
    msgs = _msgs(b"electra-pc", len(items))
    sigs = _sign(batch, items, msgs)

    def keys(j):
        return [pks[48 * int(i): 48 * int(i) + 48] for i in items[j]]

    # 2,048 keys: the drop-in wrapper against the C oracle on the same compressed bytes
    k2 = keys(2)
    s2 = bytes(sigs[192:288])
    assert shim.FastAggregateVerify(k2, msgs[2], s2) is True
    assert OC.FastAggregateVerify(k2, msgs[2], s2) is True
    assert shim.FastAggregateVerify(k2[:-1], msgs[2], s2) is False
    assert OC.FastAggregateVerify(k2[:-1], msgs[2], s2) is False
    # 131,072 keys: the drop-in wrapper against the construction and the resident oracle
    kb = keys(0)
    s0 = bytes(sigs[0:96])
    assert shim.FastAggregateVerify(kb, msgs[0], s0) is True
    assert shim.FastAggregateVerify(kb, msgs[1], s0) is False
    swapped = kb[:]
    swapped[BIG // 2] = pks[48 * int(items[1][0]): 48 * int(items[1][0]) + 48]
    assert shim.FastAggregateVerify(swapped, msgs[0], s0) is bool(items[1][0] == items[0][BIG // 2])
    idx = np.concatenate([items[0], items[0]])
    offs = batch.offsets_from_lengths([BIG, BIG])
    ref = OC.fav_batch_resident(reg96, idx, offs, msgs[0] + msgs[1], s0 + s0, b"\x5e" * 32, 0, 2)
    assert ref == [True, False]
