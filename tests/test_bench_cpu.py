"""bench.py's workload builders and shard arithmetic (host only, no GPU): the C3 epoch shards partition the
2,048 committees of one epoch at every world size with distinct indices per committee, the C4 firehose shards
cover 10^6 items in 125,000-item jobs, and the adversarial plan puts the same number of bad items of every
SURVEY.md §8(d) kind at distinct positions."""
import numpy as np
import pytest

import bench


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c3_shards_partition_the_epoch(world):
    seen = []
    for r in range(world):
        idx, offs, msgs, sks, (lo, hi) = bench.c3_shard(1 << 20, 0x5EED, r, world)
        B = hi - lo
        assert idx.size == 512 * B and offs[-1] == 512 * B and len(msgs) == 32 * B and len(sks) == 32 * B
        seen.append((lo, hi))
        two = idx.reshape(B, 512)
        assert all(len(set(row.tolist())) == 512 for row in two[:4])
    assert seen[0][0] == 0 and seen[-1][1] == 2048
    assert all(a[1] == b[0] for a, b in zip(seen, seen[1:]))


@pytest.mark.parametrize("world,chunks", [(1, 8), (2, 4), (4, 2), (8, 1)])
def test_c4_shards_and_jobs(world, chunks):
    total = 8000  # the same arithmetic as 10^6 in 125,000-item jobs, scaled down
    lo_hi = []
    for r in range(world):
        idx, offs, msgs, sks, ch, (lo, hi) = bench.c4_shard(total, 1, r, world, chunk=1000)
        assert ch == chunks and idx[0] == lo and idx.size == hi - lo and offs[-1] == hi - lo
        assert sks[:32] == (lo + 1).to_bytes(32, "big")
        lo_hi.append((lo, hi))
    assert lo_hi[0][0] == 0 and lo_hi[-1][1] == total


def test_adversarial_plan_every_kind():
    plan = bench.adversarial_plan(1024, 8, 5)
    assert len(plan) == 48 and all(0 <= j < 1024 for j in plan)
    assert {k: list(plan.values()).count(k) for k in bench.BAD_KINDS} == {k: 8 for k in bench.BAD_KINDS}


def test_corrupt_kinds():
    B = 4
    sigs = bytearray(bytes(range(96)) * B)
    idx2d = np.zeros((B, 8), dtype=np.uint32)
    bench.corrupt(sigs, idx2d, 0, "ff_tail", B)
    assert sigs[92:96] == b"\xff" * 4
    bench.corrupt(sigs, idx2d, 1, "inf_sig", B)
    assert sigs[96:192] == b"\xc0" + bytes(95)
    bench.corrupt(sigs, idx2d, 2, "g1_inf_pk", B)
    bench.corrupt(sigs, idx2d, 3, "pk_0x40", B)
    assert idx2d[2, 7] == bench.IDX_INF and idx2d[3, 0] == bench.IDX_0x40
    with pytest.raises(ValueError):
        bench.corrupt(sigs, idx2d, 0, "nope", B)
