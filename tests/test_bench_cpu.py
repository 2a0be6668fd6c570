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


def _run_bench(args, **env_over):
    import os
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_over)
    return subprocess.run([sys.executable, bench.__file__, *args], env=env, capture_output=True, text=True,
                          timeout=300)


@pytest.mark.parametrize("n", [2, 8])
def test_launcher_dry_run_rank_envs(n):
    """`python bench.py --gpus N` (no WORLD_SIZE) starts one process per GPU; the dry run prints what each child
    would get and stops before anything touches HIP."""
    import json

    p = _run_bench(["--gpus", str(n), "--steps", "3", "--launch-dry-run"])
    assert p.returncode == 0, p.stderr
    plan = json.loads(p.stdout.strip().splitlines()[-1])["launcher"]
    assert plan["ranks"] == n and plan["cmd"][-5:] == ["--gpus", str(n), "--steps", "3", "--launch-dry-run"]
    ch = plan["children"]
    assert [c["RANK"] for c in ch] == [str(r) for r in range(n)] == [c["LOCAL_RANK"] for c in ch]
    assert {c["WORLD_SIZE"] for c in ch} == {str(n)} and {c["MASTER_ADDR"] for c in ch} == {"127.0.0.1"}
    assert len({c["MASTER_PORT"] for c in ch}) == 1 and int(ch[0]["MASTER_PORT"]) > 0


def test_launcher_refuses_world_mismatch_and_missing_gpus():
    p = _run_bench(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr and "--gpus 2" in p.stderr
    # this container has no GPU (the one-GPU box has 1): --gpus 2 must fail loudly, never run one rank and print
    # n_gpus 1
    p = _run_bench(["--gpus", "2", "--no-cpu"])
    assert p.returncode != 0 and "needs 2 GPUs" in p.stderr and '"n_gpus"' not in p.stdout


def test_rank_envs():
    envs = bench.rank_envs(4, 12345, base={"PATH": "/bin", "WORLD_SIZE": "9"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"] and all(e["WORLD_SIZE"] == "4" for e in envs)
    assert all(e["PATH"] == "/bin" and e["MASTER_PORT"] == "12345" for e in envs)


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
