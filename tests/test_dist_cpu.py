"""world_size-2 gloo test of the multi-GPU combination protocol (SURVEY.md
§8(e), bls_mi355x.dist / bls_fav_job_check_comm): each rank holds the Miller
product of its shard, the 576-byte partials are all-gathered, every rank
multiplies and final-exponentiates; when the product fails, every rank
re-checks its own partial first (bls_fav_job_finish_dev with batch_ok = 0),
so only the bad shard bisects.  Partials here come from the oracle and the
all-gather is gloo's (no GPU on CPU); the library's RCCL all-gather of the
same bytes is exercised on the GPU (tests/test_gpu_comm.py)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from oracle import bls_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _partial_bytes(f):
    return b"".join(c[0].to_bytes(48, "big") + c[1].to_bytes(48, "big") for c in O.f12_to_coeffs(f))


def _from_bytes(b):
    return O.f12_from_coeffs([(int.from_bytes(b[96 * k: 96 * k + 48], "big"),
                               int.from_bytes(b[96 * k + 48: 96 * k + 96], "big")) for k in range(6)])


def _allgather(partial):
    import torch
    import torch.distributed as dist

    t = torch.frombuffer(bytearray(partial), dtype=torch.uint8)
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return b"".join(bytes(o.numpy()) for o in outs)


def _worker(rank, world, port, tamper, q):
    import torch.distributed as dist

    from bls_mi355x.dist import shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # shard r: one aggregate with sk = 3 + r over message m_r; pair (pk, H(m)) and (-G1, sig)
    sk = 3 + rank
    m = bytes([rank]) * 32
    pk = O.g1_mul(O.G1_GEN, sk)
    sig = O.g2_decompress(O.Sign(sk if not (tamper and rank == 1) else sk + 1, m))
    f = O.f12_mul(O.miller_loop(pk, O.hash_to_g2(m)), O.miller_loop(O.g1_neg(O.G1_GEN), sig))
    allp = _allgather(_partial_bytes(f))
    prod = O.F12_ONE
    for k in range(world):
        prod = O.f12_mul(prod, _from_bytes(allp[576 * k: 576 * k + 576]))
    ok = O.final_exponentiation(prod) == O.F12_ONE
    # a failing product: each rank re-checks its own partial (finish_dev's root re-check)
    own_ok = True if ok else O.final_exponentiation(f) == O.F12_ONE
    assert shard_bounds(10, rank, world) == ((0, 5), (5, 10))[rank]
    q.put((rank, (ok, own_ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("tamper", [False, True])
def test_two_rank_partials(tamper):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, tamper, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: (not tamper, True), 1: (not tamper, not tamper)}  # only rank 1's shard is bad


# ---- shards balanced by work (contiguous blocks of aggregates, balanced by
# total pubkey count).  Electra aggregates carry up to MAX_VALIDATORS_PER_COMMITTEE * MAX_COMMITTEES_PER_SLOT =
# 2,048 * 64 = 131,072 indices (specs/electra/beacon-chain.md:365), beside committees of a few hundred.
ELECTRA_SIZES = [131072, 64, 2048, 512, 3, 131072 // 2, 1, 2047] * 4 + [512] * 40


def _check_partition(bounds, offs, per_item, world):
    from bls_mi355x.dist import ITEM_WORK_KEYS  # noqa: F401  (the default weight is the §8(d) model's)

    B = len(offs) - 1
    assert bounds[0][0] == 0 and bounds[-1][1] == B
    assert all(bounds[r][1] == bounds[r + 1][0] for r in range(world - 1))
    work = [int(offs[hi] - offs[lo]) + per_item * (hi - lo) for lo, hi in bounds]
    item_max = max(int(offs[i + 1] - offs[i]) for i in range(B)) + per_item
    total = sum(work)
    assert all(abs(w - total / world) <= item_max for w in work), (work, total / world, item_max)
    return work


def test_shard_bounds_by_work_balances_variable_committees():
    import numpy as np

    from bls_mi355x.dist import ITEM_WORK_KEYS, shard_bounds, shard_bounds_by_work

    for sizes in (ELECTRA_SIZES, [512] * 2048, [1] * 1000 + [131072], list(range(1, 300))):
        offs = np.concatenate([[0], np.cumsum(sizes)])
        for world in (1, 2, 3, 4, 8):
            for per_item in (0, ITEM_WORK_KEYS):
                bounds = [shard_bounds_by_work(offs, r, world, per_item) for r in range(world)]
                _check_partition(bounds, offs, per_item, world)
    # uniform committees: the same blocks as the item-count split
    offs = np.arange(2049) * 512
    assert [shard_bounds_by_work(offs, r, 8) for r in range(8)] == [shard_bounds(2048, r, 8) for r in range(8)]
    # the item-count split is what the work split fixes: one rank would hold both 131,072-key aggregates
    offs = np.concatenate([[0], np.cumsum(ELECTRA_SIZES)])
    naive = [shard_bounds(len(ELECTRA_SIZES), r, 8) for r in range(8)]
    naive_work = [int(offs[hi] - offs[lo]) for lo, hi in naive]
    assert max(naive_work) > 4 * min(naive_work)


def test_shard_bounds_by_work_no_empty_rank():
    """with skewed committees the nearest-cut rule put several cuts on the same aggregate (ranks 1..6
    of [1] * 1000 + [131072] at world 8 got (1000, 1000)), and an empty shard cannot submit a job.  Every block is
    non-empty when B >= world; below that the empty ranks are the tail of a partition that still covers B."""
    import numpy as np

    from bls_mi355x.dist import ITEM_WORK_KEYS, shard_bounds_by_work, work_cuts

    for sizes in ([1] * 1000 + [131072], [131072] + [1] * 1000, [1] * 3 + [131072] * 2 + [1] * 3,
                  ELECTRA_SIZES, [5] * 8, [7] * 9):
        offs = np.concatenate([[0], np.cumsum(sizes)])
        for world in (2, 3, 4, 8):
            for per_item in (0, ITEM_WORK_KEYS):
                bounds = [shard_bounds_by_work(offs, r, world, per_item) for r in range(world)]
                _check_partition(bounds, offs, per_item, world)
                assert all(hi > lo for lo, hi in bounds), (sizes[:4], world, per_item, bounds)
    for B in range(0, 8):  # fewer aggregates than ranks: a partition of B, non-decreasing cuts
        offs = np.arange(B + 1) * 512
        c = work_cuts(offs, 8)
        assert c[0] == 0 and c[-1] == B and all(a <= b for a, b in zip(c, c[1:]))
        assert sum(c[r + 1] - c[r] for r in range(8)) == B


def _balance_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist

    from bls_mi355x.dist import ITEM_WORK_KEYS, shard_bounds_by_work

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    offs = np.concatenate([[0], np.cumsum(ELECTRA_SIZES)])
    mine = shard_bounds_by_work(offs, rank, world)  # each rank from the same offsets, no exchange of bounds
    allb = [None] * world
    dist.all_gather_object(allb, (rank, mine))
    q.put((rank, sorted(allb), ITEM_WORK_KEYS))
    dist.destroy_process_group()


def test_two_rank_electra_shards():
    """world 2 over gloo: the ranks' independently computed blocks partition the batch, balanced by work."""
    import numpy as np

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balance_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (b, w)) for r, b, w in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
    assert res[0][0] == res[1][0]
    bounds = [b for _, b in res[0][0]]
    offs = np.concatenate([[0], np.cumsum(ELECTRA_SIZES)])
    _check_partition(bounds, offs, res[0][1], 2)
