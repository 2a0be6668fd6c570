"""The multi-GPU exchange inside the C ABI: the RCCL
communicator of a context (bls_comm_init, world 1 on this one-GPU box) and
bls_fav_job_check_comm, which all-gathers each job's 576-byte partial on the
device and final-exponentiates the product; plus two ranks on one GPU whose
partials cross through gloo into bls_fav_job_check, covering the
bad-shard localisation of bls_fav_job_finish_dev (only the rank whose own
partial fails bisects).  The 8-rank RCCL run itself is bench.py --gpus 8."""
import hashlib
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inputs(batch, B, n, reg_n, seed):
    rng = np.random.default_rng(seed)
    idx = np.stack([rng.choice(reg_n, size=n, replace=False) for _ in range(B)]).astype(np.uint32)
    msgs = [hashlib.sha256(b"comm" + seed.to_bytes(4, "little") + j.to_bytes(4, "little")).digest() for j in range(B)]
    agg = (idx.astype(np.int64) + 1).sum(axis=1)
    sigs = bytearray(batch.sign_batch(b"".join(int(a).to_bytes(32, "big") for a in agg), b"".join(msgs)))
    return idx.reshape(-1), np.arange(B + 1, dtype=np.uint64) * n, b"".join(msgs), sigs


class DictStore(dict):
    def set(self, k, v):
        self[k] = v

    def get(self, k):
        return self[k]


def test_rccl_world1_pipeline():
    from bls_mi355x import _native, batch, dist

    ctx = _native.context()
    batch.Registry(ctx).generate(1 << 12, first_sk=1)
    dist.init_comm(ctx, 0, 1, DictStore())
    try:
        idx, offs, msgs, sigs = _inputs(batch, 300, 16, 1 << 12, seed=3)
        rb = batch.ResidentFavBatch(idx, offs, msgs, bytes(sigs), ctx=ctx)
        oks = rb.run_pipelined([os.urandom(32) for _ in range(7)], comm=True)
        assert oks == [True] * 7 and rb.verdicts().all()
        rb.free()
        sigs[96 * 11: 96 * 12] = sigs[96 * 12: 96 * 13]  # item 11 invalid
        rb = batch.ResidentFavBatch(idx, offs, msgs, bytes(sigs), ctx=ctx)
        oks = rb.run_pipelined([os.urandom(32) for _ in range(3)], comm=True)
        v = rb.verdicts()
        assert oks == [False] * 3 and not v[11] and v.sum() == 299
        rb.free()
    finally:
        dist.destroy_comm(ctx)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, tamper, q):
    import torch
    import torch.distributed as tdist

    from bls_mi355x import _native, batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = _native.context()
        batch.Registry(ctx).generate(1 << 12, first_sk=1)
        idx, offs, msgs, sigs = _inputs(batch, 200, 16, 1 << 12, seed=10 + rank)
        if tamper and rank == 1:
            sigs[96 * 42: 96 * 43] = sigs[96 * 43: 96 * 44]

        def exchange(part):
            t = torch.frombuffer(bytearray(part), dtype=torch.uint8)
            outs = [torch.empty_like(t) for _ in range(world)]
            tdist.all_gather(outs, t)
            return b"".join(bytes(o.numpy()) for o in outs)

        rb = batch.ResidentFavBatch(idx, offs, msgs, bytes(sigs), ctx=ctx)
        oks = rb.run_pipelined([os.urandom(32) for _ in range(2)], exchange=exchange)
        v = rb.verdicts()
        q.put((rank, oks, int(v.sum()), bool(v[42])))
        rb.free()
    finally:
        tdist.destroy_process_group()


@pytest.mark.parametrize("tamper", [False, True])
def test_two_ranks_one_gpu_bad_shard(tamper):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, tamper, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, oks, nvalid, v42 = q.get(timeout=240)
        res[r] = (oks, nvalid, v42)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if not tamper:
        assert res == {0: ([True, True], 200, True), 1: ([True, True], 200, True)}
    else:  # the global check fails on both ranks; only rank 1 (its own partial fails) loses item 42
        assert res == {0: ([False, False], 200, True), 1: ([False, False], 199, False)}
