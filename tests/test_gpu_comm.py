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


def test_rccl_empty_shard_joins_the_exchange():
    """A rank with no aggregates (B < world) submits an empty job: its partial is the identity and it still takes
    part in the submit-time all-gather (bls_fav_job_submit_dev with B = 0, device exchange only)."""
    import ctypes

    from bls_mi355x import _native, batch, dist

    ctx = _native.context()
    batch.Registry(ctx).generate(1 << 10, first_sk=1)
    offs = batch.DeviceBuffer(ctx, np.zeros(1, dtype=np.uint64))
    seed = os.urandom(32)
    # no communicator: an empty job is an argument error
    assert ctx.lib.bls_fav_job_submit_dev(ctx.h, 1, None, offs.ptr, 0, None, None, seed) == -2  # BLS_E_ARG
    dist.init_comm(ctx, 0, 1, DictStore())
    try:
        assert ctx.lib.bls_fav_job_submit_dev(ctx.h, 1, None, offs.ptr, 0, None, None, seed) == 1
        part = ctypes.create_string_buffer(576)
        assert ctx.lib.bls_fav_job_partial(ctx.h, 1, part) == 1
        one = bytearray(576)
        one[47] = 1  # Fp12 one: c0 of the w^0 coefficient (big-endian 48-byte words, c0 then c1 per w-power)
        assert part.raw == bytes(one)
        assert ctx.lib.bls_fav_job_check_comm(ctx.h, 1) == 1
        assert ctx.lib.bls_fav_job_finish_dev(ctx.h, 1, 1, None) == 1
        # a real batch on the same job afterwards
        idx, offs2, msgs, sigs = _inputs(batch, 40, 8, 1 << 10, seed=5)
        rb = batch.ResidentFavBatch(idx, offs2, msgs, bytes(sigs), ctx=ctx)
        assert rb.run_pipelined([os.urandom(32) for _ in range(3)], comm=True) == [True] * 3 and rb.verdicts().all()
        rb.free()
    finally:
        dist.destroy_comm(ctx)
        offs.free()


def test_finish_after_interleaved_host_batch_bisects_from_root():
    """a job slot's own verdict belongs to the batch its submit prepared.  A host-buffer batch on job 0
    in between (bls_fav_batch_indexed) replaces the slot's batch state, so bls_fav_batch_finish_dev(0) must
    bisect that batch from the root instead of reusing the earlier batch's passing verdict."""
    from bls_mi355x import _native, batch

    ctx = _native.context()
    batch.Registry(ctx).generate(1 << 10, first_sk=1)
    idx, offs, msgs, sigs = _inputs(batch, 30, 8, 1 << 10, seed=6)
    rb = batch.ResidentFavBatch(idx, offs, msgs, bytes(sigs), ctx=ctx)
    rb.submit(0, os.urandom(32))
    assert rb.job_check_own(0)  # the valid device batch passes (its own verdict: 1)
    bad = bytearray(sigs)
    bad[96 * 4: 96 * 5] = bad[96 * 5: 96 * 6]  # item 4 signs another message
    host = batch.fast_aggregate_verify_batch(idx, offs, msgs, bytes(bad), ctx=ctx)  # job 0's state is now this batch
    assert not host[4] and host.sum() == 29
    out = batch.DeviceBuffer(ctx, nbytes=30)
    ctx.check(ctx.lib.bls_fav_batch_finish_dev(ctx.h, 0, out.ptr))
    v = out.to_host().astype(bool)
    assert not v[4] and v.sum() == 29, v
    out.free()
    rb.free()


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
