#!/usr/bin/env python3
"""Throughput of the other BASELINE.json configs on one
MI355X -- parity-tested cases, measured here as secondary lines (bench.py's
headline stays C2).  Prints one JSON line per config.

  C3 epoch replay: a seeded permutation of the 2^20 registry split into
     32 slots x 64 committees of 512 -> 2048 FastAggregateVerify, one RLC batch
     (device-resident inputs; passes pipelined like bench.py).
  C4 gossip: Verify with pk_i = registry[i], distinct m_i (the per-GPU shard of
     10^6 over 8 GPUs = 125,000), host-buffer C-ABI call (PCIe included).
  C5 AggregateVerify: one call with N distinct messages, N = 128 .. 8192
     (drop-in bls_aggregate_verify), and batches of 16 AggregateVerify items
     (bls_aggregate_verify_batch); adversarial FAV batches (1024 x 512 with k
     bad items, bisection fallback).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "eth-consensus-specs_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _line(**kw):
    print(json.dumps(kw), flush=True)


def _msgs(tag: bytes, n: int) -> list[bytes]:
    return [hashlib.sha256(tag + j.to_bytes(8, "little")).digest() for j in range(n)]


def c3(batch, ctx, reg_n, steps):
    rng = np.random.default_rng(0x5EED)
    perm = rng.permutation(reg_n).astype(np.uint32)
    B, n = 2048, reg_n // 2048
    offs = np.arange(B + 1, dtype=np.uint64) * n
    msgs = _msgs(b"epoch", B)
    agg = (perm.reshape(B, n).astype(np.int64) + 1).sum(axis=1)
    sigs = batch.sign_batch(b"".join((int(a) % R).to_bytes(32, "big") for a in agg), b"".join(msgs), ctx=ctx)
    rb = batch.ResidentFavBatch(perm, offs, b"".join(msgs), sigs, ctx=ctx)
    assert all(rb.run_pipelined([os.urandom(32)]))
    ctx.check(ctx.lib.bls_sync(ctx.h))
    t = time.perf_counter()
    oks = rb.run_pipelined([os.urandom(32) for _ in range(steps)])
    ctx.check(ctx.lib.bls_sync(ctx.h))
    dt = time.perf_counter() - t
    assert all(oks) and rb.verdicts().all()
    rb.free()
    _line(config="C3 epoch replay: 32 slots x 64 committees of 512 (2^20 registry), one RLC batch per epoch",
          value=round(B * steps / dt, 1), unit="FAV/s", ms_per_epoch=round(dt / steps * 1e3, 3), steps=steps)


def c4(batch, ctx, reg_n, B):
    idx = np.arange(B, dtype=np.uint32) % reg_n
    msgs = _msgs(b"gossip", B)
    sigs = batch.sign_batch(b"".join(int(k + 1).to_bytes(32, "big") for k in idx), b"".join(msgs), ctx=ctx)
    m = b"".join(msgs)
    assert batch.verify_batch(idx, m, sigs, ctx=ctx).all()
    t = time.perf_counter()
    v = batch.verify_batch(idx, m, sigs, ctx=ctx)
    dt = time.perf_counter() - t
    assert v.all()
    _line(config=f"C4 gossip firehose: {B} single-signature Verify, distinct messages (per-GPU shard of 10^6 / 8)",
          value=round(B / dt, 1), unit="Verify/s", ms=round(dt * 1e3, 2), note="host buffers (PCIe included)")


def c5(batch, ctx):
    from bls_mi355x.backend import mi355x_bls

    for N in (128, 512, 2048, 8192):
        sks = [(7919 * (i + 1)) % R for i in range(N)]
        pks = batch.sk_to_pk_batch(b"".join(k.to_bytes(32, "big") for k in sks), ctx=ctx)
        pkl = [pks[48 * i: 48 * i + 48] for i in range(N)]
        msgs = _msgs(b"av%d" % N, N)
        s = batch.sign_batch(b"".join(k.to_bytes(32, "big") for k in sks), b"".join(msgs), ctx=ctx)
        agg = mi355x_bls.Aggregate([s[96 * i: 96 * i + 96] for i in range(N)])
        assert mi355x_bls.AggregateVerify(pkl, msgs, agg)
        reps = max(1, 4096 // N)
        t = time.perf_counter()
        for _ in range(reps):
            ok = mi355x_bls.AggregateVerify(pkl, msgs, agg)
        dt = (time.perf_counter() - t) / reps
        assert ok
        # 16 such items in one bls_aggregate_verify_batch call
        items = 16
        t = time.perf_counter()
        v = batch.aggregate_verify_batch([pkl] * items, [msgs] * items, [agg] * items, ctx=ctx)
        dtb = time.perf_counter() - t
        assert v.all()
        _line(config=f"C5 AggregateVerify, N={N} distinct messages", value=round(N / dt, 1), unit="pairs/s",
              ms_per_call=round(dt * 1e3, 3), batch16_pairs_s=round(items * N / dtb, 1),
              batch16_ms=round(dtb * 1e3, 2))


def c5_adversarial(batch, ctx, reg_n):
    B, n = 1024, 512
    rng = np.random.default_rng(5)
    idx = np.concatenate([rng.permutation(reg_n)[: B * n // 2] for _ in range(2)]).astype(np.uint32)
    offs = np.arange(B + 1, dtype=np.uint64) * n
    msgs = _msgs(b"adv", B)
    agg = (idx.reshape(B, n).astype(np.int64) + 1).sum(axis=1)
    sigs0 = batch.sign_batch(b"".join((int(a) % R).to_bytes(32, "big") for a in agg), b"".join(msgs), ctx=ctx)
    for k in (0, 1, 8, 64):
        sigs = bytearray(sigs0)
        bad = rng.choice(B, size=k, replace=False)
        for j in bad:  # wrong-message signature: a valid G2 point, only the pairing check catches it
            o = (int(j) + 1) % B
            sigs[96 * j: 96 * j + 96] = sigs0[96 * o: 96 * o + 96]
        t = time.perf_counter()
        v = batch.fast_aggregate_verify_batch(idx, offs, b"".join(msgs), bytes(sigs), ctx=ctx)
        dt = time.perf_counter() - t
        expect = np.ones(B, dtype=bool)
        expect[bad] = False
        assert (v == expect).all()
        checks, rounds = batch.fallback_stats(ctx=ctx)
        _line(config=f"C5 adversarial FAV batch: {B} x {n}, k={k} wrong-message signatures", value=round(B / dt, 1),
              unit="FAV/s", ms=round(dt * 1e3, 2), fe_checks=checks, bisection_rounds=rounds)


def main():
    from bls_mi355x import _native, batch

    ctx = _native.context()
    reg_n = 1 << 20
    batch.Registry(ctx).generate(reg_n, first_sk=1)
    c3(batch, ctx, reg_n, steps=8)
    c4(batch, ctx, reg_n, 125000)
    c5_adversarial(batch, ctx, reg_n)
    c5(batch, ctx)


if __name__ == "__main__":
    main()
