#!/usr/bin/env python3
"""bench.py -- FastAggregateVerify throughput on MI355X (BASELINE.json metric).

Headline workload (--config c2, the default; BASELINE.json configs[1], SURVEY.md
§8(d) C2): sync-committee FastAggregateVerify, 10,000 aggregates x 512 pubkeys
per GPU, pubkeys named by index into a 2^20-key registry resident in HBM
(sk_i = i + 1), distinct 32-byte messages SHA256(seed||rank||j), valid
aggregate signatures made on the device.  One step = one pass of the hot path
over the batch: registry gather + aggregate pubkeys, signature decode/subgroup
checks, hash_to_G2, random-linear-combination Miller loops, one shared final
exponentiation (per-item fallback only on failure), verdicts written to HBM.

The other BASELINE configs are selectable (the driver runs c2; every config
runs at any world size through the same RCCL exchange):
  --config c3  mainnet epoch replay (configs[2]): a seeded permutation of the
               2^20 registry, 32 slots x 64 committees of 512 = 2,048 FAV per
               epoch; the epoch is sharded over the ranks (strong scaling), each
               rank's Miller partial all-gathered over RCCL, one verdict per
               epoch.  One step = one epoch.
  --config c4  gossip firehose (configs[3]): 10^6 single-signature Verify with
               distinct messages, contiguous shards of 10^6 / world (125,000 at
               8 GPUs), each shard in 125,000-item jobs.  One step = 10^6 Verify.
  --config c5  adversarial FAV batches (configs[4]): 1,024 x 512 per rank with
               k bad items of every SURVEY §8(d) kind (bisection fallback each
               step), plus AggregateVerify with N = 128 .. 8,192 distinct
               messages as secondary figures.
The c2 line also carries the registry-load figure (`registry_load`: bls_registry_load of the 2^20 compressed
keys the passes then read, keys/s), a C3 epoch-replay figure (`c3`), a C4 figure (`c4`: one 125,000-Verify shard
per GPU, Verify/s), a C5 figure (`c5`: adversarial 1,024 x 512 batches with 8 bad items, FAV/s, plus
AggregateVerify N = 128 / 1,024 / 8,192 in pairs/s) and, on rank 0, a
parity sample (`parity`): an adversarial 1,024 x 512 slice with 8 bad items of
each kind checked against the construction and, on 16 sampled items, against
the C oracle; hash_to_G2 of the golden messages against their committed
points; the deposit-cli known answer through the per-call API.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N): the ranks' 576-byte Fp12 Miller partials are all-gathered by the
library over RCCL (bls_fav_job_check_comm: ncclAllGather on the device, xGMI)
and every rank final-exponentiates the product.  torch.distributed (gloo) is
only the control plane: rendezvous, the RCCL unique id, barriers, max over
ranks.

Roofline: after the timed region, a few passes run one batch at a time with
per-kernel hipEvent timing (bls_profile_*), so each kernel's average is its
own execution time (with five batches in flight a hipEvent pair also spans
the wait for the queue and CUs); `roofline` uses those averages.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

# before torch / HIP start (multi-GPU ranks initialise HIP through torch first): see _native.hw_queue_policy
if not os.environ.get("BLSMI355X_KEEP_HW_QUEUES") and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "eth-consensus-specs_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "BLS sig verifications/sec (FastAggregateVerify, 1/8 GPU) + % int VALU peak"
PEAK_INT_OPS = 256 * 4 * 32 / 2 * 2.4e9  # v_mad_u64_u32 is half rate on gfx950: 39.3e12 lane-ops/s
FME_OPS = 288  # one 381-bit Montgomery multiplication = 288 v_mad_u64_u32
SHA_OPS = 2400  # one SHA-256 compression
MEASURED_MAD_OPS = 31.3e12  # sustained v_mad_u64_u32 lane-ops/s, profiles/r01_s2_madrate_microbench.txt
SINGLE_KERNEL = ("miller", "miller_lines", "fav_gather")
# a FAV batch's Miller loops run split (k_miller_lines2 + k_miller_acc4q) unless BLS_MILLER_FUSED=1 selects the
# fused kernel (k_miller_fused: G2 lines and f accumulation in one workgroup, lines in LDS; bls_capi.hip)
MILLER_FUSED = os.environ.get("BLS_MILLER_FUSED") == "1"
MSM_PAIRS = 64  # the MSM's bit-sum pairs (-2^b G1, U_b) join every batch's Miller loops (bls_msm.hip)
# pairs per f of k_miller_acc4q<G> on batches of >= ACC_SHARED_MIN items (bls_capi.hip fav_prepare: BLS_ACC_G, default
# 4), one pair per f below
ACC_G = {"1": 1, "2": 2, "8": 8}.get(os.environ.get("BLS_ACC_G", "4"), 4)
ACC_SHARED_MIN = int(os.environ.get("BLS_ACC_SHARED_MIN", "4096"))


def acc_g(items: int) -> int:
    return ACC_G if items >= ACC_SHARED_MIN else 1


def lane_kernels(items: int) -> dict:
    """Lanes per item of the lane kernels (full register file, one wave per SIMD): k_miller_acc4q<G> four lanes per
    G pairs (bls_miller_pair.hip), k_miller_lines2 two per pair (bls_miller_lane.hip), k_sig_lane2 one for the G1
    chain and two for the G2 chain of an item (bls_chain_lane.hip)."""
    return {"miller": 3 if MILLER_FUSED else 4 / acc_g(items), "miller_lines": 2, "sig_vm": 3}


GATHER_BYTES_PER_KEY = 4 + 96  # u32 index + one 96-B registry record (affine x, y; validity in x's top bit)


def kernel_symbol(kernel: str, items: int) -> str | None:
    """profile entry -> kernel symbol in the rocprofv3 summaries (profiles/*kernel_stats*.md)."""
    return {"miller": "k_miller_fused<2>" if MILLER_FUSED else f"k_miller_acc4q<{acc_g(items)}>",
            "miller_lines": "k_miller_lines2", "fav_gather": "k_fav_gather_q<16>"}.get(kernel)
ROCPROF_AVG = os.path.join(ROOT, "profiles", "rocprof_kernel_avg.json")
LIB = os.path.join(ROOT, "eth-consensus-specs_amd", "libblsmi355x.so")

REG_N = 1 << 20
G1_INF = b"\xc0" + bytes(47)
PK_0x40 = b"\x40" + bytes(47)
IDX_INF, IDX_0x40 = REG_N, REG_N + 1  # invalid keys appended after the 2^20 generated ones
BAD_KINDS = ("wrong_msg", "inf_sig", "zero_sig", "ff_tail", "g1_inf_pk", "pk_0x40")
C3_SLOTS, C3_PER_SLOT, C3_N = 32, 64, 512  # presets/mainnet/phase0.yaml: SLOTS_PER_EPOCH, MAX_COMMITTEES_PER_SLOT
C4_TOTAL, C4_CHUNK = 10 ** 6, 125_000


def launch_grid(kernel: str, items: int) -> int | None:
    """Threads of one launch of the roofline kernel over `items` FAV items (rocprofv3's grid_x).  The Miller
    kernels run items + 64 pairs (the MSM's bit-sum pairs): k_miller_fused<2> one 192-thread workgroup per 64 pairs,
    k_miller_acc4q<G> 4 lanes per G pairs in 64-lane workgroups, k_miller_lines2 2 lanes per pair;
    k_fav_gather_q<16> 16 lanes per aggregate (bls_miller_pair.hip, bls_miller_lane.hip, bls_kernels.hip)."""
    np_ = items + MSM_PAIRS
    if kernel == "miller" and MILLER_FUSED:
        return (np_ + 63) // 64 * 192
    g = acc_g(items)
    lanes = {"miller": 4 * ((np_ + g - 1) // g), "miller_lines": 2 * np_, "fav_gather": 16 * items}.get(kernel)
    return None if lanes is None else (lanes + 63) // 64 * 64


def model_fme(n: int):
    """Per-item algorithmic work of FAV(n) with a resident registry."""
    return {
        "fav_gather": 11 * (n - 1),
        "sig_decode": 1200,             # signature decompression (Fp2 square root)
        "sig_vm": 1200 + 1000 + 400,    # G2 subgroup check, RLC G1, RLC G2 (MSM share)
        "fav_hash": 6600,
        # Miller loop, 4400 FME per pair: all of it in the fused kernel, or split between the two kernels of
        # the split form in the proportion of the products each executes per pair with f shared by two pairs
        # (k_miller_acc4q: 62 Fp12 squarings x 36 / 2 + 68 sparse line products x 43 = 4040; k_miller_lines2, T:
        # 63 doublings x 26 + 5 additions x 35 = 1813).  The share is the model's, fixed whatever G the shipped
        # kernel runs (with four pairs per f it executes 62 x 36 / 4 + 68 x 43 = 3,482 FME per pair).  (The MSM's 64
        # extra pairs per batch are not counted.)
        "miller": 4400 if MILLER_FUSED else 4400 * 4040 / 5853,
        "miller_lines": 4400 * 1813 / 5853,
    }


def item_ops(n: int) -> int:
    """SURVEY.md §8(d) int ops of one registry-resident FAV(n) (Verify: n = 1)."""
    return (11 * (n - 1) + 14789) * FME_OPS + 19 * SHA_OPS


BATCH_OPS = 9268 * FME_OPS  # shared per batch: 63 Fp12 squarings x 36 + final exponentiation (§8(d))


# ------------------------------------------------------------------ workloads --
def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """C4: contiguous equal blocks of single-key Verify items (bls_mi355x.dist.shard_bounds)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_bounds_by_work(offsets, rank: int, world: int) -> tuple[int, int]:
    """C2 / C3 / C5: contiguous blocks of aggregates balanced by work (pubkeys + the per-aggregate constant;
    bls_mi355x.dist.shard_bounds_by_work)."""
    from bls_mi355x.dist import shard_bounds_by_work as f

    return f(offsets, rank, world)


def _msg(tag: bytes, seed: int, j: int) -> bytes:
    return hashlib.sha256(tag + seed.to_bytes(8, "little") + int(j).to_bytes(8, "little")).digest()


def _agg_sks(idx2d: np.ndarray) -> bytes:
    """Aggregate secret key of each committee (sk_i = i + 1; the sum stays far below r)."""
    agg = (idx2d.astype(np.int64) + 1).sum(axis=1)
    return b"".join(int(a).to_bytes(32, "big") for a in agg)


def build_inputs(B: int, n: int, reg_n: int, seed: int, rank: int):
    """C2: B committees of n distinct indices, messages and aggregate secret keys (host, numpy)."""
    rng = np.random.default_rng(seed * 1000003 + rank)
    total = B * n
    perms = []
    while sum(p.size for p in perms) < total:
        perms.append(rng.permutation(reg_n).astype(np.uint32))
    idx = np.concatenate(perms)[:total] if len(perms) > 1 else perms[0][:total]
    assert reg_n % n == 0  # committees never straddle two permutations: indices distinct per committee
    offs = np.arange(B + 1, dtype=np.uint64) * n
    msgs = b"".join(hashlib.sha256(b"bench" + seed.to_bytes(8, "little") + rank.to_bytes(4, "little")
                                   + j.to_bytes(8, "little")).digest() for j in range(B))
    return idx, offs, msgs, _agg_sks(idx.reshape(B, n))


def c3_shard(reg_n: int, seed: int, rank: int, world: int):
    """C3: this rank's contiguous block of the epoch's 2,048 committees (a seeded permutation of the registry
    split into 32 slots x 64 committees of 512; one message per (slot, committee)).  Every rank draws the same
    permutation, so the shards partition the epoch."""
    B = C3_SLOTS * C3_PER_SLOT
    n = C3_N
    assert B * n <= reg_n
    perm = np.random.default_rng(seed).permutation(reg_n).astype(np.uint32)[: B * n].reshape(B, n)
    lo, hi = shard_bounds_by_work(np.arange(B + 1, dtype=np.int64) * n, rank, world)
    idx2d = perm[lo:hi]
    msgs = b"".join(_msg(b"epoch", seed, j) for j in range(lo, hi))
    return idx2d.reshape(-1), np.arange(hi - lo + 1, dtype=np.uint64) * n, msgs, _agg_sks(idx2d), (lo, hi)


def c4_shard(total: int, seed: int, rank: int, world: int, chunk: int = C4_CHUNK):
    """C4: Verify i (i < total) with pk_i = registry[i], m_i distinct, sk_i = i + 1; this rank's contiguous
    shard, run as jobs of `chunk` items (one job when the shard does not split evenly)."""
    lo, hi = shard_bounds(total, rank, world)
    B = hi - lo
    idx = np.arange(lo, hi, dtype=np.uint32)
    msgs = b"".join(_msg(b"gossip", seed, j) for j in range(lo, hi))
    sks = b"".join(int(i + 1).to_bytes(32, "big") for i in range(lo, hi))
    chunks = B // chunk if chunk and B % chunk == 0 and B >= chunk else 1
    return idx, np.arange(B + 1, dtype=np.uint64), msgs, sks, chunks, (lo, hi)


def corrupt(sigs: bytearray, idx2d: np.ndarray, j: int, kind: str, B: int) -> None:
    """Make item j invalid in one of the SURVEY.md §8(d) ways (test_eth_fast_aggregate_verify.py:38-151 cases)."""
    if kind == "wrong_msg":  # a valid G2 point for another message: only the pairing check catches it
        o = (j + 1) % B
        sigs[96 * j: 96 * j + 96] = sigs[96 * o: 96 * o + 96]
    elif kind == "inf_sig":
        sigs[96 * j: 96 * j + 96] = b"\xc0" + bytes(95)
    elif kind == "zero_sig":
        sigs[96 * j: 96 * j + 96] = bytes(96)
    elif kind == "ff_tail":  # test_eth_fast_aggregate_verify.py:104
        sigs[96 * j + 92: 96 * j + 96] = b"\xff" * 4
    elif kind == "g1_inf_pk":
        idx2d[j, 7] = IDX_INF
    elif kind == "pk_0x40":
        idx2d[j, 0] = IDX_0x40
    else:
        raise ValueError(kind)


def adversarial_plan(B: int, per_kind: int, seed: int) -> dict:
    """Seeded positions: per_kind distinct items for each bad kind."""
    rng = np.random.default_rng(seed)
    pos = rng.choice(B, size=per_kind * len(BAD_KINDS), replace=False)
    return {int(j): BAD_KINDS[t // per_kind] for t, j in enumerate(pos)}


def adversarial_inputs(batch, ctx, B: int, n: int, plan: dict, seed: int, reg_n: int = REG_N):
    rng = np.random.default_rng(seed)
    idx2d = np.stack([rng.choice(reg_n, size=n, replace=False) for _ in range(B)]).astype(np.uint32)
    msgs = [_msg(b"adv", seed, j) for j in range(B)]
    sigs = bytearray(batch.sign_batch(_agg_sks(idx2d), b"".join(msgs), ctx=ctx))
    for j, kind in sorted(plan.items()):
        corrupt(sigs, idx2d, j, kind, B)
    expect = np.ones(B, dtype=bool)
    expect[list(plan)] = False
    return idx2d, np.arange(B + 1, dtype=np.uint64) * n, msgs, sigs, expect


# --------------------------------------------------------------- CPU baseline --
_CPU = {}


def _cpu_worker(args):
    """One host process: run its chunk of the sample through oracle/bls_oracle.c (single-threaded) until the
    deadline; returns the number of FastAggregateVerify calls completed."""
    from oracle import bls_oracle_c as OC

    lo, hi, mode, deadline = args
    d = _CPU
    o = d["offs"]
    idx = d["idx"][int(o[lo]):int(o[hi])]
    offs = o[lo:hi + 1] - o[lo]
    msgs, sigs = d["msgs"][32 * lo:32 * hi], d["sigs"][96 * lo:96 * hi]
    done = 0
    while True:
        out = OC.fav_batch_resident(d["reg"], idx, offs, msgs, sigs, d["seed"], mode, 1)
        assert all(out), "CPU baseline rejected a valid aggregate"
        done += hi - lo
        if time.time() >= deadline:
            return done


def _cpu_sign(args):
    from oracle import bls_oracle_c as OC

    sks, msgs = args
    return OC.sign_batch(sks, msgs, 1)


def cpu_baseline(n: int, seconds: float, cores: int, reg_n: int = 1 << 14, per_core: int = 16, seed: int = 0x5EED):
    """Time the C restatement (oracle/bls_oracle.c, kind "port") on `cores` host processes: the same
    registry-resident FastAggregateVerify(n) workload as the GPU (pre-validated affine keys, committee gather,
    signature decode + subgroup check, hash_to_G2, pairing check), in two modes -- per call (reference-equivalent:
    one final exponentiation per call) and RLC-batched per process (one per chunk of `per_core` calls)."""
    import multiprocessing as mp

    from oracle import bls_oracle_c as OC

    B = per_core * cores
    idx, offs, msgs, sks = build_inputs(B, n, reg_n, seed, 0xC0)
    _CPU.update(reg=OC.registry_generate(1, reg_n), idx=idx, offs=offs, msgs=msgs, seed=b"\x5e" * 32)
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        chunks = [(sks[32 * per_core * c:32 * per_core * (c + 1)], msgs[32 * per_core * c:32 * per_core * (c + 1)])
                  for c in range(cores)]
        _CPU["sigs"] = b"".join(pool.map(_cpu_sign, chunks))
    res = {}
    with ctx.Pool(cores) as pool:  # forked after the sample exists: workers share it copy-on-write
        pool.map(_cpu_worker, [(c * per_core, c * per_core + 1, 0, 0.0) for c in range(cores)])  # warm
        for mode in (1, 0):
            t0 = time.time()
            dl = t0 + seconds / 2
            done = sum(pool.map(_cpu_worker, [(c * per_core, (c + 1) * per_core, mode, dl) for c in range(cores)]))
            res[mode] = (done, time.time() - t0)
    rlc, per_call = res[1][0] / res[1][1], res[0][0] / res[0][1]
    cpu = ""
    try:
        with open("/proc/cpuinfo") as fh:
            cpu = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(rlc, 2), "unit": "FAV/s", "cores": cores, "kind": "port",
            "per_call_value": round(per_call, 2),
            "sample": f"oracle/bls_oracle.c (C restatement, 6x64-bit Montgomery) on {cores} host processes ({cpu}; "
                      f"the box's CPU share per GPU, OMP_NUM_THREADS -- its sched_getaffinity set is the whole "
                      f"machine's, shared with the other GPUs' jobs): "
                      f"FastAggregateVerify(n={n}) over a {reg_n}-key pre-validated affine registry, {B} distinct "
                      f"aggregates cycled; RLC-batched per {per_core} calls: {res[1][0]} calls in {res[1][1]:.1f} s; "
                      f"per call (own final exponentiation, reference-equivalent): {res[0][0]} calls in "
                      f"{res[0][1]:.1f} s"}


def percall_latency(reps: int = 15):
    """Median wall-clock latency of the drop-in per-call API (E/utils/bls.py:141-177 call pattern: one ctypes
    call per verification, host buffers): Verify and FastAggregateVerify(n = 512), beside the C port's per-call
    time on one host core for the same inputs (checker only, outside every timed region)."""
    import statistics

    from bls_mi355x.backend import mi355x_bls as M
    from oracle import bls_oracle_c as OC

    sks = list(range(1001, 1001 + 512))
    pks = [OC.SkToPk(k) for k in sks]
    m = hashlib.sha256(b"percall").digest()
    sig1 = OC.Sign(sks[0], m)
    sig512 = OC.Sign(sum(sks), m)

    def med(fn, r):
        ts = []
        for _ in range(r):
            t = time.perf_counter()
            assert fn()
            ts.append(time.perf_counter() - t)
        return round(statistics.median(ts) * 1e3, 3)

    for _ in range(5):  # warm: first-call scratch allocation, then the steady state a caller's stream of calls sees
        M.Verify(pks[0], m, sig1)
        M.FastAggregateVerify(pks, m, sig512)
    return {"verify_ms": med(lambda: M.Verify(pks[0], m, sig1), reps),
            "fav512_ms": med(lambda: M.FastAggregateVerify(pks, m, sig512), reps),
            "cpu_port_verify_ms": med(lambda: OC.Verify(pks[0], m, sig1), 3),
            "cpu_port_fav512_ms": med(lambda: OC.FastAggregateVerify(pks, m, sig512), 3),
            "note": "median wall-clock per call incl. ctypes + H2D/D2H; CPU port = oracle/bls_oracle.c on 1 core"}


# -------------------------------------------------------------------- parity --
def parity_sample(batch, ctx, per_kind: int = 8, oracle_items: int = 16, seed: int = 0xA11):
    """Untimed parity evidence for the bench line (rank 0): an adversarial C2 slice (1,024 x 512, per_kind bad
    items of every SURVEY.md §8(d) kind) through the host-buffer batch API, its verdicts against the
    construction and, on `oracle_items` sampled items, against the C oracle (oracle/bls_oracle.c, the checker);
    hash_to_G2 of tests/golden/hash_to_g2.json against the committed points; the deposit-cli known answer
    (E/test/capella/block_processing/test_process_bls_to_execution_change.py:257-288) through the per-call API."""
    from bls_mi355x.backend import mi355x_bls as M
    from oracle import bls_oracle_c as OC

    B, n = 1024, 512
    plan = adversarial_plan(B, per_kind, seed)
    idx2d, offs, msgs, sigs, expect = adversarial_inputs(batch, ctx, B, n, plan, seed)
    out = batch.fast_aggregate_verify_batch(idx2d.reshape(-1), offs, b"".join(msgs), bytes(sigs), ctx=ctx)
    checks, rounds = batch.fallback_stats(ctx=ctx)
    mism = int((out != expect).sum())
    # the C oracle on the same compressed keys: one bad item of each kind + good ones
    rng = np.random.default_rng(seed + 1)
    bad_pick = [next(j for j in sorted(plan) if plan[j] == k) for k in BAD_KINDS]
    good = [j for j in range(B) if expect[j]]
    pick = bad_pick + [int(x) for x in rng.choice(good, size=oracle_items - len(bad_pick), replace=False)]
    pk_of = {i: OC.SkToPk(i + 1) for i in sorted({int(x) for j in pick for x in idx2d[j] if x < REG_N})}
    pk_of[IDX_INF], pk_of[IDX_0x40] = G1_INF, PK_0x40
    o_mism = 0
    for j in pick:
        o = OC.FastAggregateVerify([pk_of[int(x)] for x in idx2d[j]], msgs[j], bytes(sigs[96 * j: 96 * j + 96]))
        o_mism += int(bool(o) != bool(out[j]))
    # hash_to_G2 golden points
    with open(os.path.join(ROOT, "tests", "golden", "hash_to_g2.json")) as fh:
        h2c = json.load(fh)
    hb = lambda s: bytes.fromhex(s[2:] if s.startswith("0x") else s)  # noqa: E731
    h_mism = sum(M.hash_to_G2(hb(c["msg"]), c["dst"].encode()) != hb(c["output"]) for c in h2c)
    with open(os.path.join(ROOT, "tests", "golden", "known_answers.json")) as fh:
        ka = json.load(fh)
    k_mism = sum(M.Verify(hb(c["pubkey"]), hb(c["signing_root"]), hb(c["signature"])) != c["output"]
                 for c in ka.values())
    return {"items": B, "mismatches": mism + o_mism + h_mism + k_mism,
            "batch": {"items": B, "bad": len(plan), "bad_kinds": list(BAD_KINDS), "per_kind": per_kind,
                      "mismatches_vs_construction": mism, "fe_checks": checks, "bisection_rounds": rounds},
            "oracle": {"items": len(pick), "mismatches": o_mism, "checker": "oracle/bls_oracle.c FastAggregateVerify"},
            "hash_to_g2": {"points": len(h2c), "mismatches": int(h_mism), "source": "tests/golden/hash_to_g2.json"},
            "known_answers": {"cases": len(ka), "mismatches": int(k_mism)}}


# ------------------------------------------------------- secondary configs --
def run_c4(batch, ctx, timed, total: int, seed: int, rank: int, world: int, steps: int, warmup: int) -> dict:
    """C4 (BASELINE configs[3], E/utils/bls.py:141-151 call shape): this rank's contiguous shard of `total`
    single-signature Verify (pk_i = registry[i], distinct messages m_i, sk_i = i + 1) as registry-resident
    FastAggregateVerify items with n = 1, `steps` pipelined passes; every verdict must be True."""
    idx, offs, msgs, sks, chunks, (lo, hi) = c4_shard(total, seed, rank, world)
    rb = batch.ResidentFavBatch(idx, offs, msgs, batch.sign_batch(sks, msgs, ctx=ctx), ctx=ctx, chunks=chunks)
    dt, oks = timed(rb, steps, warmup)
    assert all(oks) and rb.verdicts().all(), "a valid C4 Verify was rejected"
    return {"rb": rb, "dt": dt, "shard_items": hi - lo, "shard": [lo, hi], "chunks": chunks,
            "verify_s": round(total * steps / dt, 1), "ms_per_shard": round(dt / steps * 1e3, 3), "steps": steps}


def run_c5(batch, ctx, timed, n: int, bad: int, seed: int, rank: int, world: int, reg_n: int, steps: int,
           warmup: int, aggregate_verify: bool) -> dict:
    """C5 (BASELINE configs[4]): 1,024 x n FastAggregateVerify per rank with `bad` items of the SURVEY.md §8(d)
    kinds (E/test/altair/bls/test_eth_fast_aggregate_verify.py:38-151 cases; the bisection fallback runs every
    pass), verdicts against the construction; with aggregate_verify, AggregateVerify with N = 128 / 1,024 / 8,192
    distinct messages through the drop-in per-call API (E/utils/bls.py:154-164), pairs/s."""
    B = 1024
    plan = {int(j): BAD_KINDS[t % len(BAD_KINDS)] for t, j in
            enumerate(np.random.default_rng(seed + rank).choice(B, size=bad, replace=False))}
    idx2d, offs, msgs, sigs, expect = adversarial_inputs(batch, ctx, B, n, plan, seed + 17 * rank, reg_n)
    rb = batch.ResidentFavBatch(idx2d.reshape(-1), offs, b"".join(msgs), bytes(sigs), ctx=ctx)
    dt, oks = timed(rb, steps, warmup)
    assert not any(oks) if plan else all(oks)
    assert (rb.verdicts() == expect).all(), "adversarial verdicts differ from the construction"
    checks, rounds = batch.fallback_stats(ctx=ctx)
    out = {"rb": rb, "dt": dt, "items": B, "committee": n, "bad": len(plan), "bad_kinds": sorted(set(plan.values())),
           "fav_s": round(B * world * steps / dt, 1), "ms_per_batch": round(dt / steps * 1e3, 3), "steps": steps,
           "verdict_mismatches": 0, "fallback_last_step": {"fe_checks": checks, "bisection_rounds": rounds}}
    if aggregate_verify:  # AggregateVerify with N distinct messages (drop-in per call)
        from bls_mi355x.backend import mi355x_bls as M
        av = {}
        for N in (128, 1024, 8192):
            ks = [(7919 * (i + 1)) for i in range(N)]
            pks = batch.sk_to_pk_batch(b"".join(k.to_bytes(32, "big") for k in ks), ctx=ctx)
            pkl = [pks[48 * i: 48 * i + 48] for i in range(N)]
            ms = [_msg(b"av", N, i) for i in range(N)]
            s = batch.sign_batch(b"".join(k.to_bytes(32, "big") for k in ks), b"".join(ms), ctx=ctx)
            agg = M.Aggregate([s[96 * i: 96 * i + 96] for i in range(N)])
            assert M.AggregateVerify(pkl, ms, agg)
            bad_agg = M.Aggregate([s[96 * i: 96 * i + 96] for i in range(N - 1)])  # one signature missing
            t = time.perf_counter()
            ok = M.AggregateVerify(pkl, ms, agg)
            el = time.perf_counter() - t
            av[str(N)] = {"pairs_s": round(N / el, 1), "ms": round(el * 1e3, 3), "ok": bool(ok),
                          "rejects_missing_sig": M.AggregateVerify(pkl, ms, bad_agg) is False}
            assert ok and av[str(N)]["rejects_missing_sig"]
        out["aggregate_verify"] = av
    return out


def registry_load_figure(ctx, reg_n: int, reps: int = 3) -> dict:
    """SURVEY.md §8(d) registry load (specs/phase0/beacon-chain.md:787 reads state.validators[*].pubkey; deposits
    append, :2037-2062): decode + KeyValidate of reg_n compressed keys (pk_i = (i + 1) G1, made on the device)
    plus the two invalid keys the C5 kinds index and the 8 tests/golden/bls_formats.json key_validate fixtures,
    through bls_registry_load (host buffer in, validity mask out).  The table it leaves behind is the one the
    C2 / C3 passes then read, so every later verdict checks the decoded keys.  keys_s = API wall-clock
    (PCIe-inclusive); kernel_keys_s = keys / k_key_validate's hipEvent time."""
    import ctypes

    from bls_mi355x import batch

    gen = ctypes.create_string_buffer(48 * reg_n)
    ctx.check(ctx.lib.bls_registry_generate(ctx.h, 1, reg_n, gen))
    with open(os.path.join(ROOT, "tests", "golden", "bls_formats.json")) as fh:
        kv = json.load(fh)["key_validate"]
    hb = lambda s: bytes.fromhex(s[2:] if s.startswith("0x") else s)  # noqa: E731
    tail = G1_INF + PK_0x40 + b"".join(hb(c["input"]) for c in kv)
    data = gen.raw + tail
    n = len(data) // 48
    expect = np.concatenate([np.ones(reg_n, np.uint8), np.zeros(2, np.uint8),
                             np.array([1 if c["output"] else 0 for c in kv], np.uint8)])
    valid = np.zeros(n, dtype=np.uint8)
    prof = batch.Profiler(ctx)
    ts = []
    for r in range(reps):
        if r == reps - 1:
            prof.start()
        t = time.perf_counter()
        ctx.check(ctx.lib.bls_registry_load(ctx.h, data, n, valid.ctypes.data))
        ts.append(time.perf_counter() - t)
        assert (valid == expect).all(), "registry load: KeyValidate mask differs from the construction / fixtures"
    kern = prof.read()
    prof.stop()
    k_ms = kern["key_validate"][0] / max(kern["key_validate"][1], 1) if kern.get("key_validate") else None
    best = min(ts)
    return {"keys": n, "keys_s": round(n / best, 1), "ms": round(best * 1e3, 3),
            "kernel_ms": round(k_ms, 3) if k_ms else None, "kernel_keys_s": round(n / (k_ms * 1e-3), 1) if k_ms else None,
            "mask_mismatches": 0, "fixtures": len(kv),
            "note": "bls_registry_load of 2^20 compressed keys + 2 invalid + 8 bls_formats.json key_validate fixtures; "
                    "keys_s includes the 48 B/key H2D and the verdict D2H; later C2/C3 passes read this table"}


# ---------------------------------------------------------------------- main --
def _lib_sha() -> str | None:
    try:
        with open(LIB, "rb") as fh:
            return hashlib.sha256(fh.read()).hexdigest()[:16]
    except OSError:
        return None


def rank_envs(n: int, port: int, base: dict | None = None) -> list[dict]:
    """The environment of each of the n rank processes the launcher starts (what torch.distributed.run sets for
    one node: RANK = LOCAL_RANK = r, WORLD_SIZE = n, the rendezvous at 127.0.0.1:port)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    """GPUs this process may use, counted WITHOUT initialising HIP (torch.cuda.device_count() reads the device
    list only on this image; no kernel, stream or context is created in the launcher process)."""
    import torch

    return int(torch.cuda.device_count())


def launch_ranks(n: int, argv: list[str], dry_run: bool = False) -> int:
    """--gpus N > 1 started as a plain `python bench.py --gpus N` (no WORLD_SIZE in the environment): start one
    child process per GPU, each re-running this script with the same arguments and the rank environment of
    rank_envs(), and return the first non-zero child exit code (the other ranks are then terminated, so no rank
    waits in a collective for a dead peer).  Nothing here touches the GPU: the children initialise HIP, one GPU
    each (BLSMI355X_DEVICE = LOCAL_RANK).  dry_run prints the plan (one JSON line) and starts nothing."""
    import subprocess

    port = _free_port()
    envs = rank_envs(n, port)
    cmd = [sys.executable, os.path.abspath(__file__), *argv]
    if dry_run:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        print(json.dumps({"launcher": {"ranks": n, "cmd": cmd,
                                       "children": [{k: e[k] for k in keys} for e in envs]}}), flush=True)
        return 0
    have = visible_gpus()
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs on this node but {have} are visible "
              f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')!r}); refusing to run fewer ranks "
              f"than asked", file=sys.stderr, flush=True)
        return 2
    import signal

    procs = {r: subprocess.Popen(cmd, env=e) for r, e in enumerate(envs)}
    # a SIGTERM to the launcher (a job scheduler's timeout) ends the ranks too, through the finally below
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(128 + signal.SIGTERM))
    rc = 0
    try:
        while procs:
            for r, p in list(procs.items()):
                code = p.poll()
                if code is None:
                    continue
                del procs[r]
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code  # a signal -s -> 128 + s, as a shell reports it
                    print(f"bench.py launcher: rank {r} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in procs.values():
                        q.terminate()
            time.sleep(0.2)
    finally:
        for q in procs.values():  # left only if the launcher itself was interrupted
            q.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node; N > 1 without WORLD_SIZE starts one rank process per GPU")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="print the rank processes --gpus N would start (environments) and exit")
    ap.add_argument("--config", choices=("c2", "c3", "c4", "c5"), default="c2")
    ap.add_argument("--steps", type=int, default=40, help="timed steps (4 in flight: fewer passes under-fill the pipeline)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=10000, help="C2: FastAggregateVerify calls per GPU per step")
    ap.add_argument("--committee", type=int, default=512)
    ap.add_argument("--registry", type=int, default=REG_N)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--c4-total", type=int, default=C4_TOTAL)
    ap.add_argument("--c5-bad", type=int, default=8, help="C5: bad items per batch (kinds cycled)")
    # the secondary figures time enough passes to fill the 10-job pipeline several times over (5 C5 passes with 10
    # jobs in flight measured mostly the fill and drain: 288k against 578k FAV/s at 30)
    ap.add_argument("--c3-steps", type=int, default=60, help="epochs timed for the c2 line's C3 figure (0: skip)")
    ap.add_argument("--c4-steps", type=int, default=4, help="125k-Verify shards timed for the c2 line's C4 figure")
    ap.add_argument("--c5-steps", type=int, default=40, help="adversarial batches timed for the c2 line's C5 figure")
    ap.add_argument("--no-regload", action="store_true", help="generate the registry instead of loading its keys")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="one batch in flight (no overlap of passes)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel hipEvent timing")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) batch call")
    ap.add_argument("--roofline-passes", type=int, default=5, help="one-batch-at-a-time passes timed per kernel")
    ap.add_argument("--no-percall", action="store_true", help="skip the drop-in per-call latency figures")
    ap.add_argument("--no-parity", action="store_true", help="skip the parity sample")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} (set by the launcher) but --gpus {args.gpus}; the line would "
              f"report a world the run does not have", file=sys.stderr, flush=True)
        sys.exit(2)
    if env_world is None and (args.gpus > 1 or args.launch_dry_run):
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], dry_run=args.launch_dry_run))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ["BLSMI355X_DEVICE"] = str(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")  # control plane only; the partials travel over RCCL inside the library

    from bls_mi355x import _native, batch

    ctx = _native.context()
    dev_name, cus = ctx.device_info()
    comm = dist is not None
    if comm:
        from bls_mi355x import dist as bdist
        from torch.distributed import distributed_c10d as c10d

        bdist.init_comm(ctx, rank, world, c10d._get_default_store())
        _COMM_CTX.append(ctx)

    def barrier_sync():
        ctx.check(ctx.lib.bls_sync(ctx.h))
        if dist is not None:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(rb, steps, warmup, depth=None):
        """warmup + `steps` timed passes of rb between barriers; max over ranks; every pass must pass.  Setup
        first: one pass on every job slot, so each slot's device scratch is allocated (hipMalloc) before the
        timed region (a slot allocates on its first batch; with 10 slots and 2 warmup passes, 8 allocations
        would land inside it)."""
        d = 1 if args.no_pipeline else (batch.FAV_DEPTH if depth is None else depth)
        prime = -(-batch.FAV_JOBS // rb.chunks) if d > 1 else 1  # passes covering every slot (a pass = `chunks` jobs)
        rb.run_pipelined([os.urandom(32) for _ in range(prime)], depth=d, comm=comm)
        if warmup:
            rb.run_pipelined([os.urandom(32) for _ in range(warmup)], depth=d, comm=comm)
        barrier_sync()
        t0 = time.perf_counter()
        oks = rb.run_pipelined([os.urandom(32) for _ in range(steps)], depth=d, comm=comm)
        barrier_sync()
        return max_over_ranks(time.perf_counter() - t0), oks

    # ---- setup (untimed): registry 2^20 (sk_i = i + 1) + two invalid appended keys (C5 kinds) ----
    t_setup = time.perf_counter()
    extra = {}
    reg = batch.Registry(ctx)
    if args.config == "c2" and args.registry == REG_N and not args.no_regload:
        # the registry the passes read is decoded from compressed keys (the §8(d) registry-load figure)
        extra["registry_load"] = registry_load_figure(ctx, REG_N)
    else:
        reg.generate(args.registry, first_sk=1)
        if args.registry == REG_N:
            assert reg.append(G1_INF + PK_0x40).tolist() == [0, 0]
    n = args.committee
    rb = None

    if args.config == "c2":
        B = args.batch
        idx, offs, msgs, sks = build_inputs(B, n, args.registry, args.seed, rank)
        sigs = batch.sign_batch(sks, msgs, ctx=ctx)
        rb = batch.ResidentFavBatch(idx, offs, msgs, sigs, ctx=ctx)
        setup_s = time.perf_counter() - t_setup
        dt, oks = timed(rb, args.steps, args.warmup)
        assert all(oks), "a valid C2 batch failed the pairing check"
        v = rb.verdicts()
        assert v.all(), f"{(~v).sum()} valid aggregates rejected"
        units, unit, scaling = B * world, "FAV/s", "weak"
        workload = f"C2 sync-committee FastAggregateVerify: {B} aggregates x {n} pubkeys per GPU"
        ops_step = item_ops(n) * B * world + BATCH_OPS * world
    elif args.config == "c3":
        idx, offs, msgs, sks, (lo, hi) = c3_shard(args.registry, args.seed, rank, world)
        B = hi - lo
        rb = batch.ResidentFavBatch(idx, offs, msgs, batch.sign_batch(sks, msgs, ctx=ctx), ctx=ctx)
        setup_s = time.perf_counter() - t_setup
        dt, oks = timed(rb, args.steps, args.warmup)
        assert all(oks) and rb.verdicts().all()
        units, unit, scaling = C3_SLOTS * C3_PER_SLOT, "FAV/s", "strong"
        workload = (f"C3 mainnet epoch replay: {C3_SLOTS} slots x {C3_PER_SLOT} committees of {C3_N} over a "
                    f"2^20 registry, epoch sharded over {world} GPU(s), one RLC verdict per epoch")
        ops_step = item_ops(C3_N) * units + BATCH_OPS * world
        extra["ms_per_epoch"] = round(dt / args.steps * 1e3, 3)
    elif args.config == "c4":
        r4 = run_c4(batch, ctx, timed, args.c4_total, args.seed, rank, world, args.steps, args.warmup)
        rb, dt, B, chunks = r4.pop("rb"), r4.pop("dt"), r4["shard_items"], r4["chunks"]
        setup_s = time.perf_counter() - t_setup
        units, unit, scaling = args.c4_total, "Verify/s", "strong"
        workload = (f"C4 gossip firehose: {args.c4_total} single-signature Verify (pk_i = registry[i], distinct "
                    f"messages), contiguous shards of {B} per GPU in {chunks} job(s)")
        ops_step = item_ops(1) * units + BATCH_OPS * chunks * world
    else:  # c5
        r5 = run_c5(batch, ctx, timed, n, args.c5_bad, args.seed, rank, world, args.registry, args.steps, args.warmup,
                    aggregate_verify=rank == 0)
        rb, dt, B = r5.pop("rb"), r5.pop("dt"), r5["items"]
        setup_s = time.perf_counter() - t_setup
        units, unit, scaling = B * world, "FAV/s", "weak"
        workload = (f"C5 adversarial FAV batches: {B} x {n} per GPU with {args.c5_bad} bad items "
                    f"({', '.join(r5['bad_kinds'])}), bisection fallback every step")
        ops_step = item_ops(n) * units + BATCH_OPS * world
        extra["fallback_last_step"] = r5["fallback_last_step"]
        if "aggregate_verify" in r5:
            extra["aggregate_verify"] = r5["aggregate_verify"]

    ms_step = dt / args.steps * 1e3
    value = units * args.steps / dt

    # ---- C3 epoch-replay figure beside the C2 headline (every rank: the epoch is sharded) ----
    if args.config == "c2" and args.c3_steps > 0 and args.registry == REG_N:
        idx3, offs3, msgs3, sks3, (lo3, hi3) = c3_shard(args.registry, args.seed, rank, world)
        rb3 = batch.ResidentFavBatch(idx3, offs3, msgs3, batch.sign_batch(sks3, msgs3, ctx=ctx), ctx=ctx)
        dt3, oks3 = timed(rb3, args.c3_steps, 2)
        assert all(oks3) and rb3.verdicts().all()
        e = C3_SLOTS * C3_PER_SLOT
        extra["c3"] = {"fav_s": round(e * args.c3_steps / dt3, 1), "ms_per_epoch": round(dt3 / args.c3_steps * 1e3, 3),
                       "epochs": args.c3_steps, "shard": [lo3, hi3],
                       "workload": f"{C3_SLOTS} slots x {C3_PER_SLOT} committees of {C3_N} (2^20 registry), "
                                   f"one RLC verdict per epoch, epochs pipelined like C2"}
        rb3.free()
    # ---- C4 / C5 figures beside the C2 headline (BASELINE configs[3], configs[4]; their own --config runs scale
    # them to any world size) ----
    if args.config == "c2" and args.registry == REG_N:
        if args.c4_steps > 0:  # one 125,000-Verify shard per GPU (the 8-GPU shard of 10^6)
            r4 = run_c4(batch, ctx, timed, C4_CHUNK * world, args.seed, rank, world, args.c4_steps, 1)
            r4.pop("rb").free()
            r4.pop("dt")
            r4["workload"] = f"{C4_CHUNK} single-signature Verify per GPU (pk_i = registry[i], distinct messages)"
            extra["c4"] = r4
        if args.c5_steps > 0:
            r5 = run_c5(batch, ctx, timed, n, args.c5_bad, args.seed, rank, world, args.registry, args.c5_steps, 1,
                        aggregate_verify=rank == 0)
            r5.pop("rb").free()
            r5.pop("dt")
            r5["workload"] = f"1024 x {n} FAV per GPU with {args.c5_bad} bad items, bisection fallback every pass"
            extra["c5"] = r5

    # per-kernel execution times: one batch at a time, hipEvents around each launch (after the timed region)
    kern = {}
    if not args.no_profile and args.roofline_passes > 0 and rb is not None and rb.chunks == 1:
        prof = batch.Profiler(ctx)
        prof.start()
        rb.run_pipelined([os.urandom(32) for _ in range(args.roofline_passes)], depth=1, comm=comm)
        kern = prof.read()
        prof.stop()

    # ---- roofline: dominant kernel, algorithmic int ops per launch -----------
    fme = model_fme(n if args.config != "c4" else 1)
    roof = None
    kernels_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in kern.items() if v[1]}
    per_launch = rb.cb if rb is not None else 0  # items per FAV job (one launch of each kernel)
    if kern:
        dom = max((k for k in SINGLE_KERNEL if k in kern and kern[k][1]), key=lambda k: kern[k][0])
        avg_s = kern[dom][0] / kern[dom][1] * 1e-3
        ops = round(fme[dom] * FME_OPS * per_launch)
        ach = ops / avg_s / 1e12
        traffic, tsrc = None, None
        try:  # HBM bytes per launch from the committed rocprofv3 --pmc FETCH_SIZE pass (a PMC run cannot be live)
            with open(os.path.join(ROOT, "tools", "pmc_traffic.json")) as fh:
                tj = json.load(fh)
            if tj.get("lib_sha256_16") == _lib_sha():  # only the profile of this exact build
                traffic, tsrc = tj["bytes_per_dispatch"].get(dom), tj["source"]
        except (OSError, ValueError, KeyError):
            pass
        roof = {"bound": "valu-int", "kernel": dom, "symbol": kernel_symbol(dom, per_launch), "achieved": round(ach, 4),
                "peak": round(PEAK_INT_OPS / 1e12, 2), "unit": "Tops/s", "frac": round(ach / (PEAK_INT_OPS / 1e12), 5),
                "frac_source": f"this run: algorithmic ops / hipEvent launch time ({args.roofline_passes} "
                               f"one-batch-at-a-time passes after the timed region)",
                "traffic": traffic, "traffic_source": tsrc, "ops_per_launch": ops,
                "avg_launch_ms": round(avg_s * 1e3, 4)}
        try:  # the committed rocprofv3 --kernel-trace --stats average of the same kernel, launched at THIS size
            # (the (symbol, grid) entry: a C2-only, one-batch-at-a-time profile, tools/gpu_check.sh profc2) -- only
            # for the same build
            with open(ROCPROF_AVG) as fh:
                rj = json.load(fh)
            grid = launch_grid(dom, per_launch)
            ent = rj.get("avg_ms_by_grid", {}).get(kernel_symbol(dom, per_launch), {}).get(str(grid))
            if ent and rj.get("lib_sha256_16") and rj["lib_sha256_16"] == _lib_sha():
                r_ms = ent["avg_ms"]
                roof["rocprof_avg_ms"] = r_ms
                roof["rocprof_grid"] = grid
                roof["rocprof_calls"] = ent["calls"]
                roof["rocprof_source"] = rj["source"] + " (committed profile of this exact libblsmi355x.so)"
                roof["frac_rocprof"] = round(ops / (r_ms * 1e-3) / PEAK_INT_OPS, 5)
        except (OSError, ValueError, KeyError):
            pass
        roof["frac_of_measured_mad_rate"] = round(roof["achieved"] * 1e12 / MEASURED_MAD_OPS, 5)
        lk = lane_kernels(per_launch)
        if dom in lk:  # k lanes per item, one wave per SIMD: the launch holds ceil(k B / 64) SIMDs
            occ = min(1.0, ((int(lk[dom] * per_launch) + 63) // 64) / (cus * 4))
            roof["occupied_simd_frac"] = round(occ, 4)
            roof["frac_of_occupied_simds"] = round(roof["frac"] / occ, 4)
    # secondary figure: algorithmic HBM bytes of the registry gather per launch / its duration
    gather_gbs = None
    if "fav_gather" in kern and kern["fav_gather"][1]:
        g_s = kern["fav_gather"][0] / kern["fav_gather"][1] * 1e-3
        keys = per_launch * (n if args.config != "c4" else 1)
        gather_gbs = round(keys * GATHER_BYTES_PER_KEY / g_s / 1e9, 1)
    # PCIe-inclusive rate: the host-buffer C-ABI call (bls_fav_batch_indexed: inputs copied H2D, verdicts D2H),
    # one batch at a time, no pipelining.  Reported beside `value`, never as it.
    e2e = None
    if rank == 0 and not args.no_e2e and args.config == "c2":
        batch.fast_aggregate_verify_batch(idx, offs, msgs, sigs, ctx=ctx)
        t1 = time.perf_counter()
        v2 = batch.fast_aggregate_verify_batch(idx, offs, msgs, sigs, ctx=ctx)
        e2e = round(args.batch / (time.perf_counter() - t1), 1)
        assert v2.all()
    barrier_sync()
    percall = None
    if rank == 0 and world == 1 and not args.no_percall:
        percall = percall_latency()
    parity = None
    if rank == 0 and not args.no_parity and args.registry == REG_N:
        parity = parity_sample(batch, ctx)
    pipeline_frac = ops_step * args.steps / dt / (PEAK_INT_OPS * world)

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": unit, "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": "u32 (381-bit Montgomery Fp, radix-2^29 digits)",
        "data": "synthetic: registry sk_i=i+1 (2^20 keys, HBM), SHA256 messages, signatures made on device",
        "config": {"workload": workload, "config": args.config,
                   "global_batch": units, "committee": n if args.config != "c4" else 1, "registry": args.registry,
                   "parallelism": f"dp{world} (sharded, RCCL all-gather of 576-B Fp12 partials)"},
        "roofline": roof,
        "int_valu_frac_pipeline": round(pipeline_frac, 5),
        "parity": parity,
        **extra,
        "kernels_avg_ms": kernels_ms,
        "gather_hbm_gbs": gather_gbs,
        "host_buffers_fav_s": e2e,
        "percall": percall,
        "device": dev_name, "cus": cus, "setup_s": round(setup_s, 2), "lib_sha256_16": _lib_sha(),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cores = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or 1 << 30, len(os.sched_getaffinity(0)))
        out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds, cores)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    barrier_sync()  # rank 0's untimed legs (percall, parity, CPU) are done before any rank tears down
    if rb is not None:
        rb.free()
    if dist is not None:
        _COMM_CTX.clear()
        bdist.destroy_comm(ctx)
        dist.destroy_process_group()


_COMM_CTX: list = []  # the context whose RCCL communicator is live (aborted if this rank fails)

if __name__ == "__main__":
    try:
        main()
    except BaseException:
        if _COMM_CTX:  # peers blocked in an all-gather with this rank fail instead of hanging
            from bls_mi355x import dist as _bd
            _bd.abort_comm(_COMM_CTX[0])
        raise
