#!/usr/bin/env python3
"""bench.py -- FastAggregateVerify throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): sync-committee
FastAggregateVerify, 10,000 aggregates x 512 pubkeys per GPU, pubkeys named
by index into a 2^20-key registry resident in HBM (sk_i = i + 1), distinct
32-byte messages SHA256(seed||rank||j), valid aggregate signatures made on
the device.  One step = one pass of the hot path over the batch: registry
gather + aggregate pubkeys, signature decode/subgroup checks, hash_to_G2,
random-linear-combination Miller loops, one shared final exponentiation
(per-item fallback only on failure), verdicts written to HBM.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N): weak scaling, each rank owns its own batch; the ranks' 576-byte
Fp12 Miller partials are all-gathered by the library over RCCL
(bls_fav_job_check_comm: ncclAllGather on the device, xGMI) and every rank
final-exponentiates the product.  torch.distributed (gloo) is only the
control plane: rendezvous, the RCCL unique id, barriers, max over ranks.

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
if not os.environ.get("BLSMI355X_KEEP_HW_QUEUES") and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 20:
    os.environ["GPU_MAX_HW_QUEUES"] = "20"

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
# lanes per item of the lane kernels (full register file, one wave per SIMD): k_miller_acc4<2> four lanes per two
# pairs (bls_miller_pair.hip), k_miller_lines2 two per pair (bls_miller_lane.hip), k_sig_lane2 one for the G1
# chain and two for the G2 chain of an item (bls_chain_lane.hip)
LANE_KERNELS = {"miller": 2, "miller_lines": 2, "sig_vm": 3}
GATHER_BYTES_PER_KEY = 4 + 96  # u32 index + one 96-B registry record (affine x, y; validity in x's top bit)
# profile entry -> kernel symbol in the rocprofv3 summaries (profiles/*kernel_stats*.md)
KERNEL_SYMBOL = {"miller": "k_miller_acc4<2>", "miller_lines": "k_miller_lines2", "fav_gather": "k_fav_gather_q<16>"}
ROCPROF_AVG = os.path.join(ROOT, "profiles", "rocprof_kernel_avg.json")


def model_fme(n: int):
    """Per-item algorithmic work of FAV(n) with a resident registry."""
    return {
        "fav_gather": 11 * (n - 1),
        "sig_decode": 1200,             # signature decompression (Fp2 square root)
        "sig_vm": 1200 + 1000 + 400,    # G2 subgroup check, RLC G1, RLC G2 (MSM share)
        "fav_hash": 6600,
        # Miller loop, 4400 FME per pair, split between its two kernels in proportion to the products each
        # executes per pair: k_miller_acc4<2> (f shared by two pairs: 62 Fp12 squarings x 36 / 2 + 68 sparse
        # line products x 43 = 4040) and k_miller_lines2 (T: 63 doublings x 26 + 5 additions x 35 = 1813)
        "miller": 4400 * 4040 / 5853,
        "miller_lines": 4400 * 1813 / 5853,
    }


def build_inputs(B: int, n: int, reg_n: int, seed: int, rank: int):
    """Committees, messages and aggregate secret keys (host, numpy)."""
    rng = np.random.default_rng(seed * 1000003 + rank)
    total = B * n
    perms = []
    while sum(p.size for p in perms) < total:
        perms.append(rng.permutation(reg_n).astype(np.uint32))
    idx = np.concatenate(perms)[:total] if len(perms) > 1 else perms[0][:total]
    assert reg_n % n == 0  # committees never straddle two permutations: indices distinct per committee
    offs = np.arange(B + 1, dtype=np.uint64) * n
    agg = (idx.reshape(B, n).astype(np.int64) + 1).sum(axis=1)  # < r, fits int64
    sks = b"".join(int(a).to_bytes(32, "big") for a in agg)
    msgs = b"".join(hashlib.sha256(b"bench" + seed.to_bytes(8, "little") + rank.to_bytes(4, "little")
                                   + j.to_bytes(8, "little")).digest() for j in range(B))
    return idx, offs, msgs, sks


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
            "sample": f"oracle/bls_oracle.c (C restatement, 6x64-bit Montgomery) on {cores} host processes ({cpu}): "
                      f"FastAggregateVerify(n={n}) over a {reg_n}-key pre-validated affine registry, {B} distinct "
                      f"aggregates cycled; RLC-batched per {per_core} calls: {res[1][0]} calls in {res[1][1]:.1f} s; "
                      f"per call (own final exponentiation, reference-equivalent): {res[0][0]} calls in "
                      f"{res[0][1]:.1f} s"}


def percall_latency(reps: int = 15):
    """Median wall-clock latency of the drop-in per-call API (E/utils/bls.py:141-177 call pattern: one ctypes
    call per verification, host buffers): Verify and FastAggregateVerify(n = 512), beside the C port's per-call
    time on one host core for the same inputs."""
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

    M.Verify(pks[0], m, sig1)  # warm (first-call scratch allocation)
    M.FastAggregateVerify(pks, m, sig512)
    return {"verify_ms": med(lambda: M.Verify(pks[0], m, sig1), reps),
            "fav512_ms": med(lambda: M.FastAggregateVerify(pks, m, sig512), reps),
            "cpu_port_verify_ms": med(lambda: OC.Verify(pks[0], m, sig1), 3),
            "cpu_port_fav512_ms": med(lambda: OC.FastAggregateVerify(pks, m, sig512), 3),
            "note": "median wall-clock per call incl. ctypes + H2D/D2H; CPU port = oracle/bls_oracle.c on 1 core"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40, help="timed passes (4 in flight: fewer passes under-fill the pipeline)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=10000, help="FastAggregateVerify calls per GPU per step")
    ap.add_argument("--committee", type=int, default=512)
    ap.add_argument("--registry", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="one batch in flight (no overlap of passes)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-kernel hipEvent timing")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) batch call")
    ap.add_argument("--roofline-passes", type=int, default=5, help="one-batch-at-a-time passes timed per kernel")
    ap.add_argument("--no-percall", action="store_true", help="skip the drop-in per-call latency figures")
    args = ap.parse_args()

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
    if dist is not None:
        from bls_mi355x import dist as bdist
        from torch.distributed import distributed_c10d as c10d

        bdist.init_comm(ctx, rank, world, c10d._get_default_store())

    def barrier_sync():
        ctx.check(ctx.lib.bls_sync(ctx.h))
        if dist is not None:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()
            dist.barrier()

    # ---- setup (untimed) ----------------------------------------------------
    t_setup = time.perf_counter()
    reg = batch.Registry(ctx)
    reg.generate(args.registry, first_sk=1)
    idx, offs, msgs, sks = build_inputs(args.batch, args.committee, args.registry, args.seed, rank)
    sigs = batch.sign_batch(sks, msgs, ctx=ctx)
    rb = batch.ResidentFavBatch(idx, offs, msgs, sigs, ctx=ctx)
    setup_s = time.perf_counter() - t_setup

    def passes(k: int, depth: int | None = None) -> list:
        """k passes over the batch; by default pass j+1.. are submitted before pass j is final-exponentiated
        (up to FAV_DEPTH batches in flight, bls_fav_job_*), so every pass completes inside the call."""
        if args.no_pipeline:
            depth = 1
        d = batch.FAV_DEPTH if depth is None else depth
        return rb.run_pipelined([os.urandom(32) for _ in range(k)], depth=d, comm=dist is not None)

    if args.warmup:
        assert all(passes(args.warmup)), "warmup batch failed the pairing check"
    v = rb.verdicts()
    assert v.all(), f"{(~v).sum()} valid aggregates rejected"

    barrier_sync()
    t0 = time.perf_counter()
    oks = passes(args.steps)
    barrier_sync()
    dt = time.perf_counter() - t0
    assert all(oks)
    if dist is not None:
        import torch

        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # per-kernel execution times: one batch at a time, hipEvents around each launch (after the timed region)
    kern = {}
    if not args.no_profile and args.roofline_passes > 0:
        prof = batch.Profiler(ctx)
        prof.start()
        assert all(passes(args.roofline_passes, depth=1))
        kern = prof.read()
        prof.stop()
    B, n = args.batch, args.committee
    ms_step = dt / args.steps * 1e3
    value = B * world * args.steps / dt

    # ---- roofline: dominant kernel, algorithmic int ops per launch -----------
    fme = model_fme(n)
    roof = None
    kernels_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in kern.items() if v[1]}
    if kern:
        # candidates: the profile entries that time exactly one kernel (k_miller_lane, k_fav_gather<16>), so the
        # rocprofv3 summary's average for that kernel can be set beside this hipEvent figure
        dom = max((k for k in SINGLE_KERNEL if k in kern and kern[k][1]), key=lambda k: kern[k][0])
        avg_s = kern[dom][0] / kern[dom][1] * 1e-3
        units = B
        ops = round(fme[dom] * FME_OPS * units) + (19 * SHA_OPS * B if dom == "fav_hash" else 0)
        ach = ops / avg_s / 1e12
        traffic, tsrc = None, None
        try:  # HBM bytes per launch from the committed rocprofv3 --pmc FETCH_SIZE pass (a PMC run cannot be live)
            with open(os.path.join(ROOT, "tools", "pmc_traffic.json")) as fh:
                tj = json.load(fh)
            traffic, tsrc = tj["bytes_per_dispatch"].get(dom), tj["source"]
        except (OSError, ValueError, KeyError):
            pass
        roof = {"bound": "valu-int", "kernel": dom, "symbol": KERNEL_SYMBOL.get(dom), "achieved": round(ach, 4),
                "peak": round(PEAK_INT_OPS / 1e12, 2), "unit": "Tops/s", "frac": round(ach / (PEAK_INT_OPS / 1e12), 5),
                "traffic": traffic, "traffic_source": tsrc, "ops_per_launch": ops,
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "avg_source": f"hipEvents around each launch, {args.roofline_passes} one-batch-at-a-time passes"}
        try:  # the committed rocprofv3 --kernel-trace --stats average of the same kernel (same build)
            with open(ROCPROF_AVG) as fh:
                rj = json.load(fh)
            r_ms = rj["avg_ms"].get(KERNEL_SYMBOL.get(dom))
            if r_ms:
                roof["rocprof_avg_ms"] = r_ms
                roof["rocprof_source"] = rj["source"]
                roof["frac_rocprof"] = round(ops / (r_ms * 1e-3) / PEAK_INT_OPS, 5)
        except (OSError, ValueError, KeyError):
            pass
    if roof is not None:
        roof["frac_of_measured_mad_rate"] = round(roof["achieved"] * 1e12 / MEASURED_MAD_OPS, 5)
        if dom in LANE_KERNELS:  # k lanes per item, one wave per SIMD: the launch holds ceil(k B / 64) SIMDs
            occ = min(1.0, ((LANE_KERNELS[dom] * B + 63) // 64) / (cus * 4))
            roof["occupied_simd_frac"] = round(occ, 4)
            roof["frac_of_occupied_simds"] = round(roof["frac"] / occ, 4)
    # secondary figure: algorithmic HBM bytes of the registry gather per launch / its duration
    gather_gbs = None
    if "fav_gather" in kern and kern["fav_gather"][1]:
        g_s = kern["fav_gather"][0] / kern["fav_gather"][1] * 1e-3
        gather_gbs = round(B * n * GATHER_BYTES_PER_KEY / g_s / 1e9, 1)
    # PCIe-inclusive rate: the host-buffer C-ABI call (bls_fav_batch_indexed: inputs copied H2D, verdicts D2H),
    # one batch at a time, no pipelining.  Reported beside `value`, never as it.
    e2e = None
    if rank == 0 and not args.no_e2e:
        batch.fast_aggregate_verify_batch(idx, offs, msgs, sigs, ctx=ctx)
        t1 = time.perf_counter()
        v2 = batch.fast_aggregate_verify_batch(idx, offs, msgs, sigs, ctx=ctx)
        e2e = round(B / (time.perf_counter() - t1), 1)
        assert v2.all()
    percall = None
    if rank == 0 and world == 1 and not args.no_percall:
        percall = percall_latency()
    total_fme = 11 * n + 14789
    pipeline_ops = (total_fme * FME_OPS + 19 * SHA_OPS) * B * world * args.steps + 9268 * FME_OPS * args.steps
    pipeline_frac = pipeline_ops / dt / (PEAK_INT_OPS * world)

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "FAV/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32-limb Fp (381-bit Montgomery)",
        "data": "synthetic: registry sk_i=i+1 (2^20 keys, HBM), SHA256 messages, signatures made on device",
        "config": {"workload": f"C2 sync-committee FastAggregateVerify: {B} aggregates x {n} pubkeys per GPU",
                   "global_batch": B * world, "committee": n, "registry": args.registry,
                   "parallelism": f"dp{world} (aggregates sharded, RCCL all-gather of 576-B Fp12 partials)"},
        "roofline": roof,
        "int_valu_frac_pipeline": round(pipeline_frac, 5),
        "kernels_avg_ms": kernels_ms,
        "gather_hbm_gbs": gather_gbs,
        "host_buffers_fav_s": e2e,
        "percall": percall,
        "device": dev_name, "cus": cus, "setup_s": round(setup_s, 2),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cores = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or 1 << 30, len(os.sched_getaffinity(0)))
        out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds, cores)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    rb.free()
    if dist is not None:
        bdist.destroy_comm(ctx)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
