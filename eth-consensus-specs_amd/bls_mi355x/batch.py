"""Batch / registry API (the throughput path).

The per-call drop-in API (``backend.mi355x_bls``) verifies one signature per
ctypes call.  Spec call sites that verify many aggregates against the
validator registry (``is_valid_indexed_attestation``,
specs/phase0/beacon-chain.md:776-790; ``process_sync_aggregate``,
specs/altair/beacon-chain.md:575-610) use these instead: the registry's
pubkeys are decoded and KeyValidated once into HBM and each aggregate is
named by registry indices.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native

# per-context job slots with streams: BLS_FAV_JOBS_INIT (default 10: two streams per job, the batch checks on the
# jobs' own streams, 21 of the 24 hardware queues -- profiles/r05h_jobs_streams_ab.txt: C2 +3 %, C3 +13 % over 7
# three-stream jobs with one shared FE stream; 11 jobs and more, or more streams than queues, collapse) of the
# BLS_FAV_JOBS = 16 in include/blsmi355x.h, read by the library at bls_ctx_create
FAV_JOBS = max(1, min(16, int(os.environ.get("BLS_FAV_JOBS_INIT", "10"))))
# batches kept in flight by run_pipelined (<= FAV_JOBS)
FAV_DEPTH = max(1, min(FAV_JOBS, int(os.environ.get("BLS_FAV_DEPTH", str(FAV_JOBS)))))
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001  # the BLS12-381 group order r


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u8(b) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b, np.uint8)


class Registry:
    """HBM-resident affine pubkey table of one context.

    The host keeps a pubkey-bytes -> index map for the keys loaded or appended through this object.  It is
    tied to the library's registry generation (``bls_registry_generation``, bumped whenever any caller
    replaces the device table): after a replacement by another object or by ``generate()``, lookups return
    None instead of indices that now name other keys."""

    def __init__(self, ctx: _native.Context | None = None):
        self.ctx = ctx or _native.context()
        self._index: dict[bytes, int] = {}  # pubkey bytes -> first registry index (host-side lookup)
        self._gen = None  # library registry generation the map belongs to

    def _generation(self) -> int:
        return int(self.ctx.lib.bls_registry_generation(self.ctx.h))

    def _remember(self, buf: np.ndarray, first: int) -> None:
        raw = buf.tobytes()
        for i in range(len(raw) // 48):
            self._index.setdefault(raw[48 * i: 48 * i + 48], first + i)

    def load(self, pubkeys48: bytes | np.ndarray) -> np.ndarray:
        """Decode + KeyValidate ``n`` compressed keys; returns the validity mask."""
        buf = _u8(pubkeys48)
        if buf.size % 48:
            raise ValueError("pubkeys must be a multiple of 48 bytes")
        n = buf.size // 48
        valid = np.zeros(n, dtype=np.uint8)
        c = self.ctx
        self._index, self._gen = {}, None
        c.check(c.lib.bls_registry_load(c.h, buf.tobytes(), n, _ptr(valid)))
        self._remember(buf, 0)
        self._gen = self._generation()
        return valid

    def append(self, pubkeys48: bytes | np.ndarray) -> np.ndarray:
        """Deposits: append keys as validator indices len(self) .. (decode + KeyValidate on the
        device, existing indices unchanged; specs/phase0/beacon-chain.md:2037-2062).  Returns the
        validity mask of the new keys."""
        buf = _u8(pubkeys48)
        if buf.size % 48:
            raise ValueError("pubkeys must be a multiple of 48 bytes")
        n = buf.size // 48
        first = len(self)
        valid = np.zeros(n, dtype=np.uint8)
        c = self.ctx
        c.check(c.lib.bls_registry_append(c.h, buf.tobytes(), n, _ptr(valid)))
        if self._gen is not None and self._gen == self._generation():
            self._remember(buf, first)
        return valid

    def _current(self) -> bool:
        return self._gen is not None and self._gen == self._generation()

    def index_of(self, pubkey48: bytes) -> int | None:
        """Registry index of a compressed pubkey loaded or appended through this object, else None (also
        None once the device table was replaced)."""
        if not self._current():
            return None
        return self._index.get(bytes(pubkey48))

    def indices(self, pubkeys) -> np.ndarray | None:
        """u32 registry indices of every key, or None if any key is not resident (or the map is stale)."""
        if not self._current():
            return None
        out = np.empty(len(pubkeys), dtype=np.uint32)
        for i, pk in enumerate(pubkeys):
            k = self._index.get(bytes(pk))
            if k is None:
                return None
            out[i] = k
        return out

    def generate(self, n: int, first_sk: int = 1, want_bytes: bool = False):
        """Synthetic registry pk_i = (first_sk + i)*G1 built on the device (benchmarks).  With want_bytes the
        compressed keys are returned and the pubkey -> index map covers them."""
        c = self.ctx
        out = ctypes.create_string_buffer(48 * n) if want_bytes else None
        self._index, self._gen = {}, None
        c.check(c.lib.bls_registry_generate(c.h, first_sk, n, out))
        if want_bytes:
            self._remember(np.frombuffer(out.raw, dtype=np.uint8), 0)
            self._gen = self._generation()
            return out.raw
        return None

    def __len__(self):
        return int(self.ctx.lib.bls_registry_size(self.ctx.h))


def offsets_from_lengths(lengths) -> np.ndarray:
    offs = np.zeros(len(lengths) + 1, dtype=np.uint64)
    np.cumsum(np.asarray(lengths, dtype=np.uint64), out=offs[1:])
    return offs


def fast_aggregate_verify_batch(indices: np.ndarray, offsets: np.ndarray, msgs32, sigs96, ctx=None) -> np.ndarray:
    """B FastAggregateVerify calls over registry indices -> bool array."""
    c = ctx or _native.context()
    idx = np.ascontiguousarray(indices, dtype=np.uint32)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    B = offs.size - 1
    m, s = _u8(msgs32), _u8(sigs96)
    if m.size != 32 * B or s.size != 96 * B:
        raise ValueError("need 32-byte messages and 96-byte signatures, one per aggregate")
    out = np.zeros(B, dtype=np.uint8)
    c.check(c.lib.bls_fav_batch_indexed(c.h, _ptr(idx), _ptr(offs), B, m.tobytes(), s.tobytes(), _ptr(out)))
    return out.astype(bool)


def verify_batch(indices: np.ndarray, msgs32, sigs96, ctx=None) -> np.ndarray:
    """B Verify calls with registry-resident pubkeys -> bool array."""
    c = ctx or _native.context()
    idx = np.ascontiguousarray(indices, dtype=np.uint32)
    B = idx.size
    m, s = _u8(msgs32), _u8(sigs96)
    if m.size != 32 * B or s.size != 96 * B:
        raise ValueError("need 32-byte messages and 96-byte signatures")
    out = np.zeros(B, dtype=np.uint8)
    c.check(c.lib.bls_verify_batch_indexed(c.h, _ptr(idx), B, m.tobytes(), s.tobytes(), _ptr(out)))
    return out.astype(bool)


def aggregate_verify_batch(pubkeys, messages, signatures, ctx=None) -> np.ndarray:
    """B AggregateVerify calls -> bool array.  pubkeys[b] / messages[b]: item b's lists of 48-byte keys
    and messages (any lengths, equal list lengths); signatures[b]: 96 bytes.  An item whose lists differ
    in length, or with a key other than 48 bytes or a signature other than 96, is False
    (E/utils/bls.py:154-164 returns False on any exception); the rest are checked in one batch
    (bls_aggregate_verify_batch)."""
    c = ctx or _native.context()
    B = len(signatures)
    if len(pubkeys) != B or len(messages) != B:
        raise ValueError("need one pubkey list, one message list and one signature per item")
    good = np.array([len(p) == len(m) and len(bytes(s)) == 96 and all(len(bytes(k)) == 48 for k in p)
                     for p, m, s in zip(pubkeys, messages, signatures)], dtype=bool)
    lens = [len(p) if g else 0 for p, g in zip(pubkeys, good)]
    io = offsets_from_lengths(lens)
    flat_pk = [bytes(k) for p, g in zip(pubkeys, good) if g for k in p]
    flat_m = [bytes(m) for ms, g in zip(messages, good) if g for m in ms]
    mo = offsets_from_lengths([len(m) for m in flat_m])
    sigs = b"".join(bytes(s) if g else bytes(96) for s, g in zip(signatures, good))
    out = np.zeros(B, dtype=np.uint8)
    if B:
        c.check(c.lib.bls_aggregate_verify_batch(c.h, b"".join(flat_pk), b"".join(flat_m), _ptr(mo), _ptr(io), B,
                                                 sigs, _ptr(out)))
    return out.astype(bool) & good


def compute_signing_roots(object_roots, domains, ctx=None) -> list[bytes]:
    """compute_signing_root for many objects on the device (specs/phase0/beacon-chain.md:953-962):
    SHA-256(object_root || domain).  ``domains``: one 32-byte domain for all, or one per root."""
    c = ctx or _native.context()
    roots = [bytes(r) for r in object_roots]
    if any(len(r) != 32 for r in roots):
        raise ValueError("object roots must be 32 bytes")
    if isinstance(domains, (bytes, bytearray)) and len(domains) == 32:
        dom, stride = bytes(domains), 0
    else:
        dl = [bytes(d) for d in domains]
        if len(dl) != len(roots) or any(len(d) != 32 for d in dl):
            raise ValueError("need one 32-byte domain, or one per root")
        dom, stride = b"".join(dl), 32
    n = len(roots)
    out = ctypes.create_string_buffer(32 * n) if n else None
    c.check(c.lib.bls_signing_roots(c.h, b"".join(roots), dom, stride, n, out))
    return [out.raw[32 * i: 32 * i + 32] for i in range(n)]


def merkleize(chunks, limit: int | None = None, ctx=None) -> bytes:
    """SSZ merkleize(chunks, limit) on the device: the tree has next_pow2(limit or len(chunks)) leaves."""
    c = ctx or _native.context()
    ch = [bytes(x) for x in chunks]
    if any(len(x) != 32 for x in ch):
        raise ValueError("chunks must be 32 bytes")
    n = len(ch)
    size = n if limit is None else limit
    if size < n:
        raise ValueError("more chunks than the limit")
    depth = max(size - 1, 0).bit_length()
    out = ctypes.create_string_buffer(32)
    c.check(c.lib.bls_merkleize(c.h, b"".join(ch) if n else None, n, depth, out))
    return out.raw


def mix_in_length(root: bytes, length: int) -> bytes:
    """hash_tree_root of a list: SHA-256(root || uint256 length little-endian) -- one node, host hashlib."""
    import hashlib

    return hashlib.sha256(bytes(root) + int(length).to_bytes(32, "little")).digest()


def pairing_check(pairs, ctx=None) -> bool:
    """KZG pairing_check (E/utils/bls.py; specs/deneb/polynomial-commitments.md:284,407,451):
    prod e(P_i, Q_i) == 1 over compressed (48-byte G1, 96-byte G2) pairs; the identity is allowed,
    an invalid encoding gives False."""
    c = ctx or _native.context()
    g1 = [bytes(p) for p, _ in pairs]
    g2 = [bytes(q) for _, q in pairs]
    if any(len(p) != 48 for p in g1) or any(len(q) != 96 for q in g2):
        raise ValueError("need 48-byte G1 and 96-byte G2 encodings")
    return c.check(c.lib.bls_pairing_check(c.h, b"".join(g1), b"".join(g2), len(g1))) == 1


def g1_multi_exp(points48, scalars, ctx=None, subgroup_check: bool = False) -> bytes:
    """KZG multi_exp / g1_lincomb on compressed points: sum [k_i] P_i (E/utils/bls.py:262-296 -> arkworks
    G1.multiexp_unchecked, i.e. no subgroup check unless asked); scalars are ints (0 <= k < 2^256).  Raises on
    an empty input (E/utils/bls.py:270-271) and on an invalid encoding, like the reference."""
    c = ctx or _native.context()
    pts = [bytes(p) for p in points48]
    ks = [int(k) for k in scalars]
    if not pts or not ks:
        raise ValueError("Cannot call multi_exp with zero points or zero scalars")
    if len(pts) != len(ks):
        raise ValueError("one scalar per point")
    if any(len(p) != 48 for p in pts) or any(not 0 <= k < 1 << 256 for k in ks):
        raise ValueError("need 48-byte points and 256-bit scalars")
    # reduced mod r as curve.Scalar / curve._k32 do (arkworks' Scalar): for a point decoded without the subgroup
    # check, [k]P and [k mod r]P differ, and both entry points must give the same result
    ks = [k % R_ORDER for k in ks]
    out = ctypes.create_string_buffer(48)
    rc = c.check(c.lib.bls_multi_exp(c.h, 1, b"".join(pts), b"".join(k.to_bytes(32, "big") for k in ks), len(pts),
                                     1 if subgroup_check else 0, out))
    if rc != 1:
        raise ValueError("invalid G1 point encoding")
    return out.raw


def fallback_stats(ctx=None) -> tuple[int, int]:
    """(batched final-exponentiation checks, bisection rounds) of the last batch call; (0, 0) if it passed."""
    c = ctx or _native.context()
    checks, rounds = ctypes.c_uint64(), ctypes.c_uint64()
    c.check(c.lib.bls_last_fallback_stats(c.h, ctypes.byref(checks), ctypes.byref(rounds)))
    return int(checks.value), int(rounds.value)


def sign_batch(sks32, msgs32, ctx=None) -> bytes:
    c = ctx or _native.context()
    sk, m = _u8(sks32), _u8(msgs32)
    B = sk.size // 32
    out = ctypes.create_string_buffer(96 * B)
    if c.check(c.lib.bls_sign_batch(c.h, sk.tobytes(), m.tobytes(), B, out)) != 1:
        raise ValueError("invalid secret key in batch")
    return out.raw


def sk_to_pk_batch(sks32, ctx=None) -> bytes:
    c = ctx or _native.context()
    sk = _u8(sks32)
    B = sk.size // 32
    out = ctypes.create_string_buffer(48 * B)
    if c.check(c.lib.bls_sk_to_pk_batch(c.h, sk.tobytes(), B, out)) != 1:
        raise ValueError("invalid secret key in batch")
    return out.raw


class DeviceBuffer:
    """HBM buffer owned by a context (inputs resident before a timed region)."""

    def __init__(self, ctx: _native.Context, data: np.ndarray | bytes | None = None, nbytes: int | None = None):
        self.ctx = ctx
        arr = None if data is None else (np.ascontiguousarray(data) if isinstance(data, np.ndarray) else _u8(data))
        self.nbytes = int(arr.nbytes if arr is not None else nbytes)
        self.ptr = ctx.lib.bls_dev_alloc(ctx.h, max(self.nbytes, 1))
        if not self.ptr:
            raise _native.NativeError("bls_dev_alloc failed")
        if arr is not None and self.nbytes:
            ctx.check(ctx.lib.bls_h2d(ctx.h, self.ptr, _ptr(arr), self.nbytes))

    def to_host(self) -> np.ndarray:
        out = np.empty(self.nbytes, dtype=np.uint8)
        self.ctx.check(self.ctx.lib.bls_d2h(self.ctx.h, _ptr(out), self.ptr, self.nbytes))
        return out

    def free(self):
        if self.ptr:
            self.ctx.lib.bls_dev_free(self.ctx.h, self.ptr)
            self.ptr = None


class ResidentFavBatch:
    """A FastAggregateVerify batch whose inputs live in HBM (bench / multi-GPU).

    ``partial()`` runs this shard's checks and Miller loops and returns the
    576-byte Fp12 partial; partials of all shards are multiplied and
    final-exponentiated by ``check_partials``; ``finish()`` writes verdicts.
    """

    def __init__(self, indices, offsets, msgs32, sigs96, ctx=None, chunks: int = 1):
        """chunks > 1 splits the batch into that many equal sub-batches (uniform committee size only), each
        submitted as its own FAV job: a pass over the batch is `chunks` jobs (large shards, e.g. the C4 firehose,
        stay within one job's scratch)."""
        self.ctx = ctx or _native.context()
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.B = int(offs.size - 1)
        self.chunks = max(1, int(chunks))
        if self.chunks > 1:
            n = int(offs[1] - offs[0]) if self.B else 0
            if self.B % self.chunks or not np.array_equal(offs, np.arange(self.B + 1, dtype=np.uint64) * n):
                raise ValueError("chunks > 1 needs B divisible by chunks and one committee size")
            self.cb, self.n = self.B // self.chunks, n
            offs = offs[: self.cb + 1]  # every chunk has the same relative offsets
        else:
            self.cb, self.n = self.B, None
        self.idx = DeviceBuffer(self.ctx, np.ascontiguousarray(indices, dtype=np.uint32))
        self.offs = DeviceBuffer(self.ctx, offs)
        self.msgs = DeviceBuffer(self.ctx, _u8(msgs32))
        self.sigs = DeviceBuffer(self.ctx, _u8(sigs96))
        self.outs = [DeviceBuffer(self.ctx, nbytes=self.B) for _ in range(FAV_JOBS)]
        self.out = self.outs[0]
        self.last_job = 0
        self._chunk_job = [0] * self.chunks  # job whose buffer holds each chunk's latest verdicts

    def partial(self, seed32: bytes | None = None) -> bytes:
        if self.chunks > 1:
            raise ValueError("a chunked batch runs through the job API (run_pipelined)")
        seed = seed32 if seed32 is not None else os.urandom(32)
        buf = ctypes.create_string_buffer(576)
        c = self.ctx
        c.check(c.lib.bls_fav_batch_partial_dev(c.h, self.idx.ptr, self.offs.ptr, self.B, self.msgs.ptr,
                                                self.sigs.ptr, seed, buf))
        return buf.raw

    def check_partials(self, partials: bytes) -> bool:
        c = self.ctx
        n = len(partials) // 576
        return c.check(c.lib.bls_partials_check(c.h, partials, n)) == 1

    def finish(self, batch_ok: bool) -> None:
        c = self.ctx
        c.check(c.lib.bls_fav_batch_finish_dev(c.h, 1 if batch_ok else 0, self.out.ptr))
        self.last_job = 0

    # ---- pipelined passes (bls_fav_job_*): up to FAV_JOBS batches in flight --
    def _chunk_ptrs(self, c: int):
        lo = c * self.cb
        nidx = lo * self.n if self.chunks > 1 else 0
        return self.idx.ptr + 4 * nidx, self.msgs.ptr + 32 * lo, self.sigs.ptr + 96 * lo, lo

    def submit(self, job: int, seed32: bytes, chunk: int = 0) -> None:
        c = self.ctx
        idx, msgs, sigs, _ = self._chunk_ptrs(chunk)
        c.check(c.lib.bls_fav_job_submit_dev(c.h, job, idx, self.offs.ptr, self.cb, msgs, sigs, seed32))

    def job_partial(self, job: int) -> bytes:
        buf = ctypes.create_string_buffer(576)
        c = self.ctx
        c.check(c.lib.bls_fav_job_partial(c.h, job, buf))
        return buf.raw

    def job_check(self, job: int, partials: bytes) -> bool:
        c = self.ctx
        return c.check(c.lib.bls_fav_job_check(c.h, job, partials, len(partials) // 576)) == 1

    def job_check_own(self, job: int) -> bool:
        """The job's own product alone (bls_fav_job_check_own: the check submit enqueued behind it)."""
        c = self.ctx
        return c.check(c.lib.bls_fav_job_check_own(c.h, job)) == 1

    def job_finish(self, job: int, batch_ok: bool, chunk: int = 0) -> None:
        c = self.ctx
        lo = self._chunk_ptrs(chunk)[3]
        c.check(c.lib.bls_fav_job_finish_dev(c.h, job, 1 if batch_ok else 0, self.outs[job].ptr + lo))
        self.last_job = job
        self._chunk_job[chunk] = job

    def job_check_comm(self, job: int) -> bool:
        """RCCL all-gather of the job's device-resident partial + the product's final exponentiation
        (bls_fav_job_check_comm; the context's communicator must be initialised: dist.init_comm)."""
        c = self.ctx
        return c.check(c.lib.bls_fav_job_check_comm(c.h, job)) == 1

    def run_pipelined(self, seeds, exchange=None, depth: int = FAV_DEPTH, comm: bool = False) -> list:
        """One pass over the batch per seed (a pass = `chunks` jobs) with up to `depth` jobs in flight:
        job k+1.. are submitted before job k is final-exponentiated (their front kernels overlap job k's
        tail).  Multi-GPU: comm=True exchanges each job's partial inside the library over RCCL
        (bls_fav_job_check_comm); otherwise exchange(partial) -> concatenated partials of all ranks (a
        host-side all-gather, e.g. gloo in the CPU tests).  Every pass is complete (verdicts written) on
        return; returns one bool per pass (all of its chunks' batch checks passed)."""
        seeds = list(seeds)
        depth = max(1, min(depth, FAV_JOBS))
        units = [(k, ch) for k in range(len(seeds)) for ch in range(self.chunks)]
        oks = [True] * len(seeds)
        for u in range(min(depth, len(units))):
            k, ch = units[u]
            self.submit(u % FAV_JOBS, seeds[k], ch)
        for u, (k, ch) in enumerate(units):
            job = u % FAV_JOBS
            if comm:
                ok = self.job_check_comm(job)
            elif exchange is None:  # one shard: its own check, already enqueued behind its product
                ok = self.job_check_own(job)
            else:
                part = self.job_partial(job)
                ok = self.job_check(job, exchange(part))
            self.job_finish(job, ok, ch)
            oks[k] = oks[k] and ok
            if u + depth < len(units):
                k2, ch2 = units[u + depth]
                self.submit((u + depth) % FAV_JOBS, seeds[k2], ch2)
        self.ctx.check(self.ctx.lib.bls_sync(self.ctx.h))  # a failing job's bisection writes its verdicts async
        return oks

    def verdicts(self) -> np.ndarray:
        if self.chunks == 1:
            return self.outs[self.last_job].to_host().astype(bool)
        bufs = {j: self.outs[j].to_host() for j in set(self._chunk_job)}
        return np.concatenate([bufs[j][c * self.cb:(c + 1) * self.cb] for c, j in enumerate(self._chunk_job)]
                              ).astype(bool)

    def run(self) -> np.ndarray:
        ok = self.check_partials(self.partial())
        self.finish(ok)
        return self.verdicts()

    def free(self):
        for b in (self.idx, self.offs, self.msgs, self.sigs, *self.outs):
            b.free()


class Profiler:
    """hipEvent timing of each kernel of the FAV path (C-ABI bls_profile_*)."""

    def __init__(self, ctx=None):
        self.ctx = ctx or _native.context()

    def start(self):
        self.ctx.check(self.ctx.lib.bls_profile_enable(self.ctx.h, 1))

    def stop(self):
        self.ctx.check(self.ctx.lib.bls_profile_enable(self.ctx.h, 0))

    def read(self) -> dict:
        c = self.ctx
        ms = (ctypes.c_double * 16)()
        cnt = (ctypes.c_uint64 * 16)()
        n = c.check(c.lib.bls_profile_read(c.h, ms, cnt, 16))
        return {c.lib.bls_profile_name(i).decode(): (ms[i], int(cnt[i])) for i in range(n)}
