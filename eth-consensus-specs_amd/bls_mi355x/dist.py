"""Multi-GPU combination of FastAggregateVerify shards.

Each rank reduces its shard to one 576-byte Fp12 Miller partial.  The
partials are all-gathered by the library itself over RCCL (``ncclAllGather``
over xGMI inside ``bls_fav_job_check_comm``), and every rank multiplies them
and runs one final exponentiation -- no broadcast, and no framework on the
data path.  Fp12 multiplication is not an element-wise sum, so this is an
all-gather, not an all-reduce.

The only host-side step is handing the 128-byte RCCL unique id from rank 0 to
the other ranks; ``init_comm`` takes any key-value store with ``set`` /
``get`` (bench.py passes the torchrun TCP store).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native

PARTIAL_BYTES = 576
UID_BYTES = 128
_UID_KEY = "blsmi355x/rccl_uid"


def init_comm(ctx: _native.Context, rank: int, world: int, store) -> None:
    """Create the context's RCCL communicator (rank `rank` of `world`)."""
    if rank == 0:
        uid = ctypes.create_string_buffer(UID_BYTES)
        ctx.check(ctx.lib.bls_comm_unique_id(uid))
        store.set(_UID_KEY, uid.raw)
        raw = uid.raw
    else:
        raw = bytes(store.get(_UID_KEY))
    if len(raw) != UID_BYTES:
        raise ValueError("RCCL unique id must be 128 bytes")
    ctx.check(ctx.lib.bls_comm_init(ctx.h, raw, rank, world))


def destroy_comm(ctx: _native.Context) -> None:
    ctx.check(ctx.lib.bls_comm_destroy(ctx.h))


def abort_comm(ctx: _native.Context) -> None:
    """ncclCommAbort: peers blocked in a collective with this rank fail instead of hanging (call on an error
    path before leaving the exchange)."""
    ctx.lib.bls_comm_abort(ctx.h)


def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) block of `total` items owned by `rank`."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


# per-aggregate work that does not scale with its committee, in pubkey additions: the SURVEY.md §8(d) model
# prices FAV(n) at 11 (n - 1) + 14,789 FME, i.e. ~1,344 additions' worth per aggregate beside its n - 1 additions
ITEM_WORK_KEYS = 14789 // 11


def shard_bounds_by_work(offsets, rank: int, world: int, per_item: int = ITEM_WORK_KEYS) -> tuple[int, int]:
    """Contiguous [lo, hi) block of aggregates owned by `rank`, balanced by work ("contiguous
    blocks of aggregates, balanced by total pubkey count"): aggregate i costs n_i + per_item, n_i =
    offsets[i + 1] - offsets[i] (per_item = 0: pure pubkey count).  Rank r's block starts at the aggregate whose
    cumulative work is nearest r / world of the total, so every rank's share is within one aggregate's work of
    total / world; uniform committees give shard_bounds' blocks.  Every rank computes the same cut points from
    the same offsets (no exchange).

    No rank's block is empty when B >= world: the cut points are made strictly increasing (a heavily skewed
    committee, e.g. one of 131,072 keys after a thousand of one, would otherwise leave the ranks between two cuts
    with nothing, and a rank with no aggregates cannot take part in a job).  Only B < world leaves ranks empty;
    those submit an empty shard, whose partial is the identity, so they still join every all-gather
    (bls_fav_job_submit_dev with B = 0)."""
    cuts = work_cuts(offsets, world, per_item)
    return cuts[rank], cuts[rank + 1]


def work_cuts(offsets, world: int, per_item: int = ITEM_WORK_KEYS) -> list[int]:
    """The world + 1 cut points of shard_bounds_by_work: 0 = c_0 <= c_1 <= ... <= c_world = B, strictly increasing
    when B >= world."""
    offs = np.asarray(offsets, dtype=np.int64)
    B = int(offs.size) - 1
    if B <= 0:
        return [0] * (world + 1)
    cum = offs - offs[0] + per_item * np.arange(B + 1, dtype=np.int64)  # work before aggregate i
    total = int(cum[-1])

    def cut(r: int) -> int:
        t = total * r / world
        i = int(np.searchsorted(cum, t))  # first boundary with work >= t
        if i > 0 and (i > B or t - cum[i - 1] <= cum[i] - t):
            i -= 1
        return min(max(i, 0), B)

    c = [0] + [cut(r) for r in range(1, world)] + [B]
    if B >= world:  # every block non-empty: c_r >= c_{r-1} + 1 going up, then c_r <= c_{r+1} - 1 going down
        for r in range(1, world):
            c[r] = max(c[r], c[r - 1] + 1)
        for r in range(world - 1, 0, -1):
            c[r] = min(c[r], c[r + 1] - 1)
    else:
        for r in range(1, world):
            c[r] = max(c[r], c[r - 1])
    return c
