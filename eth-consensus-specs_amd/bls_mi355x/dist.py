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
