"""Multi-GPU combination of FastAggregateVerify shards.

Each rank reduces its shard to one 576-byte Fp12 Miller partial; the partials
are all-gathered (torch.distributed: "nccl" = RCCL over xGMI on MI355X,
"gloo" on CPU for tests) and every rank multiplies them and runs one final
exponentiation -- no broadcast needed.  Fp12 multiplication is not an
element-wise sum, so this is an all-gather, not an all-reduce.
"""
from __future__ import annotations

PARTIAL_BYTES = 576


def allgather_partials(partial: bytes, device=None) -> bytes:
    """Concatenation (rank order) of every rank's 576-byte partial."""
    import torch
    import torch.distributed as dist

    if len(partial) != PARTIAL_BYTES:
        raise ValueError("a partial is one Fp12 = 576 bytes")
    world = dist.get_world_size()
    t = torch.frombuffer(bytearray(partial), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return b"".join(bytes(o.cpu().numpy()) for o in outs)
