"""world_size-2 gloo test of the multi-GPU combination protocol
(bls_mi355x.dist): each rank holds the Miller product of its shard, the
576-byte partials are all-gathered, every rank multiplies and final-
exponentiates.  Partials here come from the oracle (no GPU on CPU)."""
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


def _worker(rank, world, port, tamper, q):
    import torch.distributed as dist

    from bls_mi355x.dist import allgather_partials

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # shard r: one aggregate with sk = 3 + r over message m_r; pair (pk, H(m)) and (-G1, sig)
    sk = 3 + rank
    m = bytes([rank]) * 32
    pk = O.g1_mul(O.G1_GEN, sk)
    sig = O.g2_decompress(O.Sign(sk if not (tamper and rank == 1) else sk + 1, m))
    f = O.f12_mul(O.miller_loop(pk, O.hash_to_g2(m)), O.miller_loop(O.g1_neg(O.G1_GEN), sig))
    allp = allgather_partials(_partial_bytes(f))
    prod = O.F12_ONE
    for k in range(world):
        prod = O.f12_mul(prod, _from_bytes(allp[576 * k: 576 * k + 576]))
    q.put((rank, O.final_exponentiation(prod) == O.F12_ONE))
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
    assert res == {0: not tamper, 1: not tamper}
