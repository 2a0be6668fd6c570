#!/usr/bin/env python3
"""Latency of the per-call AggregateVerify (E/utils/bls.py AggregateVerify, one ctypes call) at n pairs: median
wall clock over REPS calls, one JSON line (for rocprofv3 --kernel-trace --stats runs of the per-call AV path)."""
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "eth-consensus-specs_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from bls_mi355x.backend import mi355x_bls as M  # noqa: E402
from oracle import bls_oracle_c as OC  # noqa: E402


def main(reps=int(os.environ.get("REPS", "9"))):
    out = {}
    for n in [int(x) for x in os.environ.get("AV_N", "2,16,128").split(",")]:
        sks = list(range(2001, 2001 + n))
        msgs = [hashlib.sha256(b"av" + k.to_bytes(4, "little")).digest() for k in sks]
        pks = [OC.SkToPk(k) for k in sks]
        sig = OC.Aggregate([OC.Sign(k, m) for k, m in zip(sks, msgs)])
        assert M.AggregateVerify(pks, msgs, sig)
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            assert M.AggregateVerify(pks, msgs, sig)
            ts.append(time.perf_counter() - t)
        out[f"av{n}_ms"] = round(statistics.median(ts) * 1e3, 3)
    # bls_pairing_check_ex of 2 pairs (the KZG verification shape): e(P, Q) e(-P, Q) == 1
    from bls_mi355x import _native
    from oracle import bls_oracle as O

    ctx = _native.context()
    P, Q = O.g1_mul(O.G1_GEN, 12345), O.g2_mul(O.G2_GEN, 678)
    g1 = O.g1_compress(P) + O.g1_compress(O.g1_neg(P))
    g2 = O.g2_compress(Q) * 2
    assert ctx.check(ctx.lib.bls_pairing_check_ex(ctx.h, g1, g2, 2, 1)) == 1
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.check(ctx.lib.bls_pairing_check_ex(ctx.h, g1, g2, 2, 1))
        ts.append(time.perf_counter() - t)
    out["pairing_check2_ms"] = round(statistics.median(ts) * 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
