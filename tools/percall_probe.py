#!/usr/bin/env python3
"""Latency of the drop-in per-call API (one ctypes call per verification, as
E/utils/bls.py:141-177 calls milagro): Verify and FastAggregateVerify(n) with
host buffers.  BLS_PERCALL=lane selects the previous one-lane kernels for an
A/B.  Prints one JSON line."""
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


def main(reps=int(os.environ.get("REPS", "15"))):
    sks = list(range(1001, 1001 + 512))
    pks = [OC.SkToPk(k) for k in sks]
    m = hashlib.sha256(b"percall").digest()
    sig1, sig512, sig16 = OC.Sign(sks[0], m), OC.Sign(sum(sks), m), OC.Sign(sum(sks[:16]), m)
    out = {"mode": os.environ.get("BLS_PERCALL", "phased")}
    for name, fn in (("verify_ms", lambda: M.Verify(pks[0], m, sig1)),
                     ("fav512_ms", lambda: M.FastAggregateVerify(pks, m, sig512)),
                     ("fav16_ms", lambda: M.FastAggregateVerify(pks[:16], m, sig16))):
        assert fn()
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            assert fn()
            ts.append(time.perf_counter() - t)
        out[name] = round(statistics.median(ts) * 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
