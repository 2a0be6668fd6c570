#!/usr/bin/env python3
"""Final-exponentiation check latency probe (tool): `reps` bls_partials_check calls on a random 576-byte
partial (one k_fe_check launch each, one workgroup); prints the median wall time per call.  Run under
rocprofv3 --kernel-trace / --pmc to read the kernel itself."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "eth-consensus-specs_amd"))

from bls_mi355x import _native  # noqa: E402

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def main(reps=40):
    ctx = _native.context()
    rnd = int.from_bytes(os.urandom(48), "big")
    part = b"".join(((rnd * (k + 3)) % P).to_bytes(48, "big") for k in range(12))
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ok = ctx.check(ctx.lib.bls_partials_check(ctx.h, part, 1))
        ts.append(time.perf_counter() - t)
        assert ok == 0
    print(f"bls_partials_check median {statistics.median(ts) * 1e3:.3f} ms over {reps}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40)
