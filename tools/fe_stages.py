"""Stage clocks of the six-wave final-exponentiation check (k_fe_wide, bls_test_final_check wide=2): load, easy
part (wave 0, lane-parallel), the hard part's first x-power chain, the rest.  Prints one JSON line (microseconds,
median of REPS runs)."""
import ctypes
import json
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "eth-consensus-specs_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bls_mi355x import _native  # noqa: E402

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def main():
    ctx = _native.context()
    rnd = random.Random(1)
    f = b"".join(rnd.randrange(P).to_bytes(48, "little") for _ in range(12))
    names = ["load", "easy", "powx0", "rest"]
    runs = []
    for _ in range(int(os.environ.get("REPS", "9"))):
        out = (ctypes.c_int32 * 18)()
        ctx.check(ctx.lib.bls_test_final_check(ctx.h, f, 1, 2, out))
        ts = [int.from_bytes(bytes(out)[8 + 8 * i: 16 + 8 * i], "little") for i in range(5)]
        runs.append([(ts[i + 1] - ts[i]) / 100.0 for i in range(4)])
    print(json.dumps({n: round(statistics.median(r[i] for r in runs), 1) for i, n in enumerate(names)}))


if __name__ == "__main__":
    main()
