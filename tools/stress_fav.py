#!/usr/bin/env python3
"""Replays tests/test_gpu_sigsets.py::test_registry_append_and_lookup's sequence of small FAV batches ITERS times,
each iteration with its own RLC seed written to a file the library reads (bls_set_entropy_source), and prints one JSON
line per mismatch with the seed that produced it, then a summary line.  A small-batch verdict that depends on the
RLC scalars shows up here with a seed that replays it."""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "eth-consensus-specs_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from bls_mi355x import _native, batch as b  # noqa: E402
from oracle import bls_oracle_c as OC  # noqa: E402

G1_INF = b"\xc0" + bytes(47)


def keys(sks):
    pks = b.sk_to_pk_batch(b"".join(k.to_bytes(32, "big") for k in sks))
    return [pks[48 * i: 48 * i + 48] for i in range(len(sks))]


def main(iters=int(os.environ.get("ITERS", "200")), seed0=int(os.environ.get("SEED0", "1"))):
    lib = _native.context().lib
    fd, path = tempfile.mkstemp()
    os.close(fd)
    m = hashlib.sha256(b"deposit").digest()
    sig13, sig7, sig400 = OC.Sign(13, m), OC.Sign(7, m), OC.Sign(1 + 399, m)
    first, more = keys([1, 2, 3, 4]), keys([5, 6]) + [G1_INF]
    big = keys(list(range(100, 400)))
    bad = 0
    try:
        assert lib.bls_set_entropy_source(path.encode()) == 0
        for it in range(iters):
            seed = hashlib.sha256(b"stress" + (seed0 + it).to_bytes(8, "little")).digest()
            with open(path, "wb") as f:
                f.write(seed)
            reg = b.Registry()
            reg.load(b"".join(first))
            reg.append(b"".join(more))
            got = []
            got.append(list(b.fast_aggregate_verify_batch(np.array([1, 4, 5, 0], dtype=np.uint32),
                                                          b.offsets_from_lengths([3, 1]), m + m, sig13 + sig7)))
            got.append(list(b.fast_aggregate_verify_batch(np.array([6, 0], dtype=np.uint32),
                                                          b.offsets_from_lengths([2]), m, sig13)))
            reg.append(b"".join(big))
            got.append(list(b.fast_aggregate_verify_batch(np.array([0, 306], dtype=np.uint32),
                                                          b.offsets_from_lengths([2]), m, sig400)))
            want = [[True, False], [False], [True]]
            got = [[bool(x) for x in g] for g in got]
            if got != want:
                bad += 1
                print(json.dumps({"iter": it, "seed": seed.hex(), "got": got, "want": want}), flush=True)
            if it % 50 == 0:
                print(json.dumps({"progress": it, "bad": bad}), flush=True)
    finally:
        lib.bls_set_entropy_source(b"/dev/urandom")
        os.unlink(path)
    print(json.dumps({"iters": iters, "bad": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
