"""GPU tests of the wavefront-cooperative ("wide") arithmetic of the per-call path (csrc/bls_wide.h): the device
self-test against the lane form (bls_fq.h) on random and edge inputs.  Requires an MI355X."""
import random

import pytest

from oracle import bls_oracle as O

pytestmark = pytest.mark.gpu


def test_wide_products_match_lane_form():
    import ctypes

    import numpy as np

    from bls_mi355x import _native

    ctx = _native.context()
    rnd = random.Random(0x31DE)
    edge = [0, 1, 2, O.P - 1, O.P - 2, (1 << 380) - 1, O.P >> 1, (O.P + 1) // 2]
    vals = edge + [rnd.randrange(O.P) for _ in range(4 * 512 - len(edge))]
    nw = len(vals) // 4
    buf = b"".join(v.to_bytes(48, "big") for v in vals)
    bad = np.zeros(nw, dtype=np.int32)
    ctx.check(ctx.lib.bls_test_wide_selftest(ctx.h, buf, nw, bad.ctypes.data_as(ctypes.c_void_p)))
    assert not bad.any(), [(int(w), hex(int(bad[w]))) for w in np.nonzero(bad)[0][:8]]
