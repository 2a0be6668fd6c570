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


def test_h2c_wide_matches_oracle():
    """hash_to_G2 through the one-wave-per-message kernel of the per-call path (SSWU + isogeny in the two halves,
    cofactor clearing in wide Jacobian arithmetic) equals the C oracle's and the FAV batch kernels' points."""
    import ctypes
    import hashlib

    from bls_mi355x import _native
    from oracle import bls_oracle_c as OC

    ctx = _native.context()
    msgs = [hashlib.sha256(b"wide" + j.to_bytes(4, "little")).digest() for j in range(70)]
    msgs += [bytes(32), b"\xff" * 32]
    n = len(msgs)
    wide = ctypes.create_string_buffer(96 * n)
    ctx.check(ctx.lib.bls_test_hash_to_g2_wide(ctx.h, b"".join(msgs), n, wide))
    lane = ctypes.create_string_buffer(96 * n)
    ctx.check(ctx.lib.bls_test_hash_to_g2_batch(ctx.h, b"".join(msgs), n, lane))
    assert wide.raw == lane.raw
    for j in list(range(0, n, 7)) + [n - 2, n - 1]:
        assert wide.raw[96 * j: 96 * j + 96] == OC.hash_to_g2(msgs[j]), j


@pytest.mark.parametrize("mlen", [0, 1, 31, 32, 33, 100])
def test_percall_verify_message_lengths(mlen):
    """Per-call Verify / FastAggregateVerify / AggregateVerify with messages of every length class (the wide hash's
    byte-streaming and 32-byte paths) against the C oracle's signatures: valid -> True, wrong message -> False."""
    from bls_mi355x.backend import mi355x_bls as M
    from oracle import bls_oracle_c as OC

    msg = bytes((7 * k + mlen) & 0xFF for k in range(mlen))
    other = bytes([0x5A]) + msg[1:] if mlen else b"\x01"
    pk = OC.SkToPk(4242)
    sig = OC.Sign(4242, msg)
    assert M.Verify(pk, msg, sig) is True
    assert M.Verify(pk, other, sig) is False
    pks = [OC.SkToPk(k) for k in (11, 12, 13)]
    agg = OC.Sign(11 + 12 + 13, msg)
    assert M.FastAggregateVerify(pks, msg, agg) is True
    assert M.FastAggregateVerify(pks[:2], msg, agg) is False
    msgs = [msg + bytes([k]) for k in range(3)]
    av = OC.Aggregate([OC.Sign(k, m) for k, m in zip((21, 22, 23), msgs)])
    avpks = [OC.SkToPk(k) for k in (21, 22, 23)]
    assert M.AggregateVerify(avpks, msgs, av) is True
    assert M.AggregateVerify(avpks, [msgs[1], msgs[0], msgs[2]], av) is False


def test_percall_signature_edge_cases():
    """The one-wave signature check of the per-call path on the signature edge cases: identity, bad flags, x >= p,
    not on the curve, outside G2 (points of order 13 and 23 from the batch tests' construction are covered there),
    and both y signs, against the C oracle's Verify."""
    from bls_mi355x.backend import mi355x_bls as M
    from oracle import bls_oracle_c as OC

    msg = b"\x42" * 32
    pk = OC.SkToPk(77)
    sig = OC.Sign(77, msg)
    cases = [sig, b"\xc0" + bytes(95), bytes(96), b"\x80" + bytes(95), b"\xe0" + bytes(95),
             sig[:1] + b"\xff" * 47 + sig[48:], bytes([sig[0] ^ 0x20]) + sig[1:], sig[:95] + bytes([sig[95] ^ 1]),
             b"\x9a\x01\x11\xea\x39\x7f\xe6\x9a\x4b\x1b\xa7\xb6\x43\x4b\xac\xd7\x64\x77\x4b\x84\xf3\x85\x12\xbf\x67"
             b"\x30\xd2\xa0\xf6\xb0\xf6\x24\x1e\xab\xff\xfe\xb1\x53\xff\xff\xb9\xfe\xff\xff\xff\xff\xaa\xab" + bytes(48)]
    for k in range(1, 6):  # both signs of several valid points (other messages: the verdict is False)
        s = OC.Sign(k, msg)
        cases += [s, bytes([s[0] ^ 0x20]) + s[1:]]
    for c in cases:
        assert M.Verify(pk, msg, c) == OC.Verify(pk, msg, c), c.hex()


def test_wide_key_validate_edge_cases():
    """KeyValidate through the two-keys-per-wave kernel (per-call keys, AggregatePKs, AggregateVerify) on small x
    (on-curve points almost all outside G1, off-curve x, both sign bits), valid keys and the fixtures' malformed
    encodings, against the C oracle; and a 515-key AggregatePKs (odd count: the last wave's second half idles)."""
    from bls_mi355x.backend import mi355x_bls as M
    from oracle import bls_oracle_c as OC

    keys = []
    for x in range(1, 24):
        for flag in (0x80, 0xA0):
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= flag
            keys.append(bytes(b))
    keys += [OC.SkToPk(k) for k in (1, 2, 3, 0xDEADBEEF)]
    keys += [b"\xc0" + bytes(47), b"\x40" + bytes(47), bytes(48), b"\x80" + bytes(47)]
    for pk in keys:
        assert M.KeyValidate(pk) == OC.KeyValidate(pk), pk.hex()
    pks = [OC.SkToPk(k) for k in range(1, 516)]
    assert M._AggregatePKs(pks) == OC.AggregatePKs(pks)


def test_pairing_decode_wide_matches_lane_kernel():
    """The pairing APIs' checked decodes (the wide KeyValidate kernel with the identity accepted, the one-wave signature
    check) against the lane kernel's checked decode (bls_point_decode, k_pt_decode): each point is paired with the
    other group's identity, so bls_pairing_check_ex(subgroup) is 1 exactly when the point decodes into its group."""
    import ctypes

    from bls_mi355x import _native
    from oracle import bls_oracle_c as OC

    ctx = _native.context()
    g1s = [b"\xc0" + bytes(47), b"\xe0" + bytes(47), b"\xc0" + bytes(46) + b"\x01", b"\x40" + bytes(47), bytes(48),
           b"\x80" + bytes(47)]
    for x in range(1, 16):  # small x: off the curve, or on it and (almost surely) outside G1
        for flag in (0x80, 0xA0):
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= flag
            g1s.append(bytes(b))
    g1s += [OC.SkToPk(k) for k in (1, 2, 0xDEADBEEF)]
    sig = OC.Sign(77, b"\x42" * 32)
    g2s = [sig, b"\xc0" + bytes(95), b"\xe0" + bytes(95), b"\xc0" + bytes(94) + b"\x01", bytes(96), b"\x80" + bytes(95),
           sig[:1] + b"\xff" * 47 + sig[48:], bytes([sig[0] ^ 0x20]) + sig[1:], sig[:95] + bytes([sig[95] ^ 1])]

    def lane_ok(group, pts):
        ok = (ctypes.c_uint8 * len(pts))()
        ctx.check(ctx.lib.bls_point_decode(ctx.h, group, b"".join(pts), len(pts), 1, ok))
        return [bool(v) for v in ok]

    for p, want in zip(g1s, lane_ok(1, g1s)):
        got = ctx.check(ctx.lib.bls_pairing_check_ex(ctx.h, p, b"\xc0" + bytes(95), 1, 1)) == 1
        assert got == want, p.hex()
    for q, want in zip(g2s, lane_ok(2, g2s)):
        got = ctx.check(ctx.lib.bls_pairing_check_ex(ctx.h, b"\xc0" + bytes(47), q, 1, 1)) == 1
        assert got == want, q.hex()
    assert any(lane_ok(1, g1s)) and not all(lane_ok(1, g1s))


def test_fe_wide_matches_lane_kernel():
    """The six-wave final-exponentiation check (k_fe_wide, hard part in F2 layout) against the one-wave lane kernel
    and known answers without a pairing: FE(f) = 1 for every f in Fp6 (p^6 - 1 divides (p^12 - 1) / r), so
    f conj(f) (in Fp6) and Fp6 elements pass, while a random Fp12 value, f f, and f times a perturbed conjugate
    fail.  Partial counts 1, 2 and 5 (the product inside the kernel)."""
    import ctypes

    from bls_mi355x import _native

    ctx = _native.context()
    rnd = random.Random(0xFE12)

    def raw(c):  # 12 Montgomery-form residues (any residue is some element's Montgomery form)
        return b"".join(v.to_bytes(48, "little") for v in c)

    def conj(c):
        return c[:6] + [(O.P - v) % O.P for v in c[6:]]

    def check(fs, wide):
        out = ctypes.c_int32(-1)
        ctx.check(ctx.lib.bls_test_final_check(ctx.h, b"".join(raw(f) for f in fs), len(fs), wide, ctypes.byref(out)))
        return out.value

    cases = []
    for _ in range(3):
        f = [rnd.randrange(O.P) for _ in range(12)]
        g = [rnd.randrange(O.P) for _ in range(6)] + [0] * 6
        h = [rnd.randrange(O.P) for _ in range(12)]
        cases += [([f], 0), ([g], 1), ([f, conj(f)], 1), ([f, f], 0), ([f, g, conj(f)], 1),
                  ([f, h, conj(f), conj(h), g], 1), ([f, h, conj(f), h, g], 0)]
        bad = conj(f)
        bad[7] = (bad[7] + 1) % O.P
        cases.append(([f, bad], 0))
    cases.append(([[(1 << 406) % O.P] + [0] * 11], 1))  # one (Montgomery radix 2^406)
    for fs, want in cases:
        assert check(fs, 1) == want, (len(fs), want)
        assert check(fs, 0) == want, (len(fs), want)
