#!/usr/bin/env python3
"""Stage-by-stage comparison of the one-wave hash_to_G2 (bls_test_h2c_wide_stages) with the Python oracle."""
import ctypes
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "eth-consensus-specs_amd")):
    sys.path.insert(0, p)
from bls_mi355x import _native  # noqa: E402
from oracle import bls_oracle as O  # noqa: E402

DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


def main():
    ctx = _native.context()
    for j in range(int(os.environ.get("N", "3"))):
        msg = hashlib.sha256(b"wide" + j.to_bytes(4, "little")).digest()
        buf = ctypes.create_string_buffer(72 * 48 + 320 * 4)
        ctx.check(ctx.lib.bls_test_h2c_wide_stages(ctx.h, msg, buf))
        v = [int.from_bytes(buf.raw[48 * k: 48 * k + 48], "little") for k in range(45)]
        u = O.hash_to_field_fp2(msg, 2, DST)
        res = {}
        for h in range(2):
            b = 10 * h
            res[f"u{h}"] = (v[b], v[b + 1]) == u[h]
            xy = O.map_to_curve_sswu(u[h])
            res[f"sswu{h}"] = ((v[b + 2], v[b + 3]), (v[b + 4], v[b + 5])) == xy
            iso = O.iso_map(xy)
            res[f"iso{h}"] = ((v[b + 6], v[b + 7]), (v[b + 8], v[b + 9])) == (iso[0], iso[1])
        q = O.g2_add(O.iso_map(O.map_to_curve_sswu(u[0])), O.iso_map(O.map_to_curve_sswu(u[1])))
        res["Q"] = ((v[20], v[21]), (v[22], v[23])) == (q[0], q[1])
        m = O.g2_mul(q, 0xD201000000010000)
        res["M"] = ((v[24], v[25]), (v[26], v[27])) == (m[0], m[1])
        hh = O.clear_cofactor_g2(q)
        res["H"] = ((v[28], v[29]), (v[30], v[31])) == (hh[0], hh[1])
        res["flags"] = hex(v[32])
        res["Q_lane"] = ((v[33], v[34]), (v[35], v[36])) == (q[0], q[1])
        res["z1z1"] = (v[37], v[38]) == (v[39], v[40])
        res["u1"] = (v[41], v[42]) == (v[43], v[44])
        print(j, res, flush=True)
        w = [int.from_bytes(buf.raw[48 * k: 48 * k + 48], "little") for k in range(52, 70)]
        f2 = [(w[2 * q], w[2 * q + 1]) for q in range(6)]
        f2 = [(w[2 * q], w[2 * q + 1]) for q in range(9)]
        pz, qz, zz, hh, qzz, rlz, sq, z1, z2 = f2
        print("SQ ok", sq == O.f2_sqr(O.f2_add(pz, qz)), "Z1 ok", z1 == O.f2_sqr(pz), "Z2 ok", z2 == O.f2_sqr(qz), flush=True)
        print("ZZ == 2 Pz Qz:", zz == O.f2_muls(O.f2_mul(pz, qz), 2), " Q.z == ZZ H:", qzz == O.f2_mul(zz, hh),
              " rl.z == 2 Pz Qz H:", rlz == O.f2_mul(O.f2_muls(O.f2_mul(pz, qz), 2), hh), " Q.z == -rl.z:", qzz == O.f2_neg(rlz))
        print("VALS", [hex(x) for x in w], flush=True)
        import struct
        raw = struct.unpack("<320I", buf.raw[72 * 48: 72 * 48 + 1280])
        for name, b in (("ZZ1", 0), ("SQ1", 64), ("S121", 128), ("Z11", 192), ("Z21", 256)):
            print(name, " ".join("%08x" % raw[b + l] for l in range(64)), flush=True)
        if not res["sswu0"]:
            print("  sswu0 got", hex(v[2])[:20], "want", hex(O.map_to_curve_sswu(u[0])[0][0])[:20])


if __name__ == "__main__":
    main()
