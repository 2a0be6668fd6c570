"""ctypes binding of oracle/bls_oracle.c -- TEST INFRASTRUCTURE ONLY.

The C restatement of the BLS12-381 oracle: a fast CPU parity checker for
``tests/`` and the ``cpu_baseline`` leg of ``bench.py`` (kind "port": the
build's own CPU back end of the same verification semantics, timed on all
host cores).  The product path never imports it.

Same wrapper semantics as ``oracle/bls_oracle.py`` (reference
``E/utils/bls.py:141-221,395-397``): verification functions return bools and
swallow every rejection; ``Aggregate``/``AggregatePKs``/``Sign``/``SkToPk``
raise ``ValueError`` where the reference raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libblsoracle.so")
_lib = None

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        p, sz = C.c_char_p, C.c_size_t
        sigs = {
            "oc_key_validate": [p],
            "oc_verify": [p, p, sz, p],
            "oc_fast_aggregate_verify": [p, sz, p, sz, p],
            "oc_aggregate_verify": [p, sz, p, C.POINTER(C.c_size_t), p],
            "oc_aggregate": [p, sz, p],
            "oc_aggregate_pks": [p, sz, p],
            "oc_sign": [p, p, sz, p],
            "oc_sk_to_pk": [p, p],
            "oc_hash_to_g2": [p, sz, p, sz, p],
            "oc_g2_subgroup_both": [p],
            "oc_pairing": [p, p, p],
            "oc_registry_generate": [C.c_uint64, sz, p],
            "oc_fav_batch_resident": [p, C.c_void_p, C.c_void_p, sz, p, p, p, C.c_int, C.c_int, p],
            "oc_sign_batch": [p, p, sz, C.c_int, p],
        }
        for name, args in sigs.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = C.c_int
        _lib = L
    return _lib


def _b(x) -> bytes:
    return bytes(x)


def KeyValidate(pk) -> bool:
    pk = _b(pk)
    return len(pk) == 48 and lib().oc_key_validate(pk) == 1


def Verify(pk, msg, sig) -> bool:
    pk, msg, sig = _b(pk), _b(msg), _b(sig)
    if len(pk) != 48 or len(sig) != 96:
        return False
    return lib().oc_verify(pk, msg, len(msg), sig) == 1


def FastAggregateVerify(pks, msg, sig) -> bool:
    pks = [_b(k) for k in pks]
    msg, sig = _b(msg), _b(sig)
    if any(len(k) != 48 for k in pks) or len(sig) != 96:
        return False
    return lib().oc_fast_aggregate_verify(b"".join(pks), len(pks), msg, len(msg), sig) == 1


def AggregateVerify(pks, msgs, sig) -> bool:
    pks = [_b(k) for k in pks]
    msgs = [_b(m) for m in msgs]
    sig = _b(sig)
    if len(pks) != len(msgs) or any(len(k) != 48 for k in pks) or len(sig) != 96:
        return False
    lens = (C.c_size_t * max(len(msgs), 1))(*[len(m) for m in msgs])
    return lib().oc_aggregate_verify(b"".join(pks), len(pks), b"".join(msgs), lens, sig) == 1


def Aggregate(sigs) -> bytes:
    sigs = [_b(s) for s in sigs]
    out = C.create_string_buffer(96)
    if any(len(s) != 96 for s in sigs) or lib().oc_aggregate(b"".join(sigs), len(sigs), out) != 1:
        raise ValueError("Aggregate: empty list or invalid signature")
    return out.raw


def AggregatePKs(pks) -> bytes:
    pks = [_b(k) for k in pks]
    out = C.create_string_buffer(48)
    if any(len(k) != 48 for k in pks) or lib().oc_aggregate_pks(b"".join(pks), len(pks), out) != 1:
        raise ValueError("AggregatePKs: empty list or invalid pubkey")
    return out.raw


def _sk32(sk) -> bytes:
    if isinstance(sk, int):
        if not 0 <= sk < 1 << 256:
            raise ValueError("secret key out of range")
        return sk.to_bytes(32, "big")
    return _b(sk)


def Sign(sk, msg) -> bytes:
    msg = _b(msg)
    out = C.create_string_buffer(96)
    if lib().oc_sign(_sk32(sk), msg, len(msg), out) != 1:
        raise ValueError("secret key out of range")
    return out.raw


def SkToPk(sk) -> bytes:
    out = C.create_string_buffer(48)
    if lib().oc_sk_to_pk(_sk32(sk), out) != 1:
        raise ValueError("secret key out of range")
    return out.raw


def hash_to_g2(msg, dst=DST_POP) -> bytes:
    msg, dst = _b(msg), _b(dst)
    out = C.create_string_buffer(96)
    if lib().oc_hash_to_g2(msg, len(msg), dst, len(dst), out) != 1:
        raise ValueError("DST too long")
    return out.raw


def g2_subgroup_both(sig) -> int:
    return lib().oc_g2_subgroup_both(_b(sig))


def pairing(pk, sig) -> bytes:
    out = C.create_string_buffer(576)
    if lib().oc_pairing(_b(pk), _b(sig), out) != 1:
        raise ValueError("undecodable point")
    return out.raw


def registry_generate(first_sk: int, n: int) -> bytes:
    """Affine registry keys sk = first_sk .. first_sk+n-1, 96 bytes each (x || y)."""
    out = C.create_string_buffer(96 * n)
    lib().oc_registry_generate(first_sk, n, out)
    return out.raw


def sign_batch(sks32: bytes, msgs32: bytes, threads: int) -> bytes:
    """B signatures sk_b * H(msg_b) (sks 32-byte big-endian, 32-byte messages)."""
    B = len(msgs32) // 32
    out = C.create_string_buffer(96 * max(B, 1))
    if lib().oc_sign_batch(sks32, msgs32, B, threads, out) != 1:
        raise ValueError("secret key out of range")
    return out.raw[:96 * B]


def fav_batch_resident(reg96: bytes, idx, offs, msgs32: bytes, sigs96: bytes, seed32: bytes, mode: int,
                       threads: int):
    """B registry-indexed FastAggregateVerify calls (mode 0 per call, 1 RLC batch); list of bools."""
    import numpy as np

    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    B = offs.size - 1
    out = C.create_string_buffer(max(B, 1))
    lib().oc_fav_batch_resident(reg96, idx.ctypes.data, offs.ctypes.data, B, msgs32, sigs96, seed32, mode,
                                threads, out)
    return [bool(x) for x in out.raw[:B]]
