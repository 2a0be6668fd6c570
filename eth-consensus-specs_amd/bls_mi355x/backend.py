"""The MI355X BLS backend object, attribute-compatible with the milagro
binding the reference selects by default (``fastest_bls`` /
``milagro_bls`` in E/utils/bls.py:57-68 with E = tests/core/pyspec/eth2spec).

Attribute names and argument meanings follow milagro_bls_binding:
``Sign(sk_bytes32, msg)``, ``SkToPk(sk_bytes32)``, ``Verify``,
``FastAggregateVerify``, ``AggregateVerify``, ``Aggregate``,
``_AggregatePKs``, plus ``KeyValidate``.  Functions the reference's binding
raises from (Sign, SkToPk, Aggregate, _AggregatePKs) raise ``ValueError`` on
invalid input here; the verify family returns ``False``.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

from . import _native

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


def _b(x) -> bytes:
    return bytes(x)


def _ctx():
    return _native.context()


class mi355x_bls:  # noqa: N801 -- mirrors the reference's backend class naming
    """Backend object assigned to ``bls`` by ``use_mi355x()``."""

    # -- signature API -------------------------------------------------
    @staticmethod
    def Sign(SK: bytes, message: bytes) -> bytes:
        c = _ctx()
        sk = _b(SK)
        if len(sk) != 32:
            raise ValueError("secret key must be 32 bytes")
        out = ctypes.create_string_buffer(96)
        msg = _b(message)
        if c.check(c.lib.bls_sign(c.h, sk, msg, len(msg), out)) != 1:
            raise ValueError("invalid secret key")
        return out.raw

    @staticmethod
    def SkToPk(SK: bytes) -> bytes:
        c = _ctx()
        sk = _b(SK)
        if len(sk) != 32:
            raise ValueError("secret key must be 32 bytes")
        out = ctypes.create_string_buffer(48)
        if c.check(c.lib.bls_sk_to_pk(c.h, sk, out)) != 1:
            raise ValueError("invalid secret key")
        return out.raw

    @staticmethod
    def KeyValidate(PK: bytes) -> bool:
        pk = _b(PK)
        if len(pk) != 48:
            return False
        c = _ctx()
        return c.check(c.lib.bls_key_validate(c.h, pk)) == 1

    @staticmethod
    def Verify(PK: bytes, message: bytes, signature: bytes) -> bool:
        pk, sig, msg = _b(PK), _b(signature), _b(message)
        if len(pk) != 48 or len(sig) != 96:
            return False
        c = _ctx()
        return c.check(c.lib.bls_verify(c.h, pk, msg, len(msg), sig)) == 1

    @staticmethod
    def FastAggregateVerify(PKs: Sequence[bytes], message: bytes, signature: bytes) -> bool:
        pks = [_b(p) for p in PKs]
        sig, msg = _b(signature), _b(message)
        if len(sig) != 96 or any(len(p) != 48 for p in pks):
            return False
        if not pks:
            return False
        c = _ctx()
        return c.check(c.lib.bls_fast_aggregate_verify(c.h, b"".join(pks), len(pks), msg, len(msg), sig)) == 1

    @staticmethod
    def AggregateVerify(PKs: Sequence[bytes], messages: Sequence[bytes], signature: bytes) -> bool:
        pks = [_b(p) for p in PKs]
        msgs = [_b(m) for m in messages]
        sig = _b(signature)
        if len(sig) != 96 or any(len(p) != 48 for p in pks):
            return False
        if not pks or len(pks) != len(msgs):
            return False
        lens = (ctypes.c_size_t * len(msgs))(*[len(m) for m in msgs])
        c = _ctx()
        return c.check(c.lib.bls_aggregate_verify(c.h, b"".join(pks), len(pks), b"".join(msgs), lens, sig)) == 1

    @staticmethod
    def Aggregate(signatures: Sequence[bytes]) -> bytes:
        sigs = [_b(s) for s in signatures]
        if not sigs:
            raise ValueError("Aggregate: empty signature list")
        if any(len(s) != 96 for s in sigs):
            raise ValueError("Aggregate: signatures must be 96 bytes")
        c = _ctx()
        out = ctypes.create_string_buffer(96)
        if c.check(c.lib.bls_aggregate(c.h, b"".join(sigs), len(sigs), out)) != 1:
            raise ValueError("Aggregate: invalid signature")
        return out.raw

    @staticmethod
    def _AggregatePKs(PKs: Sequence[bytes]) -> bytes:
        pks = [_b(p) for p in PKs]
        if not pks:
            raise ValueError("AggregatePKs: empty pubkey list")
        if any(len(p) != 48 for p in pks):
            raise ValueError("AggregatePKs: pubkeys must be 48 bytes")
        c = _ctx()
        out = ctypes.create_string_buffer(48)
        if c.check(c.lib.bls_aggregate_pks(c.h, b"".join(pks), len(pks), out)) != 1:
            raise ValueError("AggregatePKs: invalid pubkey")
        return out.raw

    # -- extras used by the spec helpers / tests -------------------------
    @staticmethod
    def hash_to_G2(message: bytes, dst: bytes = DST_POP) -> bytes:
        c = _ctx()
        msg, d = _b(message), _b(dst)
        out = ctypes.create_string_buffer(96)
        c.check(c.lib.bls_hash_to_g2(c.h, msg, len(msg), d, len(d), out))
        return out.raw
