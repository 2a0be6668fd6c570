"""Deferred signature sets: cross-call batching at the spec caller.

The spec verifies every signature synchronously: ``process_attestation`` ->
``is_valid_indexed_attestation`` -> ``bls.FastAggregateVerify``
(specs/phase0/beacon-chain.md:776-790, called per attestation from
``process_operations``, :1920-1928) and ``process_sync_aggregate`` ->
``eth_fast_aggregate_verify`` (specs/altair/beacon-chain.md:575-610).  A block
therefore pays one pairing check per attestation.  ``SignatureSets`` collects
the calls instead and checks them together:

* FastAggregateVerify / Verify whose keys are resident in the HBM registry
  (looked up by pubkey bytes, or given as indices) and whose message is a
  32-byte signing root -> one ``bls_fav_batch_indexed`` call (one random-
  linear-combination pairing check, bisection on failure);
* Verify with other keys or messages, and AggregateVerify -> one
  ``bls_aggregate_verify_batch`` call (Verify(pk, m, s) is AggregateVerify
  with one pair: same KeyValidate, same pairing equation);
* FastAggregateVerify with non-resident keys -> the per-call path (its
  identity-aggregate rejection has no AggregateVerify equivalent).

Every set's verdict equals the per-call verdict of ``bls_mi355x.bls``
(exceptions -> False).  ``deferred()`` routes the shim's verify functions into
a collector for the duration of a ``with`` block -- e.g. one
``state_transition`` -- and raises ``AssertionError`` at exit if any recorded
signature is invalid, which is the spec's outcome for that block.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field

import numpy as np

from . import batch as _batch

FAV, VERIFY, AV = "fav", "verify", "av"


@dataclass
class _Set:
    kind: str
    pubkeys: list = field(default_factory=list)  # bytes (48) each, or None when given as indices
    messages: list = field(default_factory=list)
    signature: bytes = b""
    indices: np.ndarray | None = None
    malformed: bool = False


def _b(x) -> bytes:
    return bytes(x)


class SignatureSets:
    """Collects verify calls; ``verify()`` checks them in as few device batches as possible."""

    def __init__(self, registry: _batch.Registry | None = None, ctx=None):
        self.registry = registry
        self.ctx = ctx
        self.sets: list[_Set] = []

    def __len__(self):
        return len(self.sets)

    def _add(self, s: _Set) -> int:
        self.sets.append(s)
        return len(self.sets) - 1

    def add_fast_aggregate_verify(self, pubkeys, message, signature) -> int:
        try:
            return self._add(_Set(FAV, [_b(k) for k in pubkeys], [_b(message)], _b(signature)))
        except Exception:
            return self._add(_Set(FAV, malformed=True))

    def add_fast_aggregate_verify_indexed(self, indices, message32, signature) -> int:
        """Registry indices instead of key bytes (is_valid_indexed_attestation already holds them)."""
        try:
            idx = np.ascontiguousarray(indices, dtype=np.uint32)
            return self._add(_Set(FAV, [None] * idx.size, [_b(message32)], _b(signature), indices=idx))
        except Exception:
            return self._add(_Set(FAV, malformed=True))

    def add_verify(self, pubkey, message, signature) -> int:
        try:
            return self._add(_Set(VERIFY, [_b(pubkey)], [_b(message)], _b(signature)))
        except Exception:
            return self._add(_Set(VERIFY, malformed=True))

    def add_aggregate_verify(self, pubkeys, messages, signature) -> int:
        try:
            return self._add(_Set(AV, [_b(k) for k in pubkeys], [_b(m) for m in messages], _b(signature)))
        except Exception:
            return self._add(_Set(AV, malformed=True))

    # ---- planning (host only) --------------------------------------------
    def _resident(self, s: _Set) -> np.ndarray | None:
        if s.indices is not None:
            return s.indices
        if self.registry is None:
            return None
        return self.registry.indices(s.pubkeys)

    def plan(self):
        """(indexed, av, single): set ids per execution route, plus the indices of the indexed ones."""
        indexed, av, single = [], [], []
        for i, s in enumerate(self.sets):
            if s.malformed:
                continue
            if s.kind in (FAV, VERIFY) and len(s.messages[0]) == 32 and len(s.signature) == 96 and s.pubkeys:
                idx = self._resident(s)
                if idx is not None:
                    indexed.append((i, idx))
                    continue
            if s.kind == FAV:
                single.append(i)
            else:
                av.append(i)
        return indexed, av, single

    # ---- execution ---------------------------------------------------------
    def verify(self) -> list[bool]:
        out = [False] * len(self.sets)
        indexed, av, single = self.plan()
        if indexed:
            ids = [i for i, _ in indexed]
            idx = np.concatenate([x for _, x in indexed]).astype(np.uint32)
            offs = _batch.offsets_from_lengths([x.size for _, x in indexed])
            msgs = b"".join(self.sets[i].messages[0] for i in ids)
            sigs = b"".join(self.sets[i].signature for i in ids)
            v = _batch.fast_aggregate_verify_batch(idx, offs, msgs, sigs, ctx=self.ctx)
            for i, ok in zip(ids, v):
                out[i] = bool(ok)
        if av:
            sets = [self.sets[i] for i in av]
            v = _batch.aggregate_verify_batch([s.pubkeys for s in sets], [s.messages for s in sets],
                                              [s.signature for s in sets], ctx=self.ctx)
            for i, ok in zip(av, v):
                out[i] = bool(ok)
        if single:
            from .backend import mi355x_bls

            for i in single:
                s = self.sets[i]
                try:
                    out[i] = bool(mi355x_bls.FastAggregateVerify(s.pubkeys, s.messages[0], s.signature))
                except Exception:
                    out[i] = False
        return out

    def clear(self):
        self.sets = []


@contextlib.contextmanager
def deferred(registry: _batch.Registry | None = None, ctx=None, check: bool = True):
    """Within the block, ``bls_mi355x.bls.Verify/FastAggregateVerify/AggregateVerify`` record their
    arguments into a ``SignatureSets`` and return True; at exit the sets are verified in batches and,
    with ``check``, an AssertionError names the first invalid one.  Yields the collector (its
    ``results`` attribute holds the verdicts after the block)."""
    from . import bls as shim

    sets = SignatureSets(registry, ctx)
    prev = shim._collector
    shim._collector = sets
    try:
        yield sets
    finally:
        shim._collector = prev
    sets.results = sets.verify()
    if check and not all(sets.results):
        bad = sets.results.index(False)
        raise AssertionError(f"signature set {bad} ({sets.sets[bad].kind}) is invalid")
