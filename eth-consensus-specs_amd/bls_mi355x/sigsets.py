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

Only calls whose result is *asserted* are deferred.  The spec asserts most
verify results (``assert bls.Verify(...)`` in process_randao, exits, slashings;
``assert is_valid_indexed_attestation(...)`` -> ``return
bls.FastAggregateVerify(...)``), and a failed assert rejects the whole block
whether it fires at the call or at the end of the block.  But some sites
*branch* on the result: ``apply_deposit``'s ``if bls.Verify(...)``
(specs/phase0/beacon-chain.md:2055) and Electra's ``if
is_valid_deposit_signature(...)`` (specs/electra/beacon-chain.md:932,1555):
an invalid proof of possession there skips the deposit and the block stays
valid (test_process_deposit.py:255-287).  Returning a recorded True there
would apply the deposit and then reject the block.  So ``try_defer`` reads the
caller's *source* (``ast`` over ``linecache``, the same lines tracebacks show:
the generated pyspec modules are ordinary files): the call is deferred only if
every call of that function on the caller's current line is the test of an
``assert`` statement, or the value of a ``return`` statement whose function's
own call site (one frame up) satisfies the same rule, and so on.  Any other use
-- ``if``, ``not``, a comparison, an argument, an assignment, a conditional
expression, a lambda or a C-level caller such as ``map`` or ``any`` in between
(it leaves no frame, so the next frame's line calls ``any``, not the function
below) -- runs the call at once and returns its real verdict, as does a caller
whose source cannot be read.  Nothing depends on the interpreter's bytecode,
so every CPython the reference supports (``requires-python = ">=3.10, <3.14"``,
pyproject.toml:10) batches the same calls; on 3.11+ the instruction's source
position narrows the match to the exact call expression.
"""
from __future__ import annotations

import ast
import contextlib
import itertools
import linecache
import sys
from dataclasses import dataclass, field

import numpy as np

from . import batch as _batch

FAV, VERIFY, AV = "fav", "verify", "av"

_AST_CACHE: dict = {}  # filename -> (linecache lines object, {callee name: [(Call node, parent node)]})


def _call_index(frame):
    """Call nodes of the frame's source file by callee name (``bls.Verify(...)`` -> "Verify", ``fn(...)`` ->
    "fn"), each with its parent node; None when the source is not available."""
    fn = frame.f_code.co_filename
    lines = linecache.getlines(fn, frame.f_globals)
    if not lines:
        return None
    ent = _AST_CACHE.get(fn)
    if ent is not None and ent[0] is lines:
        return ent[1]
    try:
        tree = ast.parse("".join(lines), fn)
    except (SyntaxError, ValueError):
        return None
    index: dict = {}
    for parent in ast.walk(tree):
        for child in ast.iter_child_nodes(parent):
            if isinstance(child, ast.Call):
                f = child.func
                name = f.id if isinstance(f, ast.Name) else (f.attr if isinstance(f, ast.Attribute) else None)
                if name:
                    index.setdefault(name, []).append((child, parent))
    _AST_CACHE[fn] = (lines, index)
    return index


def _position(frame):
    """(lineno, end_lineno, col, end_col) of the frame's current instruction (CPython 3.11+), else None."""
    positions = getattr(frame.f_code, "co_positions", None)
    if positions is None or frame.f_lasti < 0:
        return None
    try:
        return next(itertools.islice(positions(), frame.f_lasti // 2, None))
    except (StopIteration, ValueError):
        return None


def call_sites(frame, callee: str) -> list:
    """The calls of `callee` in the frame's source that its current instruction can be: every call of that name
    whose lines span the frame's line -- on 3.11+ only the one whose span is the instruction's, when exactly one
    is."""
    index = _call_index(frame)
    if index is None:
        return []
    ln = frame.f_lineno
    cands = [(c, p) for c, p in index.get(callee, ()) if c.lineno <= ln <= (c.end_lineno or c.lineno)]
    pos = _position(frame)
    if pos is not None and len(cands) > 1:
        exact = [(c, p) for c, p in cands if (c.lineno, c.end_lineno, c.col_offset, c.end_col_offset) == tuple(pos)]
        if len(exact) == 1:
            return exact
    return cands


def _use(call, parent) -> str:
    if isinstance(parent, ast.Assert) and parent.test is call:
        return "assert"
    if isinstance(parent, ast.Return) and parent.value is call:
        return "return"
    return "other"


def result_is_asserted(frame, callee: str) -> bool:
    """True iff the value that the call to `callee` (the function `frame` is executing a call into) returns
    reaches an ``assert`` through ``return`` statements only, walking up the callers.  At every level every
    call of that function on the caller's current line must be such a use: a C-level caller in between (``map``,
    ``any``, ``sorted`` ...) leaves no Python frame, so ``assert any(map(bls.Verify, ...))`` shows calls of
    ``any`` and ``map`` there, not of ``Verify``, and the verdict is computed at once."""
    depth = 0
    while frame is not None and depth < 32:
        sites = call_sites(frame, callee)
        if not sites:
            return False
        uses = {_use(c, p) for c, p in sites}
        if uses == {"assert"}:
            return True
        if uses != {"return"}:
            return False
        callee = frame.f_code.co_name
        frame = frame.f_back
        depth += 1
    return False


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
        self.eager = 0  # verify calls inside deferred() that ran at once (result not asserted)

    def try_defer(self, kind: str, args) -> bool:
        """Called by the shim's Verify / FastAggregateVerify / AggregateVerify (bls.py ``_defer``): record the
        call and return True when its result is only asserted; otherwise False (the shim verifies at once)."""
        shim_fn = sys._getframe(2)  # try_defer <- bls._defer <- bls.Verify / ...
        caller = shim_fn.f_back  # only_with_bls's wrapper (named like the shim function), calling it as `fn`
        callee = "fn" if caller is not None and caller.f_code.co_name == shim_fn.f_code.co_name else \
            shim_fn.f_code.co_name
        if not result_is_asserted(caller, callee):
            self.eager += 1
            return False
        {VERIFY: self.add_verify, FAV: self.add_fast_aggregate_verify, AV: self.add_aggregate_verify}[kind](*args)
        return True

    def __len__(self):
        return len(self.sets)

    def _add(self, s: _Set) -> int:
        self.sets.append(s)
        return len(self.sets) - 1

    @staticmethod
    def _wellformed(s: _Set) -> _Set:
        """Keys other than 48 bytes or a signature other than 96 bytes: False, as the per-call path returns."""
        if len(s.signature) != 96 or any(k is not None and len(k) != 48 for k in s.pubkeys):
            return _Set(s.kind, malformed=True)
        return s

    def add_fast_aggregate_verify(self, pubkeys, message, signature) -> int:
        try:
            return self._add(self._wellformed(_Set(FAV, [_b(k) for k in pubkeys], [_b(message)], _b(signature))))
        except Exception:
            return self._add(_Set(FAV, malformed=True))

    def add_fast_aggregate_verify_indexed(self, indices, message32, signature) -> int:
        """Registry indices instead of key bytes (is_valid_indexed_attestation already holds them)."""
        try:
            idx = np.ascontiguousarray(indices, dtype=np.uint32)
            return self._add(self._wellformed(_Set(FAV, [None] * idx.size, [_b(message32)], _b(signature),
                                                   indices=idx)))
        except Exception:
            return self._add(_Set(FAV, malformed=True))

    def add_verify(self, pubkey, message, signature) -> int:
        try:
            return self._add(self._wellformed(_Set(VERIFY, [_b(pubkey)], [_b(message)], _b(signature))))
        except Exception:
            return self._add(_Set(VERIFY, malformed=True))

    def add_aggregate_verify(self, pubkeys, messages, signature) -> int:
        try:
            return self._add(self._wellformed(_Set(AV, [_b(k) for k in pubkeys], [_b(m) for m in messages],
                                                   _b(signature))))
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
    """Within the block, ``bls_mi355x.bls.Verify/FastAggregateVerify/AggregateVerify`` calls whose result is
    asserted record their arguments into a ``SignatureSets`` and return True (every other call runs at once,
    see the module docstring); at exit the sets are verified in batches and, with ``check``, an
    AssertionError names the first invalid one.  Yields the collector (its ``results`` attribute holds the
    verdicts after the block)."""
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
