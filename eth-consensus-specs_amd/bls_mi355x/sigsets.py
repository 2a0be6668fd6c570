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
would apply the deposit and then reject the block.  So ``try_defer`` looks at
the caller's bytecode: the call is deferred only if its value flows, through
``return`` statements only, into an ``assert`` (``POP_JUMP_IF_TRUE`` followed
by ``LOAD_ASSERTION_ERROR``), and every caller on the way calls exactly the
function below it (no C-level caller such as ``map`` or ``any`` in between);
any other use -- ``if``, ``not``, a comparison, an assignment -- runs the call
at once and returns its real verdict.  The bytecode reading is for Python
3.10 (this image's interpreter); on other versions every call runs at once.
"""
from __future__ import annotations

import contextlib
import dis
import sys
import warnings
from dataclasses import dataclass, field

import numpy as np

from . import batch as _batch

FAV, VERIFY, AV = "fav", "verify", "av"

_CODE_INDEX: dict = {}  # code object -> (instructions, {offset: position})

# Python 3.10 stack effects (pops, pushes) of the opcodes that build call expressions; a span with any other
# opcode is not simulated (the call then runs at once -- never a wrong verdict, only no batching)
_LOADS = {"LOAD_GLOBAL", "LOAD_NAME", "LOAD_FAST", "LOAD_DEREF", "LOAD_CONST", "LOAD_CLOSURE", "LOAD_CLASSDEREF"}
_FIXED = {"LOAD_ATTR": (1, 1), "LOAD_METHOD": (1, 2), "BINARY_SUBSCR": (2, 1), "COMPARE_OP": (2, 1),
          "IS_OP": (2, 1), "CONTAINS_OP": (2, 1), "UNARY_NOT": (1, 1), "UNARY_NEGATIVE": (1, 1),
          "UNARY_INVERT": (1, 1), "UNARY_POSITIVE": (1, 1), "LIST_TO_TUPLE": (1, 1), "GET_ITER": (1, 1),
          "DUP_TOP": (1, 2), "NOP": (0, 0), "DICT_MERGE": (1, 0), "DICT_UPDATE": (1, 0), "LIST_EXTEND": (1, 0),
          "SET_UPDATE": (1, 0), "LIST_APPEND": (1, 0), "SET_ADD": (1, 0), "MAP_ADD": (2, 0)}


def _index(code):
    ent = _CODE_INDEX.get(code)
    if ent is None:
        ins = list(dis.get_instructions(code))
        ent = (ins, {x.offset: i for i, x in enumerate(ins)})
        _CODE_INDEX[code] = ent
    return ent


def _next_ops(code, lasti: int, k: int = 2) -> list[str]:
    """Opnames of the k instructions after the one at byte offset `lasti` ([] if unknown).  TO_BOOL (3.13+,
    before a conditional jump) is skipped: reserved for a future bytecode port, since callee_name only reads
    3.10 bytecode and nothing is deferred on other versions (SignatureSets.version_fallback counts those)."""
    ins, pos = _index(code)
    i = pos.get(lasti)
    if i is None:
        return []
    return [x.opname for x in ins[i + 1:] if x.opname != "TO_BOOL"][:k]


def _pops_pushes(x):
    op, a = x.opname, x.arg
    if op in _LOADS:
        return 0, 1
    if op in _FIXED:
        return _FIXED[op]
    if op.startswith("BINARY_") or op.startswith("INPLACE_"):
        return 2, 1
    if op in ("BUILD_TUPLE", "BUILD_LIST", "BUILD_SET", "BUILD_STRING", "BUILD_SLICE"):
        return a, 1
    if op == "BUILD_MAP":
        return 2 * a, 1
    if op == "BUILD_CONST_KEY_MAP":
        return a + 1, 1
    if op == "CALL_FUNCTION":
        return a + 1, 1
    if op in ("CALL_FUNCTION_KW", "CALL_METHOD"):
        return a + 2, 1
    if op == "CALL_FUNCTION_EX":
        return 2 + (a & 1), 1
    if op == "FORMAT_VALUE":
        return 1 + (1 if (a & 4) else 0), 1
    return None


def callee_name(code, lasti: int) -> str | None:
    """Name of the callable invoked by the call instruction at byte offset `lasti` (Python 3.10 bytecode), or
    None when it cannot be determined: the straight-line span back to the nearest jump target is simulated
    with a symbolic stack whose entries remember the name they were loaded under (``bls.Verify`` ->
    "Verify", ``is_valid_indexed_attestation`` -> itself, ``any`` -> "any")."""
    if sys.version_info[:2] != (3, 10):
        return None
    ins, pos = _index(code)
    i = pos.get(lasti)
    if i is None or not ins[i].opname.startswith("CALL_"):
        return None
    lo = i
    while lo > 0 and not ins[lo].is_jump_target:
        lo -= 1
    stack: list = []  # producer name per entry; the entries below the span are unknown (None)
    for x in ins[lo:i]:
        if "JUMP" in x.opname or x.opname in ("RETURN_VALUE", "FOR_ITER", "SETUP_FINALLY", "SETUP_WITH"):
            stack = []  # control flow inside the span: nothing below is known
            continue
        pp = _pops_pushes(x)
        if pp is None:
            return None
        pops, pushes = pp
        if x.opname == "DUP_TOP":
            top = stack[-1] if stack else None
            stack.append(top)
            continue
        for _ in range(pops):
            if stack:
                stack.pop()
        name = x.argval if x.opname in _LOADS or x.opname in ("LOAD_ATTR", "LOAD_METHOD") else None
        if x.opname == "LOAD_METHOD":
            stack.extend([name, None])  # (method, self) / (NULL, callable)
        else:
            stack.extend([name if isinstance(name, str) else None] * pushes)
    pops, _ = _pops_pushes(ins[i])
    if len(stack) < pops:
        return None
    return stack[-pops]


def result_is_asserted(frame, callee: str) -> bool:
    """True iff the value that the call to `callee` (the function `frame` is executing a call into) returns
    reaches an ``assert`` through ``return`` statements only, walking up the callers.  At every level the
    caller's instruction must be a call of exactly that function: a C-level caller in between (``map``,
    ``any``, ``sorted`` ...) leaves no Python frame, so ``assert any(map(bls.Verify, ...))`` shows a call of
    ``any`` there and the verdict is computed at once."""
    depth = 0
    while frame is not None and depth < 32:
        if callee_name(frame.f_code, frame.f_lasti) != callee:
            return False
        ops = _next_ops(frame.f_code, frame.f_lasti)
        if not ops:
            return False
        if ops[0] == "RETURN_VALUE":
            callee = frame.f_code.co_name
            frame = frame.f_back
            depth += 1
            continue
        return (ops[0].startswith("POP_JUMP") and ops[0].endswith("IF_TRUE") and len(ops) > 1
                and ops[1] == "LOAD_ASSERTION_ERROR")
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
        self.version_fallback = 0  # of those, calls run at once only because this interpreter is not 3.10

    def try_defer(self, kind: str, args) -> bool:
        """Called by the shim's Verify / FastAggregateVerify / AggregateVerify (bls.py ``_defer``): record the
        call and return True when its result is only asserted; otherwise False (the shim verifies at once)."""
        shim_fn = sys._getframe(2)  # try_defer <- bls._defer <- bls.Verify / ...
        caller = shim_fn.f_back  # only_with_bls's wrapper (named like the shim function), calling it as `fn`
        callee = "fn" if caller is not None and caller.f_code.co_name == shim_fn.f_code.co_name else \
            shim_fn.f_code.co_name
        if sys.version_info[:2] != (3, 10):  # the bytecode walk reads 3.10 only: batching is lost, say so once
            self.eager += 1
            self.version_fallback += 1
            if self.version_fallback == 1:
                warnings.warn(f"bls_mi355x.sigsets: deferred() batching needs Python 3.10 bytecode; on "
                              f"{sys.version_info[0]}.{sys.version_info[1]} every verify call runs at once",
                              RuntimeWarning, stacklevel=4)
            return False
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
