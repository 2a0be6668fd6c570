"""MI355X (gfx950) BLS12-381 backend for the Ethereum consensus pyspec.

``bls_mi355x.bls`` mirrors ``eth2spec.utils.bls``; ``bls_mi355x.batch`` is the
registry-indexed throughput API.  All compute runs in libblsmi355x.so on the
GPU (hand-written HIP kernels); nothing falls back to the CPU.
"""
from . import _native, backend, batch, bls  # noqa: F401
from ._native import NativeError, NativeUnavailable  # noqa: F401
from .backend import mi355x_bls  # noqa: F401

__all__ = ["bls", "batch", "backend", "mi355x_bls", "NativeError", "NativeUnavailable"]
