"""ctypes binding of libblsmi355x.so (C ABI: include/blsmi355x.h).

The library is the only compute path.  If it cannot be loaded, or no GPU
context can be created, every call raises ``NativeUnavailable`` -- there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

HW_QUEUES = 24  # 10 FAV jobs x 2 streams + the fallback and per-call streams share them with the default/copy streams


def hw_queue_policy() -> None:
    """The library keeps up to BLS_FAV_JOBS_INIT x BLS_JOB_STREAMS streams busy; with HIP's default of 4 hardware queues per
    process, streams share queues and a long one-lane-per-item kernel blocks every kernel queued behind it
    (measured: 687k -> 838k FAV/s at 8+ queues; 5 jobs: 1.00M at 16, 1.02M at 20).  HIP reads
    GPU_MAX_HW_QUEUES once, when it starts, so this sets it at import -- only when the variable is unset (an
    explicit setting is kept) and unless BLSMI355X_KEEP_HW_QUEUES is set.  The C library itself never changes
    the process environment (other hosts set the variable themselves)."""
    if os.environ.get("BLSMI355X_KEEP_HW_QUEUES") or "GPU_MAX_HW_QUEUES" in os.environ:
        return
    os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)


hw_queue_policy()

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BLSMI355X_LIB", os.path.join(os.path.dirname(_HERE), "libblsmi355x.so"))

BLS_E_DEVICE = -1
BLS_E_ARG = -2
BLS_E_NOREG = -3


class NativeUnavailable(RuntimeError):
    """libblsmi355x.so missing or no usable MI355X device."""


class NativeError(RuntimeError):
    """The device library reported an internal/device error (negative code)."""


_u8p = ctypes.c_char_p
_sz = ctypes.c_size_t
_vp = ctypes.c_void_p
_ip = ctypes.c_int

_SIGS = {
    "bls_ctx_create": (_ip, [_ip, ctypes.POINTER(_vp)]),
    "bls_ctx_destroy": (None, [_vp]),
    "bls_last_error": (ctypes.c_char_p, [_vp]),
    "bls_device_info": (_ip, [_vp, ctypes.c_char_p, _sz, ctypes.POINTER(_ip)]),
    "bls_verify": (_ip, [_vp, _u8p, _u8p, _sz, _u8p]),
    "bls_fast_aggregate_verify": (_ip, [_vp, _u8p, _sz, _u8p, _sz, _u8p]),
    "bls_aggregate_verify": (_ip, [_vp, _u8p, _sz, _u8p, ctypes.POINTER(_sz), _u8p]),
    "bls_aggregate": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_aggregate_pks": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_key_validate": (_ip, [_vp, _u8p]),
    "bls_sign": (_ip, [_vp, _u8p, _u8p, _sz, _vp]),
    "bls_sk_to_pk": (_ip, [_vp, _u8p, _vp]),
    "bls_hash_to_g2": (_ip, [_vp, _u8p, _sz, _u8p, _sz, _vp]),
    "bls_registry_load": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_registry_size": (_sz, [_vp]),
    "bls_fav_batch_indexed": (_ip, [_vp, _vp, _vp, _sz, _u8p, _u8p, _vp]),
    "bls_verify_batch_indexed": (_ip, [_vp, _vp, _sz, _u8p, _u8p, _vp]),
    "bls_aggregate_verify_batch": (_ip, [_vp, _u8p, _u8p, _vp, _vp, _sz, _u8p, _vp]),
    "bls_registry_append": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_signing_roots": (_ip, [_vp, _u8p, _u8p, _sz, _sz, _vp]),
    "bls_merkleize": (_ip, [_vp, _u8p, _sz, _ip, _vp]),
    "bls_pairing_check": (_ip, [_vp, _u8p, _u8p, _sz]),
    "bls_g1_multi_exp": (_ip, [_vp, _u8p, _u8p, _sz, _vp]),
    "bls_sign_batch": (_ip, [_vp, _u8p, _u8p, _sz, _vp]),
    "bls_sk_to_pk_batch": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_dev_alloc": (_vp, [_vp, _sz]),
    "bls_dev_free": (_ip, [_vp, _vp]),
    "bls_h2d": (_ip, [_vp, _vp, _vp, _sz]),
    "bls_d2h": (_ip, [_vp, _vp, _vp, _sz]),
    "bls_sync": (_ip, [_vp]),
    "bls_fav_batch_partial_dev": (_ip, [_vp, _vp, _vp, _sz, _vp, _vp, _u8p, _vp]),
    "bls_partials_check": (_ip, [_vp, _u8p, _sz]),
    "bls_fav_batch_finish_dev": (_ip, [_vp, _ip, _vp]),
    "bls_fav_job_submit_dev": (_ip, [_vp, _ip, _vp, _vp, _sz, _vp, _vp, _u8p]),
    "bls_fav_job_partial": (_ip, [_vp, _ip, _vp]),
    "bls_fav_job_check": (_ip, [_vp, _ip, _u8p, _sz]),
    "bls_fav_job_check_own": (_ip, [_vp, _ip]),
    "bls_test_miller_forms": (_ip, [_vp, _u8p, _u8p, _sz, _u8p]),
    "bls_fav_job_finish_dev": (_ip, [_vp, _ip, _ip, _vp]),
    "bls_registry_generate": (_ip, [_vp, ctypes.c_uint64, _sz, _vp]),
    "bls_last_fallback_stats": (_ip, [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "bls_profile_enable": (_ip, [_vp, _ip]),
    "bls_profile_read": (_ip, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64), _ip]),
    "bls_profile_name": (ctypes.c_char_p, [_ip]),
    "bls_registry_generation": (ctypes.c_uint64, [_vp]),
    "bls_point_decode": (_ip, [_vp, _ip, _u8p, _sz, _ip, _vp]),
    "bls_point_add": (_ip, [_vp, _ip, _u8p, _u8p, _vp]),
    "bls_point_mul": (_ip, [_vp, _ip, _u8p, _u8p, _vp]),
    "bls_point_neg": (_ip, [_vp, _ip, _u8p, _vp]),
    "bls_multi_exp": (_ip, [_vp, _ip, _u8p, _u8p, _sz, _ip, _vp]),
    "bls_multi_pairing": (_ip, [_vp, _u8p, _u8p, _sz, _ip, _vp]),
    "bls_gt_mul": (_ip, [_vp, _u8p, _u8p, _vp]),
    "bls_pairing_check_ex": (_ip, [_vp, _u8p, _u8p, _sz, _ip]),
    "bls_comm_unique_id": (_ip, [_vp]),
    "bls_comm_init": (_ip, [_vp, _u8p, _ip, _ip]),
    "bls_comm_destroy": (_ip, [_vp]),
    "bls_fav_job_check_comm": (_ip, [_vp, _ip]),
    "bls_comm_abort": (_ip, [_vp]),
    "bls_host_seed": (_ip, [_vp]),
    "bls_set_entropy_source": (_ip, [ctypes.c_char_p]),
    "bls_test_force_h2c_fallback": (_ip, [_vp, _u8p, _sz]),
    "bls_test_hash_to_g2_batch": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_test_wide_selftest": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_test_final_check": (_ip, [_vp, _u8p, _sz, _ip, _vp]),
    "bls_test_hash_to_g2_wide": (_ip, [_vp, _u8p, _sz, _vp]),
    "bls_test_h2c_wide_stages": (_ip, [_vp, _u8p, _vp]),
}

EXPORTS = tuple(_SIGS)

_lib = None
_lib_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load the shared library and declare every C-ABI signature (no device needed)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(f"{path} not found -- run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        ab_build = "BLSMI355X_LIB" in os.environ  # an older library under A/B may lack newer entry points
        for name, (res, args) in _SIGS.items():
            if ab_build and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


class Context:
    """One device context (stream + scratch arena + HBM registry)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _vp()
        rc = self.lib.bls_ctx_create(device, ctypes.byref(h))
        if rc != 0 or not h.value:
            raise NativeUnavailable(f"bls_ctx_create(device={device}) failed ({rc}): no usable GPU")
        self.h = h
        self.device = device

    def close(self):
        if self.h is not None and self.h.value:
            self.lib.bls_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int) -> int:
        if rc < 0:
            msg = self.lib.bls_last_error(self.h)
            raise NativeError(f"libblsmi355x error {rc}: {msg.decode() if msg else ''}")
        return rc

    def device_info(self):
        buf = ctypes.create_string_buffer(256)
        cu = _ip()
        self.check(self.lib.bls_device_info(self.h, buf, 256, ctypes.byref(cu)))
        return buf.value.decode(), cu.value


_ctx = None
_ctx_lock = threading.Lock()


def context() -> Context:
    global _ctx
    with _ctx_lock:
        if _ctx is None:
            _ctx = Context(int(os.environ.get("BLSMI355X_DEVICE", "0")))
        return _ctx
