"""ctypes binding of libdpk.so (the C ABI declared in include/diffpose_kernels.h).

The library is built in-tree (``python __graft_entry__.py`` → ``build()``, or
``make -C diffpose-nw_amd``).  There is no fallback: if it is missing or fails to
load, ``lib()`` raises, and every product entry point fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPK_LIB", os.path.join(_HERE, "libdpk.so"))

DPK_OK = 0
ERRORS = {-1: "DPK_E_INVALID", -2: "DPK_E_UNSUPPORTED", -3: "DPK_E_HIP", -4: "DPK_E_STATE", -5: "DPK_E_WEIGHTS"}

# every symbol include/diffpose_kernels.h declares
EXPORTS = ("dpk_version", "dpk_create", "dpk_set_graph", "dpk_load_weights", "dpk_set_mask", "dpk_set_pose_masks",
           "dpk_set_schedule", "dpk_eps", "dpk_sample", "dpk_sample_noise", "dpk_ddim_update", "dpk_ddim_update_noise",
           "dpk_pose", "dpk_pose_metrics", "dpk_gmm_sample", "dpk_gmm_sample_f64", "dpk_set_gemm_mode",
           "dpk_set_tail_plan", "dpk_debug_split", "dpk_debug_resources", "dpk_profile", "dpk_profile_read",
           "dpk_kernel_geometry", "dpk_last_error", "dpk_destroy")


class DpkConfig(ctypes.Structure):
    _fields_ = [("hid_dim", ctypes.c_int), ("num_layers", ctypes.c_int), ("n_head", ctypes.c_int),
                ("n_pts", ctypes.c_int), ("coords_in", ctypes.c_int), ("coords_out", ctypes.c_int),
                ("device", ctypes.c_int)]


class DpkError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str = ""):
        super().__init__(f"{fn} failed: {ERRORS.get(code, code)} {msg}".strip())
        self.code = code


_LIB = None


def lib() -> ctypes.CDLL:
    """Load libdpk.so once.  Imports torch first so the HIP runtime is shared with it."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libdpk.so not found at {LIB_PATH}: build it with `python __graft_entry__.py` "
                          "(build()) or `make -C diffpose-nw_amd`; there is no CPU fallback")
    import torch  # noqa: F401  (binds libamdhip64.so.7 before our library resolves it)

    L = ctypes.CDLL(LIB_PATH)
    if "DPK_LIB" in os.environ:
        # an A/B build of another version (tools/ab_bench.sh): bind what it exports
        class _Partial:
            def __init__(self, lib):
                self._lib = lib

            def __getattr__(self, name):
                try:
                    return getattr(self._lib, name)
                except AttributeError:
                    return lambda *a: -2          # DPK_E_UNSUPPORTED: not in that build
        L = _Partial(L)
    vp, i32, i64, u64, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float)
    L.dpk_version.restype = i32
    L.dpk_create.argtypes = [ctypes.POINTER(DpkConfig), ctypes.POINTER(vp)]
    L.dpk_set_graph.argtypes = [vp, fp]
    L.dpk_load_weights.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(fp), ctypes.POINTER(i64), i32]
    L.dpk_set_mask.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8)]
    L.dpk_set_pose_masks.argtypes = [vp, vp, i32]
    L.dpk_set_schedule.argtypes = [vp, fp, i32, ctypes.POINTER(i32), i32, ctypes.c_float]
    L.dpk_eps.argtypes = [vp, vp, vp, vp, i32, vp]
    L.dpk_sample.argtypes = [vp, vp, vp, vp, vp, i32, u64, vp]
    L.dpk_sample_noise.argtypes = [vp, vp, vp, vp, vp, i32, u64, vp, vp]
    L.dpk_ddim_update.argtypes = [vp, vp, vp, vp, vp, i64, i32, u64, vp]
    L.dpk_ddim_update_noise.argtypes = [vp, vp, vp, vp, vp, i64, i32, u64, vp, vp]
    L.dpk_debug_split.argtypes = [vp, i32, ctypes.POINTER(i32)]
    L.dpk_debug_resources.argtypes = [vp, ctypes.POINTER(i32), i32]
    L.dpk_pose.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp]
    L.dpk_pose_metrics.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, vp]
    L.dpk_gmm_sample.argtypes = [vp, vp, i32, i32, vp, i32, vp, u64, ctypes.c_double, vp, vp, vp, vp]
    L.dpk_gmm_sample_f64.argtypes = [vp, vp, i32, i32, vp, i32, vp, u64, ctypes.c_double, vp, vp, vp, vp]
    L.dpk_set_gemm_mode.argtypes = [vp, i32]
    L.dpk_set_tail_plan.argtypes = [vp, i32]
    L.dpk_profile.argtypes = [vp, i32]
    L.dpk_profile_read.argtypes = [vp, fp, i32, ctypes.POINTER(i32)]
    L.dpk_kernel_geometry.argtypes = [ctypes.POINTER(i32)] * 3
    L.dpk_last_error.argtypes = [vp]
    L.dpk_last_error.restype = ctypes.c_char_p
    L.dpk_destroy.argtypes = [vp]
    L.dpk_destroy.restype = None
    for name in EXPORTS:
        if name in ("dpk_last_error", "dpk_destroy"):
            continue
        getattr(L, name).restype = i32
    _LIB = L
    return L


def check(handle, fn: str, rc: int) -> None:
    if rc != DPK_OK:
        msg = ""
        if handle:
            raw = lib().dpk_last_error(handle)
            msg = raw.decode() if raw else ""
        raise DpkError(fn, rc, msg)


def kernel_geometry():
    L = lib()
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.dpk_kernel_geometry(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return {"poses_per_workgroup": a.value, "threads_per_workgroup": b.value, "lds_bytes": c.value}
