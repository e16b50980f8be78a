"""ctypes binding of libneo_hip.so (the C-ABI in include/neo_hip.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, calls raise. The library is built in-tree by
`make -C neo-dsp_amd` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.environ.get("NEO_HIP_LIBRARY") or os.path.join(_HERE, "..", "lib", "libneo_hip.so"))

NEO_HIP_OK = 0
NEO_HIP_EINVAL = 1
NEO_HIP_ERUNTIME = 2
NEO_HIP_ENOMEM = 3
NEO_HIP_ENODEV = 4

C2C, R2C, C2R = 0, 1, 2
F64 = 16  # OR into the kind: complex128 / float64 plans

class UpolsOpts(ctypes.Structure):
    """neo_hip_upols_opts (include/neo_hip.h)."""
    _fields_ = [("fused", ctypes.c_int), ("split_workgroups", ctypes.c_int), ("batch_blocks", ctypes.c_int),
                ("batch_bins", ctypes.c_int), ("levels", ctypes.c_int), ("far_level", ctypes.c_int),
                ("far_group", ctypes.c_int), ("toep_split", ctypes.c_int), ("step_group", ctypes.c_int),
                ("far_phase2", ctypes.c_int)]


# every symbol declared in include/neo_hip.h: (name, restype, argtypes)
_vp, _i, _i64, _fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_float)
SIGNATURES = {
    "neo_hip_last_error": (ctypes.c_char_p, []),
    "neo_hip_version": (_i, []),
    "neo_hip_device_count": (_i, [ctypes.POINTER(_i)]),
    "neo_hip_host_register": (_i, [_vp, _i64]),
    "neo_hip_host_unregister": (_i, [_vp]),
    "neo_hip_memory_trim": (_i, [_i]),
    "neo_hip_memory_info": (_i, [_i, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "neo_hip_fft_max_order": (_i, []),
    "neo_hip_fft_plan_create": (_i, [_i, _i64, _i, _i, ctypes.POINTER(_vp)]),
    "neo_hip_fft_plan_destroy": (_i, [_vp]),
    "neo_hip_fft_execute": (_i, [_vp, _vp, _vp, _i, _vp]),
    "neo_hip_fft_execute_host": (_i, [_vp, _vp, _vp, _i]),
    "neo_hip_upols_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "neo_hip_upola_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "neo_hip_upola2_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "neo_hip_upols_process_samples": (_i, [_vp, _vp, _i64, _vp, _i64, _i64, _i, _vp]),
    "neo_hip_upols_set_batch": (_i, [_vp, _i]),
    "neo_hip_upols_batch_info": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "neo_hip_upols_create_ex": (_i, [_i, _i, _i, _i, _i, _vp, ctypes.POINTER(_vp)]),
    "neo_hip_upols_destroy": (_i, [_vp]),
    "neo_hip_upols_set_filter": (_i, [_vp, _vp, _i]),
    "neo_hip_upols_set_impulse": (_i, [_vp, _vp, _i64, _i, _i]),
    "neo_hip_upols_process": (_i, [_vp, _vp, _i, _vp]),
    "neo_hip_upols_process_device": (_i, [_vp, _vp, _i64, _vp, _i64, _vp]),
    "neo_hip_upols_process_blocks": (_i, [_vp, _vp, _vp, _i64, _i64, _vp]),
    "neo_hip_upols_reset": (_i, [_vp]),
    "neo_hip_upols_set_ahead": (_i, [_vp, _i]),
    "neo_hip_upols_set_offline": (_i, [_vp, _i]),
    "neo_hip_upols_get_offline": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "neo_hip_upols_get_ahead": (_i, [_vp] + [ctypes.POINTER(_i)] * 4),
    "neo_hip_upols_set_timing": (_i, [_vp, _i]),
    "neo_hip_upols_timing": (_i, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64)]),
    "neo_hip_upols_timing_detail": (_i, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64)]),
    "neo_hip_upols_step_times": (_i, [_vp, ctypes.POINTER(ctypes.c_double), _i64, ctypes.POINTER(_i64)]),
    "neo_hip_upols_level_plan": (_i, [_i] + [ctypes.POINTER(_i)] * 6),
    "neo_hip_upols_part_plan": (_i, [_i] * 5 + [ctypes.POINTER(_i)] * 3 + [_i, ctypes.POINTER(_i),
                                                                          ctypes.POINTER(ctypes.c_double), _i]),
    "neo_hip_upols_get_far_group": (_i, [_vp, ctypes.POINTER(_i)]),
    "neo_hip_upols_get_step_group": (_i, [_vp, ctypes.POINTER(_i)]),
    "neo_hip_upols_join_background": (_i, [_vp, _vp]),
    "neo_hip_upols_set_paced": (_i, [_vp, _i]),
    "neo_hip_upols_set_persistent": (_i, [_vp, _i, ctypes.c_double]),
    "neo_hip_upols_get_persistent": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i64)]),
    "neo_hip_upols_persist_step_times": (_i, [_vp, ctypes.POINTER(ctypes.c_double), _i64, ctypes.POINTER(_i64)]),
    "neo_hip_upols_get_far_form": (_i, [_vp, ctypes.POINTER(_i)]),
    "neo_hip_upols_info": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "neo_hip_upols_multi_create": (_i, [_i, _i, _i, _vp, _i, _i, _vp, ctypes.POINTER(_vp)]),
    "neo_hip_upols_multi_destroy": (_i, [_vp]),
    "neo_hip_upols_multi_shards": (_i, [_vp, ctypes.POINTER(_i)]),
    "neo_hip_upols_multi_shard": (_i, [_vp, _i, ctypes.POINTER(_vp)] + [ctypes.POINTER(_i)] * 3),
    "neo_hip_upols_multi_set_filter": (_i, [_vp, _vp]),
    "neo_hip_upols_multi_set_impulse": (_i, [_vp, _vp, _i64, _i]),
    "neo_hip_upols_multi_process_samples": (_i, [_vp, _vp, _i64, _vp, _i64, _i64]),
    "neo_hip_upols_multi_reset": (_i, [_vp]),
    "neo_hip_overlap_create": (_i, [_i, _i, _i64, _i64, _i, ctypes.POINTER(_vp)]),
    "neo_hip_overlap_destroy": (_i, [_vp]),
    "neo_hip_overlap_info": (_i, [_vp] + [ctypes.POINTER(_i64)] * 3),
    "neo_hip_overlap_reset": (_i, [_vp]),
    "neo_hip_overlap_forward": (_i, [_vp, _vp, _i64, _vp, _i, _vp]),
    "neo_hip_overlap_inverse": (_i, [_vp, _vp, _vp, _i64, _i, _vp]),
    "neo_hip_upols_group_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "neo_hip_upols_group_destroy": (_i, [_vp]),
    "neo_hip_upols_group_join": (_i, [_vp, ctypes.POINTER(_i)]),
    "neo_hip_upols_group_leave": (_i, [_vp, _i]),
    "neo_hip_upols_group_set_filter": (_i, [_vp, _i, _vp, _i]),
    "neo_hip_upols_group_process": (_i, [_vp, _i, _vp]),
    "neo_hip_upols_group_reset": (_i, [_vp, _i]),
    "neo_hip_upols_group_stats": (_i, [_vp, ctypes.POINTER(_i)] + [ctypes.POINTER(_i64)] * 4),
    "neo_hip_upols_group_register": (_i, [_vp, _vp, _i64]),
    "neo_hip_upols_group_register_ex": (_i, [_vp, _vp, _i64, _i]),
    "neo_hip_upols_group_unregister": (_i, [_vp, _vp]),
    "neo_hip_num_partitions": (_i, [_i64, _i, ctypes.POINTER(_i64)]),
    "neo_hip_uniform_partition": (_i, [_vp, _i, _i64, _i, _vp, _i, _i]),
    "neo_hip_normalize_impulse": (_i, [_vp, _i, _i64, _i, _i]),
    "neo_hip_fft_convolve": (_i, [_vp, _i64, _vp, _i64, _vp, _i, _i]),
    "neo_hip_direct_convolve": (_i, [_vp, _i64, _vp, _i64, _vp, _i, _i]),
    "neo_hip_fft_convolve_f64": (_i, [_vp, _i64, _vp, _i64, _vp, _i, _i]),
    "neo_hip_direct_convolve_f64": (_i, [_vp, _i64, _vp, _i64, _vp, _i, _i]),
    "neo_hip_stft_num_frames": (_i, [_i64, _i, _i, ctypes.POINTER(_i64)]),
    "neo_hip_stft": (_i, [_vp, _i, _i64, _i, _i, _i, _vp, _vp, _i, _i]),
    "neo_hip_stft_f64": (_i, [_vp, _i, _i64, _i, _i, _i, _vp, _vp, _i, _i]),
}

ABI_VERSION = 200  # include/neo_hip.h NEO_HIP_VERSION
_lib = None
_lock = threading.Lock()


class NeoHipError(RuntimeError):
    """Raised for any nonzero neo_hip status (maps the reference's std::runtime_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"neo_hip error {code}: {msg}")
        self.code = code


def load(path: str = LIB_PATH):
    """Load libneo_hip.so and bind every exported symbol; raises if absent."""
    global _lib
    with _lock:
        if _lib is None:
            # One HIP runtime per process: torch bundles its own libamdhip64.so (same
            # soname, libamdhip64.so.7). Importing torch first makes libneo_hip.so bind
            # to that copy; loading ours first would map a second HIP/HSA runtime.
            if os.environ.get("NEO_HIP_NO_TORCH") != "1":
                try:
                    import torch  # noqa: F401
                except ImportError:
                    pass
            if not os.path.exists(path):
                raise ImportError(
                    f"{path} not found: build the HIP library first (make -C neo-dsp_amd); "
                    "there is no CPU fallback")
            lib = ctypes.CDLL(path)
            lib.neo_hip_version.restype = ctypes.c_int
            if lib.neo_hip_version() != ABI_VERSION:  # neo_hip_upols_opts' layout is tied to it
                raise ImportError(f"{path}: ABI version {lib.neo_hip_version()}, these bindings need {ABI_VERSION}")
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc: int) -> None:
    if rc != NEO_HIP_OK:
        msg = load().neo_hip_last_error()
        raise NeoHipError(rc, msg.decode() if msg else "")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = load().neo_hip_device_count(ctypes.byref(n))
    return n.value if rc == NEO_HIP_OK else 0


def require_gpu() -> None:
    if device_count() < 1:
        raise NeoHipError(NEO_HIP_ENODEV, "no HIP device visible; neo_hip has no CPU fallback")
