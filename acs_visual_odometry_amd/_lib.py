"""ctypes binding of libvo_mi355x.so (the C ABI declared in include/vo_mi355x.h).

There is no CPU fallback: if the HIP library is missing, importing the binding raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VO_LIB_PATH") or os.path.join(_HERE, "libvo_mi355x.so")   # override: diagnostic builds

VO_ABI_VERSION = 2        # include/vo_mi355x.h; VoConfig below mirrors that version's vo_config
VO_OK = 0
VO_ERR_IO = -6
VO_ERR_INTERNAL = -7
VO_RNG_SPLITMIX = 0
VO_RNG_MT19937 = 1
VO_ERR_DEGENERATE_E = -10
STATUS = {0: "OK", 1: "FIRST", 2: "MISSING", 3: "FEW_MATCHES", 4: "FEW_INLIERS", 5: "DEGENERATE",
          6: "OVERFLOW", 7: "STALLED", 8: "INCONSISTENT"}

# every symbol include/vo_mi355x.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "vo_config_default", "vo_create", "vo_destroy", "vo_strerror", "vo_abi_version", "vo_extract",
    "vo_response", "vo_match", "vo_ransac_F", "vo_ransac_run", "vo_fit_F", "vo_pose", "vo_set_ground_truth", "vo_set_sequence_starts", "vo_set_frame_origin",
    "vo_trajectory_state", "vo_ring_slots", "vo_rechain", "vo_process_frame",
    "vo_process_frames_device", "vo_process_frames_host", "vo_extract_frames_device", "vo_host_alloc", "vo_host_free", "vo_imread_gray", "vo_device_alloc", "vo_device_free", "vo_device_upload", "vo_device_error_count", "vo_reference_samples", "vo_reset",
    "vo_last_kernel_times", "vo_last_kernel_stats", "vo_enable_kernel_timing", "vo_kernel_form",
    "vo_unpack_descriptor",
]


class VoConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("max_kpts", C.c_int), ("nms_k", C.c_int),
        ("resp_thr", C.c_float), ("border_row", C.c_int), ("border_col", C.c_int),
        ("ratio", C.c_float), ("match_bits", C.c_int), ("ransac_p", C.c_double),
        ("sampson_thr", C.c_double), ("ransac_chunk_threads", C.c_int), ("seed", C.c_uint64),
        ("K", C.c_double * 9), ("device", C.c_int), ("frame_batch", C.c_int), ("rng_mode", C.c_int),
    ]


_lib = None


def load():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libvo_mi355x.so not built ({LIB_PATH}); run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    I = C.c_int
    L.vo_config_default.argtypes = [C.POINTER(VoConfig), I, I]
    L.vo_config_default.restype = None
    L.vo_create.argtypes = [C.POINTER(VoConfig), C.POINTER(P)]
    L.vo_destroy.argtypes = [P]
    L.vo_destroy.restype = None
    L.vo_strerror.argtypes = [I]
    L.vo_strerror.restype = C.c_char_p
    L.vo_extract.argtypes = [P, P, C.c_size_t, P, P, C.POINTER(I), P]
    L.vo_response.argtypes = [P, P, C.c_size_t, P]
    L.vo_match.argtypes = [P, P, I, P, I, P, C.POINTER(I)]
    L.vo_ransac_F.argtypes = [P, P, I, C.c_uint64, P, C.POINTER(I), P, C.POINTER(I), C.POINTER(I),
                              C.POINTER(I), P]
    L.vo_pose.argtypes = [P, P, P, P, I, C.c_double, P, P, P]
    L.vo_ransac_run.argtypes = [P, P, I, C.c_double, C.c_double, I, C.c_uint64, P, C.POINTER(I), P,
                                C.POINTER(I), C.POINTER(I)]
    L.vo_fit_F.argtypes = [P, P, I, P]
    L.vo_set_ground_truth.argtypes = [P, P, I]
    L.vo_set_sequence_starts.argtypes = [P, P, I]
    L.vo_set_frame_origin.argtypes = [P, I]
    L.vo_trajectory_state.argtypes = [P, P]
    L.vo_ring_slots.argtypes = [P]
    L.vo_rechain.argtypes = [P, P, I, I, P]
    L.vo_process_frame.argtypes = [P, P, C.c_size_t, P, C.POINTER(I), P]
    L.vo_process_frames_device.argtypes = [P, P, C.c_size_t, I, P, P, P]
    L.vo_extract_frames_device.argtypes = [P, P, C.c_size_t, I, P, P, P]
    L.vo_process_frames_host.argtypes = [P, P, C.c_size_t, I, P, P, P]
    L.vo_imread_gray.argtypes = [C.c_char_p, P, C.c_size_t, C.POINTER(I), C.POINTER(I)]
    L.vo_host_alloc.argtypes = [P, C.c_size_t, C.POINTER(P)]
    L.vo_host_free.argtypes = [P, P]
    L.vo_device_alloc.argtypes = [P, C.c_size_t, C.POINTER(P)]
    L.vo_device_free.argtypes = [P, P]
    L.vo_device_upload.argtypes = [P, P, P, C.c_size_t]
    L.vo_device_error_count.argtypes = [P, C.POINTER(C.c_uint32)]
    L.vo_reference_samples.argtypes = [C.c_uint32, I, I, P]
    L.vo_reset.argtypes = [P]
    L.vo_last_kernel_times.argtypes = [P, C.POINTER(C.c_char_p), C.POINTER(C.c_float), I]
    L.vo_last_kernel_stats.argtypes = [P, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.POINTER(C.c_float), I]
    L.vo_enable_kernel_timing.argtypes = [P, I]
    L.vo_kernel_form.argtypes = [P, I]
    L.vo_kernel_form.restype = C.c_char_p
    L.vo_unpack_descriptor.argtypes = [P, P]
    L.vo_unpack_descriptor.restype = None
    L.vo_selftest_arith.argtypes = [P, P, P, P, P, P, I, I]
    L.vo_selftest_nullvec9.argtypes = [P, P, P, P, I, I]
    if L.vo_abi_version() != VO_ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI version {L.vo_abi_version()}, this binding is {VO_ABI_VERSION}")
    _lib = L
    return L


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = load().vo_strerror(rc).decode()
        if rc == VO_ERR_DEGENERATE_E:
            raise RuntimeError(msg)          # PoseUpdate.hpp:71-73 throws std::runtime_error
        raise RuntimeError(f"{what}: {msg} ({rc})")
    return rc


def default_config(width: int, height: int, **overrides) -> VoConfig:
    c = VoConfig()
    load().vo_config_default(C.byref(c), width, height)
    for k, v in overrides.items():
        if k == "K":
            vals = [float(x) for x in (v.reshape(9) if hasattr(v, "reshape") else v)]
            for i in range(9):
                c.K[i] = vals[i]
        else:
            setattr(c, k, v)
    return c
