"""ctypes binding of ``include/slio.h`` (the C-ABI of libslio.so).

There is no CPU fallback: if the HIP library cannot be loaded the import of
the device API raises, so a silent non-native path cannot exist.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libslio.so")

SLIO_NUM_MATCH = 5
SLIO_NPROD = 91
SLIO_NHTH = 78
SLIO_NSUPER = 8
SLIO_CHUNK = 128
SLIO_MODE_REFERENCE = 0
SLIO_MODE_FIXED = 1
SLIO_KERNEL_SEARCH = 0
SLIO_KERNEL_REUSE = 1
SLIO_KERNEL_SUPER = 2
SLIO_PROFILE_KEEP = 16
SLIO_LIO_PROFILE_KEEP = 16
SLIO_LIO_PROFILE_SCAN = 32

ERRORS = {0: "OK", -1: "EINVAL", -2: "ENOMEM", -3: "EDEVICE", -4: "ECAPACITY", -5: "ESTATE", -6: "ETIMEOUT"}
SLIO_ETIMEOUT = -6


class SlioParams(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("max_points", C.c_int32),
        ("rank", C.c_int32),
        ("nranks", C.c_int32),
        ("grid_cell", C.c_float),
        ("plane_threshold", C.c_float),
        ("max_match_sqd", C.c_float),
        ("lanes_per_query", C.c_int32),
        ("max_grid_cells", C.c_int64),
        ("search_radius", C.c_float),
        ("far_query_margin", C.c_float),
    ]


class SlioPose(C.Structure):
    _fields_ = [
        ("rot", C.c_double * 4),
        ("pos", C.c_double * 3),
        ("rli", C.c_double * 4),
        ("tli", C.c_double * 3),
    ]


class SlioState(C.Structure):
    _fields_ = [
        ("pos", C.c_double * 3),
        ("rot", C.c_double * 4),
        ("rli", C.c_double * 4),
        ("tli", C.c_double * 3),
        ("vel", C.c_double * 3),
        ("bg", C.c_double * 3),
        ("ba", C.c_double * 3),
        ("grav", C.c_double * 3),
    ]


class SlioIkfStats(C.Structure):
    _fields_ = [
        ("passes", C.c_int32),
        ("searches", C.c_int32),
        ("valid_passes", C.c_int32),
        ("converged", C.c_int32),
        ("last_m", C.c_int64),
        ("device_ms", C.c_double),
    ]


class SlioLioParams(C.Structure):
    """slio_lio_params (include/slio_frontend.h)."""
    _fields_ = [
        ("device", C.c_int32),
        ("n_scan", C.c_int32),
        ("horizon_scan", C.c_int32),
        ("downsample_rate", C.c_int32),
        ("lidar_min_range", C.c_float),
        ("lidar_max_range", C.c_float),
        ("edge_threshold", C.c_float),
        ("surf_threshold", C.c_float),
        ("surf_leaf_size", C.c_float),
        ("max_points", C.c_int32),
        ("reserved", C.c_int32 * 4),
    ]


class SlioLioCounts(C.Structure):
    _fields_ = [("n_extracted", C.c_int64), ("n_corner", C.c_int64), ("n_surface", C.c_int64)]


class SlioLegoParams(C.Structure):
    """slio_lego_params (include/slio_frontend.h)."""
    _fields_ = [
        ("device", C.c_int32),
        ("n_scan", C.c_int32),
        ("horizon_scan", C.c_int32),
        ("ground_scan_ind", C.c_int32),
        ("segment_valid_point_num", C.c_int32),
        ("segment_valid_line_num", C.c_int32),
        ("ang_res_x", C.c_float),
        ("ang_res_y", C.c_float),
        ("ang_bottom", C.c_float),
        ("sensor_mount_angle", C.c_float),
        ("segment_theta", C.c_float),
        ("edge_threshold", C.c_float),
        ("surf_threshold", C.c_float),
        ("leaf_size", C.c_float),
        ("scan_period", C.c_float),
        ("max_points", C.c_int32),
        ("reserved", C.c_int32 * 4),
    ]


class SlioLegoImu(C.Structure):
    _fields_ = [("time", C.POINTER(C.c_double))] + [(n, C.POINTER(C.c_float)) for n in (
        "roll", "pitch", "yaw", "velo_x", "velo_y", "velo_z", "shift_x", "shift_y", "shift_z",
        "ang_x", "ang_y", "ang_z")] + [
        ("pointer_last", C.c_int32), ("pointer_last_iteration", C.c_int32), ("que_len", C.c_int32),
        ("time_scan_cur", C.c_double), ("ang_last", C.c_float * 3)]


class SlioLegoImuOut(C.Structure):
    _fields_ = [("rpy_start", C.c_float * 3), ("rpy_cur", C.c_float * 3),
                ("velo_from_start", C.c_float * 3), ("angular_from_start", C.c_float * 3),
                ("ang_last", C.c_float * 3), ("pointer_last_iteration", C.c_int32)]


class SlioLegoCounts(C.Structure):
    _fields_ = [("n_segmented", C.c_int64), ("n_outlier", C.c_int64), ("n_sharp", C.c_int64),
                ("n_less_sharp", C.c_int64), ("n_flat", C.c_int64), ("n_less_flat", C.c_int64),
                ("orientation", C.c_float * 3)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.c_void_p)

_P = C.c_void_p
_FP = C.POINTER(C.c_float)
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int32)
_I64P = C.POINTER(C.c_int64)
_U8P = C.POINTER(C.c_uint8)
_U16P = C.POINTER(C.c_uint16)

# name -> (restype, argtypes); every symbol include/*.h declares
class SlioImuSample(C.Structure):
    _fields_ = [("t", C.c_double), ("acc", C.c_double * 3), ("gyr", C.c_double * 3)]


class SlioImuPose(C.Structure):
    _fields_ = [("offset_time", C.c_double), ("acc", C.c_double * 3), ("gyr", C.c_double * 3),
                ("vel", C.c_double * 3), ("pos", C.c_double * 3), ("rot", C.c_double * 9)]


SLIO_COMM_ID_BYTES = 128
SLIO_GROUP_RCCL = 1
SLIO_GROUP_DEVICE = 2

SIGNATURES = {
    "slio_params_default": (C.c_int, [C.POINTER(SlioParams)]),
    "slio_create": (C.c_int, [C.POINTER(_P), C.POINTER(SlioParams)]),
    "slio_destroy": (C.c_int, [_P]),
    "slio_set_stream": (C.c_int, [_P, _P]),
    "slio_last_error": (C.c_char_p, []),
    "slio_build_id": (C.c_char_p, []),
    "slio_map_upload": (C.c_int, [_P, _FP, _FP, _FP, C.c_int64]),
    "slio_map_share": (C.c_int, [_P, _P]),
    "slio_create_group": (C.c_int, [C.POINTER(_P), C.c_int, _IP, C.POINTER(SlioParams)]),
    "slio_group_ikf_update": (C.c_int, [C.POINTER(_P), C.c_int, C.POINTER(SlioState), _DP, C.c_double, C.c_int,
                                        C.c_int, C.c_int, C.POINTER(SlioIkfStats)]),
    "slio_group_reduce_kind": (C.c_int, [_P]),
    "slio_comm_unique_id": (C.c_int, [_U8P]),
    "slio_comm_init": (C.c_int, [_P, _U8P]),
    "slio_map_info": (C.c_int, [_P, _IP, _FP, _I64P]),
    "slio_ikf_predict": (C.c_int, [C.POINTER(SlioState), _DP, C.c_double, _DP, _DP, _DP]),
    "slio_imu_forward": (C.c_int, [C.POINTER(SlioImuSample), C.c_int, C.c_double, C.c_double, _DP, C.c_double,
                                   _DP, _DP, _DP, _DP, _DP, _DP, C.POINTER(SlioState), _DP,
                                   C.POINTER(SlioImuPose), C.c_int, _IP]),
    "slio_undistort": (C.c_int, [_P, _FP, _FP, _FP, _FP, C.c_int64, C.POINTER(SlioImuPose), C.c_int,
                                 C.POINTER(SlioState), _FP, _FP, _FP, _FP]),
    "slio_scan_upload_undistort_voxel": (C.c_int, [_P, _FP, _FP, _FP, _FP, C.c_int64, C.POINTER(SlioImuPose),
                                                   C.c_int, C.POINTER(SlioState), C.c_float, _I64P]),
    "slio_s2m_coeffs": (C.c_int, [_P, C.c_int, _FP, _I64P]),
    "slio_s2m_get_coeffs": (C.c_int, [_P, _FP, _U8P]),
    "slio_s2m_normal_equations": (C.c_int, [_P, _P, _FP, _FP, _FP, _I64P]),
    "slio_s2m_lm_step": (C.c_int, [_FP, _FP, C.c_int64, C.c_int, _FP, _IP, _FP, _IP]),
    "slio_scan_upload_voxel": (C.c_int, [_P, _FP, _FP, _FP, C.c_int64, C.c_float, _I64P]),
    "slio_scan_download": (C.c_int, [_P, _FP, _FP, _FP]),
    "slio_map_add_points": (C.c_int, [_P, _FP, _FP, _FP, C.c_int64, C.c_int, C.c_float, _I64P]),
    "slio_map_delete_boxes": (C.c_int, [_P, _FP, C.c_int64, _I64P]),
    "slio_map_incremental": (C.c_int, [_P, C.POINTER(SlioState), C.c_double, C.c_int, _I64P]),
    "slio_map_download": (C.c_int, [_P, _FP, _FP, _FP, C.POINTER(C.c_uint32), C.c_int64, _I64P]),
    "slio_fov_segment": (C.c_int, [_DP, _FP, _FP, _IP, C.c_double, C.c_float, _FP, _IP]),
    "slio_scan_upload": (C.c_int, [_P, _FP, _FP, _FP, C.c_int64]),
    "slio_shard_range": (C.c_int, [_P, _I64P, _I64P]),
    "slio_iterate_async": (C.c_int, [_P, C.POINTER(SlioPose), C.c_int, C.c_int, C.POINTER(_DP)]),
    "slio_set_super_buffer": (C.c_int, [_P, _P]),
    "slio_super_download": (C.c_int, [_P, _DP]),
    "slio_reduce_super": (C.c_int, [_DP, _DP, _DP, _I64P]),
    "slio_iterate": (C.c_int, [_P, C.POINTER(SlioPose), C.c_int, C.c_int, _DP, _DP, _I64P]),
    "slio_get_neighbors": (C.c_int, [_P, _IP, _FP, _U8P]),
    "slio_far_queries": (C.c_int, [_P, _I64P]),
    "slio_get_planes": (C.c_int, [_P, _FP]),
    "slio_get_residuals": (C.c_int, [_P, _FP]),
    "slio_profile": (C.c_int, [_P, C.c_int]),
    "slio_profile_read": (C.c_int, [_P, C.c_int, _DP, _I64P]),
    "slio_ikf_update": (
        C.c_int,
        [_P, C.POINTER(SlioState), _DP, C.c_double, C.c_int, C.c_int, C.c_int, ALLREDUCE_FN, _P,
         C.POINTER(SlioIkfStats)],
    ),
    "slio_ikf_update_device": (
        C.c_int,
        [_P, C.POINTER(SlioState), _DP, C.c_double, C.c_int, C.c_int, C.c_int, ALLREDUCE_FN, _P,
         C.POINTER(SlioIkfStats)],
    ),
    "slio_state_boxplus": (C.c_int, [C.POINTER(SlioState), _DP, C.POINTER(SlioState)]),
    "slio_state_boxminus": (C.c_int, [C.POINTER(SlioState), C.POINTER(SlioState), _DP]),
    "slio_debug_reload_switches": (C.c_int, [_P]),
    "slio_debug_update_path": (C.c_int, [_P]),
    "slio_debug_host_stamps": (C.c_int, [_P, C.c_int, _I64P]),
    "slio_debug_knn_cert": (C.c_int, [_P, C.POINTER(C.c_uint32)]),
    "slio_debug_wait_limit": (C.c_int, [_P, C.c_int64]),
    # include/slio_frontend.h (LIO-SAM front-end)
    "slio_lio_params_default": (C.c_int, [C.POINTER(SlioLioParams)]),
    "slio_lio_create": (C.c_int, [C.POINTER(_P), C.POINTER(SlioLioParams)]),
    "slio_lio_destroy": (C.c_int, [_P]),
    "slio_lio_set_stream": (C.c_int, [_P, _P]),
    "slio_lio_set_deskew": (C.c_int, [_P, _DP, _DP, _DP, _DP, C.c_int32, C.c_double, C.c_int32]),
    "slio_lio_upload": (C.c_int, [_P, _FP, _FP, _FP, _FP, _U16P, _FP, C.c_int64]),
    "slio_lio_run_async": (C.c_int, [_P]),
    "slio_lio_run": (C.c_int, [_P, C.POINTER(SlioLioCounts)]),
    "slio_lio_get_counts": (C.c_int, [_P, C.POINTER(SlioLioCounts)]),
    "slio_lio_get_range_image": (C.c_int, [_P, _FP, _IP]),
    "slio_lio_get_cloud_info": (C.c_int, [_P, _IP, _IP, _IP, _FP, _FP]),
    "slio_lio_get_features": (C.c_int, [_P, _FP, _U8P, _IP]),
    "slio_lio_get_clouds": (C.c_int, [_P, _FP, _FP]),
    "slio_lio_profile": (C.c_int, [_P, C.c_int]),
    "slio_lio_profile_read": (C.c_int, [_P, _DP, _I64P]),
    # include/slio_frontend.h (LeGO-LOAM front-end)
    "slio_lego_params_default": (C.c_int, [C.POINTER(SlioLegoParams)]),
    "slio_lego_create": (C.c_int, [C.POINTER(_P), C.POINTER(SlioLegoParams)]),
    "slio_lego_destroy": (C.c_int, [_P]),
    "slio_lego_set_stream": (C.c_int, [_P, _P]),
    "slio_lego_set_imu": (C.c_int, [_P, C.POINTER(SlioLegoImu)]),
    "slio_lego_upload": (C.c_int, [_P, _FP, _FP, _FP, C.c_int64]),
    "slio_lego_run_async": (C.c_int, [_P]),
    "slio_lego_run": (C.c_int, [_P, C.POINTER(SlioLegoCounts)]),
    "slio_lego_get_counts": (C.c_int, [_P, C.POINTER(SlioLegoCounts)]),
    "slio_lego_get_image": (C.c_int, [_P, _FP, _IP, C.POINTER(C.c_int8), _IP]),
    "slio_lego_get_seg_info": (C.c_int, [_P, _IP, _IP, _U8P, _IP, _FP, _FP, _FP]),
    "slio_lego_get_features": (C.c_int, [_P, _FP, _FP, _U8P, _IP, C.POINTER(SlioLegoImuOut)]),
    "slio_lego_get_clouds": (C.c_int, [_P, _FP, _FP, _FP, _FP]),
    "slio_lego_profile": (C.c_int, [_P, C.c_int]),
    "slio_lego_profile_read": (C.c_int, [_P, _DP, _I64P]),
}

_lib = None


def load() -> C.CDLL:
    """Load the in-tree libslio.so once and bind every declared signature.
    The library must carry the digest of the current sources (slio_build_id):
    a stale or foreign build fails loudly.  (Diagnostic variants are bound by
    scripts/variant.py, outside the product.)"""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -m agi_lidar_slam_amd.build` "
            "(there is no CPU fallback for the device path)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the library lacks a declared symbol
        fn.restype = res
        fn.argtypes = args
    from . import build
    got, want = lib.slio_build_id().decode(), build.source_hash()
    if got != want:
        raise RuntimeError(f"{LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                           "rebuild with `python -m agi_lidar_slam_amd.build`")
    _lib = lib
    return lib


class SlioError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().slio_last_error()
        msg = msg.decode() if msg else ""
        raise SlioError(f"{what}: {ERRORS.get(rc, rc)}: {msg}")


def fptr(a: np.ndarray):
    return a.ctypes.data_as(_FP)


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_DP)


def iptr(a: np.ndarray):
    return a.ctypes.data_as(_IP)


def u8ptr(a: np.ndarray):
    return a.ctypes.data_as(_U8P)


def u16ptr(a: np.ndarray):
    return a.ctypes.data_as(_U16P)


def i64ptr(a: np.ndarray):
    return a.ctypes.data_as(_I64P)
