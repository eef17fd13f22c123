"""ctypes binding of libmage_hot.so (the C-ABI in include/mage_hot.h).

The product path has no CPU fallback: if the HIP library is missing this module raises at
import, and every call that needs a GPU fails with MageError(MAGE_EDEVICE).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

LIB_PATH = Path(__file__).resolve().parent / "_lib" / "libmage_hot.so"

MAGE_OK, MAGE_EINVAL, MAGE_EDEVICE, MAGE_ENOMEM, MAGE_EUNSUPPORTED, MAGE_ECAPACITY = range(6)
MAGE_TETHER_DISTANCE, MAGE_TETHER_ROTATION, MAGE_TETHER_TRANSFORM = range(3)
STATUS_NAMES = {0: "MAGE_OK", 1: "MAGE_EINVAL", 2: "MAGE_EDEVICE", 3: "MAGE_ENOMEM",
                4: "MAGE_EUNSUPPORTED", 5: "MAGE_ECAPACITY"}

# Every entry point declared in include/mage_hot.h (checked by tests/test_capi.py).
EXPORTS = [
    "mage_version", "mage_last_error", "mage_pool_trim", "mage_profile_enable", "mage_profile_filter", "mage_profile_reset",
    "mage_profile_report", "mage_orb_create", "mage_orb_destroy", "mage_orb_detect_and_compute",
    "mage_orb_detect_and_compute_batch_device", "mage_orb_status", "mage_orb_reset_status",
    "mage_orb_set_fast_gate", "mage_orb_fast_gate_stats",
    "mage_synth_frames_device", "mage_synth_scene_device", "mage_orb_fast_score_map",
    "mage_undistort_keypoints", "mage_undistort_keypoints_batch_device",
    "mage_undistorter_create", "mage_undistorter_destroy", "mage_undistorter_get_maps", "mage_undistort_image",
    "mage_undistort_image_batch_device", "mage_resize_linear_device", "mage_scale_for_camera_configuration",
    "mage_scale_image_for_camera_configuration_device",
    "mage_hamming_distance", "mage_hamming_match", "mage_hamming_match_batch_device",
    "mage_radius_match", "mage_radius_match_batch_device", "mage_local_map_match",
    "mage_bow_create", "mage_bow_destroy", "mage_bow_train", "mage_bow_train_kmedoid", "mage_bow_get_tree", "mage_bow_find_leaves", "mage_bow_find_leaves_device",
    "mage_indexed_match", "mage_indexed_match_batch_device",
    "mage_ba_create", "mage_ba_destroy", "mage_ba_set_cameras", "mage_ba_fix_camera",
    "mage_ba_set_points", "mage_ba_set_observations", "mage_ba_set_lambda", "mage_ba_get_lambda",
    "mage_ba_set_tethers", "mage_ba_step", "mage_ba_get_poses", "mage_ba_get_points",
    "mage_ba_get_stats", "mage_ba_get_state_f64", "mage_ba_pose_batch", "mage_ba_pose_batch_device",
    "mage_track_sequence", "mage_track_sequence_device",
]


class MageError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Calibration(C.Structure):
    """mage_calibration: CameraCalibration's linear intrinsics + OpenCV-ordered distortion."""
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("dist", C.c_float * 8), ("ndist", C.c_int32)]

    @classmethod
    def make(cls, fx, fy, cx, cy, dist=()):
        d = list(dist)
        if len(d) not in (0, 5, 8):
            raise ValueError("distortion: 0 (None), 5 (Poly3k) or 8 (Rational6k) coefficients")
        return cls(fx, fy, cx, cy, (C.c_float * 8)(*(d + [0.0] * (8 - len(d)))), len(d))


class CameraConfig(C.Structure):
    """mage_camera_config: MAGESlam::CameraConfiguration (Extrinsics M11..M44 row-major, Size) with
    its undistorted pinhole calibration."""
    _fields_ = [("extrinsics", C.c_float * 16), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float),
                ("cy", C.c_float), ("width", C.c_uint32), ("height", C.c_uint32)]

    @classmethod
    def make(cls, extrinsics, fx, fy, cx, cy, width, height):
        e = np.asarray(extrinsics, np.float32).reshape(16)
        return cls((C.c_float * 16)(*e.tolist()), fx, fy, cx, cy, width, height)


class KeyPoint(C.Structure):
    """cv::KeyPoint layout (28 B)."""

    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


class OrbSettingsC(C.Structure):
    _fields_ = [("gaussian_kernel_size", C.c_uint32), ("nfeatures", C.c_uint32),
                ("scale_factor", C.c_float), ("nlevels", C.c_uint32), ("patch_size", C.c_uint32),
                ("fast_threshold", C.c_uint32), ("use_orientation", C.c_int32),
                ("feature_factor", C.c_float), ("feature_strength", C.c_float),
                ("strong_response", C.c_int32), ("min_robust_factor", C.c_float),
                ("max_robust_factor", C.c_float), ("num_cells_x", C.c_int32),
                ("num_cells_y", C.c_int32)]


class TrackSettingsC(C.Structure):
    """mage_track_settings (include/mage_hot.h)."""
    _fields_ = [("search_radius", C.c_float), ("wider_search_radius", C.c_float),
                ("extra_wider_search_radius", C.c_float), ("small_match_ratio", C.c_double),
                ("min_matches", C.c_uint32), ("max_hamming", C.c_int32), ("min_hamming_difference", C.c_int32),
                ("initial_steps", C.c_uint32), ("initial_huber", C.c_float), ("initial_max_error", C.c_double),
                ("final_steps", C.c_uint32), ("final_huber", C.c_float), ("final_max_error", C.c_double),
                ("refinement_info", C.c_float), ("keyframe_ratio", C.c_double), ("keyframe_min", C.c_uint32),
                ("local_map_keyframes", C.c_uint32), ("match_search_radius", C.c_float),
                ("local_max_hamming", C.c_int32), ("local_min_hamming_difference", C.c_int32),
                ("min_view_cos", C.c_float), ("image_border", C.c_float), ("min_tracked", C.c_uint32),
                ("scale_factor", C.c_float), ("num_levels", C.c_uint32), ("width", C.c_int32), ("height", C.c_int32),
                ("local_ba", C.c_uint32), ("ba_huber", C.c_float), ("ba_huber_scale", C.c_float),
                ("ba_max_outlier_error", C.c_float), ("ba_steps_per_run", C.c_uint32),
                ("ba_low_connectivity_scale", C.c_float), ("ba_upper_connections", C.c_uint32),
                ("min_lambda", C.c_float), ("ba_free_keyframes", C.c_uint32),
                ("covis_min_threshold", C.c_uint32), ("covis_ba_step", C.c_uint32),
                ("ba_lower_connections", C.c_uint32), ("covis_max_steps", C.c_uint32),
                ("map_point_depth_noise", C.c_float)]


class BAStats(C.Structure):
    _fields_ = [("iterations", C.c_uint64), ("trials", C.c_uint64), ("rejected_trials", C.c_uint64),
                ("last_chi2", C.c_double), ("lambda_", C.c_double)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DM_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("img_idx", "<i4"),
                     ("distance", "<f4")])

_lib = None


def load() -> C.CDLL:
    """Load libmage_hot.so (raises ImportError if it has not been built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -m mageslam_amd.build`")
        lib = C.CDLL(str(LIB_PATH))
        _declare(lib)
        _lib = lib
    return _lib


def ptr(a):
    """Host pointer of a numpy array, or raw device pointer of a torch tensor / int."""
    if a is None:
        return None
    if isinstance(a, int):
        return C.c_void_p(a)
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    return a.ctypes.data_as(C.c_void_p)


def check(status: int) -> None:
    if status != MAGE_OK:
        msg = load().mage_last_error().decode(errors="replace")
        raise MageError(status, msg)


def profile_report() -> dict:
    """{kernel: (launches, total_ms)} from the library's event timers."""
    out = {}
    for line in load().mage_profile_report().decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out


def _declare(L: C.CDLL) -> None:
    vp, i32, u32, f32, i64, u64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_float, C.c_int64, C.c_uint64
    st = C.c_int

    def sig(name, res, *args):
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = list(args)

    sig("mage_version", C.c_char_p)
    sig("mage_last_error", C.c_char_p)
    sig("mage_pool_trim", C.c_uint64, i32)
    sig("mage_profile_enable", None, i32)
    sig("mage_profile_filter", None, C.c_char_p)
    sig("mage_profile_reset", None)
    sig("mage_profile_report", C.c_char_p)
    sig("mage_orb_create", st, vp, C.c_int, C.POINTER(vp))
    sig("mage_orb_destroy", st, vp)
    sig("mage_orb_detect_and_compute", st, vp, vp, i32, i32, i32, vp, vp, u32, C.POINTER(u32))
    sig("mage_orb_detect_and_compute_batch_device", st, vp, vp, u32, i32, i32, i32, i64, vp, vp, u32, vp, vp)
    sig("mage_orb_status", st, vp, vp)
    sig("mage_orb_reset_status", st, vp, vp)
    sig("mage_orb_set_fast_gate", st, vp, u32, i32, vp)
    sig("mage_orb_fast_gate_stats", st, vp, u32, C.POINTER(i32), C.POINTER(i32), C.POINTER(u32), vp)
    sig("mage_synth_frames_device", st, vp, u32, i32, i32, i64, u32, u64, vp)
    f64 = C.c_double
    sig("mage_synth_scene_device", st, vp, u32, i32, i32, i64, vp, f64, f64, f64, f64, f64, f64, i64, u64, vp)
    sig("mage_orb_fast_score_map", st, vp, i32, i32, i32, i32, vp, C.c_int)
    sig("mage_undistort_keypoints", st, vp, vp, vp, u32, C.c_int)
    sig("mage_undistort_keypoints_batch_device", st, vp, vp, vp, i64, vp, u32, vp)
    sig("mage_undistorter_create", st, vp, i32, i32, C.c_int, C.POINTER(vp), vp)
    sig("mage_undistorter_destroy", st, vp)
    sig("mage_undistorter_get_maps", st, vp, vp, vp)
    sig("mage_undistort_image", st, vp, vp, i32, vp, i32)
    sig("mage_undistort_image_batch_device", st, vp, vp, i32, i64, vp, i32, i64, u32, vp)
    sig("mage_resize_linear_device", st, vp, i32, i32, i32, vp, i32, i32, i32, vp)
    sig("mage_scale_for_camera_configuration", st, vp, vp, f32, vp, C.POINTER(f32), vp, C.POINTER(i32))
    sig("mage_scale_image_for_camera_configuration_device", st, vp, vp, f32, vp, i32, vp, i32, i64, vp,
        C.POINTER(f32), C.POINTER(i32), vp)
    sig("mage_hamming_distance", i32, vp, vp)
    sig("mage_hamming_match", st, vp, u32, vp, vp, u32, vp, i32, i32, vp, u32, C.POINTER(u32))
    sig("mage_hamming_match_batch_device", st, vp, i64, vp, vp, i64, vp, u32, i32, i32, vp, u32, vp, vp)
    sig("mage_radius_match", st, vp, vp, vp, vp, u32, vp, vp, vp, u32, C.c_float, i32, i32, vp, u32, C.POINTER(u32))
    sig("mage_radius_match_batch_device", st, vp, vp, vp, i64, vp, vp, vp, i64, vp, u32, C.c_float, i32, i32, vp,
        vp, u32, vp, vp, vp)
    sig("mage_local_map_match", st, vp, vp, vp, vp, u32, vp, vp, u32, vp, C.c_float, i32, i32, vp, C.c_int)
    sig("mage_bow_create", st, vp, vp, vp, u32, C.c_int, C.POINTER(vp))
    sig("mage_bow_destroy", st, vp)
    sig("mage_bow_train", st, vp, u32, u32, u32, u32, C.c_int, C.POINTER(vp))
    sig("mage_bow_train_kmedoid", st, vp, u32, u32, u32, u32, C.c_int, C.POINTER(vp))
    sig("mage_bow_get_tree", st, vp, vp, vp, vp, u32, C.POINTER(u32))
    sig("mage_bow_find_leaves", st, vp, vp, u32, vp)
    sig("mage_bow_find_leaves_device", st, vp, vp, u32, vp, vp)
    sig("mage_indexed_match", st, vp, vp, u32, vp, vp, u32, vp, i32, i32, vp, u32, C.POINTER(u32))
    sig("mage_indexed_match_batch_device", st, vp, vp, vp, i64, vp, vp, vp, vp, i64, vp, u32, i32, i32, vp, u32,
        vp, vp, vp)
    sig("mage_ba_create", st, i32, C.c_int, C.POINTER(vp))
    sig("mage_ba_destroy", st, vp)
    sig("mage_ba_set_cameras", st, vp, u32, vp, vp, vp, vp)
    sig("mage_ba_fix_camera", st, vp, u32, i32)
    sig("mage_ba_set_points", st, vp, u32, vp)
    sig("mage_ba_set_observations", st, vp, u32, vp, vp, vp, vp)
    sig("mage_ba_set_lambda", st, vp, f32)
    sig("mage_ba_get_lambda", st, vp, C.POINTER(f32))
    sig("mage_ba_set_tethers", st, vp, u32, u32, vp, vp, vp, vp)
    sig("mage_ba_step", st, vp, vp, u32, f32, vp, u32, C.POINTER(u32), C.POINTER(f32))
    sig("mage_ba_get_poses", st, vp, vp, vp)
    sig("mage_ba_get_points", st, vp, vp)
    sig("mage_ba_get_state_f64", st, vp, vp, vp)
    sig("mage_ba_get_stats", st, vp, C.POINTER(BAStats))
    sig("mage_track_sequence", st, vp, vp, vp, u32, vp, vp, C.c_double, vp, vp, vp, vp, vp, C.c_int)
    sig("mage_track_sequence_device", st, vp, vp, u32, vp, u32, vp, vp, C.c_double, vp, vp, vp, vp, vp, vp, vp)
    sig("mage_ba_pose_batch", st, u32, vp, vp, vp, vp, vp, vp, vp, u32, f32, f32, vp, vp, vp, vp, vp, vp, C.c_int)
    sig("mage_ba_pose_batch_device", st, u32, vp, vp, vp, vp, vp, vp, vp, u32, f32, f32, vp, vp, vp, vp, vp, vp, vp)
