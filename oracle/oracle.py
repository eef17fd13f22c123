"""ctypes binding of the CPU oracle (oracle/_build/libmage_oracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; the product (mageslam_amd) never imports it.
Parity unpinned: see the headers of orb_oracle.c / ba_oracle.c and DESIGN.md §Parity.
"""
from __future__ import annotations

import ctypes as C
import math
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libmage_oracle.so"
DATA = HERE.parent / "mageslam_amd" / "data"


class KeyPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


class DMatch(C.Structure):
    _fields_ = [("query_idx", C.c_int32), ("train_idx", C.c_int32), ("img_idx", C.c_int32),
                ("distance", C.c_float)]


class OrbSettings(C.Structure):
    _fields_ = [("gaussian_kernel_size", C.c_uint32), ("nfeatures", C.c_uint32),
                ("scale_factor", C.c_float), ("nlevels", C.c_uint32), ("patch_size", C.c_uint32),
                ("fast_threshold", C.c_uint32), ("use_orientation", C.c_int32),
                ("feature_factor", C.c_float), ("feature_strength", C.c_float),
                ("strong_response", C.c_int32), ("min_robust_factor", C.c_float),
                ("max_robust_factor", C.c_float), ("num_cells_x", C.c_int32),
                ("num_cells_y", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DM_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("img_idx", "<i4"),
                     ("distance", "<f4")])

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = C.CDLL(str(LIB_PATH))
        _declare(_lib)
    return _lib


def use_native_build() -> str:
    """bench.py's CPU baselines only: rebuild the oracle with -march=native for THIS host (in a
    temporary directory, never the prebuilt tree) and switch every later call to it, with the
    FAST score map of the reference's x64 build (SSE2, fast_sse2.c).  Returns a description of
    the build used; falls back to the portable build (and says so) when gcc fails here."""
    global _lib
    import tempfile

    d = tempfile.mkdtemp(prefix="mage_oracle_native_")
    r = subprocess.run(["make", "-s", "-C", str(HERE), "native", f"NATIVE_DIR={d}"], capture_output=True, text=True)
    so = Path(d) / "libmage_oracle_native.so"
    if r.returncode == 0 and so.exists():
        _lib = C.CDLL(str(so))
        _declare(_lib)
        desc = "gcc -O3 -march=native (built on this host)"
    else:
        lib()
        desc = f"portable -O3 -march=x86-64-v2 build (native build failed: {r.stderr.strip()[-200:]})"
    _lib.oracle_set_fast_sse2(1)
    return desc + ", FAST score map of the reference's x64 SSE2 build"


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _declare(L):
    vp, i32, u32, f32 = C.c_void_p, C.c_int, C.c_uint32, C.c_float
    L.oracle_fast_score_map.argtypes = [vp, i32, i32, i32, i32, vp]
    L.oracle_fast_score_map_sse2.argtypes = [vp, i32, i32, i32, i32, vp, vp]
    L.oracle_set_fast_sse2.argtypes = [i32]
    L.oracle_gaussian_blur.argtypes = [vp, i32, i32, i32, i32, vp]
    L.oracle_gaussian_taps.argtypes = [i32, C.c_double, vp]
    L.oracle_orb_detect.argtypes = [vp, vp, vp, i32, i32, i32, vp, vp, u32, C.POINTER(u32)]
    L.oracle_resize_linear.argtypes = [vp, i32, i32, i32, vp, i32, i32, i32]
    L.oracle_fast_atan2.argtypes = [f32, f32]
    L.oracle_fast_atan2.restype = f32
    L.oracle_umax.argtypes = [i32, vp]
    L.oracle_random_pattern.argtypes = [i32, vp]
    L.oracle_undistort_points.argtypes = [vp, vp, i32, vp, vp, i32]
    L.oracle_radius_match.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, u32, f32, i32, i32, vp, u32]
    L.oracle_radius_match.restype = u32
    L.oracle_ic_angle.argtypes = [vp, i32, i32, i32, vp, i32]
    L.oracle_ic_angle.restype = f32
    L.oracle_level_geometry.argtypes = [i32, i32, i32, f32, vp, vp, vp]
    L.oracle_features_per_level.argtypes = [i32, f32, i32, vp]
    L.oracle_orb_detect.restype = i32
    L.oracle_hamming.argtypes = [vp, vp]
    L.oracle_hamming.restype = i32
    L.oracle_match.argtypes = [vp, u32, vp, vp, u32, vp, i32, i32, vp, u32]
    L.oracle_match.restype = u32
    L.oracle_ba_create.argtypes = [i32]
    L.oracle_ba_create.restype = vp
    L.oracle_ba_destroy.argtypes = [vp]
    L.oracle_ba_set_cameras.argtypes = [vp, i32, vp, vp, vp, vp]
    L.oracle_ba_fix_camera.argtypes = [vp, i32, i32]
    L.oracle_ba_set_points.argtypes = [vp, i32, vp]
    L.oracle_ba_set_observations.argtypes = [vp, i32, vp, vp, vp, vp]
    L.oracle_ba_set_lambda.argtypes = [vp, f32]
    L.oracle_ba_set_tethers.argtypes = [vp, i32, i32, vp, vp, vp, vp]
    L.oracle_undistort_map.argtypes = [vp, vp, i32, vp, i32, i32, vp, vp]
    L.oracle_remap_linear.argtypes = [vp, i32, i32, i32, vp, vp, i32, i32, vp, i32]
    L.oracle_local_map_match.argtypes = [vp, vp, vp, vp, u32, vp, vp, u32, vp, f32, i32, i32, vp]
    L.oracle_scale_geometry.argtypes = [vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp]
    L.oracle_scale_geometry.restype = i32
    L.oracle_ba_pose_batch.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, u32, f32, f32, vp, vp, vp, vp, vp, vp]
    L.oracle_bow_find_leaf.argtypes = [vp, vp, vp, vp]
    L.oracle_bow_find_leaf.restype = u32
    L.oracle_indexed_match.argtypes = [vp, vp, vp, vp, u32, vp, vp, u32, vp, i32, i32, vp, u32]
    L.oracle_indexed_match.restype = u32
    L.oracle_bow_train.argtypes = [vp, u32, u32, u32, u32, vp, vp, vp, u32]
    L.oracle_bow_train.restype = u32
    L.oracle_bow_train2.argtypes = [vp, u32, u32, u32, u32, vp, vp, vp, u32, C.c_int]
    L.oracle_bow_train2.restype = u32
    L.oracle_msvc_shuffle.argtypes = [u32, vp]
    L.oracle_mt19937_first.argtypes = [u32, u32]
    L.oracle_mt19937_first.restype = u32
    L.oracle_ba_tether_linearization.argtypes = [vp, i32, vp, vp, vp]
    L.oracle_ba_tether_linearization.restype = i32
    L.oracle_ba_get_lambda.argtypes = [vp]
    L.oracle_ba_get_lambda.restype = f32
    L.oracle_ba_step.argtypes = [vp, vp, i32, f32, vp, u32, C.POINTER(u32), C.POINTER(f32)]
    L.oracle_ba_step.restype = i32
    L.oracle_ba_get_poses.argtypes = [vp, vp, vp]
    L.oracle_ba_get_points.argtypes = [vp, vp]
    L.oracle_ba_get_state.argtypes = [vp, vp, vp]
    L.oracle_ba_get_stats.argtypes = [vp, vp, vp, vp, vp, vp]
    L.oracle_ba_edge_linearization.argtypes = [vp, i32, vp, vp, vp]
    L.oracle_ba_perturb_camera.argtypes = [vp, i32, vp]
    L.oracle_ba_perturb_point.argtypes = [vp, i32, vp]


def default_settings(nfeatures: int = 440, **kw) -> OrbSettings:
    """FeatureExtractorSettings defaults (MageSettings.h:151-167)."""
    s = OrbSettings(7, nfeatures, 1.5, 1, 15, 4, 0, 1.5, 0.9, 20, 1.1, 2.0, 32, 32)
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def pattern_table(patch: int) -> np.ndarray:
    return np.fromfile(DATA / f"bit_pattern_{patch}_rotated.bin", dtype=np.int8)


def resize_linear(img: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """OpenCV 3.4.0 resize(INTER_LINEAR) 8UC1 restatement (pyramid levels > 0)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize_linear(_p(img), w, h, w, _p(out), dw, dh, dw)
    return out


def fast_atan2(y: float, x: float) -> float:
    return float(lib().oracle_fast_atan2(y, x))


def random_pattern(patch_size: int) -> np.ndarray:
    """MakeRandomPattern (OpenCVModified.cpp:551-560) as (x0, y0, x1, y1) int8 per test (256 x 4)."""
    out = np.zeros(1024, np.int8)
    lib().oracle_random_pattern(int(patch_size), _p(out))
    return out


def undistort_points(pts, k_dist, dist, k_new) -> np.ndarray:
    """cv::undistortPoints(pts, K_dist, dist, noArray(), K_new) (OrbFeatureDetector.cpp:55);
    k_* = (fx, fy, cx, cy), dist = 0, 5 or 8 OpenCV-ordered coefficients."""
    p = np.ascontiguousarray(pts, np.float32).reshape(-1, 2).copy()
    kd = np.ascontiguousarray(k_dist, np.float32)
    kn = np.ascontiguousarray(k_new, np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    lib().oracle_undistort_points(_p(kd), _p(d) if len(d) else None, len(d), _p(kn), _p(p), len(p))
    return p


def umax(half_patch: int) -> np.ndarray:
    out = np.zeros(half_patch + 2, np.int32)
    lib().oracle_umax(half_patch, _p(out))
    return out


def ic_angle(img: np.ndarray, x: int, y: int, half_patch: int) -> float:
    img = np.ascontiguousarray(img, np.uint8)
    u = umax(half_patch)
    return float(lib().oracle_ic_angle(_p(img), img.shape[1], x, y, _p(u), half_patch))


def level_geometry(w: int, h: int, nlevels: int, scale_factor: float):
    sc = np.zeros(nlevels, np.float32)
    lw = np.zeros(nlevels, np.int32)
    lh = np.zeros(nlevels, np.int32)
    lib().oracle_level_geometry(w, h, nlevels, scale_factor, _p(sc), _p(lw), _p(lh))
    return sc, lw, lh


def features_per_level(nfeatures: int, scale_factor: float, nlevels: int) -> np.ndarray:
    out = np.zeros(nlevels, np.int32)
    lib().oracle_features_per_level(nfeatures, scale_factor, nlevels, _p(out))
    return out


def fast_score_map(img: np.ndarray, threshold: int = 4) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), np.uint8)
    lib().oracle_fast_score_map(_p(img), w, h, w, threshold, _p(out))
    return out


def fast_score_map_sse2(img: np.ndarray, threshold: int = 4):
    """FAST_t<16> score map as the reference's x64 (SSE2) build computes it (fast_sse2.c):
    (score map, per-row column where the 16-pixel SIMD loop handed over to the scalar tail)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), np.uint8)
    cols = np.zeros(h, np.int32)
    lib().oracle_fast_score_map_sse2(_p(img), w, h, w, threshold, _p(out), _p(cols))
    return out, cols


def gaussian_blur(img: np.ndarray, ksize: int = 7) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), np.uint8)
    lib().oracle_gaussian_blur(_p(img), w, h, w, ksize, _p(out))
    return out


def gaussian_taps(ksize: int = 7, sigma: float = 2.0) -> np.ndarray:
    out = np.zeros(ksize, np.int32)
    lib().oracle_gaussian_taps(ksize, sigma, _p(out))
    return out


def orb_detect(img: np.ndarray, settings: OrbSettings | None = None, cap: int | None = None):
    """Returns (status, keypoints structured array, descriptors (n,32) uint8)."""
    s = settings or default_settings()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = int(cap if cap is not None else s.nfeatures)
    kp = np.zeros(max(cap, 1), KP_DTYPE)
    desc = np.zeros((max(cap, 1), 32), np.uint8)
    n = C.c_uint32(0)
    table = pattern_table(s.patch_size if s.patch_size in (15, 31) else 15)
    st = lib().oracle_orb_detect(C.byref(s), _p(table), _p(img), w, h, w, _p(kp), _p(desc), cap,
                                 C.byref(n))
    return st, kp[: n.value].copy(), desc[: n.value].copy()


def hamming(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return int(lib().oracle_hamming(_p(a), _p(b)))


def radius_match(qkp, qdesc, tkp, tdesc, radius, qpos=None, qmask=None, tmask=None, max_distance=30,
                 min_difference=1):
    """RadiusMatch (FeatureMatcher.cpp:294-446) over a target KeypointSpatialIndex; returns an
    (n,) DM_DTYPE array in query order."""
    qkp = np.ascontiguousarray(qkp, KP_DTYPE)
    tkp = np.ascontiguousarray(tkp, KP_DTYPE)
    qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
    td = np.ascontiguousarray(tdesc, np.uint8).reshape(-1, 32)
    qp = None if qpos is None else np.ascontiguousarray(qpos, np.float32).reshape(-1, 2)
    qm = None if qmask is None else np.ascontiguousarray(qmask, np.uint8)
    tm = None if tmask is None else np.ascontiguousarray(tmask, np.uint8)
    cap = max(len(qkp), 1)
    out = np.zeros(cap, DM_DTYPE)
    n = lib().oracle_radius_match(_p(qkp), _p(qp), _p(qm), _p(qd), len(qkp), _p(tkp), _p(tm), _p(td), len(tkp),
                                  float(radius), int(max_distance), int(min_difference), _p(out), cap)
    return out[:n].copy()


def local_map_match(qpos, qoct, qdesc, hide, tkp, tdesc, mask, radius=8.0, max_distance=30, min_difference=1):
    """TrackLocalMap's sequential per-map-point matching (orb_oracle.c oracle_local_map_match):
    -> (result (n,) int32 keypoint or -1, updated mask)."""
    qp = np.ascontiguousarray(qpos, np.float32).reshape(-1, 2)
    qo = np.ascontiguousarray(qoct, np.int32)
    qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
    hd = None if hide is None else np.ascontiguousarray(hide, np.int32)
    tk = np.ascontiguousarray(tkp, KP_DTYPE)
    td = np.ascontiguousarray(tdesc, np.uint8).reshape(-1, 32)
    m = np.ascontiguousarray(mask, np.uint8).copy()
    res = np.zeros(max(len(qp), 1), np.int32)
    lib().oracle_local_map_match(_p(qp), _p(qo), _p(qd), _p(hd), len(qp), _p(tk), _p(td), len(tk), _p(m),
                                 float(radius), int(max_distance), int(min_difference), _p(res))
    return res[:len(qp)].copy(), m


def match(desc_a, desc_b, mask_a=None, mask_b=None, max_distance=30, min_difference=1):
    da = np.ascontiguousarray(desc_a, np.uint8).reshape(-1, 32)
    db = np.ascontiguousarray(desc_b, np.uint8).reshape(-1, 32)
    ma = None if mask_a is None else np.ascontiguousarray(mask_a, np.uint8)
    mb = None if mask_b is None else np.ascontiguousarray(mask_b, np.uint8)
    cap = max(len(da), 1)
    out = np.zeros(cap, DM_DTYPE)
    n = lib().oracle_match(_p(da), len(da), _p(ma), _p(db), len(db), _p(mb), max_distance,
                           min_difference, _p(out), cap)
    return out[:n].copy()


def undistort_image(img, k_dist, dist):
    """ImagePreprocessor::UndistortImage (ImagePreprocessor.cpp:71-120): k_dist = (fx, fy, cx, cy),
    dist = OpenCV-ordered coefficients (0, 4, 5 or 8).  Returns (undistorted image, mapx, mapy, K')."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    kd = np.ascontiguousarray(k_dist, np.float32)
    kn = np.array([kd[0], kd[1], np.float32(w) * np.float32(0.5), np.float32(h) * np.float32(0.5)], np.float32)
    dd = np.ascontiguousarray(dist, np.float32)
    mx = np.zeros((h, w), np.float32)
    my = np.zeros((h, w), np.float32)
    lib().oracle_undistort_map(_p(kd), _p(dd), len(dd), _p(kn), w, h, _p(mx), _p(my))
    out = np.zeros((h, w), np.uint8)
    lib().oracle_remap_linear(_p(img), w, h, w, _p(mx), _p(my), w, h, _p(out), w)
    return out, mx, my, kn


def bow_find_leaves(tree, desc):
    """OnlineBow::FindLeafNode (OnlineBow.cpp:289-311) of each descriptor; tree = (node_desc,
    child_start, children)."""
    nd, cs, ch = (np.ascontiguousarray(x) for x in tree)
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    return np.array([lib().oracle_bow_find_leaf(_p(nd), _p(cs), _p(ch), _p(d[i])) for i in range(len(d))], np.uint32)


def bow_train(desc, levels=2, branching=6, max_iter=12, kmedoid=False):
    """OnlineBow::CreateTree (OnlineBow.cpp:325-337, Kmean :451-485; with kmedoid the Kmedoid
    recursion :487-521) over training descriptors (BagOfWordsSettings defaults, MageSettings.h:
    230-232); returns (node_desc, child_start, children)."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    cap = 1
    for _ in range(levels):
        cap = cap * branching + 1
    nd = np.zeros((cap, 32), np.uint8)
    cs = np.zeros(cap + 1, np.uint32)
    ch = np.zeros(max(cap, 1), np.uint32)
    n = lib().oracle_bow_train2(_p(d), len(d), levels, branching, max_iter, _p(nd), _p(cs), _p(ch), cap, int(kmedoid))
    assert n > 0
    return nd[:n].copy(), cs[: n + 1].copy(), ch[: int(cs[n])].copy()


def msvc_shuffle(n):
    """std::shuffle(0..n-1, mt19937{}) as MSVC's STL computes it (InitializeTraining, OnlineBow.cpp:404)."""
    out = np.zeros(max(n, 1), np.uint32)
    lib().oracle_msvc_shuffle(n, _p(out))
    return out[:n]


def mt19937_output(seed, k):
    return int(lib().oracle_mt19937_first(seed, k))


def indexed_match(tree, desc_a, desc_b, mask_a=None, mask_b=None, max_distance=30, min_difference=1):
    """IndexedMatch (FeatureMatcher.cpp:192-292) with BoW candidate lists; (n,) DM_DTYPE in A order."""
    nd, cs, ch = (np.ascontiguousarray(x) for x in tree)
    da = np.ascontiguousarray(desc_a, np.uint8).reshape(-1, 32)
    db = np.ascontiguousarray(desc_b, np.uint8).reshape(-1, 32)
    ma = None if mask_a is None else np.ascontiguousarray(mask_a, np.uint8)
    mb = None if mask_b is None else np.ascontiguousarray(mask_b, np.uint8)
    cap = max(len(da), 1)
    out = np.zeros(cap, DM_DTYPE)
    n = lib().oracle_indexed_match(_p(nd), _p(cs), _p(ch), _p(da), len(da), _p(ma), _p(db), len(db), _p(mb),
                                   int(max_distance), int(min_difference), _p(out), cap)
    return out[:n].copy()


def pose_batch(pb, nsteps, huber, max_error_square):
    """TrackLocalMap::OptimizeCameraPose per problem (fresh BundlerLib, ArePointsFixed); pb is a
    synth.PoseBatch.  Returns dict(pos, r9, qt7, outlier, mean_sq, stats)."""
    K = len(pb.pos)
    E = int(pb.obs_start[-1])
    out = dict(pos=np.zeros((K, 3), np.float32), r9=np.zeros((K, 9), np.float32), qt7=np.zeros((K, 7)),
               outlier=np.zeros(max(E, 1), np.uint8), mean_sq=np.zeros(K, np.float32), stats=np.zeros((K, 2), np.uint32))
    c = lambda a, t: np.ascontiguousarray(a, t)  # noqa: E731
    lib().oracle_ba_pose_batch(K, _p(c(pb.pos, np.float32)), _p(c(pb.r9, np.float32)), _p(c(pb.intr, np.float32)),
                               _p(c(pb.obs_start, np.uint32)), _p(c(pb.points, np.float32)), _p(c(pb.uv, np.float32)),
                               _p(c(pb.info, np.float32)), nsteps, huber, max_error_square, _p(out["pos"]),
                               _p(out["r9"]), _p(out["qt7"]), _p(out["outlier"]), _p(out["mean_sq"]), _p(out["stats"]))
    out["outlier"] = out["outlier"][:E]
    return out


class BundlerOracle:
    """BundlerLib restated on the CPU (same call sequence as the product's BundlerLib)."""

    def __init__(self, points_fixed: bool = False):
        self.h = lib().oracle_ba_create(int(points_fixed))
        self.nc = self.np_ = self.ne = 0

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_ba_destroy(self.h)
            self.h = None

    def set_graph(self, g):
        self.set_cameras(g.pos, g.rot_colmajor, g.intr, g.fixed)
        self.set_points(g.points)
        self.set_observations(g.uv, g.cam, g.pt, g.info)

    def set_cameras(self, pos, r9_colmajor, intr, fixed):
        pos = np.ascontiguousarray(pos, np.float32)
        r9 = np.ascontiguousarray(r9_colmajor, np.float32)
        intr = np.ascontiguousarray(intr, np.float32)
        fixed = np.ascontiguousarray(fixed, np.uint8)
        self.nc = len(pos)
        lib().oracle_ba_set_cameras(self.h, self.nc, _p(pos), _p(r9), _p(intr), _p(fixed))

    def fix_camera(self, idx, fixed=True):
        lib().oracle_ba_fix_camera(self.h, idx, int(fixed))

    def set_points(self, xyz):
        xyz = np.ascontiguousarray(xyz, np.float32)
        self.np_ = len(xyz)
        lib().oracle_ba_set_points(self.h, self.np_, _p(xyz))

    def set_observations(self, uv, cam, pt, info):
        uv = np.ascontiguousarray(uv, np.float32)
        cam = np.ascontiguousarray(cam, np.uint32)
        pt = np.ascontiguousarray(pt, np.uint32)
        info = np.ascontiguousarray(info, np.float32)
        self.ne = len(cam)
        lib().oracle_ba_set_observations(self.h, self.ne, _p(uv), _p(cam), _p(pt), _p(info))

    def set_lambda(self, lam):
        lib().oracle_ba_set_lambda(self.h, lam)

    def set_tethers(self, kind, cam1, cam2, params, weight):
        """kind 0: params (n,) distances; 1: (n, 4) quaternions x,y,z,w; 2: (n, 7) = position
        xyz + quaternion x,y,z,w (BundlerLib::Set*Constraint, BundlerLib.cpp:311-350)."""
        cam1 = np.ascontiguousarray(cam1, np.uint32)
        cam2 = np.ascontiguousarray(cam2, np.uint32)
        params = np.ascontiguousarray(params, np.float32).reshape(-1)
        weight = np.ascontiguousarray(weight, np.float32)
        lib().oracle_ba_set_tethers(self.h, kind, len(cam1), _p(cam1), _p(cam2), _p(params), _p(weight))

    def tether_linearization(self, i):
        """(error, J1, J2) of tether i (all kinds in distance, rotation, transform order)."""
        e = np.zeros(6)
        j1 = np.zeros(36)
        j2 = np.zeros(36)
        d = lib().oracle_ba_tether_linearization(self.h, i, _p(e), _p(j1), _p(j2))
        return e[:d], j1[: 6 * d].reshape(d, 6), j2[: 6 * d].reshape(d, 6)

    def get_lambda(self):
        return float(lib().oracle_ba_get_lambda(self.h))

    def step(self, huber_widths, max_error_square):
        hw = np.ascontiguousarray(huber_widths, np.float32)
        cap = max(self.ne, 1)
        outl = np.zeros(cap, np.uint32)
        n = C.c_uint32(0)
        ms = C.c_float(0)
        lib().oracle_ba_step(self.h, _p(hw), len(hw), max_error_square, _p(outl), cap, C.byref(n),
                             C.byref(ms))
        return float(ms.value), outl[: min(n.value, cap)].copy()

    def poses(self):
        pos = np.zeros((self.nc, 3), np.float32)
        r9 = np.zeros((self.nc, 9), np.float32)
        lib().oracle_ba_get_poses(self.h, _p(pos), _p(r9))
        return pos, r9

    def points(self):
        xyz = np.zeros((self.np_, 3), np.float32)
        lib().oracle_ba_get_points(self.h, _p(xyz))
        return xyz

    def state(self):
        qt = np.zeros((self.nc, 7), np.float64)
        xyz = np.zeros((self.np_, 3), np.float64)
        lib().oracle_ba_get_state(self.h, _p(qt), _p(xyz))
        return qt, xyz

    def stats(self):
        it, tr, rj = C.c_uint64(), C.c_uint64(), C.c_uint64()
        chi, lam = C.c_double(), C.c_double()
        lib().oracle_ba_get_stats(self.h, C.byref(it), C.byref(tr), C.byref(rj), C.byref(chi),
                                  C.byref(lam))
        return dict(iterations=it.value, trials=tr.value, rejected=rj.value, chi2=chi.value,
                    lambda_=lam.value)

    def edge_linearization(self, i):
        err = np.zeros(2)
        jpt = np.zeros(6)
        jp = np.zeros(12)
        lib().oracle_ba_edge_linearization(self.h, i, _p(err), _p(jpt), _p(jp))
        return err, jpt.reshape(2, 3), jp.reshape(2, 6)

    def perturb_camera(self, c, u):
        u = np.ascontiguousarray(u, np.float64)
        lib().oracle_ba_perturb_camera(self.h, c, _p(u))

    def perturb_point(self, p, u):
        u = np.ascontiguousarray(u, np.float64)
        lib().oracle_ba_perturb_point(self.h, p, _p(u))


class OnlineBowOracle:
    """Literal restatement of OnlineBow's keyframe database (OnlineBow.cpp:94-271, 340-449) over an
    oracle tree (bow_train / FindLeafNode in C), float32 throughout.  Test infrastructure only.
    Canonical orders where the reference iterates unordered_maps: ascending node and keyframe id;
    equal scores keep ascending keyframe id (std::sort is unstable)."""

    def __init__(self, tree, qualifying_candidate_score=0.75):
        self.tree = tree
        self.nodes_weight = [np.float32(0)] * len(tree[0])
        self.m_NodeKeyframeMap = {}
        self.m_imageSet = set()
        self.QualifyingCandidateScore = np.float32(qualifying_candidate_score)

    def FindLeafNode(self, desc):
        return int(bow_find_leaves(self.tree, np.asarray(desc, np.uint8).reshape(1, 32))[0])

    def SetNodeWeights(self, training_features, descriptorsCount):  # :340-394
        nImages = len(descriptorsCount)
        leafNodeImageMap = {}
        start = 0
        leaves = bow_find_leaves(self.tree, training_features)
        for imageIndex in range(nImages):
            leafNodeFound = set()
            for j in range(int(descriptorsCount[imageIndex])):
                leafNodeID = int(leaves[start + j])
                if leafNodeID not in leafNodeFound:
                    leafNodeImageMap[leafNodeID] = leafNodeImageMap.get(leafNodeID, 0) + 1
                    leafNodeFound.add(leafNodeID)
            start += int(descriptorsCount[imageIndex])
        for nodeId, count in leafNodeImageMap.items():
            self.nodes_weight[nodeId] = np.float32(math.log(float(np.float32(np.float32(nImages + 1) / np.float32(count)))))  # logf, correctly rounded

    def InsertDescriptors(self, kf, descriptors):  # :413-449
        pts = []
        s = np.float32(0)
        leaves = bow_find_leaves(self.tree, descriptors)
        for i in range(len(leaves)):
            nodeId = int(leaves[i])
            m = self.m_NodeKeyframeMap.setdefault(nodeId, {})
            if kf not in m:
                m[kf] = {"nodeValue": np.float32(0), "indexes": []}
                pts.append(m[kf])
            m[kf]["indexes"].append(i)
            m[kf]["nodeValue"] = np.float32(m[kf]["nodeValue"] + self.nodes_weight[nodeId])
            s = np.float32(s + self.nodes_weight[nodeId])
        if s == 0:
            return
        for p in pts:
            p["nodeValue"] = np.float32(p["nodeValue"] / s)
        self.m_imageSet.add(kf)

    def RemoveImage(self, kf):  # :100-113
        for m in self.m_NodeKeyframeMap.values():
            m.pop(kf, None)
        self.m_imageSet.discard(kf)

    def QueryFeatures(self, desc, kf):  # :115-133
        e = self.m_NodeKeyframeMap.get(self.FindLeafNode(desc), {}).get(kf)
        return [] if e is None else list(e["indexes"])

    def QueryUnknownImage(self, descriptors, maxResults):  # :155-271
        curMap = {}
        s = np.float32(0)
        for leaf in bow_find_leaves(self.tree, descriptors):
            w = self.nodes_weight[int(leaf)]
            curMap[int(leaf)] = np.float32(curMap[int(leaf)] + w) if int(leaf) in curMap else w
            s = np.float32(s + w)
        if s == 0:
            return []
        for k in curMap:
            curMap[k] = np.float32(curMap[k] / s)
        scores = {}
        for nodeId in sorted(curMap):
            imageNodeValue = curMap[nodeId]
            for kf in sorted(self.m_NodeKeyframeMap.get(nodeId, {})):
                keyFrameNodeValue = self.m_NodeKeyframeMap[nodeId][kf]["nodeValue"]
                value = np.float32(np.float32(np.abs(np.float32(imageNodeValue - keyFrameNodeValue)) - np.abs(imageNodeValue))
                                   - np.abs(keyFrameNodeValue))
                scores[kf] = np.float32(scores[kf] + value) if kf in scores else value
        maxScore = np.float32(0)
        for kf in scores:
            scores[kf] = np.float32(-scores[kf] / np.float32(2.0))
            if scores[kf] > maxScore:
                maxScore = scores[kf]
        qualifyingScore = np.float32(maxScore * self.QualifyingCandidateScore)
        v = [(kf, sc) for kf, sc in scores.items() if sc >= qualifyingScore]
        v.sort(key=lambda t: (-t[1], t[0]))
        return [(int(kf), float(sc)) for kf, sc in v[:maxResults]]


def scale_geometry(src_ext, src_k, src_wh, tgt_ext, tgt_k, tgt_wh, depth=2.3):
    """ScaleImageForCameraConfiguration geometry restated (image_oracle.c): k = (fx, fy, cx, cy),
    wh = (width, height).  -> (ok, crop (x, y, w, h), scale, (width, height), (fx, fy, cx, cy))."""
    se, te = np.ascontiguousarray(src_ext, np.float32).reshape(16), np.ascontiguousarray(tgt_ext, np.float32).reshape(16)
    sk, tk = np.ascontiguousarray(src_k, np.float32), np.ascontiguousarray(tgt_k, np.float32)
    sw, tw = np.ascontiguousarray(src_wh, np.uint32), np.ascontiguousarray(tgt_wh, np.uint32)
    crop = np.zeros(4, np.int32)
    scale = np.zeros(1, np.float32)
    owh = np.zeros(2, np.uint32)
    ok_k = np.zeros(4, np.float32)
    ok = lib().oracle_scale_geometry(_p(se), _p(sk), _p(sw), _p(te), _p(tk), _p(tw), float(depth), _p(crop), _p(scale),
                                     _p(owh), _p(ok_k))
    return bool(ok), tuple(int(v) for v in crop), float(scale[0]), tuple(int(v) for v in owh), tuple(ok_k.tolist())


def scale_image_for_camera_configuration(img, src_ext, src_k, tgt_ext, tgt_k, tgt_wh, depth=2.3):
    """The whole ScaleImageForCameraConfiguration: geometry, then resize INTER_LINEAR (or the clone)."""
    h, w = img.shape
    ok, crop, scale, (ow, oh), k = scale_geometry(src_ext, src_k, (w, h), tgt_ext, tgt_k, tgt_wh, depth)
    if not ok:
        return False, None, scale, k
    out = resize_linear(img, ow, oh) if scale != 1.0 else img.copy()
    return True, out, scale, k
