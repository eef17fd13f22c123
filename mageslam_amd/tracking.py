"""Tracking loop over the hot path (BASELINE.json C4).

Per frame, the reference's tracker does (Core/MAGESLAM/Source/Tracking):
  * PoseEstimator::TryEstimatePoseFromKeyframe (PoseEstimator.cpp:439-607): project the reference
    keyframe's map points with the predicted pose (ProjectUndistorted), RadiusMatch them against the
    frame's keypoints at SearchRadius, widened to WiderSearchRadius and then ExtraWiderSearchRadius
    without position overrides when too few match (PoseEstimationSettings, MageSettings.h:170-176);
  * TrackLocalMap::RunTrackLocalMap (TrackLocalMap.cpp:37-140): OptimizeCameraPose with
    InitialPoseEstimateBundleAdjustmentSteps x InitialPoseEstimateBundleAdjustmentHuberWidth at
    MaxOutlierErrorPoseEstimation^2, drop the outliers, OptimizeCameraPose again with
    BundleAdjustmentG2OSteps x BundleAdjustmentHuberWidth at MaxOutlierError^2 (MageSettings.h:182-189).
This module runs that sequence on the hot-path kernels: ORB extraction of every frame (batched),
RadiusMatch and the pose-only BundlerLib per frame.  Map creation is NOT the reference's
(MapInitialization / NewMapPointsCreation triangulate; they are outside the hot path): a new
keyframe's keypoints are back-projected onto the scene plane with the keyframe's estimated pose.

`Backend` abstracts the three kernels so the identical loop also runs on the CPU oracle (tests /
bench.py's cpu_baseline leg), which is how the pose parity of the whole loop is measured.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ._lib import KP_DTYPE


@dataclass
class TrackerSettings:
    search_radius: float = 12.0            # PoseEstimationSettings::SearchRadius
    wider_search_radius: float = 24.0      # ::WiderSearchRadius
    extra_wider_search_radius: float = 36.0  # ::ExtraWiderSearchRadius
    small_match_ratio: float = 0.333780871615353  # ::FeatureSmallMatchRatioThreshold
    min_matches: int = 20
    max_hamming: int = 30                  # OrbMatcherSettings::MaxHammingDistance
    min_hamming_difference: int = 1        # OrbMatcherSettings::MinHammingDifference
    initial_ba: tuple = (3, 4.0, 6.0)      # steps, Huber width, MaxOutlierErrorPoseEstimation
    final_ba: tuple = (4, 0.9, 4.5)        # steps, Huber width, MaxOutlierError
    refinement_info: float = float(np.float32(1.0) - np.float32(1.0) / np.float32(1.5) ** 2)  # count 0
    # NewKeyFrameDecision.cpp:196: a new keyframe when the frame tracks fewer than overlap x the
    # reference keyframe's map points + KeyframeDecisionMinTrackingPointCount; the overlap is the
    # console's 0.5 (console.cpp:141; MageSettings.h:86-87).  It has to sit above
    # small_match_ratio, or the SearchRadius match falls back to the position-free wide search first.
    keyframe_ratio: float = 0.5
    keyframe_min: int = 25


@dataclass
class Pose:
    R: np.ndarray  # world -> camera rotation (3, 3) float64
    t: np.ndarray  # view-space translation (3,)

    # elementwise products with left-to-right sums (no BLAS, no FMA): the native loop
    # (csrc/track.cpp) evaluates the same expressions in the same order
    def inverse(self) -> "Pose":
        Rt = np.ascontiguousarray(self.R.T)
        return Pose(Rt, -_mv(Rt, self.t))

    def __mul__(self, o: "Pose") -> "Pose":
        return Pose(_mm(self.R, o.R), _mv(self.R, o.t) + self.t)


def _mv(R, v):
    return np.array([(R[i, 0] * v[0] + R[i, 1] * v[1]) + R[i, 2] * v[2] for i in range(3)], np.float64)


def _mm(A, B):
    return np.array([[(A[i, 0] * B[0, j] + A[i, 1] * B[1, j]) + A[i, 2] * B[2, j] for j in range(3)]
                     for i in range(3)], np.float64)


@dataclass
class Keyframe:
    pose: Pose
    kp: np.ndarray       # its keypoints (KP_DTYPE)
    desc: np.ndarray     # (n, 32)
    points: np.ndarray   # (n, 3) float32 map point per keypoint


@dataclass
class TrackResult:
    poses: list = field(default_factory=list)      # Pose per frame
    matches: list = field(default_factory=list)    # RadiusMatch count per frame
    inliers: list = field(default_factory=list)    # associations after the outlier removal
    keyframes: list = field(default_factory=list)  # frame indices that became keyframes

    def translations(self) -> np.ndarray:
        return np.stack([p.t for p in self.poses])

    def rotations(self) -> np.ndarray:
        return np.stack([p.R for p in self.poses])


def backproject_to_plane(kp: np.ndarray, pose: Pose, K, plane_z: float) -> np.ndarray:
    """World points where the keypoints' rays meet the plane Z = plane_z (the scene's depth)."""
    fx, fy, cx, cy = K
    R = pose.R
    u = (kp["x"].astype(np.float64) - cx) / fx
    v = (kp["y"].astype(np.float64) - cy) / fy
    d = [(u * R[0, j] + v * R[1, j]) + R[2, j] for j in range(3)]  # R^T (u, v, 1)
    C = [-((R[0, j] * pose.t[0] + R[1, j] * pose.t[1]) + R[2, j] * pose.t[2]) for j in range(3)]
    lam = (plane_z - C[2]) / d[2]
    return np.stack([C[j] + lam * d[j] for j in range(3)], 1).astype(np.float32)


def project(points: np.ndarray, pose: Pose, K):
    """ProjectUndistorted (Tracking/Reprojection): float32 view matrix and camera matrix; returns
    (positions (n, 2) float32, in_front mask)."""
    fx, fy, cx, cy = (np.float32(v) for v in K)
    R = pose.R.astype(np.float32)
    t = pose.t.astype(np.float32)
    P = points.astype(np.float32)
    Xc = [((R[i, 0] * P[:, 0] + R[i, 1] * P[:, 1]) + R[i, 2] * P[:, 2]) + t[i] for i in range(3)]
    z = Xc[2]
    ok = z > 0
    zs = np.where(ok, z, np.float32(1))
    pos = np.stack([fx * Xc[0] / zs + cx, fy * Xc[1] / zs + cy], 1).astype(np.float32)
    return pos, ok


class Backend:
    """The three hot-path operations the loop needs."""

    def extract(self, frames: np.ndarray):  # -> list of (kp, desc)
        raise NotImplementedError

    def radius_match(self, qkp, qdesc, tkp, tdesc, radius, qpos, max_hamming, min_diff) -> np.ndarray:
        raise NotImplementedError

    def optimize_pose(self, pose: Pose, K, points, uv, info, steps, huber, max_err_sq):
        """-> (Pose, outlier flags (n,) bool)"""
        raise NotImplementedError


class GpuBackend(Backend):
    """libmage_hot.so: batched ORB, RadiusMatch, batched pose-only BA (one problem)."""

    def __init__(self, nfeatures: int = 2000, device: int = 0, batch: int = 64):
        from . import orb

        self.det = orb.OrbDetector(nfeatures=nfeatures, device=device)
        self.nfeatures, self.device, self.batch = nfeatures, device, batch

    def extract(self, frames):
        import torch

        N = self.nfeatures
        out = []
        if isinstance(frames, np.ndarray):
            frames = torch.from_numpy(np.ascontiguousarray(frames)).to(f"cuda:{self.device}")
        T, H, W = frames.shape
        for s in range(0, T, self.batch):
            fr = frames[s:s + self.batch]
            B = fr.shape[0]
            kp = torch.zeros((B, N * 28), dtype=torch.uint8, device=fr.device)
            desc = torch.zeros((B, N, 32), dtype=torch.uint8, device=fr.device)
            n = torch.zeros(B, dtype=torch.int32, device=fr.device)
            self.det.detect_and_compute_batch_device(fr, W, H, kp, desc, n, N)
            kp_h, desc_h, n_h = kp.cpu().numpy(), desc.cpu().numpy(), n.cpu().numpy()
            for i in range(B):
                out.append((kp_h[i, : 28 * n_h[i]].view(KP_DTYPE).copy(), desc_h[i, : n_h[i]].copy()))
        self.det.device_status()
        return out

    def radius_match(self, qkp, qdesc, tkp, tdesc, radius, qpos, max_hamming, min_diff):
        from . import matcher

        return matcher.RadiusMatch(qkp, qdesc, tkp, tdesc, radius, max_hamming, min_diff,
                                   queryKeypointPositionOverrides=qpos)

    def optimize_pose(self, pose, K, points, uv, info, steps, huber, max_err_sq):
        from . import bundler

        r = bundler.OptimizeCameraPoses(pose_problem(pose, K, points, uv, info), steps, max_err_sq, huber,
                                        device=self.device)
        return pose_from_result(r), r["outlier"].astype(bool)


@dataclass
class _Problem:
    pos: np.ndarray
    r9: np.ndarray
    intr: np.ndarray
    obs_start: np.ndarray
    points: np.ndarray
    uv: np.ndarray
    info: np.ndarray


def pose_problem(pose: Pose, K, points, uv, info) -> _Problem:
    """OptimizeCameraPose's BundlerLib inputs (TrackLocalMap.cpp:445-475): camera 0 = the frame's
    float pose, observation i on map point i."""
    fx, fy, cx, cy = K
    n = len(points)
    return _Problem(pos=pose.t.astype(np.float32)[None], r9=pose.R.astype(np.float32).T.reshape(1, 9),
                    intr=np.float32([[cx, cy, fx, fy]]), obs_start=np.array([0, n], np.uint32),
                    points=np.ascontiguousarray(points, np.float32), uv=np.ascontiguousarray(uv, np.float32),
                    info=np.full(n, info, np.float32))


def pose_from_result(r) -> Pose:
    """GetPose (BundlerLib.cpp:457-465) output -> Pose (float values, as the reference's Pose)."""
    R = r["r9"][0].reshape(3, 3).T.astype(np.float64)
    return Pose(R, r["pos"][0].astype(np.float64))


def track(features, K, first_pose: Pose, plane_z: float, backend: Backend,
          settings: TrackerSettings | None = None, frames: int | None = None) -> TrackResult:
    """Run the loop over precomputed per-frame (keypoints, descriptors); frame 0 is the first
    keyframe at `first_pose` (its map from the scene plane)."""
    s = settings or TrackerSettings()
    T = len(features) if frames is None else frames
    res = TrackResult()
    kp0, d0 = features[0]
    kf = Keyframe(first_pose, kp0, d0, backproject_to_plane(kp0, first_pose, K, plane_z))
    res.poses.append(first_pose)
    res.matches.append(len(kp0))
    res.inliers.append(len(kp0))
    res.keyframes.append(0)
    for t in range(1, T):
        kp, desc = features[t]
        # motion model: constant velocity on SE3 (the tracker's predicted pose)
        prev = res.poses[-1]
        pred = prev if t < 2 else (prev * res.poses[-2].inverse()) * prev
        qpos, front = project(kf.points, pred, K)
        sel = np.nonzero(front)[0]
        qkp, qdesc, qp = kf.kp[sel], kf.desc[sel], qpos[sel]
        m = backend.radius_match(qkp, qdesc, kp, desc, s.search_radius, qp, s.max_hamming, s.min_hamming_difference)
        if len(m) < s.min_matches or len(m) / max(len(sel), 1) < s.small_match_ratio:
            m = backend.radius_match(qkp, qdesc, kp, desc, s.wider_search_radius, qp, s.max_hamming,
                                     s.min_hamming_difference)
        if len(m) < s.min_matches or len(m) / max(len(sel), 1) < s.small_match_ratio:
            m = backend.radius_match(qkp, qdesc, kp, desc, s.extra_wider_search_radius, None, s.max_hamming,
                                     s.min_hamming_difference)
        res.matches.append(len(m))
        if len(m) < s.min_matches:  # lost: keep the prediction (relocalisation is outside the hot path)
            res.poses.append(pred)
            res.inliers.append(0)
            continue
        pts = kf.points[sel[m["query_idx"]]]
        uv = np.stack([kp["x"][m["train_idx"]], kp["y"][m["train_idx"]]], 1)
        steps, huber, err = s.initial_ba
        pose, out = backend.optimize_pose(pred, K, pts, uv, s.refinement_info, steps, huber, err * err)
        keep = ~out
        steps, huber, err = s.final_ba
        pose, out2 = backend.optimize_pose(pose, K, pts[keep], uv[keep], s.refinement_info, steps, huber, err * err)
        n_in = int((~out2).sum())
        res.poses.append(pose)
        res.inliers.append(n_in)
        if n_in < s.keyframe_ratio * len(kf.points) + s.keyframe_min:
            kf = Keyframe(pose, kp, desc, backproject_to_plane(kp, pose, K, plane_z))
            res.keyframes.append(t)
    return res


def track_native(features, K, first_pose: Pose, plane_z: float, settings: TrackerSettings | None = None,
                 device: int = 0) -> TrackResult:
    """The same loop as `track` with GpuBackend, run by the library's native host code
    (mage_track_sequence, csrc/track.cpp): no Python between the per-frame kernel calls."""
    from . import _lib

    s = settings or TrackerSettings()
    T = len(features)
    counts = np.array([len(k) for k, _ in features], np.uint32)
    start = np.zeros(T + 1, np.uint32)
    start[1:] = np.cumsum(counts)
    kp = np.ascontiguousarray(np.concatenate([k for k, _ in features]) if T else np.zeros(0, KP_DTYPE), KP_DTYPE)
    desc = np.ascontiguousarray(np.concatenate([d for _, d in features]).reshape(-1, 32) if T else
                                np.zeros((0, 32), np.uint8), np.uint8)
    cs = _settings_c(s)
    Kd = np.array(K, np.float64)
    p0 = np.concatenate([np.asarray(first_pose.R, np.float64).reshape(9), np.asarray(first_pose.t, np.float64)])
    poses = np.zeros((max(T, 1), 12))
    matches = np.zeros(max(T, 1), np.uint32)
    inliers = np.zeros(max(T, 1), np.uint32)
    kf = np.zeros(max(T, 1), np.uint8)
    import ctypes as C

    _lib.check(_lib.load().mage_track_sequence(_lib.ptr(kp), _lib.ptr(desc), _lib.ptr(start), T, _lib.ptr(Kd),
                                               _lib.ptr(p0), float(plane_z), C.byref(cs), _lib.ptr(poses),
                                               _lib.ptr(matches), _lib.ptr(inliers), _lib.ptr(kf), device))
    res = TrackResult()
    for f in range(T):
        res.poses.append(Pose(poses[f, :9].reshape(3, 3).copy(), poses[f, 9:].copy()))
    res.matches = [int(x) for x in matches[:T]]
    res.inliers = [int(x) for x in inliers[:T]]
    res.keyframes = [int(f) for f in np.nonzero(kf[:T])[0]]
    return res


def _settings_c(s: TrackerSettings):
    from . import _lib

    return _lib.TrackSettingsC(s.search_radius, s.wider_search_radius, s.extra_wider_search_radius,
                               s.small_match_ratio, s.min_matches, s.max_hamming, s.min_hamming_difference,
                               s.initial_ba[0], s.initial_ba[1], s.initial_ba[2], s.final_ba[0], s.final_ba[1],
                               s.final_ba[2], s.refinement_info, s.keyframe_ratio, s.keyframe_min)


def track_native_device(d_kp, d_desc, pitch: int, d_counts, frames: int, K, first_pose: Pose, plane_z: float,
                        settings: TrackerSettings | None = None, stream=None) -> TrackResult:
    """The same loop device-resident (mage_track_sequence_device, csrc/track.hip): features stay
    in device memory as the batched extraction leaves them (torch tensors: keypoints frame-major
    with `pitch` slots per frame, 32-byte descriptors, uint32 counts); the host enqueues every
    frame and synchronises once."""
    import ctypes as C

    from . import _lib

    s = settings or TrackerSettings()
    cs = _settings_c(s)
    Kd = np.array(K, np.float64)
    p0 = np.concatenate([np.asarray(first_pose.R, np.float64).reshape(9), np.asarray(first_pose.t, np.float64)])
    T = int(frames)
    poses = np.zeros((max(T, 1), 12))
    matches = np.zeros(max(T, 1), np.uint32)
    inliers = np.zeros(max(T, 1), np.uint32)
    kf = np.zeros(max(T, 1), np.uint8)
    _lib.check(_lib.load().mage_track_sequence_device(
        _lib.ptr(d_kp), _lib.ptr(d_desc), int(pitch), _lib.ptr(d_counts), T, _lib.ptr(Kd), _lib.ptr(p0),
        float(plane_z), C.byref(cs), _lib.ptr(poses), _lib.ptr(matches), _lib.ptr(inliers), _lib.ptr(kf),
        C.c_void_p(stream) if stream else None))
    res = TrackResult()
    for f in range(T):
        res.poses.append(Pose(poses[f, :9].reshape(3, 3).copy(), poses[f, 9:].copy()))
    res.matches = [int(x) for x in matches[:T]]
    res.inliers = [int(x) for x in inliers[:T]]
    res.keyframes = [int(f) for f in np.nonzero(kf[:T])[0]]
    return res


def features_to_device(features, pitch: int | None = None):
    """Host per-frame (keypoints, descriptors) -> (d_kp, d_desc, pitch, d_counts) torch tensors in
    the batched extraction's layout (tests)."""
    import torch

    T = len(features)
    pitch = int(pitch or max([len(k) for k, _ in features] + [1]))
    kp = np.zeros((T, pitch), KP_DTYPE)
    desc = np.zeros((T, pitch, 32), np.uint8)
    counts = np.zeros(T, np.uint32)
    for f, (k, d) in enumerate(features):
        kp[f, :len(k)] = k
        desc[f, :len(k)] = np.asarray(d).reshape(-1, 32)
        counts[f] = len(k)
    return (torch.from_numpy(kp.view(np.uint8).reshape(T, -1)).cuda(), torch.from_numpy(desc).cuda(), pitch,
            torch.from_numpy(counts.view(np.int32)).cuda())


def pose_rmse(a: TrackResult, b: TrackResult) -> tuple[float, float]:
    """(translation RMSE, rotation RMSE in radians) between two runs over the same frames."""
    n = min(len(a.poses), len(b.poses))
    dt = np.array([np.linalg.norm(a.poses[i].t - b.poses[i].t) for i in range(n)])
    # angle between rotations as 2 asin(|Ra - Rb|_F / sqrt 8): exact for rotation matrices and 0 for
    # identical ones (arccos of the trace is ~1e-4 of noise on float32-rounded matrices)
    dr = [2 * np.arcsin(min(np.linalg.norm(a.poses[i].R - b.poses[i].R) / np.sqrt(8.0), 1.0)) for i in range(n)]
    return float(np.sqrt(np.mean(dt ** 2))), float(np.sqrt(np.mean(np.square(dr))))
