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

import math
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
    # FIXED (deprecated): must stay MapPointRefinementConfidence(0) = 1 - 1/1.5^2 (ValueError
    # otherwise); the information of an observation follows its point's refinement count
    refinement_info: float = float(np.float32(1.0) - np.float32(1.0) / np.float32(1.5) ** 2)  # count 0
    # NewKeyFrameDecision.cpp:196: a new keyframe when the frame tracks fewer than overlap x the
    # reference keyframe's map points + KeyframeDecisionMinTrackingPointCount; the overlap is the
    # console's 0.5 (console.cpp:141; MageSettings.h:86-87).  It has to sit above
    # small_match_ratio, or the SearchRadius match falls back to the position-free wide search first.
    keyframe_ratio: float = 0.5
    keyframe_min: int = 25
    # TrackLocalMap's local-map search between the two OptimizeCameraPose passes
    # (TrackLocalMap.cpp:114-265; TrackLocalMapSettings, MageSettings.h:180-194); 0 keyframes = off.
    # The local map is the last `local_map_keyframes` keyframes (the covisible set of this
    # plane-backprojection map), visited in ascending keyframe id like GetConnectedMapPoints' sorted K1K2s.
    local_map_keyframes: int = 4
    match_search_radius: float = 8.0       # TrackLocalMapSettings::MatchSearchRadius
    local_max_hamming: int = 30            # TrackLocalMapSettings::OrbMatcherSettings
    local_min_hamming_difference: int = 1
    min_view_degrees: float = 60.0         # MinDegreesBetweenCurrentViewAndMapPointView
    image_border: float = 7.5              # FeatureExtractorSettings::GetImageBorder() = PatchSize / 2
    min_tracked: int = 20                  # MinTrackedFeatureCount
    scale_factor: float = 1.5              # the frames' pyramid (ComputeOctave / ComputeDMin / ComputeDMax)
    num_levels: int = 1
    width: int = 1280                      # AnalyzedImage size (PointWithinImageBorder)
    height: int = 720
    # Local bundle adjustment after every new keyframe, as MappingWorker runs it
    # (MappingWorker.cpp:228-371; BundleAdjustSettings / CovisibilitySettings / MappingSettings,
    # MageSettings.h:41-52, 74-79, 253-260): see local_bundle_adjust.  Off by default.
    local_ba: bool = False
    ba_huber: float = 1.8                  # BundleAdjustSettings::HuberWidth
    ba_huber_scale: float = 0.95           # ::HuberWidthScale
    ba_max_outlier_error: float = 7.25     # ::MaxOutlierError (the first maxErrorSquare, BundleAdjust.cpp:375)
    ba_steps_per_run: int = 1              # ::NumStepsPerRun (NumSteps = MinSteps = 1: one call per keyframe)
    ba_low_connectivity_scale: float = 1.5  # ::LowConnectivityIterationsScale
    ba_upper_connections: int = 2000       # CovisibilitySettings::UpperConnectionsForBA
    min_lambda: float = 1e-3               # MappingSettings::MinLambda (PersistLambda on)
    # The window's free keyframes.  0 (default): GetMapPointsAndDistantKeyframes' rule
    # (ThreadSafeMap.cpp:888-957) — the new keyframe Ki and the ring keyframes sharing at least
    # theta map points with it are free, every other observer is fixed (as is the sequence's first
    # keyframe, ThreadSafeMap.cpp:89), theta retuned until the associations lie in
    # [ba_lower_connections, ba_upper_connections] and persisted across windows.  N > 0: the
    # newest N ring keyframes free and the older ones fixed (the round-4/5 harness rule, studies).
    ba_free_keyframes: int = 0
    covis_min_threshold: int = 15          # CovisibilitySettings::CovisMinThreshold (theta's start and floor)
    covis_ba_step: int = 15                # ::CovisBaStepThreshold
    ba_lower_connections: int = 1500       # ::LowerConnectionsForBA
    covis_max_steps: int = 1               # ::MaxSteps (the retune loop runs MaxSteps + 1 times)
    # New map points' depth scaled by 1 + sigma g (g a seeded unit-variance variate per (keyframe
    # frame, keypoint)): the depth error a triangulated point carries (NewMapPointsCreation.cpp:254),
    # instead of the plane back-projection's exact depth; 0 = exact.
    map_point_depth_noise: float = 0.0

    def __post_init__(self):
        # every loop takes an observation's information from MapPointRefinementConfidence of its
        # point's refinement count (TrackLocalMap.cpp:473-475); this field only names the count-0 value
        if np.float32(self.refinement_info) != refinement_confidence(0):
            raise ValueError("refinement_info must be MapPointRefinementConfidence(0) = 1 - 1/1.5^2")

    def min_view_cos(self) -> np.float32:
        """std::cos(mira::deg2rad(degrees)) in float (arcana/math.h:86-90: degrees * (PI / 180))."""
        return _libm_f("cosf", np.float32(self.min_view_degrees) * (np.float32(np.pi) / np.float32(180)))

    def octave_factors(self):
        """ComputeDMax / ComputeDMin factors per keypoint octave (MappingMath.h:32-40) with powf."""
        L, s = self.num_levels, np.float32(self.scale_factor)
        dmax = np.float32([_libm_f("powf", s, np.float32(L) - (np.float32(o) + np.float32(0.5))) for o in range(8)])
        dmin = np.float32([_libm_f("powf", s, np.float32(0) - (np.float32(o) + np.float32(0.5))) for o in range(8)])
        return dmax, dmin


_LIBM = None


def _libm_f(name: str, *args) -> np.float32:
    """A float function of the C library (the host loops' cosf / powf), so every loop uses the
    same rounding."""
    import ctypes as C

    global _LIBM
    if _LIBM is None:
        _LIBM = C.CDLL("libm.so.6")
        for fn, n in (("cosf", 1), ("powf", 2)):
            f = getattr(_LIBM, fn)
            f.restype = C.c_float
            f.argtypes = [C.c_float] * n
    return np.float32(getattr(_LIBM, name)(*[float(np.float32(a)) for a in args]))


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
    id: int = 0          # frame index
    mvd: np.ndarray | None = None   # (n, 3) float32 mean viewing direction
    dmin: np.ndarray | None = None  # (n,) float32 scale-invariance distances
    dmax: np.ndarray | None = None
    # mapping side (local_ba): per point its refinement count (MapPoint::IncrementRefinementCount)
    # and whether the keyframe's own observation of it is still associated; the keyframe's
    # associations to other keyframes' points (its frame's pass-2 inliers): owner keyframe id,
    # point index, keypoint position, alive
    refine: np.ndarray | None = None
    own_alive: np.ndarray | None = None
    assoc_owner: np.ndarray | None = None
    assoc_idx: np.ndarray | None = None
    assoc_uv: np.ndarray | None = None
    assoc_alive: np.ndarray | None = None


def _dot3(a, b):
    """cv::Matx / Vec dot in float32: s = 0, s += a_i b_i left to right."""
    return ((np.float32(0) + a[..., 0] * b[..., 0]) + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def world_position_f32(pose: Pose) -> np.ndarray:
    """Pose::GetWorldSpacePosition (Data/Pose.cpp:110-113): column 3 of Invert(viewMatrix) (Utils/cv.h:
    226-262: the transposed rotation times the negated translation, float 4x4 product)."""
    R, t = pose.R.astype(np.float32), pose.t.astype(np.float32)
    C = np.zeros(3, np.float32)
    for i in range(3):
        s = np.float32(0)
        for k in range(3):
            s = np.float32(s + np.float32(R[k, i] * np.float32(-t[k])))
        C[i] = np.float32(s + np.float32(0))
    return C


DEPTH_NOISE_SEED = 0xDE9785EED
_DEPTH_INV_SD = 1.0 / (65536.0 * math.sqrt(1.0 / 3.0))  # 1 / sd of a sum of four uniform 16-bit draws


def depth_noise_factor(fid: int, n: int, sigma: float) -> np.ndarray:
    """Per keypoint i of keyframe `fid`: 1 + sigma g, g = (a + b + c + d - 131070) / sd with a..d
    the 16-bit fields of splitmix64(seed ^ fid K1 ^ i K2) (a unit-variance, nearly normal variate);
    float64, evaluated in this order by every loop (track.cpp, track.hip)."""
    from .synth import splitmix64

    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = splitmix64(np.uint64(DEPTH_NOISE_SEED) ^ (np.uint64(fid) * np.uint64(0x9E3779B97F4A7C15)) ^
                       (i * np.uint64(0xC2B2AE3D27D4EB4F)))
    m = np.uint64(0xFFFF)
    q = (z & m) + ((z >> np.uint64(16)) & m) + ((z >> np.uint64(32)) & m) + (z >> np.uint64(48))
    g = (q.astype(np.float64) - 131070.0) * _DEPTH_INV_SD
    return 1.0 + float(np.float32(sigma)) * g


def make_keyframe(fid: int, pose: Pose, kp, desc, K, plane_z: float, s: "TrackerSettings") -> Keyframe:
    """A keyframe and its map points: plane back-projection plus MapPoint::
    UpdateMeanViewDirectionAndDistances (Map/MapPoint.cpp:131-154) for a point seen by this keyframe
    alone: mean viewing direction = Normalize(Normalize(point - centre)) (cv::Vec / float scales by
    1.f / length), d = |centre - point|, dmax / dmin = d x the octave's ComputeDMax / DMin factor."""
    factor = depth_noise_factor(fid, len(kp), s.map_point_depth_noise) if s.map_point_depth_noise else None
    pts = backproject_to_plane(kp, pose, K, plane_z, factor)
    C = world_position_f32(pose)
    v = (pts - C).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.sqrt(_dot3(v, v)).astype(np.float32)
        n1 = np.where(d[:, None] == 0, v, v * (np.float32(1) / d)[:, None]).astype(np.float32)
        d2 = np.sqrt(_dot3(n1, n1)).astype(np.float32)
        mvd = np.where(d2[:, None] == 0, n1, n1 * (np.float32(1) / d2)[:, None]).astype(np.float32)
    delta = (C - pts).astype(np.float32)
    dist = np.sqrt((delta[:, 0] * delta[:, 0] + delta[:, 1] * delta[:, 1]) + delta[:, 2] * delta[:, 2]).astype(np.float32)
    fmax, fmin = s.octave_factors()
    octv = np.asarray(kp["octave"], np.int64)
    n = len(kp)
    return Keyframe(pose, kp, desc, pts, fid, mvd, (dist * fmin[octv]).astype(np.float32),
                    (dist * fmax[octv]).astype(np.float32), refine=np.zeros(n, np.uint32),
                    own_alive=np.ones(n, bool), assoc_owner=np.zeros(0, np.int64), assoc_idx=np.zeros(0, np.int64),
                    assoc_uv=np.zeros((0, 2), np.float32), assoc_alive=np.zeros(0, bool))


def point_attributes(kf: Keyframe, s: "TrackerSettings", idx: np.ndarray) -> None:
    """make_keyframe's MapPoint::UpdateMeanViewDirectionAndDistances of kf's points `idx`, again from
    its current pose and points (after a local BA moved them: UpdateData, then SetPosition)."""
    C = world_position_f32(kf.pose)
    pts = kf.points[idx]
    v = (pts - C).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = np.sqrt(_dot3(v, v)).astype(np.float32)
        n1 = np.where(d[:, None] == 0, v, v * (np.float32(1) / d)[:, None]).astype(np.float32)
        d2 = np.sqrt(_dot3(n1, n1)).astype(np.float32)
        kf.mvd[idx] = np.where(d2[:, None] == 0, n1, n1 * (np.float32(1) / d2)[:, None]).astype(np.float32)
    delta = (C - pts).astype(np.float32)
    dist = np.sqrt((delta[:, 0] * delta[:, 0] + delta[:, 1] * delta[:, 1]) + delta[:, 2] * delta[:, 2]).astype(np.float32)
    fmax, fmin = s.octave_factors()
    octv = np.asarray(kf.kp["octave"][idx], np.int64)
    kf.dmin[idx] = (dist * fmin[octv]).astype(np.float32)
    kf.dmax[idx] = (dist * fmax[octv]).astype(np.float32)


def refinement_confidence(count) -> np.ndarray:
    """MapPointRefinementConfidence (Map/MappingMath.h:42-49): 1 - 1 / powf(1.5 + count, 2) in float."""
    c = np.asarray(count, np.float32)
    return (np.float32(1.0) - np.float32(1.0) / np.power(np.float32(1.5) + c, np.float32(2.0))).astype(np.float32)


@dataclass
class BAWindow:
    """One local BA problem in BundlerLib's boundary layout (synth.BAGraph's fields) and how its
    observations map back to the keyframes' associations."""
    pos: np.ndarray
    rot: np.ndarray
    intr: np.ndarray
    fixed: np.ndarray
    points: np.ndarray
    uv: np.ndarray
    cam: np.ndarray
    pt: np.ndarray
    info: np.ndarray
    point_src: list        # (ring position of the owner, point index) per point
    obs_src: list          # ("own" | "assoc", ring position of the observer, index) per observation
    huber_widths: list
    max_error_square: float

    @property
    def rot_colmajor(self) -> np.ndarray:
        return np.ascontiguousarray(np.transpose(self.rot, (0, 2, 1)).reshape(-1, 9))


def _ring_observations(ring):
    """Every alive observation of the ring's map points, per camera: its own points (ascending
    index), then its associations in the order its frame made them (owners outside the ring are
    gone from this loop's map): (cam, owner ring position, point index, u, v, src)."""
    pos_of = {k.id: c for c, k in enumerate(ring)}
    obs = []
    for c, k in enumerate(ring):
        for i in np.nonzero(k.own_alive)[0]:
            obs.append((c, c, int(i), k.kp["x"][i], k.kp["y"][i], ("own", c, int(i))))
        for a in range(len(k.assoc_owner)):
            o = pos_of.get(int(k.assoc_owner[a]))
            if k.assoc_alive[a] and o is not None:
                obs.append((c, o, int(k.assoc_idx[a]), k.assoc_uv[a, 0], k.assoc_uv[a, 1], ("assoc", c, a)))
    return obs


def covisible_window(ring, obs, s: "TrackerSettings", theta: int):
    """GetMapPointsAndDistantKeyframes (ThreadSafeMap.cpp:888-957) over the ring: Kc = the newest
    keyframe Ki and the keyframes sharing >= theta map points with it (CovisibilityGraph::
    GetConnectedKeyframes, CovisibilityGraph.cpp:131-170: the edge weight is the shared-point
    count); the window's points are every point a Kc keyframe observes, its associations every
    observation of those points; theta steps up while the associations exceed
    UpperConnectionsForBA and down (not below CovisMinThreshold) while they are below
    LowerConnectionsForBA, MaxSteps + 1 rounds.  Returns (free ring positions, point keys, theta)."""
    last = len(ring) - 1
    seen = [set() for _ in ring]
    for c, o, i, _, _, _ in obs:
        seen[c].add((o, i))
    weight = [len(seen[c] & seen[last]) for c in range(len(ring))]
    for _ in range(s.covis_max_steps + 1):
        kc = {last} | {c for c in range(last) if weight[c] >= theta}
        pts = set()
        for c in kc:
            pts |= seen[c]
        n_assoc = sum(1 for c, o, i, _, _, _ in obs if (o, i) in pts)
        if n_assoc > s.ba_upper_connections:
            theta += s.covis_ba_step
            continue
        if n_assoc < s.ba_lower_connections and theta > s.covis_min_threshold:
            theta -= s.covis_ba_step
            continue
        break
    return kc, pts, theta


def build_ba_window(ring, K, s: "TrackerSettings", theta: int | None = None):
    """GetMapPointsAndDistantKeyframes + BuildDataForG2O (ThreadSafeMap.cpp:868-960; BundleAdjust.cpp:
    25-193) over this loop's map (the local map's keyframes, ascending id) -> (window or None, the
    covisibility threshold to persist).  Free keyframes: covisible_window's Kc (ba_free_keyframes =
    0), fixed = every other observer and the sequence's first keyframe (ThreadSafeMap.cpp:89, 939);
    or the newest ba_free_keyframes of the ring (at least one fixed).  Points: those a free
    keyframe observes, ascending (owner, index); observations: every alive association of those
    points, per camera: its own points (ascending index), then its associations in the order its
    frame made them.  info = MapPointRefinementConfidence of the point's refinement count.
    NumStepsPerRun and the Huber width scale with the connectivity ratio UpperConnectionsForBA /
    associations (MappingWorker.cpp:254-263)."""
    if theta is None:
        theta = s.covis_min_threshold
    if len(ring) < 2:
        return None, theta
    obs = _ring_observations(ring)
    if s.ba_free_keyframes > 0:
        nfix = max(len(ring) - s.ba_free_keyframes, 1)  # the oldest keyframes are fixed, at least one
        free = set(range(nfix, len(ring)))
        seen_free = {(o, i) for c, o, i, _, _, _ in obs if c in free}
    else:
        free, seen_free, theta = covisible_window(ring, obs, s, theta)
        free = {c for c in free if ring[c].id != 0}  # the map's first keyframe stays fixed
    point_src = sorted(seen_free)
    pidx = {key: n for n, key in enumerate(point_src)}
    obs = [ob for ob in obs if (ob[1], ob[2]) in pidx]
    if not obs or not free:
        return None, theta
    fx, fy, cx, cy = K
    npts = len(point_src)
    points = np.zeros((npts, 3), np.float32)
    refine = np.zeros(npts, np.uint32)
    for n, (o, i) in enumerate(point_src):
        points[n] = ring[o].points[i]
        refine[n] = ring[o].refine[i]
    pt = np.array([pidx[(ob[1], ob[2])] for ob in obs], np.uint32)
    A = len(obs)
    ratio = s.ba_upper_connections // A
    steps = s.ba_steps_per_run
    huber = np.float32(s.ba_huber)
    if ratio > 0:
        steps = steps * int(np.float32(ratio) * np.float32(s.ba_low_connectivity_scale))
        huber = np.float32(huber * _libm_f("powf", np.float32(s.ba_huber_scale), np.float32(ratio)))
    return BAWindow(pos=np.stack([k.pose.t for k in ring]).astype(np.float32),
                    rot=np.stack([k.pose.R for k in ring]).astype(np.float32),
                    intr=np.tile(np.float32([cx, cy, fx, fy]), (len(ring), 1)),
                    fixed=np.array([0 if c in free else 1 for c in range(len(ring))], np.uint8), points=points,
                    uv=np.array([[ob[3], ob[4]] for ob in obs], np.float32),
                    cam=np.array([ob[0] for ob in obs], np.uint32), pt=pt, info=refinement_confidence(refine[pt]),
                    point_src=point_src, obs_src=[ob[5] for ob in obs], huber_widths=[float(huber)] * max(steps, 1),
                    max_error_square=float(np.float32(s.ba_max_outlier_error))), theta


def apply_ba_window(ring, w: BAWindow, outliers, pos, r9, points, s: "TrackerSettings") -> None:
    """AdjustPosesAndMapPoints (ThreadSafeMap.cpp:995-1046) after UpdateData (BundleAdjust.cpp:195-226):
    the outlier associations removed, the free keyframes' poses and every point of the window from
    GetPose / GetPoint (floats), refinement counts + 1, then the points' view attributes again.
    (Map-point culling and the covisibility graph update are outside this loop's map.)"""
    for e in outliers:
        kind, c, i = w.obs_src[int(e)]
        if kind == "own":
            ring[c].own_alive[i] = False
        else:
            ring[c].assoc_alive[i] = False
    for c, k in enumerate(ring):
        if not w.fixed[c]:
            k.pose = Pose(r9[c].reshape(3, 3).T.astype(np.float64), pos[c].astype(np.float64))
    moved = [[] for _ in ring]
    for n, (o, i) in enumerate(w.point_src):
        ring[o].points[i] = points[n]
        ring[o].refine[i] += 1
        moved[o].append(i)
    for c, k in enumerate(ring):  # the moved points' attributes (their owners' poses already updated)
        if moved[c]:
            point_attributes(k, s, np.asarray(moved[c], np.int64))


def local_bundle_adjust(ring, K, s: "TrackerSettings", backend: "Backend", lam, theta=None):
    """One MappingWorker local BA after a new keyframe (NumSteps = 1: one StepBundleAdjustment at
    MaxOutlierError, BundleAdjust.cpp:375-404, with the persisted lambda and covisibility threshold,
    MappingWorker.cpp:237-293).  Returns (the next lambda, the outlier observation count or None when
    there is no window, the next theta)."""
    w, theta = build_ba_window(ring, K, s, theta)
    if w is None:
        return lam, None, theta
    outl, pos, r9, pts, lam_out = backend.bundle_adjust(w, lam)
    apply_ba_window(ring, w, outl, pos, r9, pts, s)
    return max(lam_out, s.min_lambda), len(outl), theta


def local_map_queries(kfs, ref: Keyframe, visited_ref: np.ndarray, hide_ref: np.ndarray, pose: Pose, K,
                      s: "TrackerSettings"):
    """TrackLocalMap.cpp:175-223: the connected keyframes' map points in order (keyframe id, then
    point index), skipping the visited ones (the frame's inlier associations), through
    ProjectMapPointIntoCurrentFrame (:325-370): ProjectUndistorted with the updated pose, IsGoodCandidate
    (:519-554: in front, inside the image border, viewing angle, scale-invariance distance) and
    ComputeOctave (MappingMath.h:13-16).  Returns (positions (n, 2), octaves, descriptors, hidden
    keypoint or -1, (keyframe, point) of each query)."""
    fx, fy, cx, cy = (np.float32(v) for v in K)
    R, t = pose.R.astype(np.float32), pose.t.astype(np.float32)
    C = world_position_f32(pose)
    fwd = R[2].astype(np.float32)  # GetWorldSpaceForward: column 2 of the inverse view matrix
    cmin = s.min_view_cos()
    border, W, H = np.float32(s.image_border), np.float32(s.width), np.float32(s.height)
    log2s = np.float32(math.log2(float(np.float32(s.scale_factor))))
    out_pos, out_oct, out_desc, out_hide, out_src = [], [], [], [], []
    for kf in sorted(kfs, key=lambda k: k.id):
        P = kf.points
        n = len(P)
        if n == 0:
            continue
        cs = [(((np.float32(0) + R[r, 0] * P[:, 0]) + R[r, 1] * P[:, 1]) + R[r, 2] * P[:, 2]) + t[r] * np.float32(1)
              for r in range(3)]
        depth = cs[2].astype(np.float32)
        div = np.where(depth != 0, depth, np.float32(1)).astype(np.float32)
        px = ((cs[0] / div) * fx + cx).astype(np.float32)
        py = ((cs[1] / div) * fy + cy).astype(np.float32)
        ok = ~(depth < 0)
        ok &= (border <= px) & (border <= py) & (px < W - border) & (py < H - border)
        ok &= ~(_dot3(kf.mvd, np.broadcast_to(fwd, kf.mvd.shape)) < cmin)
        dl = (P - C).astype(np.float32)
        d2 = ((dl[:, 0] * dl[:, 0] + dl[:, 1] * dl[:, 1]) + dl[:, 2] * dl[:, 2]).astype(np.float32)
        ok &= ~((d2 < kf.dmin * kf.dmin) | (kf.dmax * kf.dmax < d2))
        is_ref = kf is ref
        if is_ref:
            ok &= ~visited_ref
        idx = np.nonzero(ok)[0]
        octv = []
        keep = []
        for i in idx:
            # (int)roundf(log2f(d / dmin) / log2f(scale) - 0.5f); log2 taken in double and rounded
            r = np.float32(np.sqrt(d2[i]) / kf.dmin[i])
            x = np.float32(np.float32(np.float32(math.log2(float(r))) / log2s) - np.float32(0.5))
            o = int(np.copysign(np.floor(abs(float(x)) + 0.5), float(x)))
            if 0 <= o <= s.num_levels:
                keep.append(i)
                octv.append(o)
        keep = np.asarray(keep, np.int64)
        out_pos.append(np.stack([px[keep], py[keep]], 1))
        out_oct.append(np.asarray(octv, np.int32))
        out_desc.append(kf.desc[keep])
        out_hide.append(hide_ref[keep] if is_ref else np.full(len(keep), -1, np.int32))
        out_src.append((kf, keep))
    if not out_pos:
        return np.zeros((0, 2), np.float32), np.zeros(0, np.int32), np.zeros((0, 32), np.uint8), np.zeros(0, np.int32), []
    return (np.concatenate(out_pos).astype(np.float32), np.concatenate(out_oct), np.concatenate(out_desc),
            np.concatenate(out_hide).astype(np.int32), out_src)


@dataclass
class TrackResult:
    poses: list = field(default_factory=list)      # Pose per frame
    matches: list = field(default_factory=list)    # RadiusMatch count per frame
    inliers: list = field(default_factory=list)    # associations after the outlier removal
    keyframes: list = field(default_factory=list)  # frame indices that became keyframes
    local_matches: list = field(default_factory=list)  # new associations of the local-map search
    ba_outliers: list = field(default_factory=list)  # (keyframe frame, outlier count) per local BA

    def translations(self) -> np.ndarray:
        return np.stack([p.t for p in self.poses])

    def rotations(self) -> np.ndarray:
        return np.stack([p.R for p in self.poses])


def backproject_to_plane(kp: np.ndarray, pose: Pose, K, plane_z: float, factor=None) -> np.ndarray:
    """World points where the keypoints' rays meet the plane Z = plane_z (the scene's depth), the
    ray parameter scaled by `factor` (depth_noise_factor) when given."""
    fx, fy, cx, cy = K
    R = pose.R
    u = (kp["x"].astype(np.float64) - cx) / fx
    v = (kp["y"].astype(np.float64) - cy) / fy
    d = [(u * R[0, j] + v * R[1, j]) + R[2, j] for j in range(3)]  # R^T (u, v, 1)
    C = [-((R[0, j] * pose.t[0] + R[1, j] * pose.t[1]) + R[2, j] * pose.t[2]) for j in range(3)]
    lam = (plane_z - C[2]) / d[2]
    if factor is not None:
        lam = lam * factor
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
    pos = np.stack([(Xc[0] / zs) * fx + cx, (Xc[1] / zs) * fy + cy], 1).astype(np.float32)
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

    def local_map_match(self, qpos, qoct, qdesc, qhide, tkp, tdesc, mask, radius, max_hamming, min_diff):
        """TrackLocalMap's sequential per-point matching -> (keypoint per query or -1, updated mask)"""
        raise NotImplementedError

    def bundle_adjust(self, w: "BAWindow", lam):
        """BuildDataForG2O(w) + SetCurrentLambda(lam) (unless None) + one StepBundleAdjustment(
        w.huber_widths, w.max_error_square) + GetPose / GetPoint -> (outliers, pos (C, 3), r9 (C, 9)
        column-major, points (P, 3), GetCurrentLambda())."""
        raise NotImplementedError


def run_bundler(b, w: "BAWindow", lam, set_lambda, get_lambda):
    """Backend.bundle_adjust on a BundlerLib-shaped object (GPU BundlerLib or the CPU oracle's)."""
    b.set_graph(w)
    if lam is not None:
        set_lambda(lam)
    _, outl = b.step(w.huber_widths, w.max_error_square)
    pos, r9 = b.poses()
    return np.asarray(outl, np.int64), pos, r9, b.points(), float(get_lambda())


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

    def local_map_match(self, qpos, qoct, qdesc, qhide, tkp, tdesc, mask, radius, max_hamming, min_diff):
        from . import matcher

        return matcher.LocalMapMatch(qpos, qoct, qdesc, tkp, tdesc, mask, radius, max_hamming, min_diff,
                                     queryHidden=qhide, device=self.device)

    def bundle_adjust(self, w, lam):
        from . import bundler

        b = bundler.BundlerLib(device=self.device)  # MakeBundler: a fresh BundlerLib per task
        try:
            return run_bundler(b, w, lam, b.SetCurrentLambda, b.GetCurrentLambda)
        finally:
            b.close()


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
                    info=np.broadcast_to(np.asarray(info, np.float32), (n,)).copy())


def pose_from_result(r) -> Pose:
    """GetPose (BundlerLib.cpp:457-465) output -> Pose (float values, as the reference's Pose)."""
    R = r["r9"][0].reshape(3, 3).T.astype(np.float64)
    return Pose(R, r["pos"][0].astype(np.float64))


def track(features, K, first_pose: Pose, plane_z: float, backend: Backend,
          settings: TrackerSettings | None = None, frames: int | None = None) -> TrackResult:
    """Run the loop over precomputed per-frame (keypoints, descriptors); frame 0 is the first
    keyframe at `first_pose` (its map from the scene plane).  Per frame: prediction, RadiusMatch of
    the reference keyframe's points (three radii), OptimizeCameraPose 1, and — with
    local_map_keyframes > 0 — TrackLocalMap's local-map search (TrackLocalMap.cpp:114-265): the
    pass-1 outliers are unassociated (their keypoints hidden from their own points), the local map's
    unvisited points are projected with the updated pose and matched one by one against the
    still-unassociated keypoints, and OptimizeCameraPose 2 runs over the pass-1 inliers followed by
    the new associations; fewer than MinTrackedFeatureCount associations after it is a lost frame."""
    s = settings or TrackerSettings()
    T = len(features) if frames is None else frames
    res = TrackResult()
    kp0, d0 = features[0]
    kf = make_keyframe(0, first_pose, kp0, d0, K, plane_z, s)
    kfs = [kf]
    res.poses.append(first_pose)
    res.matches.append(len(kp0))
    res.inliers.append(len(kp0))
    res.keyframes.append(0)
    res.local_matches.append(0)
    lam = None  # the persisted local-BA lambda (MappingWorker: CurrentLambda)
    theta = s.covis_min_threshold  # the persisted covisibility threshold (MappingWorker: CosVisThreashold)
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

        def lost():  # keep the prediction (relocalisation is outside the hot path)
            res.poses.append(pred)
            res.inliers.append(0)
            res.local_matches.append(0)

        if len(m) < s.min_matches:
            lost()
            continue
        qidx = sel[m["query_idx"]]              # the reference keyframe's matched points
        tidx = m["train_idx"].astype(np.int64)  # their keypoints
        pts = kf.points[qidx]
        uv = np.stack([kp["x"][tidx], kp["y"][tidx]], 1)
        # information per observation: MapPointRefinementConfidence of the point's refinement count
        # (TrackLocalMap.cpp:473-475; every count is 0 without the local BA)
        info = refinement_confidence(kf.refine[qidx])
        steps, huber, err = s.initial_ba
        pose, out = backend.optimize_pose(pred, K, pts, uv, info, steps, huber, err * err)
        keep = ~out
        pts2, uv2, info2 = pts[keep], uv[keep], info[keep]
        own2, idx2 = np.full(int(keep.sum()), kf.id, np.int64), qidx[keep].astype(np.int64)  # the points' sources
        n_new = 0
        if s.local_map_keyframes > 0:
            if not keep.any():  # mapPoints.empty() after the outliers are unassociated (:149-150)
                lost()
                continue
            mask = np.ones(len(kp), bool)
            mask[tidx[keep]] = False
            visited = np.zeros(len(kf.points), bool)
            visited[qidx[keep]] = True
            hide = np.full(len(kf.points), -1, np.int32)
            hide[qidx[out]] = tidx[out]
            lp, lo, ld, lh, src = local_map_queries(kfs, kf, visited, hide, pose, K, s)
            if len(lp):
                r, _ = backend.local_map_match(lp, lo, ld, lh, kp, desc, mask, s.match_search_radius,
                                               s.local_max_hamming, s.local_min_hamming_difference)
                qpts = np.concatenate([k.points[i] for k, i in src]).reshape(-1, 3)
                qown = np.concatenate([np.full(len(i), k.id, np.int64) for k, i in src])
                qidx2 = np.concatenate([np.asarray(i, np.int64) for _, i in src])
                qinfo = np.concatenate([refinement_confidence(k.refine[i]) for k, i in src])
                hit = r >= 0
                n_new = int(hit.sum())
                pts2 = np.concatenate([pts2, qpts[hit]]).astype(np.float32)
                uv2 = np.concatenate([uv2, np.stack([kp["x"][r[hit]], kp["y"][r[hit]]], 1)]).astype(np.float32)
                info2 = np.concatenate([info2, qinfo[hit]]).astype(np.float32)
                own2 = np.concatenate([own2, qown[hit]])
                idx2 = np.concatenate([idx2, qidx2[hit]])
        steps, huber, err = s.final_ba
        pose, out2 = backend.optimize_pose(pose, K, pts2, uv2, info2, steps, huber, err * err)
        n_in = int((~out2).sum())
        if s.local_map_keyframes > 0 and n_in < s.min_tracked:  # TrackLocalMap.cpp:309-314
            lost()
            continue
        res.poses.append(pose)
        res.inliers.append(n_in)
        res.local_matches.append(n_new)
        if n_in < s.keyframe_ratio * len(kf.points) + s.keyframe_min:
            kf = make_keyframe(t, pose, kp, desc, K, plane_z, s)
            inl = ~out2  # the new keyframe's associations: its frame's pass-2 inliers
            kf.assoc_owner, kf.assoc_idx = own2[inl], idx2[inl]
            kf.assoc_uv, kf.assoc_alive = uv2[inl].astype(np.float32), np.ones(int(inl.sum()), bool)
            kfs = (kfs + [kf])[-max(s.local_map_keyframes, 1):]
            res.keyframes.append(t)
            if s.local_ba:
                lam, n_out, theta = local_bundle_adjust(kfs, K, s, backend, lam, theta)
                if n_out is not None:
                    res.ba_outliers.append((t, n_out))
                    res.poses[-1] = kf.pose  # this frame's pose as the BA left its keyframe
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
                               s.final_ba[2], s.refinement_info, s.keyframe_ratio, s.keyframe_min,
                               s.local_map_keyframes, s.match_search_radius, s.local_max_hamming,
                               s.local_min_hamming_difference, float(s.min_view_cos()), s.image_border, s.min_tracked,
                               s.scale_factor, s.num_levels, s.width, s.height, int(s.local_ba), s.ba_huber,
                               s.ba_huber_scale, s.ba_max_outlier_error, s.ba_steps_per_run, s.ba_low_connectivity_scale,
                               s.ba_upper_connections, s.min_lambda, s.ba_free_keyframes, s.covis_min_threshold,
                               s.covis_ba_step, s.ba_lower_connections, s.covis_max_steps, s.map_point_depth_noise)


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
    bo = np.full(max(T, 1), 0xFFFFFFFF, np.uint32)
    _lib.check(_lib.load().mage_track_sequence_device(
        _lib.ptr(d_kp), _lib.ptr(d_desc), int(pitch), _lib.ptr(d_counts), T, _lib.ptr(Kd), _lib.ptr(p0),
        float(plane_z), C.byref(cs), _lib.ptr(poses), _lib.ptr(matches), _lib.ptr(inliers), _lib.ptr(kf),
        _lib.ptr(bo), C.c_void_p(stream) if stream else None))
    res = TrackResult()
    for f in range(T):
        res.poses.append(Pose(poses[f, :9].reshape(3, 3).copy(), poses[f, 9:].copy()))
    res.matches = [int(x) for x in matches[:T]]
    res.inliers = [int(x) for x in inliers[:T]]
    res.keyframes = [int(f) for f in np.nonzero(kf[:T])[0]]
    res.ba_outliers = [(int(f), int(bo[f])) for f in range(T) if bo[f] != 0xFFFFFFFF]
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
