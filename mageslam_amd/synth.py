"""Seeded synthetic inputs for the hot path.

Frames: a world texture T(u, v) of 8x8-px cells with a uniform gray level from a splitmix64
hash, plus a 3x3-px layer of +-24, clamped to [0, 255]; frame t = T(x + 3t, y + 2t), an
integer pan so consecutive frames overlap and have true matches.  The same function is
implemented on the GPU (`mage_synth_frames` in csrc/synth.hip) so the benchmark's frames are
generated in HBM; tests check both agree byte for byte.

BA graph (C3): 50 pinhole cameras on a line looking +z, 5000 points each seen by 20
consecutive cameras (100k observations), 0.5 px noise, 1% outliers, cameras 0-9 fixed.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

FRAME_SEED = 0x5EEDF00D
BA_SEED = 0xBA5EBA11
K1 = np.uint64(0x9E3779B97F4A7C15)
K2 = np.uint64(0xC2B2AE3D27D4EB4F)
FINE_SALT = np.uint64(0xA5A5A5A5)


def splitmix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (z + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def texture(u: np.ndarray, v: np.ndarray, seed: int = FRAME_SEED) -> np.ndarray:
    """World texture T(u, v) for non-negative integer coordinates (uint8)."""
    s = np.uint64(seed)
    u = u.astype(np.uint64)
    v = v.astype(np.uint64)
    with np.errstate(over="ignore"):
        base = splitmix64(s ^ ((u >> np.uint64(3)) * K1) ^ ((v >> np.uint64(3)) * K2))
        fine = splitmix64(s ^ FINE_SALT ^ ((u // np.uint64(3)) * K1) ^ ((v // np.uint64(3)) * K2))
    g = (base >> np.uint64(56)).astype(np.int32)
    f = ((fine >> np.uint64(56)) % np.uint64(49)).astype(np.int32) - 24
    return np.clip(g + f, 0, 255).astype(np.uint8)


def frame(t: int, width: int, height: int, seed: int = FRAME_SEED) -> np.ndarray:
    """Frame t of the panning sequence, shape (height, width), uint8."""
    y, x = np.mgrid[0:height, 0:width]
    return texture(x + 3 * t, y + 2 * t, seed)


def frames(t0: int, count: int, width: int, height: int, seed: int = FRAME_SEED) -> np.ndarray:
    return np.stack([frame(t0 + i, width, height, seed) for i in range(count)])


@dataclass
class BAGraph:
    """Inputs of one BundlerLib problem in the reference's boundary layout."""

    pos: np.ndarray  # (C,3) float32 view-space translation t (X_cam = R X + t)
    rot: np.ndarray  # (C,3,3) float32 rotation R (row-major here; C-ABI takes column-major)
    intr: np.ndarray  # (C,4) float32 {cx, cy, fx, fy}
    fixed: np.ndarray  # (C,) uint8
    points: np.ndarray  # (P,3) float32 initial (perturbed) positions
    uv: np.ndarray  # (E,2) float32 observations
    cam: np.ndarray  # (E,) uint32
    pt: np.ndarray  # (E,) uint32
    info: np.ndarray  # (E,) float32
    true_points: np.ndarray
    true_pos: np.ndarray
    true_rot: np.ndarray

    @property
    def rot_colmajor(self) -> np.ndarray:
        """(C,9) Eigen column-major layout used by SetCameraPose (BundleAdjust.cpp:46-55)."""
        return np.ascontiguousarray(np.transpose(self.rot, (0, 2, 1)).reshape(-1, 9))


def _rot(yaw: float, pitch: float = 0.0, roll: float = 0.0) -> np.ndarray:
    cy, sy = np.cos(yaw), np.sin(yaw)
    cp, sp = np.cos(pitch), np.sin(pitch)
    cr, sr = np.cos(roll), np.sin(roll)
    ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
    rz = np.array([[cr, -sr, 0], [sr, cr, 0], [0, 0, 1]])
    return rz @ rx @ ry


def refinement_confidence(count: np.ndarray) -> np.ndarray:
    """MapPointRefinementConfidence (Core/.../Source/Map/MappingMath.h:42-49), float32."""
    c = count.astype(np.float32)
    return (np.float32(1.0) - np.float32(1.0) / np.power(np.float32(1.5) + c, np.float32(2.0))).astype(np.float32)


def ba_graph(
    cameras: int = 50,
    points: int = 5000,
    obs_per_point: int = 20,
    fixed_cameras: int = 10,
    seed: int = BA_SEED,
    noise_px: float = 0.5,
    outlier_frac: float = 0.01,
) -> BAGraph:
    """Synthetic local-BA window (SURVEY.md §8(d) 'BA graph (C3)')."""
    rng = np.random.default_rng(seed)
    f, cx, cy = 900.0, 640.0, 360.0
    obs_per_point = min(obs_per_point, cameras)
    # true cameras: centres at x = 0.1 i, looking +z, yaw ~ U(-5, 5) deg
    true_rot = np.zeros((cameras, 3, 3))
    true_pos = np.zeros((cameras, 3))
    for i in range(cameras):
        R = _rot(np.deg2rad(rng.uniform(-5, 5)))
        centre = np.array([0.1 * i, 0.0, 0.0])
        true_rot[i] = R
        true_pos[i] = -R @ centre  # t = -R c
    span = max(cameras - obs_per_point + 1, 1)
    xs = rng.uniform(-1, 6, points) if cameras >= 50 else rng.uniform(-1, 0.1 * cameras + 1, points)
    true_pts = np.stack([xs, rng.uniform(-1.5, 1.5, points), rng.uniform(4, 8, points)], axis=1)
    starts = rng.integers(0, span, points)
    cam = (starts[:, None] + np.arange(obs_per_point)[None, :]).reshape(-1).astype(np.uint32)
    pt = np.repeat(np.arange(points), obs_per_point).astype(np.uint32)
    Xc = np.einsum("eij,ej->ei", true_rot[cam], true_pts[pt]) + true_pos[cam]
    uv = np.stack([f * Xc[:, 0] / Xc[:, 2] + cx, f * Xc[:, 1] / Xc[:, 2] + cy], axis=1)
    uv += rng.normal(0, noise_px, uv.shape)
    n_out = int(round(outlier_frac * len(cam)))
    out_idx = rng.choice(len(cam), n_out, replace=False)
    ang = rng.uniform(0, 2 * np.pi, n_out)
    mag = rng.uniform(15, 30, n_out)
    uv[out_idx] += np.stack([mag * np.cos(ang), mag * np.sin(ang)], axis=1)
    # initial estimates: rotation N(0, 0.3 deg) per axis, translation N(0, 0.01); points N(0, 0.02)
    rot0 = np.zeros_like(true_rot)
    pos0 = np.zeros_like(true_pos)
    for i in range(cameras):
        if i < fixed_cameras:
            rot0[i], pos0[i] = true_rot[i], true_pos[i]
        else:
            d = np.deg2rad(rng.normal(0, 0.3, 3))
            rot0[i] = _rot(d[0], d[1], d[2]) @ true_rot[i]
            pos0[i] = true_pos[i] + rng.normal(0, 0.01, 3)
    pts0 = true_pts + rng.normal(0, 0.02, true_pts.shape)
    fixed = np.zeros(cameras, np.uint8)
    fixed[:fixed_cameras] = 1
    info = refinement_confidence(np.arange(points)[pt] % 6)
    intr = np.tile(np.array([cx, cy, f, f], np.float32), (cameras, 1))
    return BAGraph(
        pos=pos0.astype(np.float32),
        rot=rot0.astype(np.float32),
        intr=intr,
        fixed=fixed,
        points=pts0.astype(np.float32),
        uv=uv.astype(np.float32),
        cam=cam,
        pt=pt,
        info=info,
        true_points=true_pts,
        true_pos=true_pos,
        true_rot=true_rot,
    )


def quat_from_rot(R: np.ndarray) -> np.ndarray:
    """Unit quaternion (x, y, z, w) of a rotation matrix (w >= 0)."""
    R = np.asarray(R, np.float64)
    w = np.sqrt(max(0.0, 1.0 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.sqrt(max(0.0, 1.0 + R[0, 0] - R[1, 1] - R[2, 2])) / 2
    y = np.sqrt(max(0.0, 1.0 - R[0, 0] + R[1, 1] - R[2, 2])) / 2
    z = np.sqrt(max(0.0, 1.0 - R[0, 0] - R[1, 1] + R[2, 2])) / 2
    x = np.copysign(x, R[2, 1] - R[1, 2])
    y = np.copysign(y, R[0, 2] - R[2, 0])
    z = np.copysign(z, R[1, 0] - R[0, 1])
    q = np.array([x, y, z, w])
    return q / np.linalg.norm(q)


@dataclass
class Tethers:
    """Camera-camera constraints in the BundlerLib setter shapes (BundlerLib.cpp:311-350):
    distance (cam1, cam2, distance, weight), rotation (cam1, cam2, quaternion xyzw, weight),
    transform (cam1, cam2, position xyz + quaternion xyzw, weight)."""
    distance: tuple
    rotation: tuple
    transform: tuple


def ba_tethers(g: BAGraph, seed: int = BA_SEED + 7, count: int = 4, weight: float = 50.0) -> Tethers:
    """Tethers measured on the true poses of `g` (slightly perturbed), mirroring KeyframeBuilder's
    distance / three-dof / extrinsic tethers (BundleAdjust.cpp:57-105, 155-189).  Pairs mix free
    and fixed cameras; one pair of fixed cameras is included (an inactive edge)."""
    rng = np.random.default_rng(seed)
    C = len(g.pos)
    nfix = int(g.fixed.sum())
    free = np.arange(nfix, C)

    def pairs(k):
        a = rng.choice(free, k)
        b = np.where(rng.random(k) < 0.3, rng.integers(0, max(nfix, 1), k), rng.choice(free, k))
        b = np.where(b == a, (a + 1) % C, b)
        return a.astype(np.uint32), b.astype(np.uint32)

    R, t = g.true_rot, g.true_pos
    # distance between the SE3Quat translations (EdgeScaleConstraint::computeError)
    c1, c2 = pairs(count)
    if nfix >= 2:
        c1[-1], c2[-1] = 0, 1  # both fixed: not an active edge
    d = np.linalg.norm(t[c2] - t[c1], axis=1) * (1 + rng.normal(0, 0.01, count))
    dist = (c1, c2, d.astype(np.float32), np.full(count, weight, np.float32))
    # relative rotation (T1^-1 T2).rotation()
    c1, c2 = pairs(count)
    q = np.stack([quat_from_rot(R[a].T @ R[b]) for a, b in zip(c1, c2)]).astype(np.float32)
    rot = (c1, c2, q, np.full(count, weight / 5, np.float32))
    # relative transform C with log(T2^-1 C T1) = 0 at the truth: C = T2 T1^-1
    c1, c2 = pairs(count)
    p7 = []
    for a, b in zip(c1, c2):
        Rc = R[b] @ R[a].T
        tc = t[b] - Rc @ t[a]
        p7.append(np.concatenate([tc + rng.normal(0, 0.002, 3), quat_from_rot(Rc)]))
    tr = (c1, c2, np.asarray(p7, np.float32), np.full(count, weight, np.float32))
    return Tethers(distance=dist, rotation=rot, transform=tr)


def _hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(len(a), len(b)) Hamming distances of 32-byte descriptors."""
    ab = np.unpackbits(np.ascontiguousarray(a, np.uint8).reshape(-1, 32), axis=1).astype(np.int32)
    bb = np.unpackbits(np.ascontiguousarray(b, np.uint8).reshape(-1, 32), axis=1).astype(np.int32)
    return ab @ (1 - bb).T + (1 - ab) @ bb.T


def msvc_shuffle(n: int) -> np.ndarray:
    """std::shuffle(0..n-1, mt19937{}) as MSVC's STL computes it (OnlineBow::InitializeTraining,
    OnlineBow.cpp:404): a default-seeded (5489) engine, target t swapped with _Rng_from_urng(t + 1)
    = one 32-bit draw r kept when r // (t+1) < 0xFFFFFFFF // (t+1) or 0xFFFFFFFF % (t+1) == t,
    giving r % (t+1).  numpy's MT19937 with legacy seeding is std::mt19937 (same raw outputs)."""
    bg = np.random.MT19937(0)
    bg._legacy_seeding(5489)
    perm = list(range(n))
    mask = 0xFFFFFFFF
    raw = iter(())
    for t in range(1, n):
        index = t + 1
        while True:
            r = next(raw, None)
            if r is None:
                raw = iter(bg.random_raw(4096).tolist())
                r = next(raw)
            if r // index < mask // index or mask % index == index - 1:
                off = r % index
                break
        if off != t:
            perm[t], perm[off] = perm[off], perm[t]
    return np.array(perm, np.int64)


def bow_tree(train: np.ndarray, levels: int = 2, branching: int = 6, max_iter: int = 12):
    """OnlineBow::CreateTree (OnlineBow.cpp:325-337) restated in numpy: Kmean (:451-485) with
    InitializeTraining's shuffle (msvc_shuffle), IterateClusteringKmean (:587-614: the groups are
    those of the last iteration's assignment, made before its center update), KmeanCenter (:551-585)
    and FindCluster (:631-638, first smallest distance); BagOfWordsSettings defaults
    (MageSettings.h:230-232).  Returns (node_desc (N, 32) u8, child_start (N + 1,) u32,
    children (N - 1,) u32)."""
    train = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
    nodes = [np.zeros(32, np.uint8)]
    kids: list[list[int]] = [[]]

    def kmean(parent: int, desc: np.ndarray, level: int) -> None:
        perm = msvc_shuffle(len(desc))
        centers = [desc[i].copy() for i in perm[:branching]]
        it = 0
        while True:
            it += 1
            d = _hamming_matrix(desc, np.stack(centers))
            assign = np.argmin(d, axis=1)  # first minimum, as std::min_element
            changed = 0
            for g in range(len(centers)):
                members = desc[assign == g]
                bits = np.unpackbits(members, axis=1).reshape(-1, 32, 8)[:, :, ::-1]  # LSB first
                half = (len(members) + 1) // 2
                newbits = (bits.sum(axis=0) >= half).astype(np.uint8)  # KmeanCenter majority
                new = np.packbits(newbits[:, ::-1], axis=1).reshape(32)
                if not np.array_equal(new, centers[g]):
                    changed += 1
                centers[g] = new
            if not (it < max_iter and changed > 0):
                break
        ids = []
        for c in centers:
            ids.append(len(nodes))
            nodes.append(c)
            kids.append([])
        kids[parent].extend(ids)
        if level < levels:
            for g, nid in enumerate(ids):
                sub = desc[assign == g]
                if len(sub) > 1:
                    kmean(nid, sub, level + 1)

    if len(train):
        kmean(0, train, 1)
    child_start = np.zeros(len(nodes) + 1, np.uint32)
    child_start[1:] = np.cumsum([len(k) for k in kids])
    children = np.array([c for k in kids for c in k], np.uint32)
    return np.stack(nodes).astype(np.uint8), child_start, children


@dataclass
class PoseBatch:
    """Independent pose-only problems (TrackLocalMap::OptimizeCameraPose inputs, TrackLocalMap.cpp:
    421-501): one camera each, observations obs_start[k] .. obs_start[k+1]-1 on fixed map points."""
    pos: np.ndarray  # (K, 3) f32 view-space t
    r9: np.ndarray  # (K, 9) f32 column-major R
    intr: np.ndarray  # (K, 4) f32 {cx, cy, fx, fy}
    obs_start: np.ndarray  # (K + 1,) u32
    points: np.ndarray  # (E, 3) f32
    uv: np.ndarray  # (E, 2) f32
    info: np.ndarray  # (E,) f32
    true_pos: np.ndarray
    true_rot: np.ndarray


def pose_batch(problems: int = 256, obs: int = 600, seed: int = BA_SEED + 1, noise_px: float = 0.5,
               outlier_frac: float = 0.05, vary: bool = True) -> PoseBatch:
    """K frames of a 720p camera (fx = fy = 900) tracking map points 3-10 m ahead: observation =
    projection + N(0, noise_px) with outlier_frac offset by U(10, 40) px; initial pose = the true
    one perturbed by N(0, 0.5 deg) per axis and N(0, 0.02) in translation (a motion-model
    prediction); refinement counts 0..5.  With `vary`, per-problem observation counts vary."""
    rng = np.random.default_rng(seed)
    f, cx, cy = 900.0, 640.0, 360.0
    counts = rng.integers(max(obs // 2, 1), obs + obs // 2 + 1, problems) if vary else np.full(problems, obs)
    obs_start = np.zeros(problems + 1, np.uint32)
    obs_start[1:] = np.cumsum(counts)
    E = int(obs_start[-1])
    pos = np.zeros((problems, 3))
    r9 = np.zeros((problems, 9))
    true_pos = np.zeros((problems, 3))
    true_rot = np.zeros((problems, 3, 3))
    pts = np.zeros((E, 3))
    uv = np.zeros((E, 2))
    for k in range(problems):
        R = _rot(rng.uniform(-0.5, 0.5), rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1))
        c = rng.normal(0, 2, 3)
        t = -R @ c
        true_pos[k], true_rot[k] = t, R
        n = int(counts[k])
        # points in the camera frustum: pixel uniform, depth 3-10 m
        u = rng.uniform(20, 1260, n)
        v = rng.uniform(20, 700, n)
        z = rng.uniform(3, 10, n)
        Xc = np.stack([(u - cx) / f * z, (v - cy) / f * z, z], axis=1)
        Xw = (Xc - t) @ R  # R^T (Xc - t)
        s = slice(int(obs_start[k]), int(obs_start[k + 1]))
        pts[s] = Xw
        o = np.stack([u, v], axis=1) + rng.normal(0, noise_px, (n, 2))
        bad = rng.random(n) < outlier_frac
        ang = rng.uniform(0, 2 * np.pi, n)
        mag = rng.uniform(10, 40, n)
        o[bad] += np.stack([mag * np.cos(ang), mag * np.sin(ang)], axis=1)[bad]
        uv[s] = o
        d = np.deg2rad(rng.normal(0, 0.5, 3))
        R0 = _rot(d[0], d[1], d[2]) @ R
        pos[k] = t + rng.normal(0, 0.02, 3)
        r9[k] = R0.T.reshape(9)  # column-major
    info = refinement_confidence(rng.integers(0, 6, E))
    intr = np.tile(np.array([cx, cy, f, f], np.float32), (problems, 1))
    return PoseBatch(pos=pos.astype(np.float32), r9=r9.astype(np.float32), intr=intr, obs_start=obs_start,
                     points=pts.astype(np.float32), uv=uv.astype(np.float32), info=info, true_pos=true_pos,
                     true_rot=true_rot)


# ------------------------------------------------------------------------------------------
# C4 tracking sequence: a textured plane seen by a moving 720p camera
# ------------------------------------------------------------------------------------------
SCENE_PLANE_Z = 5.0
SCENE_TEXEL_SCALE = 180.0  # texels per metre: ~1 texel per pixel at 5 m with f = 900
SCENE_TEXEL_OFFSET = 1 << 20


@dataclass
class SceneSequence:
    """Ground truth of a tracking sequence: per frame world -> camera rotation R (row-major), the
    camera centre C and the view-space translation t = -R C (Pose::GetViewSpacePosition)."""
    R: np.ndarray  # (T, 3, 3)
    C: np.ndarray  # (T, 3)
    fx: float
    fy: float
    cx: float
    cy: float
    width: int
    height: int

    @property
    def t(self) -> np.ndarray:
        return -np.einsum("tij,tj->ti", self.R, self.C)

    def cams(self) -> np.ndarray:
        """(T, 12) float64: R row-major, C — mage_synth_scene_device's camera records."""
        return np.ascontiguousarray(np.concatenate([self.R.reshape(-1, 9), self.C], 1), np.float64)


def scene_sequence(frames: int, width: int = 1280, height: int = 720, step: float = 0.015,
                   origin: tuple = (0.0, 0.0)) -> SceneSequence:
    """A 'video.mp4-shaped' hand-held pan over the plane: ~2.7 px of motion per frame at 720p plus
    slow yaw / pitch / roll and depth oscillations (BASELINE.json C4).  `origin` shifts the camera
    path over the plane (C5: every rank's sequence starts elsewhere, rank_origin)."""
    f = 900.0 * width / 1280.0
    t = np.arange(frames, dtype=np.float64)
    yaw = 0.03 * np.sin(t / 17.0)
    pitch = 0.02 * np.sin(t / 23.0)
    roll = 0.01 * np.sin(t / 31.0)
    R = np.stack([_rot(a, b, c) for a, b, c in zip(yaw, pitch, roll)])
    C = np.stack([step * t + origin[0], 0.08 * np.sin(t / 19.0) + origin[1], 0.15 * np.sin(t / 29.0)], 1)
    return SceneSequence(R=R, C=C, fx=f, fy=f, cx=width / 2.0, cy=height / 2.0, width=width, height=height)


def rank_origin(rank: int) -> tuple:
    """Start of rank r's camera path on the plane (C5: independent sequences)."""
    return (0.37 * rank, -0.21 * rank)


def scene_frames(seq: SceneSequence, first: int = 0, count: int | None = None, seed: int = FRAME_SEED) -> np.ndarray:
    """(count, H, W) uint8 renderings, byte-identical to mage_synth_scene_device (same fp64 order)."""
    count = len(seq.R) - first if count is None else count
    y, x = np.mgrid[0:seq.height, 0:seq.width]
    dx = (x.astype(np.float64) - seq.cx) / seq.fx
    dy = (y.astype(np.float64) - seq.cy) / seq.fy
    out = np.zeros((count, seq.height, seq.width), np.uint8)
    for i in range(count):
        c = seq.cams()[first + i]
        dwx = (c[0] * dx + c[3] * dy) + c[6]
        dwy = (c[1] * dx + c[4] * dy) + c[7]
        dwz = (c[2] * dx + c[5] * dy) + c[8]
        lam = (SCENE_PLANE_Z - c[11]) / dwz
        X = c[9] + lam * dwx
        Y = c[10] + lam * dwy
        u = np.floor(X * SCENE_TEXEL_SCALE).astype(np.int64) + SCENE_TEXEL_OFFSET
        v = np.floor(Y * SCENE_TEXEL_SCALE).astype(np.int64) + SCENE_TEXEL_OFFSET
        out[i] = texture(u, v, seed)
    return out
