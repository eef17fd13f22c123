"""The local-BA composition of the tracking loop (tracking.build_ba_window / apply_ba_window /
local_bundle_adjust, MappingWorker.cpp:228-371) on the CPU: the window's structure on a hand-made
keyframe ring, the write-back, and the whole loop over the oracle backend."""
import numpy as np

from mageslam_amd import synth, tracking
from mageslam_amd._lib import KP_DTYPE


def _kf(fid, n, t):
    kp = np.zeros(n, KP_DTYPE)
    kp["x"] = 100 + 10 * np.arange(n)
    kp["y"] = 50 + fid
    pose = tracking.Pose(np.eye(3), np.array([t, 0.0, 0.0]))
    pts = np.stack([np.arange(n, dtype=np.float32), np.zeros(n, np.float32), np.full(n, 5, np.float32)], 1)
    k = tracking.Keyframe(pose, kp, np.zeros((n, 32), np.uint8), pts, fid, refine=np.zeros(n, np.uint32),
                          own_alive=np.ones(n, bool), assoc_owner=np.zeros(0, np.int64), assoc_idx=np.zeros(0, np.int64),
                          assoc_uv=np.zeros((0, 2), np.float32), assoc_alive=np.zeros(0, bool),
                          mvd=np.zeros((n, 3), np.float32), dmin=np.zeros(n, np.float32), dmax=np.zeros(n, np.float32))
    return k


def test_window_structure():
    s = tracking.TrackerSettings(ba_free_keyframes=2)  # the newest-N rule
    k0, k1, k2 = _kf(0, 3, 0.0), _kf(10, 2, 0.1), _kf(20, 2, 0.2)
    # k1 observes k0's point 1 and 2 (the second association dead); k2 observes k1's point 0
    k1.assoc_owner, k1.assoc_idx = np.array([0, 0]), np.array([1, 2])
    k1.assoc_uv, k1.assoc_alive = np.float32([[1, 2], [3, 4]]), np.array([True, False])
    k2.assoc_owner, k2.assoc_idx = np.array([10, 99]), np.array([0, 0])  # keyframe 99 is not in the ring
    k2.assoc_uv, k2.assoc_alive = np.float32([[5, 6], [7, 8]]), np.array([True, True])
    k0.refine[1] = 2
    k1.own_alive[1] = False
    w, _ = tracking.build_ba_window([k0, k1, k2], (900.0, 900.0, 640.0, 360.0), s)
    # points a free keyframe observes: k0's point 1 (by k1), k1's point 0 (own + k2), k2's points
    assert w.point_src == [(0, 1), (1, 0), (2, 0), (2, 1)]
    assert list(w.fixed) == [1, 0, 0]
    # per camera: own alive points in the window, then its associations in order
    assert [src for src in w.obs_src] == [("own", 0, 1), ("own", 1, 0), ("assoc", 1, 0), ("own", 2, 0),
                                          ("own", 2, 1), ("assoc", 2, 0)]
    assert list(w.cam) == [0, 1, 1, 2, 2, 2] and list(w.pt) == [0, 1, 0, 2, 3, 1]
    assert np.allclose(w.uv[2], [1, 2]) and np.allclose(w.uv[5], [5, 6])
    assert w.info[0] == tracking.refinement_confidence(2) and w.info[1] == tracking.refinement_confidence(0)
    assert np.array_equal(w.intr[0], np.float32([640, 360, 900, 900]))
    # 6 associations: ratio 2000 // 6 = 333 steps x 1.5 and Huber 1.8 x 0.95^333 (MappingWorker.cpp:254-263)
    assert len(w.huber_widths) == int(np.float32(333) * np.float32(1.5))
    # write-back: outliers, free poses, points + refinement counts
    pos = np.float32([[0, 0, 0], [0.11, 0, 0], [0.21, 0, 0]])
    r9 = np.tile(np.eye(3, dtype=np.float32).reshape(9), (3, 1))
    pts = np.float32([[9, 9, 9], [8, 8, 8], [7, 7, 7], [6, 6, 6]])
    tracking.apply_ba_window([k0, k1, k2], w, [2, 3], pos, r9, pts, s)
    assert not k1.assoc_alive[0] and not k2.own_alive[0]
    assert k0.pose.t[0] == 0.0 and np.isclose(k1.pose.t[0], 0.11) and np.isclose(k2.pose.t[0], 0.21)
    assert np.array_equal(k0.points[1], [9, 9, 9]) and np.array_equal(k2.points[1], [6, 6, 6])
    assert k0.refine[1] == 3 and k0.refine[0] == 0 and k1.refine[0] == 1
    assert k0.dmax[1] > 0 and k0.dmax[0] == 0  # attributes of the moved points only


def test_single_keyframe_has_no_window():
    w, theta = tracking.build_ba_window([_kf(0, 3, 0.0)], (900.0, 900.0, 640.0, 360.0), tracking.TrackerSettings())
    assert w is None and theta == 15


def _covis_ring():
    # k1 (id 10) shares 2 points with the newest keyframe k3, k2 shares 1, k0 (id 0) none
    k0, k1, k2, k3 = _kf(0, 2, 0.0), _kf(10, 2, 0.1), _kf(20, 2, 0.2), _kf(30, 3, 0.3)
    k2.assoc_owner, k2.assoc_idx = np.array([10]), np.array([0])
    k2.assoc_uv, k2.assoc_alive = np.float32([[1, 1]]), np.array([True])
    k3.assoc_owner, k3.assoc_idx = np.array([10, 10]), np.array([0, 1])
    k3.assoc_uv, k3.assoc_alive = np.float32([[2, 2], [3, 3]]), np.array([True, True])
    return [k0, k1, k2, k3]


def test_covisibility_window():
    """GetMapPointsAndDistantKeyframes (ThreadSafeMap.cpp:888-957): Kc = the new keyframe and the
    ones sharing >= theta points with it; theta steps up while the associations exceed the upper
    bound; the window holds every point a Kc keyframe observes, the other observers fixed."""
    K = (900.0, 900.0, 640.0, 360.0)
    # theta 1: Kc = {k3, k1, k2}, 10 associations > 9 -> theta 2: Kc = {k3, k1}, 8 associations
    s = tracking.TrackerSettings(covis_min_threshold=1, covis_ba_step=1, ba_lower_connections=0,
                                 ba_upper_connections=9)
    w, theta = tracking.build_ba_window(_covis_ring(), K, s, 1)
    assert theta == 2
    assert list(w.fixed) == [1, 0, 1, 0]
    assert w.point_src == [(1, 0), (1, 1), (3, 0), (3, 1), (3, 2)]
    assert w.obs_src == [("own", 1, 0), ("own", 1, 1), ("assoc", 2, 0), ("own", 3, 0), ("own", 3, 1), ("own", 3, 2),
                         ("assoc", 3, 0), ("assoc", 3, 1)]
    assert list(w.cam) == [1, 1, 2, 3, 3, 3, 3, 3] and list(w.pt) == [0, 1, 0, 2, 3, 4, 0, 1]
    # one retune round only (MaxSteps 0): theta 1 stays too wide, the loop ends with theta 2 and
    # the last round's window (Kc = {k3, k1, k2})
    s0 = tracking.TrackerSettings(covis_min_threshold=1, covis_ba_step=1, ba_lower_connections=0,
                                  ba_upper_connections=9, covis_max_steps=0)
    w0, theta0 = tracking.build_ba_window(_covis_ring(), K, s0, 1)
    assert theta0 == 2 and list(w0.fixed) == [1, 0, 0, 0] and len(w0.obs_src) == 10
    # too few associations: theta steps down (3 -> 2 -> 1) while above CovisMinThreshold; the
    # window is the last round's (theta 2: Kc = {k3, k1}), the returned theta already lowered
    s1 = tracking.TrackerSettings(covis_min_threshold=1, covis_ba_step=1, ba_lower_connections=100)
    w1, theta1 = tracking.build_ba_window(_covis_ring(), K, s1, 3)
    assert theta1 == 1 and list(w1.fixed) == [1, 0, 1, 0]
    w1b, theta1b = tracking.build_ba_window(_covis_ring(), K, s1, 1)  # at the floor: no step
    assert theta1b == 1 and list(w1b.fixed) == [1, 0, 0, 0]
    # the sequence's first keyframe (id 0) is never free, even when covisible; its points count
    ring = _covis_ring()
    ring[3].assoc_owner = np.array([0, 10, 10])
    ring[3].assoc_idx = np.array([1, 0, 1])
    ring[3].assoc_uv, ring[3].assoc_alive = np.float32([[4, 4], [2, 2], [3, 3]]), np.array([True, True, True])
    w2, _ = tracking.build_ba_window(ring, K, tracking.TrackerSettings(covis_min_threshold=1, covis_ba_step=1,
                                                                       ba_lower_connections=0), 1)
    assert w2.fixed[0] == 1 and (0, 0) in w2.point_src and (0, 1) in w2.point_src


def test_depth_noise_factor():
    f = tracking.depth_noise_factor(7, 20000, 0.02)
    assert np.array_equal(f, tracking.depth_noise_factor(7, 20000, 0.02))
    assert not np.array_equal(f, tracking.depth_noise_factor(8, 20000, 0.02))
    assert abs(f.mean() - 1.0) < 1e-3 and abs(f.std() - 0.02) < 1e-3
    # an independent restatement of one entry (splitmix64 in Python integers)
    M = (1 << 64) - 1
    z = (0xDE9785EED ^ ((7 * 0x9E3779B97F4A7C15) & M) ^ ((5 * 0xC2B2AE3D27D4EB4F) & M))
    z = (z + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    z ^= z >> 31
    q = sum((z >> (16 * k)) & 0xFFFF for k in range(4))
    g = (q - 131070.0) * (1.0 / (65536.0 * np.sqrt(1.0 / 3.0)))
    assert f[5] == 1.0 + float(np.float32(0.02)) * g


def test_oracle_loop_with_local_ba(oracle):
    from oracle.tracking_backend import OracleBackend

    seq = synth.scene_sequence(64, 640, 480, step=0.06)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    ob = OracleBackend(1000)
    feats = ob.extract(frames)
    s = tracking.TrackerSettings(local_ba=True, width=640, height=480)
    r = tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, ob, s)
    gt = tracking.TrackResult(poses=[tracking.Pose(seq.R[i], seq.t[i]) for i in range(len(seq.R))])
    assert len(r.ba_outliers) >= 1 and [f for f, _ in r.ba_outliers] == r.keyframes[1:]
    assert tracking.pose_rmse(r, gt)[0] < 0.03 and min(r.inliers[1:]) >= 100
