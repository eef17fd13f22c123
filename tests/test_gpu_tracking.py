"""GPU parity of the whole tracking loop (BASELINE.json C4): ORB extraction, RadiusMatch, the
pose-only BundlerLib and TrackLocalMap's local-map search on the GPU vs the same loop on the CPU
oracle, over a synthetic hand-held sequence of a textured plane.  Bar (north star): pose RMSE <=
1e-4 (translation, rotation in rad); the per-frame match / inlier / local-map association counts
and keyframe decisions must be identical."""
import numpy as np
import pytest

from mageslam_amd import synth, tracking

pytestmark = pytest.mark.gpu


def test_scene_renderer_matches_numpy(gpu):
    import torch

    from mageslam_amd import _lib

    seq = synth.scene_sequence(6, 640, 480)
    cams = torch.from_numpy(seq.cams()).cuda()
    out = torch.zeros((6, 480, 640), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().mage_synth_scene_device(_lib.ptr(out), 6, 640, 480, 640 * 480, _lib.ptr(cams), seq.fx,
                                                   seq.fy, seq.cx, seq.cy, synth.SCENE_PLANE_Z,
                                                   synth.SCENE_TEXEL_SCALE, synth.SCENE_TEXEL_OFFSET,
                                                   synth.FRAME_SEED, None))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), synth.scene_frames(seq))


def _same(a, b):
    assert a.matches == b.matches and a.inliers == b.inliers and a.keyframes == b.keyframes
    assert all(np.array_equal(x.R, y.R) and np.array_equal(x.t, y.t) for x, y in zip(a.poses, b.poses))


def test_tracking_loop_gpu_vs_oracle(gpu, oracle):
    from oracle.tracking_backend import OracleBackend

    seq = synth.scene_sequence(36, 640, 480)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gb, ob = tracking.GpuBackend(1000), OracleBackend(1000)
    gf, of = gb.extract(frames), ob.extract(frames)
    for (k1, d1), (k2, d2) in zip(gf, of):
        assert np.array_equal(k1.view(np.uint8), k2.view(np.uint8)) and np.array_equal(d1, d2)
    gt = tracking.TrackResult(poses=[tracking.Pose(seq.R[i], seq.t[i]) for i in range(len(seq.R))])
    for nk in (4, 0):  # with and without TrackLocalMap's local-map search
        s = tracking.TrackerSettings(local_map_keyframes=nk, width=640, height=480)
        g = tracking.track(gf, K, p0, synth.SCENE_PLANE_Z, gb, s)
        o = tracking.track(of, K, p0, synth.SCENE_PLANE_Z, ob, s)
        assert g.matches == o.matches and g.inliers == o.inliers and g.keyframes == o.keyframes
        assert g.local_matches == o.local_matches
        rt, rr = tracking.pose_rmse(g, o)
        assert rt <= 1e-4 and rr <= 1e-4, (rt, rr)
        # and the loop actually tracks: within a couple of centimetres of the ground truth at 5 m
        assert tracking.pose_rmse(g, gt)[0] < 0.03
        assert min(g.inliers[1:]) >= 100
        if nk:
            assert sum(g.local_matches) > 0
        # the native loops (mage_track_sequence, mage_track_sequence_device) are the same specification
        n = tracking.track_native(gf, K, p0, synth.SCENE_PLANE_Z, settings=s)
        _same(n, g)
        d = tracking.track_native_device(*tracking.features_to_device(gf), len(gf), K, p0, synth.SCENE_PLANE_Z,
                                         settings=s)
        _same(d, g)


def test_tracking_loop_720p_gpu_vs_oracle(gpu, oracle):
    """C4 at 1280 x 720 over 64 frames with keyframe switches: the device-resident loop
    (mage_track_sequence_device, local map on) against the oracle loop, frame by frame."""
    from oracle.tracking_backend import OracleBackend

    seq = synth.scene_sequence(64, 1280, 720, step=0.06)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gf = tracking.GpuBackend(2000).extract(frames)
    ob = OracleBackend(2000)
    of = ob.extract(frames)
    for (k1, d1), (k2, d2) in zip(gf, of):
        assert np.array_equal(k1.view(np.uint8), k2.view(np.uint8)) and np.array_equal(d1, d2)
    s = tracking.TrackerSettings()
    d = tracking.track_native_device(*tracking.features_to_device(gf), len(gf), K, p0, synth.SCENE_PLANE_Z,
                                     settings=s)
    o = tracking.track(of, K, p0, synth.SCENE_PLANE_Z, ob, s)
    assert len(o.keyframes) >= 3 and sum(o.local_matches) > 0
    assert d.matches == o.matches and d.inliers == o.inliers and d.keyframes == o.keyframes
    rt, rr = tracking.pose_rmse(d, o)
    assert rt <= 1e-4 and rr <= 1e-4, (rt, rr)


@pytest.mark.parametrize("noise,free", [(0.0, 0), (0.02, 0), (0.0, 2)])
def test_tracking_loop_local_ba_720p_device_vs_oracle(gpu, oracle, noise, free):
    """C4 composed with the local BA MappingWorker runs after every new keyframe
    (tracking.local_bundle_adjust: the covisibility window of GetMapPointsAndDistantKeyframes — or
    the newest `free` keyframes — one StepBundleAdjustment at MaxOutlierError with the persisted
    lambda and theta, poses / points / refinement counts written back before the next frame
    tracks), with exact and with noisy map-point depth: the device loop (mage_track_sequence_device,
    BundlerLib between frames) and the Python loop on the GPU backend against the oracle loop at
    1280 x 720 over 96 frames — identical matches, inliers, keyframes and BA outlier counts, pose
    RMSE <= 1e-4."""
    from oracle.tracking_backend import OracleBackend

    seq = synth.scene_sequence(96, 1280, 720, step=0.06)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gb = tracking.GpuBackend(2000)
    gf = gb.extract(frames)
    ob = OracleBackend(2000)
    of = ob.extract(frames)
    s = tracking.TrackerSettings(local_ba=True, map_point_depth_noise=noise, ba_free_keyframes=free)
    o = tracking.track(of, K, p0, synth.SCENE_PLANE_Z, ob, s)
    g = tracking.track(gf, K, p0, synth.SCENE_PLANE_Z, gb, s)
    d = tracking.track_native_device(*tracking.features_to_device(gf), len(gf), K, p0, synth.SCENE_PLANE_Z,
                                     settings=s)
    assert len(o.ba_outliers) >= 2, o.ba_outliers  # at least two windows
    for r in (g, d):
        assert r.matches == o.matches and r.inliers == o.inliers and r.keyframes == o.keyframes
        assert r.ba_outliers == o.ba_outliers
        rt, rr = tracking.pose_rmse(r, o)
        assert rt <= 1e-4 and rr <= 1e-4, (rt, rr)
    _same(d, g)  # the device loop and the Python loop over the same GPU kernels: bit-identical
    # the BA changed the map: without it the same frames give other poses
    n = tracking.track(gf, K, p0, synth.SCENE_PLANE_Z, gb, tracking.TrackerSettings(map_point_depth_noise=noise))
    assert any(not np.array_equal(a.t, b.t) for a, b in zip(n.poses, g.poses))


def test_native_tracking_loop_depth_noise(gpu):
    """The seeded map-point depth error (depth_noise.hpp / tracking.depth_noise_factor) is the same
    arithmetic in the host loop (mage_track_sequence), the device loop and the Python loop:
    bit-identical poses, and different ones from the exact-depth map."""
    seq = synth.scene_sequence(100, 1280, 720, step=0.06)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gb = tracking.GpuBackend(2000)
    gf = gb.extract(frames)
    s = tracking.TrackerSettings(map_point_depth_noise=0.05)
    g = tracking.track(gf, K, p0, synth.SCENE_PLANE_Z, gb, s)
    n = tracking.track_native(gf, K, p0, synth.SCENE_PLANE_Z, settings=s)
    d = tracking.track_native_device(*tracking.features_to_device(gf), len(gf), K, p0, synth.SCENE_PLANE_Z, settings=s)
    assert len(g.keyframes) >= 2
    _same(n, g)
    _same(d, g)
    e = tracking.track(gf, K, p0, synth.SCENE_PLANE_Z, gb, tracking.TrackerSettings())
    assert any(not np.array_equal(a.t, b.t) for a, b in zip(e.poses, g.poses))


def test_native_tracking_loop_720p_keyframes(gpu):
    """A 720p pan long enough for keyframe switches: native loop == Python loop over the GPU
    kernels, frame by frame (poses bit-identical), and within a centimetre of the ground truth."""
    seq = synth.scene_sequence(160, 1280, 720)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gb = tracking.GpuBackend(2000)
    gf = gb.extract(frames)
    g = tracking.track(gf, K, p0, synth.SCENE_PLANE_Z, gb)
    n = tracking.track_native(gf, K, p0, synth.SCENE_PLANE_Z)
    assert len(g.keyframes) >= 2 and sum(g.local_matches) > 0
    assert n.matches == g.matches and n.inliers == g.inliers and n.keyframes == g.keyframes
    assert all(np.array_equal(a.R, b.R) and np.array_equal(a.t, b.t) for a, b in zip(n.poses, g.poses))
    gt = tracking.TrackResult(poses=[tracking.Pose(seq.R[i], seq.t[i]) for i in range(len(seq.R))])
    assert tracking.pose_rmse(n, gt)[0] < 0.01


def test_native_tracking_errors(gpu):
    from mageslam_amd._lib import MageError

    p0 = tracking.Pose(np.eye(3), np.zeros(3))
    assert tracking.track_native([], (500.0, 500.0, 320.0, 240.0), p0, 5.0).poses == []
    with pytest.raises(MageError):
        from mageslam_amd import _lib

        _lib.check(_lib.load().mage_track_sequence(None, None, None, 3, None, None, 5.0, None, None, None, None, None, 0))


def test_device_tracking_loop_equals_native(gpu):
    """mage_track_sequence_device (every per-frame decision on the device) == the host-driven
    native loop, frame by frame, over a 720p pan with keyframe switches."""
    seq = synth.scene_sequence(120, 1280, 720)
    frames = synth.scene_frames(seq)
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gf = tracking.GpuBackend(2000).extract(frames)
    for nk in (4, 1, 0):
        s = tracking.TrackerSettings(local_map_keyframes=nk)
        n = tracking.track_native(gf, K, p0, synth.SCENE_PLANE_Z, settings=s)
        d = tracking.track_native_device(*tracking.features_to_device(gf), len(gf), K, p0, synth.SCENE_PLANE_Z,
                                         settings=s)
        assert len(n.keyframes) >= 2
        _same(d, n)


def test_device_tracking_loop_fallbacks_and_lost(gpu):
    """The device-side decisions of the fallback radii and of lost frames: a sequence with
    feature-less frames (lost: prediction kept, no keyframe) and strict settings that force the
    wider and the position-free searches."""
    seq = synth.scene_sequence(30, 640, 480)
    frames = synth.scene_frames(seq).copy()
    frames[10:13] = 128  # blank: no keypoints at all
    frames[20] = np.roll(frames[20], 9, axis=1)  # a jump the 12 px search misses
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gf = tracking.GpuBackend(1000).extract(frames)
    for s in (tracking.TrackerSettings(width=640, height=480),
              tracking.TrackerSettings(small_match_ratio=0.9, min_matches=200, width=640, height=480),
              tracking.TrackerSettings(min_tracked=900, width=640, height=480),  # lost after the local map
              tracking.TrackerSettings(local_map_keyframes=0, width=640, height=480)):
        n = tracking.track_native(gf, K, p0, synth.SCENE_PLANE_Z, settings=s)
        d = tracking.track_native_device(*tracking.features_to_device(gf, pitch=1000), len(gf), K, p0,
                                         synth.SCENE_PLANE_Z, settings=s)
        assert 0 in n.inliers[1:]
        _same(d, n)
