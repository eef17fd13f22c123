"""GPU parity: ORB extraction through the C-ABI vs the CPU oracle (bit-exact).

Parity unpinned against the reference itself; the oracle restates it.
"""
import numpy as np
import pytest

from mageslam_amd import orb, synth

pytestmark = pytest.mark.gpu


def kp_bytes(k):
    return np.ascontiguousarray(k).view(np.uint8)


@pytest.mark.parametrize("shape", [(480, 640), (720, 1280), (37, 53), (7, 7), (200, 131)])
def test_fast_score_map_matches_oracle(gpu, oracle, shape):
    h, w = shape
    rng = np.random.default_rng(h * 1000 + w)
    for img in (synth.frame(3, w, h), rng.integers(0, 256, (h, w), dtype=np.uint8),
                np.full((h, w), 77, np.uint8)):
        for t in (4, 20, 0):
            g = orb.fast_score_map(img, t)
            o = oracle.fast_score_map(img, t)
            assert np.array_equal(g, o), (shape, t)


def test_fast_score_map_extremes(gpu, oracle):
    # saturated rings: 0/255 checkerboards and single bright / dark pixels
    img = np.zeros((64, 64), np.uint8)
    img[::2, ::2] = 255
    img[31, 31] = 255
    img[10:20, 40:50] = 255
    for t in (0, 4, 100, 254, 255):
        assert np.array_equal(orb.fast_score_map(img, t), oracle.fast_score_map(img, t))


@pytest.mark.parametrize("size,nfeat", [((640, 480), 2000), ((1280, 720), 2000), ((640, 480), 440),
                                        ((320, 180), 440)])
def test_detect_and_compute_matches_oracle(gpu, oracle, size, nfeat):
    w, h = size
    det = orb.OrbDetector(nfeatures=nfeat)
    for t in (0, 1, 7):
        img = synth.frame(t, w, h)
        kp, d = det.DetectAndCompute(img)
        st, okp, od = oracle.orb_detect(img, oracle.default_settings(nfeat))
        assert st == 0
        assert len(kp) == len(okp)
        assert np.array_equal(kp_bytes(kp), kp_bytes(okp))
        assert np.array_equal(d, od)


@pytest.mark.parametrize("kw", [dict(patchSize=31), dict(gaussianKernelSize=5), dict(gaussianKernelSize=1),
                                dict(gaussianKernelSize=15), dict(numCellsX=16, numCellsY=8),
                                dict(numCellsX=64, numCellsY=64), dict(fastThreshold=12),
                                dict(strongResponseANMS=60, minRobustFactor=1.0, maxRobustFactor=3.0),
                                dict(featureFactorANMS=1.0, featureStrengthANMS=0.5)])
def test_detect_settings_variants(gpu, oracle, kw):
    det = orb.OrbDetector(nfeatures=1000, **kw)
    m = {"patchSize": "patch_size", "gaussianKernelSize": "gaussian_kernel_size", "numCellsX": "num_cells_x",
         "numCellsY": "num_cells_y", "fastThreshold": "fast_threshold", "strongResponseANMS": "strong_response",
         "minRobustFactor": "min_robust_factor", "maxRobustFactor": "max_robust_factor",
         "featureFactorANMS": "feature_factor", "featureStrengthANMS": "feature_strength"}
    s = oracle.default_settings(1000, **{m[k]: v for k, v in kw.items()})
    rng = np.random.default_rng(5)
    imgs = [synth.frame(2, 640, 480), (rng.random((240, 320)) * 40 + 100).astype(np.uint8)]
    for img in imgs:
        kp, d = det.DetectAndCompute(img)
        st, okp, od = oracle.orb_detect(img, s)
        assert st == 0
        assert np.array_equal(kp_bytes(kp), kp_bytes(okp)), kw
        assert np.array_equal(d, od), kw


def test_raster_path_and_capacity(gpu, oracle):
    # few corners: no retain/ANMS, raster order; capacity smaller than the count truncates
    img = np.full((120, 160), 100, np.uint8)
    rng = np.random.default_rng(4)
    ys, xs = rng.integers(10, 110, 40), rng.integers(10, 150, 40)
    img[ys, xs] = rng.integers(130, 250, 40)  # isolated dots: strict local maxima
    det = orb.OrbDetector(nfeatures=440)
    kp, d = det.DetectAndCompute(img)
    _, okp, od = oracle.orb_detect(img, oracle.default_settings(440))
    assert 0 < len(kp) < 440
    assert np.array_equal(kp_bytes(kp), kp_bytes(okp))
    assert np.array_equal(d, od)
    kp2, d2 = det.DetectAndCompute(img, capacity=3)
    assert np.array_equal(kp_bytes(kp2), kp_bytes(okp[:3]))


def test_empty_and_blank(gpu, oracle):
    det = orb.OrbDetector(nfeatures=440)
    for img in (np.zeros((100, 100), np.uint8), np.zeros((10, 10), np.uint8), np.zeros((1, 1), np.uint8)):
        kp, d = det.DetectAndCompute(img)
        assert len(kp) == 0 and d.shape == (0, 32)


def test_rejects_bad_input(gpu):
    det = orb.OrbDetector()
    with pytest.raises(ValueError):
        det.DetectAndCompute(np.zeros((10, 10, 3), np.uint8))
    from mageslam_amd._lib import MageError

    with pytest.raises(MageError):
        orb.OrbDetector(patchSize=1)
    with pytest.raises(MageError):
        orb.OrbDetector(nlevels=9)
    with pytest.raises(MageError):
        orb.OrbDetector(nlevels=2, scaleFactor=1.0)
    with pytest.raises(MageError):  # random-pattern radius 20 > 18
        orb.OrbDetector(patchSize=41)


def test_batch_device_equals_single(gpu):
    import torch

    w, h, B, cap = 640, 480, 6, 2000
    frames = torch.empty((B, h, w), dtype=torch.uint8, device="cuda")
    orb.synth_frames_device(frames, B, w, h, 10, synth.FRAME_SEED)
    torch.cuda.synchronize()
    host = frames.cpu().numpy()
    for i in range(B):
        assert np.array_equal(host[i], synth.frame(10 + i, w, h)), "GPU frame generator differs from numpy"
    det = orb.OrbDetector(nfeatures=cap)
    kp = torch.zeros((B, cap * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    det.detect_and_compute_batch_device(frames, w, h, kp, desc, n, cap)
    det.device_status()
    kp_h, desc_h, n_h = kp.cpu().numpy(), desc.cpu().numpy(), n.cpu().numpy()
    for i in range(B):
        k1, d1 = det.DetectAndCompute(host[i])
        assert n_h[i] == len(k1)
        assert np.array_equal(kp_h[i, : 28 * n_h[i]], kp_bytes(k1).reshape(-1))
        assert np.array_equal(desc_h[i, : n_h[i]], d1)


def test_720p_properties(gpu):
    # size-independent properties at the benchmark size: unique positions, border respected,
    # canonical order is non-increasing in (r, response) -> responses bounded, count == N
    det = orb.OrbDetector(nfeatures=2000)
    img = synth.frame(100, 1280, 720)
    kp, d = det.DetectAndCompute(img)
    assert len(kp) == 2000
    xy = kp["x"].astype(int) * 10000 + kp["y"].astype(int)
    assert len(np.unique(xy)) == len(xy)
    assert kp["x"].min() >= 7 and kp["x"].max() < 1280 - 7
    assert kp["y"].min() >= 7 and kp["y"].max() < 720 - 7
    assert (kp["size"] == 15).all() and (kp["angle"] == 0).all() and (kp["class_id"] == -1).all()
    kp2, d2 = det.DetectAndCompute(img)
    assert np.array_equal(kp_bytes(kp), kp_bytes(kp2)) and np.array_equal(d, d2)  # deterministic


# ------------------------- pyramid + orientation (the rBRIEF-31 variant) -------------


@pytest.mark.parametrize("kw", [dict(nlevels=4, patchSize=31, useOrientation=True),
                                dict(nlevels=4, patchSize=31, useOrientation=True, gaussianKernelSize=5),
                                dict(nlevels=3, patchSize=31),
                                dict(nlevels=2, patchSize=15, useOrientation=True, scaleFactor=1.2),
                                dict(nlevels=1, patchSize=31, useOrientation=True),
                                dict(nlevels=8, patchSize=31, useOrientation=True, scaleFactor=1.3),
                                # exact 2x levels: cv::resize's INTER_AREA fast path
                                dict(nlevels=3, patchSize=31, useOrientation=True, scaleFactor=2.0)])
@pytest.mark.parametrize("size", [(640, 480), (1280, 720), (333, 211), (1000, 600)])
def test_pyramid_orientation_matches_oracle(gpu, oracle, kw, size):
    w, h = size
    nfeat = 2000
    det = orb.OrbDetector(nfeatures=nfeat, **kw)
    m = {"nlevels": "nlevels", "patchSize": "patch_size", "useOrientation": "use_orientation",
         "gaussianKernelSize": "gaussian_kernel_size", "scaleFactor": "scale_factor"}
    s = oracle.default_settings(nfeat, **{m[k]: v for k, v in kw.items()})
    for t in (0, 5):
        img = synth.frame(t, w, h)
        kp, d = det.DetectAndCompute(img)
        st, okp, od = oracle.orb_detect(img, s)
        assert st == 0
        assert len(kp) == len(okp), (kw, size, t)
        assert np.array_equal(kp_bytes(kp), kp_bytes(okp)), (kw, size, t)
        assert np.array_equal(d, od), (kw, size, t)


@pytest.mark.parametrize("kw", [dict(patchSize=21),
                                dict(patchSize=9, useOrientation=True, nlevels=3),
                                dict(patchSize=25, useOrientation=True),
                                dict(patchSize=21, gaussianKernelSize=5, useOrientation=True, nlevels=2),
                                dict(patchSize=35)])
@pytest.mark.parametrize("size", [(640, 480), (333, 211)])
def test_random_pattern_matches_oracle(gpu, oracle, kw, size):
    # patch sizes other than 15 / 31: MakeRandomPattern + ComputeOrbDescriptors (per-keypoint
    # f32 rotation of the pattern), OpenCVModified.cpp:877-884
    w, h = size
    nfeat = 1500
    det = orb.OrbDetector(nfeatures=nfeat, **kw)
    m = {"nlevels": "nlevels", "patchSize": "patch_size", "useOrientation": "use_orientation",
         "gaussianKernelSize": "gaussian_kernel_size", "scaleFactor": "scale_factor"}
    s = oracle.default_settings(nfeat, **{m[k]: v for k, v in kw.items()})
    for t in (0, 3):
        img = synth.frame(t, w, h)
        kp, d = det.DetectAndCompute(img)
        st, okp, od = oracle.orb_detect(img, s)
        assert st == 0 and len(kp) == len(okp) > 0, (kw, size, t)
        assert np.array_equal(kp_bytes(kp), kp_bytes(okp)), (kw, size, t)
        assert np.array_equal(d, od), (kw, size, t)


def test_pyramid_batch_device_equals_single(gpu):
    import torch

    w, h, B, cap = 640, 480, 5, 2000
    frames = torch.empty((B, h, w), dtype=torch.uint8, device="cuda")
    orb.synth_frames_device(frames, B, w, h, 3, synth.FRAME_SEED)
    det = orb.OrbDetector(nfeatures=cap, nlevels=4, patchSize=31, useOrientation=True)
    kp = torch.zeros((B, cap * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    det.detect_and_compute_batch_device(frames, w, h, kp, desc, n, cap)
    torch.cuda.synchronize()
    host = frames.cpu().numpy()
    for i in range(B):
        k1, d1 = det.DetectAndCompute(host[i])
        ni = int(n[i])
        assert ni == len(k1)
        assert np.array_equal(kp[i, : ni * 28].cpu().numpy(), kp_bytes(k1))
        assert np.array_equal(desc[i, :ni].cpu().numpy(), d1)


# ------------------------- UndistortKeypoints (OrbFeatureDetector.cpp:30-62) -------------------------


@pytest.mark.parametrize("dist", [(-0.12, 0.03, 1e-4, -2e-4, 0.0),
                                  (0.05, -0.01, -3e-4, 1e-4, 0.002, 0.02, -0.005, 0.001),
                                  (-0.3, 0.1, 0.0, 0.0, -0.02)])
def test_undistort_keypoints_matches_oracle(gpu, oracle, dist):
    from mageslam_amd._lib import Calibration

    img = synth.frame(2, 1280, 720)
    kp, _ = orb.OrbDetector(nfeatures=2000).DetectAndCompute(img)
    cd = Calibration.make(900.0, 905.0, 640.0, 360.0, dist)
    cu = Calibration.make(880.0, 880.0, 642.5, 358.0)
    g = orb.UndistortKeypoints(kp, cd, cu)
    pts = np.stack([kp["x"], kp["y"]], 1)
    o = oracle.undistort_points(pts, (900.0, 905.0, 640.0, 360.0), dist, (880.0, 880.0, 642.5, 358.0))
    assert np.array_equal(g["x"], o[:, 0]) and np.array_equal(g["y"], o[:, 1])
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(g[f], kp[f])


def test_undistort_batch_device_and_process(gpu, oracle):
    import torch

    from mageslam_amd._lib import KP_DTYPE, Calibration, MageError

    w, h, B, cap = 640, 480, 3, 1000
    frames = torch.empty((B, h, w), dtype=torch.uint8, device="cuda")
    orb.synth_frames_device(frames, B, w, h, 0, synth.FRAME_SEED)
    det = orb.OrbDetector(nfeatures=cap)
    kp = torch.zeros((B, cap * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    det.detect_and_compute_batch_device(frames, w, h, kp, desc, n, cap)
    before = kp.cpu().numpy().copy()
    cd = Calibration.make(500.0, 500.0, 320.0, 240.0, (-0.2, 0.05, 0.0, 0.0, 0.0))
    cu = Calibration.make(500.0, 500.0, 320.0, 240.0)
    from mageslam_amd import _lib
    import ctypes as C

    _lib.check(_lib.load().mage_undistort_keypoints_batch_device(C.byref(cd), C.byref(cu), _lib.ptr(kp), cap,
                                                                  _lib.ptr(n), B, None))
    torch.cuda.synchronize()
    after = kp.cpu().numpy()
    for i in range(B):
        ni = int(n[i])
        k0 = before[i, : 28 * ni].view(KP_DTYPE)
        k1 = after[i, : 28 * ni].view(KP_DTYPE)
        assert np.array_equal(k1, orb.UndistortKeypoints(k0, cd, cu))
        assert np.array_equal(after[i, 28 * ni:], before[i, 28 * ni:])  # beyond the count: untouched
    # Process: undistortion only when the calibrations differ (OrbFeatureDetector.cpp:96-99)
    fd = orb.OrbFeatureDetector(orb.FeatureExtractorSettings(NumFeatures=cap))
    img = frames[0].cpu().numpy()
    k_same, _ = fd.Process(cu, cu, img)
    k_plain, _ = det.DetectAndCompute(img)
    assert np.array_equal(k_same, k_plain)
    k_und, _ = fd.Process(cd, cu, img)
    assert np.array_equal(k_und, orb.UndistortKeypoints(k_plain, cd, cu))
    with pytest.raises(MageError):
        orb.UndistortKeypoints(k_plain, Calibration(500.0, 500.0, 320.0, 240.0, (C.c_float * 8)(), 3), cu)


# ------------------------- candidate gate (speed-only state, DESIGN.md §2 ORB) -------------------------


def _batch_vs_oracle(det, oracle, frames_np, settings, cap):
    """Runs one device batch of `frames_np` and checks every frame against the oracle."""
    import torch

    B, h, w = frames_np.shape
    frames = torch.from_numpy(frames_np).cuda()
    kp = torch.zeros((B, cap * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(B, dtype=torch.int32, device="cuda")
    det.detect_and_compute_batch_device(frames, w, h, kp, desc, n, cap)
    det.device_status()
    kp_h, desc_h, n_h = kp.cpu().numpy(), desc.cpu().numpy(), n.cpu().numpy()
    for i in range(B):
        st, okp, od = oracle.orb_detect(frames_np[i], settings)
        assert st == 0
        assert n_h[i] == len(okp), i
        assert np.array_equal(kp_h[i, : 28 * n_h[i]], kp_bytes(okp).reshape(-1)), i
        assert np.array_equal(desc_h[i, : n_h[i]], od), i


def test_fast_gate_from_previous_batch(gpu, oracle):
    # batch 1 runs ungated and sets a gate; batch 2 (later frames of the stream) runs gated
    w, h, cap = 640, 480, 2000
    det = orb.OrbDetector(nfeatures=cap)
    s = oracle.default_settings(cap)
    _batch_vs_oracle(det, oracle, np.stack([synth.frame(t, w, h) for t in range(4)]), s, cap)
    st = det.fast_gate_stats()
    assert st["last_gate"] == 0 and st["next_gate"] > 4 and st["last_redo"] == 0
    _batch_vs_oracle(det, oracle, np.stack([synth.frame(t, w, h) for t in range(4, 10)]), s, cap)
    st2 = det.fast_gate_stats()
    assert st2["last_gate"] == st["next_gate"] and st2["last_redo"] == 0


@pytest.mark.parametrize("gate", [250, 120, 60, 5])
def test_fast_gate_forced_mixed_frames(gpu, oracle, gate):
    # forced gates over frames the gate does and does not fit: blank, low-texture, noise,
    # textured; frames above their retain bound take the exact path again
    w, h, cap = 640, 480, 1500
    rng = np.random.default_rng(gate)
    yy, xx = np.mgrid[0:h, 0:w]
    frames = np.stack([synth.frame(3, w, h),
                       np.full((h, w), 128, np.uint8),
                       ((xx + yy) // 5 % 256).astype(np.uint8),
                       rng.integers(0, 256, (h, w), dtype=np.uint8),
                       np.clip(synth.frame(9, w, h).astype(int) // 8 + 100, 0, 255).astype(np.uint8),
                       synth.frame(20, w, h)])
    det = orb.OrbDetector(nfeatures=cap)
    det.set_fast_gate(gate)
    _batch_vs_oracle(det, oracle, frames, oracle.default_settings(cap), cap)
    st = det.fast_gate_stats()
    assert st["last_gate"] == gate
    if gate == 250:
        assert st["last_redo"] == len(frames)
    if gate == 5:
        assert st["last_redo"] >= 1  # the blank frame has no candidates above the gate


def test_fast_gate_pyramid(gpu, oracle):
    # per-level gates (nlevels 4, oriented rBRIEF-31) over two batches, one level forced high
    w, h, cap = 640, 480, 2000
    kw = dict(nlevels=4, patchSize=31, useOrientation=True)
    det = orb.OrbDetector(nfeatures=cap, **kw)
    s = oracle.default_settings(cap, nlevels=4, patch_size=31, use_orientation=True)
    _batch_vs_oracle(det, oracle, np.stack([synth.frame(t, w, h) for t in range(3)]), s, cap)
    det.set_fast_gate(200, level=2)
    _batch_vs_oracle(det, oracle, np.stack([synth.frame(t, w, h) for t in range(3, 7)]), s, cap)
    assert det.fast_gate_stats(level=2)["last_redo"] == 4
    assert det.fast_gate_stats(level=0)["last_gate"] > 4


WIN_BLUR_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from mageslam_amd import orb, synth
from oracle import oracle as O
for (w, h), nfeat in (((640, 480), 2000), ((1280, 720), 2000), ((320, 180), 440)):
    det = orb.OrbDetector(nfeatures=nfeat)
    for t in (0, 3):
        img = synth.frame(t, w, h)
        kp, d = det.DetectAndCompute(img)
        st, okp, od = O.orb_detect(img, O.default_settings(nfeat))
        assert st == 0 and len(kp) == len(okp), (w, h, t)
        assert np.array_equal(np.ascontiguousarray(kp).view(np.uint8), np.ascontiguousarray(okp).view(np.uint8))
        assert np.array_equal(d, od), (w, h, t)
        # keypoints whose 7x7 support leaves the frame take the reflect-101 path
        assert ((kp["x"] < 10) | (kp["y"] < 10) | (kp["x"] > w - 11) | (kp["y"] > h - 11)).any() or w > 640
print("ok")
"""


def test_window_blur_descriptors_match_oracle(gpu):
    """MAGE_WIN_BLUR=1 (describe_win_kernel: the Gaussian per keypoint window on the matrix cores,
    reflect-101 gathers at the border) is bit-exact vs the oracle; the switch is read once per
    process, so the case runs in a child."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parent.parent)
    r = subprocess.run([sys.executable, "-c", WIN_BLUR_CHILD, root], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MAGE_WIN_BLUR="1"), cwd=root)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("kw", [dict(), dict(nlevels=4, patchSize=31, useOrientation=True), dict(patchSize=21),
                                dict(gaussianKernelSize=5)])
def test_describe_partial_waves(gpu, oracle, kw):
    """describe_blurred_kernel / describe_kernel run KP keypoints per wave (8 for the default
    windows, 2 for the rotated ones) and 4 waves per workgroup, each wave staging its keypoints'
    windows in its own LDS region: keypoint counts that end inside a wave or a workgroup (the last
    wave's loads clamp to the last keypoint, its tests stop at n) must stay bit-exact (the audit
    after the matcher's stage-buffer race)."""
    m = {"nlevels": "nlevels", "patchSize": "patch_size", "useOrientation": "use_orientation",
         "gaussianKernelSize": "gaussian_kernel_size"}
    img = synth.frame(4, 640, 480)
    for nfeat in (1, 7, 9, 33, 257, 1001):
        det = orb.OrbDetector(nfeatures=nfeat, **kw)
        kp, d = det.DetectAndCompute(img)
        st, okp, od = oracle.orb_detect(img, oracle.default_settings(nfeat, **{m[k]: v for k, v in kw.items()}))
        assert st == 0 and len(kp) == len(okp) and len(kp) > 0, (kw, nfeat)
        assert np.array_equal(kp_bytes(kp), kp_bytes(okp)), (kw, nfeat)
        assert np.array_equal(d, od), (kw, nfeat)
