"""ImagePreprocessor::ScaleImageForCameraConfiguration (ImagePreprocessor.cpp:18-65, SURVEY.md
§8(f)3): the overlap-crop geometry and scaled intrinsics bit-exact against the oracle
restatement (oracle/image_oracle.c), and the prepared image byte for byte against the oracle's
OpenCV 3.4.0 resize(INTER_LINEAR) restatement.  Parity with OpenCV itself is unpinned (no
OpenCV here); the geometry's own known answers are checked on the oracle."""
import numpy as np
import pytest

from mageslam_amd import synth


def rigid(yaw=0.0, pitch=0.0, t=(0.0, 0.0, 0.0)):
    R = synth._rot(yaw, pitch)
    M = np.eye(4, dtype=np.float32)
    M[:3, :3] = R
    M[:3, 3] = t
    return M


# (source extrinsics, source (fx, fy, cx, cy), source size, target extrinsics, target K, target size)
CASES = [
    # identical cameras: the crop is the whole frame, scale 1 (the clone branch)
    (rigid(), (900, 900, 640, 360), (1280, 720), rigid(), (900, 900, 640, 360), (1280, 720)),
    # 10 cm stereo baseline, half-resolution target: scale ~0.5
    (rigid(t=(0.1, 0, 0)), (900, 900, 640, 360), (1280, 720), rigid(), (450, 450, 320, 180), (640, 360)),
    # rotated, higher-resolution target (upscale)
    (rigid(0.02, -0.01, (0.06, 0.01, 0)), (500, 505, 320, 240), (640, 480), rigid(-0.01, 0.0, (-0.02, 0, 0.01)),
     (800, 800, 400, 300), (800, 600)),
    # a different aspect and principal point
    (rigid(0.0, 0.03, (0.0, 0.05, 0.02)), (600, 610, 330, 230), (640, 480), rigid(), (900, 900, 640, 360),
     (1280, 720)),
    # a 5 m baseline: the source frame lies right of the target frame, entirely offscreen
    (rigid(t=(-5.0, 0, 0)), (900, 900, 640, 360), (1280, 720), rigid(), (900, 900, 640, 360), (1280, 720)),
    # ... and left of it: every corner projects to x < 0, so the maximum keeps its initial value
    # FLT_MIN (numeric_limits<float>::min(), MageUtil.cpp:31) and the crop reaches x = 0 — not
    # offscreen, as in the reference
    (rigid(t=(5.0, 0, 0)), (900, 900, 640, 360), (1280, 720), rigid(), (900, 900, 640, 360), (1280, 720)),
]


def test_oracle_geometry_known_answers():
    from oracle import oracle as O

    ok, crop, scale, wh, k = O.scale_geometry(*CASES[0][:3], *CASES[0][3:])
    assert ok and crop == (0, 0, 1280, 720) and scale == 1.0 and wh == (1280, 720)
    assert k == (900.0, 900.0, 640.0, 360.0)
    # baseline b at depth d shifts the frame by f b / d pixels; the half-resolution target halves it
    ok, crop, scale, wh, k = O.scale_geometry(*CASES[1][:3], *CASES[1][3:])
    assert ok
    assert abs(crop[0] - (-450 * 0.1 / 2.3)) <= 1 and crop[1] == 0
    assert crop[2] in (640, 641) and scale == pytest.approx(crop[2] / 1280, abs=1e-6)
    assert wh == (int(1280 * np.float32(scale)), int(720 * np.float32(scale)))
    ok, crop, scale, _, _ = O.scale_geometry(*CASES[4][:3], *CASES[4][3:])
    assert not ok  # IsEntirelyOffscreen: the reference returns false
    ok, crop, scale, _, _ = O.scale_geometry(*CASES[5][:3], *CASES[5][3:])
    assert ok and crop[0] == -1956 and crop[0] + crop[2] == 1


def test_oracle_lu_inverse_matches_numpy():
    """The restated cv::Matx44f LU inverse agrees with float64 numpy to float precision (its exact
    rounding is OpenCV's LUImpl order, pinned only by this restatement)."""
    from oracle import oracle as O

    rng = np.random.default_rng(0)
    for _ in range(20):
        T = rigid(*rng.normal(0, 0.3, 2), rng.normal(0, 1, 3))
        ok, crop, scale, wh, k = O.scale_geometry(T, (900, 900, 640, 360), (1280, 720), T, (900, 900, 640, 360),
                                                  (1280, 720))
        # same camera twice: targetToSource = T T^-1 ~ I, so the crop is the whole frame
        assert ok and abs(crop[0]) <= 1 and abs(crop[1]) <= 1 and abs(crop[2] - 1280) <= 1, crop


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)))
def test_scale_image_matches_oracle(gpu, case):
    from oracle import oracle as O

    from mageslam_amd import image
    from mageslam_amd._lib import CameraConfig

    se, sk, swh, te, tk, twh = CASES[case]
    src = CameraConfig.make(se, *sk, *swh)
    tgt = CameraConfig.make(te, *tk, *twh)
    img = synth.frame(case, *swh)
    ok, crop, scale, prep = image.scale_geometry(src, tgt)
    ook, ocrop, oscale, owh, ok_k = O.scale_geometry(se, sk, swh, te, tk, twh)
    assert (ok, crop, np.float32(scale)) == (ook, ocrop, np.float32(oscale))
    assert (prep.width, prep.height) == owh
    assert np.array_equal(np.float32([prep.fx, prep.fy, prep.cx, prep.cy]), np.float32(ok_k))
    gok, gimg, gprep, gscale = image.ScaleImageForCameraConfiguration(src, tgt, img)
    cok, cimg, cscale, _ = O.scale_image_for_camera_configuration(img, se, sk, te, tk, twh)
    assert gok == cok
    if cok:
        assert gimg.shape == cimg.shape and np.array_equal(gimg, cimg)
        assert np.float32(gscale) == np.float32(cscale)


@pytest.mark.gpu
@pytest.mark.parametrize("dst", [(640, 360), (1920, 1080), (977, 533), (1280, 720), (640, 480), (33, 17)])
def test_resize_linear_any_scale(gpu, dst):
    """cv::resize(INTER_LINEAR) 8UC1 at scales the pyramid never uses (up, down, non-uniform, exact 2x
    = INTER_AREA, identity) against the oracle restatement."""
    import torch

    from oracle import oracle as O

    from mageslam_amd import image

    img = synth.frame(3, 1280, 720)
    g = image.resize_linear_device(torch.from_numpy(img).cuda(), *dst)
    torch.cuda.synchronize()
    assert np.array_equal(g.cpu().numpy(), O.resize_linear(img, *dst))
