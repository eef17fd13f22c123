"""GPU parity: frame undistortion (ImagePreprocessor::UndistortImage, ImagePreprocessor.cpp:71-120)
and NV12 / GRAYSCALE8 ingest (CreateGrayCVMat, Utils/cv.cpp:8-28) vs the CPU oracle.

Bit-exact: the CV_32FC1 maps (float bits) and the remapped frames.
"""
import numpy as np
import pytest

from mageslam_amd import image, orb, synth
from mageslam_amd._lib import Calibration

pytestmark = pytest.mark.gpu

DISTS = [[], [-0.28, 0.07, 0.001, -0.0005, 0.01],
         [0.9, -0.3, 0.0007, 0.0002, 0.02, 1.2, -0.2, 0.05]]


@pytest.mark.parametrize("dist", DISTS)
def test_undistort_maps_and_frames(gpu, oracle, dist):
    w, h = 1280, 720
    kd = (910.0, 905.0, 652.5, 349.0)
    cal = Calibration.make(*kd, dist)
    u = image.Undistorter(cal, w, h)
    img = synth.frame(3, w, h)
    ref, mx, my, kn = oracle.undistort_image(img, kd, np.float32(dist))
    gx, gy = u.maps()
    assert np.array_equal(gx.view(np.uint32), mx.view(np.uint32)) and np.array_equal(gy.view(np.uint32), my.view(np.uint32))
    assert (u.undistorted.cx, u.undistorted.cy, u.undistorted.fx, u.undistorted.ndist) == (kn[2], kn[3], kn[0], 0)
    assert np.array_equal(u(img), ref)


def test_undistort_odd_size_shift_and_preprocessor_cache(gpu, oracle):
    w, h = 333, 97  # width not a multiple of 4: scalar tail path
    img = synth.frame(1, w, h)
    kd = (150.0, 150.0, w * 0.5 + 2.0, h * 0.5 - 1.0)
    ref, *_ = oracle.undistort_image(img, kd, np.zeros(5, np.float32))
    pp = image.ImagePreprocessor()
    out, ucal = pp.UndistortImage(img, Calibration.make(*kd, [0, 0, 0, 0, 0]))
    assert np.array_equal(out, ref)
    u0 = pp._u
    pp.UndistortImage(img, Calibration.make(*kd, [0, 0, 0, 0, 0]))
    assert pp._u is u0  # CachedUndistortDataValid: same size and calibration reuse the maps


def test_undistort_batch_device_nv12(gpu, oracle):
    """A batch of NV12 frames (Y plane first, pitch 1.5 w h) undistorted in place of a copy."""
    import torch

    w, h, B = 640, 480, 5
    kd = (520.0, 515.0, 322.0, 236.0)
    dist = [-0.2, 0.05, 0.0005, -0.0003, 0.0]
    u = image.Undistorter(Calibration.make(*kd, dist), w, h)
    pitch = image.frame_pitch(w, h, image.NV12)
    host = np.zeros((B, pitch), np.uint8)
    frames = [synth.frame(t, w, h) for t in range(B)]
    for i, f in enumerate(frames):
        host[i, : w * h] = f.reshape(-1)
        host[i, w * h:] = 128  # chroma
    src = torch.from_numpy(host).cuda()
    dst = torch.zeros((B, w * h), dtype=torch.uint8, device="cuda")
    u.batch_device(src, w, pitch, dst, w, w * h, B)
    torch.cuda.synchronize()
    for i, f in enumerate(frames):
        assert np.array_equal(image.gray_view(host[i], w, h, image.NV12), f)
        ref, *_ = oracle.undistort_image(f, kd, np.float32(dist))
        assert np.array_equal(dst[i].cpu().numpy().reshape(h, w), ref), i


def test_orb_batch_reads_nv12_luma_in_place(gpu):
    """The batched detector consumes NV12 frames through its frame pitch (no CreateGrayCVMat clone)."""
    import torch

    w, h, B = 640, 480, 3
    pitch = image.frame_pitch(w, h, image.NV12)
    host = np.full((B, pitch), 77, np.uint8)
    frames = [synth.frame(t, w, h) for t in range(B)]
    for i, f in enumerate(frames):
        host[i, : w * h] = f.reshape(-1)
    det = orb.OrbDetector(nfeatures=2000)
    cap = 2000
    kp_b = torch.zeros((B, cap * 28), dtype=torch.uint8, device="cuda")
    desc_b = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    n_b = torch.zeros(B, dtype=torch.int32, device="cuda")
    dev = torch.from_numpy(host).cuda()
    det.detect_and_compute_batch_device(dev, w, h, kp_b, desc_b, n_b, cap, stride=w, frame_pitch=pitch)
    det.device_status()
    for i, f in enumerate(frames):
        kp, d = det.DetectAndCompute(f)
        n = int(n_b[i])
        assert n == len(kp)
        assert np.array_equal(kp_b[i, : 28 * n].cpu().numpy(), kp.view(np.uint8).reshape(-1))
        assert np.array_equal(desc_b[i, :n].cpu().numpy(), d)
