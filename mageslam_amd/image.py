"""Frame ingest and undistortion — host mirror of ImagePreprocessor (Core/MAGESLAM/Source/Image/
ImagePreprocessor.cpp:71-120) and CreateGrayCVMat (Utils/cv.cpp:8-28).

`ScaleImageForCameraConfiguration` (ImagePreprocessor.cpp:18-65) brings a stereo frame to the other
camera's resolution (overlap-crop geometry on the host, resize on the GPU).
`ImagePreprocessor.UndistortImage(distortedImage, distortedCalibration)` returns the undistorted
frame and calibration like the reference, caching the device-resident CV_32FC1 maps per
(size, calibration) as `CachedUndistortDataValid` does.  `gray_view` is CreateGrayCVMat without the
clone: a GRAYSCALE8 frame or the Y plane of an NV12 frame, as (array, stride, pitch) for the
batched device entry points.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import Calibration, CameraConfig, check, load, ptr

GRAYSCALE8, NV12 = 0, 1


def frame_pitch(width: int, height: int, fmt: int) -> int:
    """Bytes per frame of a packed sequence: w*h (GRAYSCALE8) or w*h*3/2 (NV12); the luma plane
    comes first in both, so the ORB / undistortion batch kernels read it in place."""
    return width * height if fmt == GRAYSCALE8 else width * height * 3 // 2


def gray_view(buf: np.ndarray, width: int, height: int, fmt: int) -> np.ndarray:
    """CreateGrayCVMat (Utils/cv.cpp:8-28) as a view: the first width*height bytes."""
    if fmt not in (GRAYSCALE8, NV12):
        raise ValueError("unsupported pixel format")
    flat = np.ascontiguousarray(buf, np.uint8).reshape(-1)
    if flat.size < frame_pitch(width, height, fmt):
        raise ValueError("buffer smaller than one frame")
    return flat[: width * height].reshape(height, width)


class Undistorter:
    def __init__(self, distorted: Calibration, width: int, height: int, device: int = 0):
        self._h = C.c_void_p()
        self.undistorted = Calibration()
        self.width, self.height = width, height
        check(_lib.load().mage_undistorter_create(C.byref(distorted), width, height, device, C.byref(self._h),
                                                  C.byref(self.undistorted)))

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().mage_undistorter_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def maps(self):
        mx = np.zeros((self.height, self.width), np.float32)
        my = np.zeros((self.height, self.width), np.float32)
        check(_lib.load().mage_undistorter_get_maps(self._h, ptr(mx), ptr(my)))
        return mx, my

    def __call__(self, img: np.ndarray) -> np.ndarray:
        src = np.ascontiguousarray(img, np.uint8)
        if src.shape != (self.height, self.width):
            raise ValueError("image size differs from the undistorter's")
        out = np.zeros_like(src)
        check(_lib.load().mage_undistort_image(self._h, ptr(src), self.width, ptr(out), self.width))
        return out

    def batch_device(self, src, src_stride: int, src_pitch: int, dst, dst_stride: int, dst_pitch: int, batch: int,
                     stream=None) -> None:
        check(_lib.load().mage_undistort_image_batch_device(self._h, ptr(src), src_stride, src_pitch, ptr(dst),
                                                            dst_stride, dst_pitch, batch,
                                                            C.c_void_p(stream) if stream else None))


def _key(cal: Calibration):
    return (cal.fx, cal.fy, cal.cx, cal.cy, tuple(cal.dist), cal.ndist)


class ImagePreprocessor:
    def __init__(self, device: int = 0):
        self.device = device
        self._u: Undistorter | None = None
        self._key = None

    def UndistortImage(self, distortedImage: np.ndarray, distortedCameraCal: Calibration):
        """-> (undistortedImage, undistortedCameraCal)."""
        h, w = distortedImage.shape
        key = ((w, h), _key(distortedCameraCal))
        if self._u is None or self._key != key:  # CachedUndistortDataValid
            self._u = Undistorter(distortedCameraCal, w, h, self.device)
            self._key = key
        return self._u(distortedImage), self._u.undistorted


def scale_geometry(source: CameraConfig, target: CameraConfig, max_depth_meters: float = 2.3):
    """ScaleImageForCameraConfiguration's geometry (mage_scale_for_camera_configuration):
    (ok, crop (x, y, w, h), scaleSourceToTarget, prepared CameraConfig).  max_depth_meters defaults
    to StereoMapInitializationSettings::MaxDepthMeters (MageSettings.h:144)."""
    crop = (C.c_int32 * 4)()
    scale, ok = C.c_float(0), C.c_int32(0)
    prepared = CameraConfig()
    check(load().mage_scale_for_camera_configuration(C.byref(source), C.byref(target), float(max_depth_meters), crop,
                                                      C.byref(scale), C.byref(prepared), C.byref(ok)))
    return bool(ok.value), tuple(crop), float(scale.value), prepared


def ScaleImageForCameraConfiguration(source: CameraConfig, target: CameraConfig, rawSourceImage,
                                     max_depth_meters: float = 2.3, device: int = 0):
    """ImagePreprocessor::ScaleImageForCameraConfiguration (ImagePreprocessor.cpp:18-65) on the GPU:
    -> (ok, preparedImage, prepared CameraConfig, scaleSourceToTarget).  The image (H x W uint8,
    numpy or a CUDA tensor) is resized with cv::resize INTER_LINEAR (or copied when the scale is 1)
    by mage_scale_image_for_camera_configuration_device; preparedImage is None when there is no overlap."""
    import torch

    dev = torch.device("cuda", device)
    src = rawSourceImage if isinstance(rawSourceImage, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(rawSourceImage, np.uint8))
    src = src.to(dev).contiguous()
    h, w = src.shape
    if (w, h) != (source.width, source.height):
        raise ValueError("the image size must match the source camera configuration")
    ok, _, scale, prepared = scale_geometry(source, target, max_depth_meters)
    if not ok:
        return False, None, prepared, scale
    out = torch.empty((prepared.height, prepared.width), dtype=torch.uint8, device=dev)
    s2, k2, p2 = C.c_float(0), C.c_int32(0), CameraConfig()
    check(load().mage_scale_image_for_camera_configuration_device(
        C.byref(source), C.byref(target), float(max_depth_meters), ptr(src), w, ptr(out), prepared.width,
        out.numel(), C.byref(p2), C.byref(s2), C.byref(k2), None))
    torch.cuda.synchronize(dev)
    res = out if isinstance(rawSourceImage, torch.Tensor) else out.cpu().numpy()
    return True, res, p2, float(s2.value)


def resize_linear_device(src, dw: int, dh: int, stream=None):
    """cv::resize(INTER_LINEAR) 8UC1 of a CUDA tensor (mage_resize_linear_device)."""
    import torch

    h, w = src.shape
    out = torch.empty((dh, dw), dtype=torch.uint8, device=src.device)
    check(load().mage_resize_linear_device(ptr(src), w, h, w, ptr(out), dw, dh, dw,
                                           C.c_void_p(stream) if stream else None))
    return out
