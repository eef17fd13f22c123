"""Frame ingest and undistortion — host mirror of ImagePreprocessor (Core/MAGESLAM/Source/Image/
ImagePreprocessor.cpp:71-120) and CreateGrayCVMat (Utils/cv.cpp:8-28).

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
from ._lib import Calibration, check, ptr

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
