"""OrbDetector — host mirror of the reference extractor interface.

Mirrors `class OrbDetector` (Core/MAGESLAM/Source/Image/OpenCVModified.h:64-173): same 14
constructor arguments in the same order, `DetectAndCompute(image) -> (keypoints, descriptors)`
where keypoints are cv::KeyPoint-layout records in the canonical order and
descriptors are the 32-byte ORBDescriptors.  Backed by libmage_hot.so on a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import KP_DTYPE, OrbSettingsC, check, ptr


@dataclass
class FeatureExtractorSettings:
    """Defaults of FeatureExtractorSettings (Core/MAGESLAM/Source/MageSettings.h:151-167)."""

    NumFeatures: int = 440
    ScaleFactor: float = 1.5
    GaussianKernelSize: int = 7
    NumLevels: int = 1
    FastThreshold: int = 4
    PatchSize: int = 15
    UseOrientation: bool = False
    FeatureFactor: float = 1.5
    FeatureStrength: float = 0.9
    StrongResponse: int = 20
    MinRobustnessFactor: float = 1.1
    MaxRobustnessFactor: float = 2.0
    NumCellsX: int = 32
    NumCellsY: int = 32

    def to_c(self) -> OrbSettingsC:
        return OrbSettingsC(self.GaussianKernelSize, self.NumFeatures, self.ScaleFactor,
                            self.NumLevels, self.PatchSize, self.FastThreshold,
                            int(bool(self.UseOrientation)), self.FeatureFactor,
                            self.FeatureStrength, self.StrongResponse, self.MinRobustnessFactor,
                            self.MaxRobustnessFactor, self.NumCellsX, self.NumCellsY)


class OrbDetector:
    def __init__(self, gaussianKernelSize=7, nfeatures=440, scaleFactor=1.5, nlevels=1,
                 patchSize=15, fastThreshold=4, useOrientation=False, featureFactorANMS=1.5,
                 featureStrengthANMS=0.9, strongResponseANMS=20, minRobustFactor=1.1,
                 maxRobustFactor=2.0, numCellsX=32, numCellsY=32, device: int = 0):
        self.settings = FeatureExtractorSettings(
            NumFeatures=nfeatures, ScaleFactor=scaleFactor, GaussianKernelSize=gaussianKernelSize,
            NumLevels=nlevels, FastThreshold=fastThreshold, PatchSize=patchSize,
            UseOrientation=useOrientation, FeatureFactor=featureFactorANMS,
            FeatureStrength=featureStrengthANMS, StrongResponse=strongResponseANMS,
            MinRobustnessFactor=minRobustFactor, MaxRobustnessFactor=maxRobustFactor,
            NumCellsX=numCellsX, NumCellsY=numCellsY)
        self._c = self.settings.to_c()
        self._h = C.c_void_p()
        self.device = device
        check(_lib.load().mage_orb_create(C.byref(self._c), device, C.byref(self._h)))

    @classmethod
    def from_settings(cls, s: FeatureExtractorSettings, device: int = 0) -> "OrbDetector":
        """OrbFeatureDetector ctor (Core/MAGESLAM/Source/Image/OrbFeatureDetector.cpp:64-82)."""
        return cls(s.GaussianKernelSize, s.NumFeatures, s.ScaleFactor, s.NumLevels, s.PatchSize,
                   s.FastThreshold, s.UseOrientation, s.FeatureFactor, s.FeatureStrength,
                   s.StrongResponse, s.MinRobustnessFactor, s.MaxRobustnessFactor, s.NumCellsX,
                   s.NumCellsY, device=device)

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().mage_orb_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def DetectAndCompute(self, image: np.ndarray, capacity: int | None = None):
        """OrbDetector::DetectAndCompute (OpenCVModified.cpp:771-886).

        `image` is an 8-bit single-channel (H, W) array (CV_Assert(type == CV_8UC1) → ValueError).
        `capacity` is the ImageData capacity (default NumFeatures, ImageFactory.h:67-79).
        """
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("image must be CV_8UC1: a 2-D uint8 array")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = int(self.settings.NumFeatures if capacity is None else capacity)
        kp = np.zeros(max(cap, 1), KP_DTYPE)
        desc = np.zeros((max(cap, 1), 32), np.uint8)
        n = C.c_uint32(0)
        check(_lib.load().mage_orb_detect_and_compute(self._h, ptr(img), w, h, w, ptr(kp), ptr(desc),
                                                      cap, C.byref(n)))
        return kp[: n.value].copy(), desc[: n.value].copy()

    def detect_and_compute_batch_device(self, frames, width: int, height: int, keypoints,
                                        descriptors, counts, capacity: int, stride: int | None = None,
                                        frame_pitch: int | None = None, stream=None) -> None:
        """Batched device path: `frames` (B, H, W) uint8 torch tensor on the GPU; outputs are
        preallocated device tensors (B*cap*28 bytes, B*cap*32 bytes, B uint32)."""
        b = frames.shape[0]
        stride = width if stride is None else stride
        pitch = stride * height if frame_pitch is None else frame_pitch
        check(_lib.load().mage_orb_detect_and_compute_batch_device(
            self._h, ptr(frames), b, width, height, stride, pitch, ptr(keypoints), ptr(descriptors),
            capacity, ptr(counts), C.c_void_p(stream) if stream else None))

    def set_fast_gate(self, gate: int, level: int = 0, stream=None) -> None:
        """Gate of the next batch's FAST pass on `level` (0: none).  Speed only: outputs are
        identical for every gate (frames it does not fit run the exact path again)."""
        check(_lib.load().mage_orb_set_fast_gate(self._h, level, int(gate), C.c_void_p(stream) if stream else None))

    def fast_gate_stats(self, level: int = 0, stream=None) -> dict:
        """{'last_gate', 'next_gate', 'last_redo'}: the gate the last batch ran with, the gate of
        the next batch and the number of the last batch's frames that took the exact path."""
        lg, ng, rd = C.c_int32(0), C.c_int32(0), C.c_uint32(0)
        check(_lib.load().mage_orb_fast_gate_stats(self._h, level, C.byref(lg), C.byref(ng), C.byref(rd),
                                                   C.c_void_p(stream) if stream else None))
        return {"last_gate": lg.value, "next_gate": ng.value, "last_redo": rd.value}

    def device_status(self, stream=None) -> None:
        check(_lib.load().mage_orb_status(self._h, C.c_void_p(stream) if stream else None))


def fast_score_map(image: np.ndarray, threshold: int = 4, device: int = 0) -> np.ndarray:
    """FAST_t<16> score map (0 where the segment test fails), computed on the GPU."""
    img = np.ascontiguousarray(image, np.uint8)
    h, w = img.shape
    out = np.zeros((h, w), np.uint8)
    check(_lib.load().mage_orb_fast_score_map(ptr(img), w, h, w, threshold, ptr(out), device))
    return out


def synth_frames_device(out, count: int, width: int, height: int, t0: int, seed: int,
                        frame_pitch: int | None = None, stream=None) -> None:
    """Writes frames t0..t0+count-1 of the synthetic sequence into a device tensor."""
    pitch = width * height if frame_pitch is None else frame_pitch
    check(_lib.load().mage_synth_frames_device(ptr(out), count, width, height, pitch, t0, seed,
                                               C.c_void_p(stream) if stream else None))


def _cal_key(c):
    return (c.fx, c.fy, c.cx, c.cy, c.ndist, tuple(c.dist[: c.ndist]))


def UndistortKeypoints(keypoints: np.ndarray, distortedCalibration, undistortedCalibration,
                       device: int = 0) -> np.ndarray:
    """OrbFeatureDetector::UndistortKeypoints (OrbFeatureDetector.cpp:30-62) on the GPU: returns a
    copy of the keypoints with positions through cv::undistortPoints(distorted K, distortion,
    noArray(), undistorted K).  Calibrations are `_lib.Calibration` records."""
    kp = np.array(keypoints, dtype=KP_DTYPE, copy=True)
    check(_lib.load().mage_undistort_keypoints(C.byref(distortedCalibration), C.byref(undistortedCalibration),
                                               ptr(kp), len(kp), int(device)))
    return kp


def undistort_keypoints_batch_device(distortedCalibration, undistortedCalibration, keypoints, pitch: int, counts,
                                     batch: int, stream=None) -> None:
    """Batched device form: frame f's keypoints at keypoints + f * pitch (in keypoints), counts[f]
    of them, undistorted in place (torch device tensors)."""
    check(_lib.load().mage_undistort_keypoints_batch_device(
        C.byref(distortedCalibration), C.byref(undistortedCalibration), ptr(keypoints), pitch, ptr(counts), batch,
        C.c_void_p(stream) if stream else None))


class OrbFeatureDetector:
    """OrbFeatureDetector (Image/OrbFeatureDetector.cpp:64-100): DetectAndCompute, then keypoint
    undistortion when the distorted and undistorted calibrations differ (operator!=)."""

    def __init__(self, settings: FeatureExtractorSettings | None = None, device: int = 0):
        s = settings or FeatureExtractorSettings()
        self.detector = OrbDetector(s.GaussianKernelSize, s.NumFeatures, s.ScaleFactor, s.NumLevels, s.PatchSize,
                                    s.FastThreshold, s.UseOrientation, s.FeatureFactor, s.FeatureStrength,
                                    s.StrongResponse, s.MinRobustnessFactor, s.MaxRobustnessFactor, s.NumCellsX,
                                    s.NumCellsY, device=device)
        self.device = device

    def Process(self, distortedCalibration, undistortedCalibration, image: np.ndarray):
        kp, desc = self.detector.DetectAndCompute(image)
        if _cal_key(distortedCalibration) != _cal_key(undistortedCalibration):
            kp = UndistortKeypoints(kp, distortedCalibration, undistortedCalibration, self.device)
        return kp, desc
