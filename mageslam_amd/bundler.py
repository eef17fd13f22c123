"""BundlerLib — host mirror of the reference bundle adjuster interface.

Mirrors `class BundlerLib` (Dependencies/BundlerLib/Include/BundlerLib.h:20-66) method for
method; the Eigen::Map arguments become numpy arrays (orientation is the logical 3x3 matrix;
the column-major Eigen layout is produced here).  Setters buffer on the host and the problem
is handed to libmage_hot.so (gfx950) at the first StepBundleAdjustment.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import BAStats, check, ptr


@dataclass
class BundlerParameters:
    ArePointsFixed: bool = False


class BundlerLib:
    def __init__(self, params: BundlerParameters | None = None, device: int = 0):
        self.params = params or BundlerParameters()
        self._h = C.c_void_p()
        check(_lib.load().mage_ba_create(int(self.params.ArePointsFixed), device, C.byref(self._h)))
        self._cams = None
        self._pts = None
        self._obs = None
        self._teth = {}
        self._uploaded = {"cams": False, "pts": False, "obs": False, "teth": True}

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().mage_ba_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- allocation / setters (BundlerLib.cpp:198-309) ---
    def AllocateCameras(self, count: int) -> None:
        if self._cams is not None:
            raise RuntimeError("can only allocate once")
        self._cams = dict(pos=np.zeros((count, 3), np.float32), r9=np.zeros((count, 9), np.float32),
                          intr=np.zeros((count, 4), np.float32), fixed=np.zeros(count, np.uint8))

    def SetCameraPose(self, idx: int, position, orientation, intrinsics, isFixed: bool) -> None:
        c = self._cams
        c["pos"][idx] = np.asarray(position, np.float32).reshape(3)
        c["r9"][idx] = np.asarray(orientation, np.float32).reshape(3, 3).T.reshape(9)  # column-major
        c["intr"][idx] = np.asarray(intrinsics, np.float32).reshape(4)
        c["fixed"][idx] = 1 if isFixed else 0
        self._uploaded["cams"] = False

    def FixCameraPose(self, idx: int, value: bool) -> None:
        self._cams["fixed"][idx] = 1 if value else 0
        if self._uploaded["cams"]:
            check(_lib.load().mage_ba_fix_camera(self._h, idx, int(value)))

    def AllocateMapPoints(self, count: int) -> None:
        self._pts = np.zeros((count, 3), np.float32)
        self._uploaded["pts"] = False

    def SetMapPoint(self, idx: int, point) -> None:
        self._pts[idx] = np.asarray(point, np.float32).reshape(3)
        self._uploaded["pts"] = False

    def AllocateObservations(self, count: int) -> None:
        self._obs = dict(uv=np.zeros((count, 2), np.float32), cam=np.zeros(count, np.uint32),
                         pt=np.zeros(count, np.uint32), info=np.zeros(count, np.float32))
        self._uploaded["obs"] = False

    def SetObservation(self, idx: int, position, cameraIndex: int, mapPointIndex: int,
                       informationMatrixScalar: float) -> None:
        o = self._obs
        o["uv"][idx] = np.asarray(position, np.float32).reshape(2)
        o["cam"][idx] = cameraIndex
        o["pt"][idx] = mapPointIndex
        o["info"][idx] = informationMatrixScalar
        self._uploaded["obs"] = False

    def set_graph(self, g) -> None:
        """Bulk form of the setters for a synth.BAGraph-like object."""
        n = len(g.pos)
        self._cams = dict(pos=np.ascontiguousarray(g.pos, np.float32), r9=g.rot_colmajor.astype(np.float32),
                          intr=np.ascontiguousarray(g.intr, np.float32),
                          fixed=np.ascontiguousarray(g.fixed, np.uint8))
        assert len(self._cams["r9"]) == n
        self._pts = np.ascontiguousarray(g.points, np.float32)
        self._obs = dict(uv=np.ascontiguousarray(g.uv, np.float32), cam=np.ascontiguousarray(g.cam, np.uint32),
                         pt=np.ascontiguousarray(g.pt, np.uint32), info=np.ascontiguousarray(g.info, np.float32))
        for kind in range(3):  # a fresh graph carries no tethers until set_tethers
            self._alloc_tethers(kind, 0)
        self._uploaded.update(cams=False, pts=False, obs=False, teth=False)

    # --- tether constraints (BundlerLib.cpp:229-257, 311-350) ---
    _TETHER_STRIDE = (1, 4, 7)

    def _alloc_tethers(self, kind: int, count: int) -> None:
        self._teth[kind] = dict(c1=np.zeros(count, np.uint32), c2=np.zeros(count, np.uint32),
                                params=np.zeros((count, self._TETHER_STRIDE[kind]), np.float32),
                                weight=np.ones(count, np.float32))
        self._uploaded["teth"] = False

    def _set_tether(self, kind: int, idx: int, c1: int, c2: int, params, weight: float) -> None:
        t = self._teth[kind]
        t["c1"][idx], t["c2"][idx] = c1, c2
        t["params"][idx] = np.asarray(params, np.float32).reshape(-1)
        t["weight"][idx] = weight
        self._uploaded["teth"] = False

    def AllocateFixedDistanceConstraints(self, count: int) -> None:
        self._alloc_tethers(_lib.MAGE_TETHER_DISTANCE, count)

    def SetFixedDistanceConstraint(self, idx: int, cameraIndex1: int, cameraIndex2: int, distance: float = 1.0,
                                   weight: float = 1.0) -> None:
        self._set_tether(_lib.MAGE_TETHER_DISTANCE, idx, cameraIndex1, cameraIndex2, [distance], weight)

    def AllocateRelativeRotationConstraints(self, count: int) -> None:
        self._alloc_tethers(_lib.MAGE_TETHER_ROTATION, count)

    def SetRelativeRotationConstraint(self, idx: int, cameraIndex1: int, cameraIndex2: int, deltaRotation,
                                      weight: float = 1.0) -> None:
        """deltaRotation: quaternion (x, y, z, w) (Eigen::Quaternionf coefficient order)."""
        self._set_tether(_lib.MAGE_TETHER_ROTATION, idx, cameraIndex1, cameraIndex2, deltaRotation, weight)

    def AllocateRelativeTransformConstraints(self, count: int) -> None:
        self._alloc_tethers(_lib.MAGE_TETHER_TRANSFORM, count)

    def SetRelativeTransformConstraint(self, idx: int, cameraIndex1: int, cameraIndex2: int, deltaPosition,
                                       deltaRotation, weight: float) -> None:
        p = np.concatenate([np.asarray(deltaPosition, np.float32).reshape(3),
                            np.asarray(deltaRotation, np.float32).reshape(4)])
        self._set_tether(_lib.MAGE_TETHER_TRANSFORM, idx, cameraIndex1, cameraIndex2, p, weight)

    def set_tethers(self, t) -> None:
        """Bulk form for a synth.Tethers-like object (distance, rotation, transform tuples of
        (cam1, cam2, params, weight))."""
        for kind, (c1, c2, params, w) in enumerate((t.distance, t.rotation, t.transform)):
            self._alloc_tethers(kind, len(c1))
            tt = self._teth[kind]
            tt["c1"][:] = c1
            tt["c2"][:] = c2
            tt["params"][:] = np.asarray(params, np.float32).reshape(len(c1), self._TETHER_STRIDE[kind])
            tt["weight"][:] = w

    def SetCurrentLambda(self, userLambda: float) -> None:
        check(_lib.load().mage_ba_set_lambda(self._h, float(userLambda)))

    def GetCurrentLambda(self) -> float:
        v = C.c_float()
        check(_lib.load().mage_ba_get_lambda(self._h, C.byref(v)))
        return float(v.value)

    def _upload(self) -> None:
        L = _lib.load()
        if not self._uploaded["cams"] and self._cams is not None:
            c = self._cams
            check(L.mage_ba_set_cameras(self._h, len(c["pos"]), ptr(c["pos"]), ptr(c["r9"]), ptr(c["intr"]),
                                        ptr(c["fixed"])))
            self._uploaded["cams"] = True
        if not self._uploaded["pts"] and self._pts is not None:
            check(L.mage_ba_set_points(self._h, len(self._pts), ptr(self._pts)))
            self._uploaded["pts"] = True
        if not self._uploaded["obs"] and self._obs is not None:
            o = self._obs
            check(L.mage_ba_set_observations(self._h, len(o["cam"]), ptr(o["uv"]), ptr(o["cam"]), ptr(o["pt"]),
                                             ptr(o["info"])))
            self._uploaded["obs"] = True
        if not self._uploaded["teth"]:
            for kind, t in sorted(self._teth.items()):
                check(L.mage_ba_set_tethers(self._h, kind, len(t["c1"]), ptr(t["c1"]), ptr(t["c2"]),
                                            ptr(np.ascontiguousarray(t["params"])), ptr(t["weight"])))
            self._uploaded["teth"] = True

    def StepBundleAdjustment(self, huberWidthPerIteration, maxErrorSquare: float, outliers: list | None = None) -> float:
        """BundlerLib::StepBundleAdjustment (BundlerLib.cpp:364-447): returns the mean squared
        error of the kept edges and appends outlier observation indices to `outliers`."""
        self._upload()
        # per-call Python work kept to a minimum (the mapping thread calls this once per BA step,
        # ~190 us at C3): the huber array, the outlier buffer and the out-parameters are reused,
        # and raw addresses replace ndarray.ctypes.data_as (several us each)
        key = None if isinstance(huberWidthPerIteration, np.ndarray) else tuple(huberWidthPerIteration)
        if key is None or key != getattr(self, "_hw_key", None):
            hw = np.ascontiguousarray(np.asarray(huberWidthPerIteration, np.float32).reshape(-1))
            self._hw, self._hw_key, self._hw_ptr = hw, key, C.c_void_p(hw.ctypes.data)
        cap = max(len(self._obs["cam"]) if self._obs is not None else 0, 1)
        if getattr(self, "_outbuf", None) is None or len(self._outbuf) < cap:
            self._outbuf = np.empty(cap, np.uint32)  # reused: the call writes only the first n entries
            self._out_ptr = C.c_void_p(self._outbuf.ctypes.data)
            self._n, self._ms = C.c_uint32(0), C.c_float(0)
            self._n_ref, self._ms_ref = C.byref(self._n), C.byref(self._ms)
        check(_lib.load().mage_ba_step(self._h, self._hw_ptr, len(self._hw), float(maxErrorSquare), self._out_ptr, cap,
                                       self._n_ref, self._ms_ref))
        n = self._n.value
        if outliers is not None and n:
            outliers.extend(self._outbuf[:n].tolist())
        return float(self._ms.value)

    def step(self, huber_widths, max_error_square):
        """Convenience form: returns (mean_sq, outliers ndarray)."""
        outl: list = []
        ms = self.StepBundleAdjustment(huber_widths, max_error_square, outl)
        return ms, np.asarray(outl, np.uint32)

    # GetPose / GetPoint run after every StepBundleAdjustment (UpdateData): fresh output arrays,
    # raw addresses instead of ndarray.ctypes.data_as (several us each)
    def poses(self):
        n = len(self._cams["pos"])
        pos = np.empty((n, 3), np.float32)
        r9 = np.empty((n, 9), np.float32)
        self._upload()
        check(_lib.load().mage_ba_get_poses(self._h, pos.ctypes.data, r9.ctypes.data))
        return pos, r9

    def points(self):
        xyz = np.empty((len(self._pts), 3), np.float32)
        self._upload()
        check(_lib.load().mage_ba_get_points(self._h, xyz.ctypes.data))
        return xyz

    def state(self):
        """fp64 state: (C,7) [qx,qy,qz,qw,tx,ty,tz] and (P,3) points."""
        self._upload()
        qt = np.zeros((len(self._cams["pos"]), 7), np.float64)
        xyz = np.zeros((len(self._pts), 3), np.float64)
        check(_lib.load().mage_ba_get_state_f64(self._h, ptr(qt), ptr(xyz)))
        return qt, xyz

    def GetPose(self, idx: int):
        """(position (3,), orientation (3,3)) of camera idx (BundlerLib.cpp:457-465)."""
        pos, r9 = self.poses()
        return pos[idx], r9[idx].reshape(3, 3).T

    def GetPoint(self, idx: int):
        return self.points()[idx]

    def stats(self) -> dict:
        s = BAStats()
        check(_lib.load().mage_ba_get_stats(self._h, C.byref(s)))
        return dict(iterations=s.iterations, trials=s.trials, rejected=s.rejected_trials, chi2=s.last_chi2,
                    lambda_=s.lambda_)


def OptimizeCameraPoses(pb, numIterations: int, maxOutlierErrorSquared: float, huberWidth: float, device: int = 0):
    """TrackLocalMap::OptimizeCameraPose (TrackLocalMap.cpp:421-501) for a batch of frames in one
    launch.  `pb` holds pos (K,3), r9 (K,9 column-major), intr (K,4), obs_start (K+1), points (E,3),
    uv (E,2), info (E) (synth.PoseBatch).  Returns dict(pos, r9, qt7, outlier (E,) u8, mean_sq,
    stats (K, 2) = LM iterations / trials); outlierIndices of problem k are the flagged entries of
    its observation range."""
    K = len(pb.pos)
    E = int(pb.obs_start[-1])
    c = np.ascontiguousarray
    out = dict(pos=np.zeros((K, 3), np.float32), r9=np.zeros((K, 9), np.float32), qt7=np.zeros((K, 7)),
               outlier=np.zeros(max(E, 1), np.uint8), mean_sq=np.zeros(K, np.float32),
               stats=np.zeros((K, 2), np.uint32))
    check(_lib.load().mage_ba_pose_batch(
        K, ptr(c(pb.pos, np.float32)), ptr(c(pb.r9, np.float32)), ptr(c(pb.intr, np.float32)),
        ptr(c(pb.obs_start, np.uint32)), ptr(c(pb.points, np.float32)), ptr(c(pb.uv, np.float32)),
        ptr(c(pb.info, np.float32)), int(numIterations), float(huberWidth), float(maxOutlierErrorSquared),
        ptr(out["pos"]), ptr(out["r9"]), ptr(out["qt7"]), ptr(out["outlier"]), ptr(out["mean_sq"]),
        ptr(out["stats"]), device))
    out["outlier"] = out["outlier"][:E]
    return out


def pose_batch_device(problems: int, pos3, r9, intr4, obs_start, points3, uv, info, nsteps: int, huber: float,
                      max_error_square: float, pos3_out, r9_out, qt7_out, outlier, mean_sq, stats=None,
                      stream=None) -> None:
    """Device form of OptimizeCameraPoses over torch device tensors (asynchronous)."""
    check(_lib.load().mage_ba_pose_batch_device(
        problems, ptr(pos3), ptr(r9), ptr(intr4), ptr(obs_start), ptr(points3), ptr(uv), ptr(info), nsteps,
        float(huber), float(max_error_square), ptr(pos3_out), ptr(r9_out), ptr(qt7_out), ptr(outlier), ptr(mean_sq),
        ptr(stats), C.c_void_p(stream) if stream else None))
