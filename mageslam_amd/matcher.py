"""Hamming matching — host mirror of FeatureMatcher's brute-force entry points.

`Match` mirrors `unsigned Match(imageA, imageB, maskA, maskB, countA, countB, maxHammingDist,
minHammingDifference, goodMatches)` (Core/MAGESLAM/Source/Tracking/FeatureMatcher.h:68-77):
descriptors are passed directly instead of AnalyzedImage, masks are boolean arrays, and the
result is an array of cv::DMatch-layout records.  `GetDescriptorDistance` mirrors
FeatureMatcher.cpp:453-504.  `RadiusMatch` mirrors the batch RadiusMatch (FeatureMatcher.cpp:294-378)
over a target KeypointSpatialIndex (built on the device from the target keypoints).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import DM_DTYPE, KP_DTYPE, check, load, ptr


def GetDescriptorDistance(d0: np.ndarray, d1: np.ndarray) -> int:
    a = np.ascontiguousarray(d0, np.uint8)
    b = np.ascontiguousarray(d1, np.uint8)
    if a.size != 32 or b.size != 32:
        raise ValueError("ORB descriptors are 32 bytes")
    return int(_lib.load().mage_hamming_distance(ptr(a), ptr(b)))


def Match(descA: np.ndarray, descB: np.ndarray, maskA=None, maskB=None, maxHammingDist: int = 30,
          minHammingDifference: int = 1) -> np.ndarray:
    """Two-way brute-force match on the GPU; returns DMatch records in ascending A index.

    Returns an empty array (and 0 matches) when either mask selects nothing
    (FeatureMatcher.cpp:72-77)."""
    da = np.ascontiguousarray(descA, np.uint8).reshape(-1, 32)
    db = np.ascontiguousarray(descB, np.uint8).reshape(-1, 32)
    ma = None if maskA is None else np.ascontiguousarray(np.asarray(maskA, bool), np.uint8)
    mb = None if maskB is None else np.ascontiguousarray(np.asarray(maskB, bool), np.uint8)
    if ma is not None and len(ma) != len(da):
        raise ValueError("maskA length must equal the number of A descriptors")
    if mb is not None and len(mb) != len(db):
        raise ValueError("maskB length must equal the number of B descriptors")
    cap = max(len(da), 1)
    out = np.zeros(cap, DM_DTYPE)
    n = C.c_uint32(0)
    check(_lib.load().mage_hamming_match(ptr(da), len(da), ptr(ma), ptr(db), len(db), ptr(mb),
                                         int(maxHammingDist), int(minHammingDifference), ptr(out),
                                         cap, C.byref(n)))
    return out[: n.value].copy()


def match_batch_device(desc_a, a_pitch: int, n_a, desc_b, b_pitch: int, n_b, pairs: int,
                       max_distance: int, min_difference: int, out, capacity: int, n_out,
                       stream=None) -> None:
    """Batched device path over `pairs` (A_p, B_p) descriptor sets (torch device tensors)."""
    check(_lib.load().mage_hamming_match_batch_device(
        ptr(desc_a), a_pitch, ptr(n_a), ptr(desc_b), b_pitch, ptr(n_b), pairs, max_distance,
        min_difference, ptr(out), capacity, ptr(n_out), C.c_void_p(stream) if stream else None))


def RadiusMatch(queryKeypoints, queryDescriptors, targetKeypoints, targetDescriptors, radius: float,
                maxHammingDist: int = 30, minHammingDifference: int = 1, queryKeypointPositionOverrides=None,
                queryKeypointsMask=None, targetKeypointsMask=None) -> np.ndarray:
    """RadiusMatch on the GPU (FeatureMatcher.cpp:294-446): keypoints are cv::KeyPoint-layout
    records (KP_DTYPE), descriptors (n, 32) uint8; returns DMatch records in query order
    (queryIdx = query index, trainIdx = target index)."""
    from ._lib import KP_DTYPE

    qk = np.ascontiguousarray(queryKeypoints, KP_DTYPE)
    tk = np.ascontiguousarray(targetKeypoints, KP_DTYPE)
    qd = np.ascontiguousarray(queryDescriptors, np.uint8).reshape(-1, 32)
    td = np.ascontiguousarray(targetDescriptors, np.uint8).reshape(-1, 32)
    if len(qd) != len(qk) or len(td) != len(tk):
        raise ValueError("one descriptor per keypoint")
    qp = None
    if queryKeypointPositionOverrides is not None:
        qp = np.ascontiguousarray(queryKeypointPositionOverrides, np.float32).reshape(-1, 2)
        if len(qp) != len(qk):
            raise ValueError("one position override per query keypoint")
    qm = None if queryKeypointsMask is None else np.ascontiguousarray(np.asarray(queryKeypointsMask, bool), np.uint8)
    tm = None if targetKeypointsMask is None else np.ascontiguousarray(np.asarray(targetKeypointsMask, bool), np.uint8)
    cap = max(len(qk), 1)
    out = np.zeros(cap, DM_DTYPE)
    n = C.c_uint32(0)
    check(_lib.load().mage_radius_match(ptr(qk), ptr(qp), ptr(qm), ptr(qd), len(qk), ptr(tk), ptr(tm), ptr(td),
                                        len(tk), float(radius), int(maxHammingDist), int(minHammingDifference),
                                        ptr(out), cap, C.byref(n)))
    return out[: n.value].copy()


def radius_match_batch_device(query_kp, query_pos, query_desc, query_pitch: int, n_query, target_kp, target_desc,
                              target_pitch: int, n_target, pairs: int, radius: float, max_distance: int,
                              min_difference: int, scratch, out, capacity: int, n_out, status, stream=None) -> None:
    """Batched device RadiusMatch over `pairs` (query set, target set) pairs (torch device tensors)."""
    check(_lib.load().mage_radius_match_batch_device(
        ptr(query_kp), ptr(query_pos), ptr(query_desc), query_pitch, ptr(n_query), ptr(target_kp), ptr(target_desc),
        target_pitch, ptr(n_target), pairs, float(radius), max_distance, min_difference, ptr(scratch), ptr(out),
        capacity, ptr(n_out), ptr(status), C.c_void_p(stream) if stream else None))


def LocalMapMatch(queryPositions, queryOctaves, queryDescriptors, targetKeypoints, targetDescriptors, unassociatedMask,
                  radius: float = 8.0, maxHammingDist: int = 30, minHammingDifference: int = 1, queryHidden=None,
                  device: int = 0):
    """TrackLocalMap's per-map-point matching over projected map points in order
    (TrackLocalMap.cpp:175-256 -> MatchMapPointToCurrentFrame -> RadiusMatch, FeatureMatcher.cpp:386-446),
    through mage_local_map_match: -> (result (n,) int32 keypoint index or -1, updated mask (True =
    still unassociated))."""
    qp = np.ascontiguousarray(queryPositions, np.float32).reshape(-1, 2)
    n = len(qp)
    qo = np.ascontiguousarray(queryOctaves, np.int32).reshape(n)
    qd = np.ascontiguousarray(queryDescriptors, np.uint8).reshape(n, 32)
    qh = None if queryHidden is None else np.ascontiguousarray(queryHidden, np.int32).reshape(n)
    tk = np.ascontiguousarray(targetKeypoints, KP_DTYPE)
    td = np.ascontiguousarray(targetDescriptors, np.uint8).reshape(-1, 32)
    m = np.ascontiguousarray(unassociatedMask, np.uint8).reshape(len(tk)).copy()
    res = np.full(max(n, 1), -1, np.int32)
    check(load().mage_local_map_match(ptr(qp), ptr(qo), ptr(qd), ptr(qh), n, ptr(tk), ptr(td), len(tk), ptr(m),
                                      float(radius), int(maxHammingDist), int(minHammingDifference), ptr(res), device))
    return res[:n].copy(), m.astype(bool)
