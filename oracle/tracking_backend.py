"""CPU oracle backend of the tracking loop (TEST INFRASTRUCTURE ONLY: tests/ and bench.py's
cpu_baseline leg): the same mageslam_amd.tracking loop with ORB extraction, RadiusMatch and the
pose-only BundlerLib restated on the CPU, so the loop's pose parity can be measured."""
from __future__ import annotations

import numpy as np

from mageslam_amd import tracking

from . import oracle as O


class OracleBackend(tracking.Backend):
    def __init__(self, nfeatures: int = 2000):
        self.settings = O.default_settings(nfeatures)

    def extract(self, frames):
        out = []
        for f in frames:
            _, kp, d = O.orb_detect(np.ascontiguousarray(f), self.settings)
            out.append((kp, d))
        return out

    def radius_match(self, qkp, qdesc, tkp, tdesc, radius, qpos, max_hamming, min_diff):
        return O.radius_match(qkp, qdesc, tkp, tdesc, radius, qpos=qpos, max_distance=max_hamming,
                              min_difference=min_diff)

    def optimize_pose(self, pose, K, points, uv, info, steps, huber, max_err_sq):
        r = O.pose_batch(tracking.pose_problem(pose, K, points, uv, info), steps, huber, max_err_sq)
        return tracking.pose_from_result(r), r["outlier"].astype(bool)

    def local_map_match(self, qpos, qoct, qdesc, qhide, tkp, tdesc, mask, radius, max_hamming, min_diff):
        r, m = O.local_map_match(qpos, qoct, qdesc, qhide, tkp, tdesc, mask.astype(np.uint8), radius, max_hamming,
                                 min_diff)
        return r, m.astype(bool)

    def bundle_adjust(self, w, lam):
        b = O.BundlerOracle()  # a fresh BundlerLib per task (BundleAdjust.cpp MakeBundler)
        return tracking.run_bundler(b, w, lam, b.set_lambda, b.get_lambda)
