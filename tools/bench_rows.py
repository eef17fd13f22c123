#!/usr/bin/env python3
"""Per-row measurements of the §8 kernels the headline bench.py does not exercise.

Each leg runs one batched device entry point on HBM-resident synthetic inputs, times K launches
with the library's dispatch-timestamp timers (the same as bench.py), and prints one JSON object per
leg: kernel average, throughput in the row's unit, algorithmic bytes per launch and the HBM
fraction.  Run under `rocprofv3 --kernel-trace --stats` for the committed summary
(tools/profile_round.sh does both).

  radius    RadiusMatch (FeatureMatcher.cpp:294-378): 256 frame pairs x 2000 keypoints, r = 15 px
  indexed   OnlineBow FindLeafNode + IndexedMatch (FeatureMatcher.cpp:192-292): 256 pairs, default tree
  remap     UndistortImage (ImagePreprocessor.cpp:106-120): 256 x 720p Rational6k frames
  kpundist  UndistortKeypoints (OrbFeatureDetector.cpp:30-62): 256 x 2000 keypoints
  pose      batched pose-only BA (TrackLocalMap::OptimizeCameraPose, TrackLocalMap.cpp:421-501): bench.py's
            pose leg (2048 problems x ~600 observations, 3 LM steps) alone, for its own counters
  train     OnlineBow::CreateTree (OnlineBow.cpp:325-337): TrainingFrames (15) x 2000 descriptors,
            2 levels x 6 branches, <= 12 Kmean iterations (host-driven: wall time per tree)
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0


def timed(lib, fn, iters, torch):
    from mageslam_amd import _lib

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    lib.mage_profile_reset()
    lib.mage_profile_enable(1)
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    lib.mage_profile_enable(0)
    return wall, {k: (c, ms / c) for k, (c, ms) in _lib.profile_report().items()}


def frames_features(torch, B, W, H, N):
    """B + 1 consecutive synthetic frames through the batched detector: (kp, desc, counts) tensors."""
    from mageslam_amd import orb, synth

    det = orb.OrbDetector(nfeatures=N)
    frames = torch.empty((B + 1, H, W), dtype=torch.uint8, device="cuda")
    orb.synth_frames_device(frames, B + 1, W, H, 0, synth.FRAME_SEED)
    kp = torch.zeros((B + 1, N * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B + 1, N, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(B + 1, dtype=torch.int32, device="cuda")
    det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
    torch.cuda.synchronize()
    return frames, kp, desc, cnt


def leg(name, unit, units_per_launch, wall, kern, tag, bytes_per_launch):
    c, avg_ms = kern[tag]
    out = {"row": name, "kernel": tag, "avg_launch_ms": avg_ms, "wall_ms_per_launch": wall * 1e3,
           "value": units_per_launch / (avg_ms / 1e3), "unit": unit, "units_per_launch": units_per_launch,
           "algorithmic_bytes_per_launch": bytes_per_launch,
           "roofline": {"bound": "hbm", "achieved": bytes_per_launch / (avg_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s"},
           "kernels": {k: {"launches": n, "avg_ms": v} for k, (n, v) in kern.items()}}
    out["roofline"]["frac"] = out["roofline"]["achieved"] / HBM_PEAK_GBS
    print(json.dumps(out), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--legs", default="radius,indexed,remap,kpundist,pose,train")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--iters", type=int, default=10)
    a = p.parse_args()
    import torch

    from mageslam_amd import _lib, bow, image, matcher, orb, synth
    from mageslam_amd._lib import Calibration

    lib = _lib.load()
    B, W, H, N = a.batch, 1280, 720, 2000
    legs = a.legs.split(",")
    frames = kp = desc = cnt = None
    if {"radius", "indexed", "kpundist", "train"} & set(legs):
        frames, kp, desc, cnt = frames_features(torch, B, W, H, N)
    if "radius" in legs:
        scratch = torch.zeros(B * N, dtype=torch.int32, device="cuda")
        out = torch.zeros((B, N * 16), dtype=torch.uint8, device="cuda")
        nout = torch.zeros(B, dtype=torch.int32, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")

        def radius():
            matcher.radius_match_batch_device(kp[1:], None, desc[1:], N, cnt[1:], kp[:-1], desc[:-1], N, cnt[:-1], B,
                                              15.0, 30, 1, scratch, out, N, nout, status)

        wall, kern = timed(lib, radius, a.iters, torch)
        # query kp + desc, target kp + desc, matches out
        leg("a15 RadiusMatch", "frame pairs/s", B, wall, kern, "match.radius", B * N * (28 + 32) * 2 + B * N * 16)
    if "indexed" in legs:
        host_desc = desc[:2].cpu().numpy().reshape(-1, 32)
        tree = bow.OnlineBowTree(*synth.bow_tree(host_desc))
        leaves = torch.zeros((B + 1, N), dtype=torch.int32, device="cuda")
        out = torch.zeros((B, N * 16), dtype=torch.uint8, device="cuda")
        nout = torch.zeros(B, dtype=torch.int32, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")

        def indexed():
            tree.find_leaves_device(desc, (B + 1) * N, leaves)
            bow.indexed_match_batch_device(desc[1:], leaves[1:], None, N, cnt[1:], desc[:-1], leaves[:-1], None, N,
                                           cnt[:-1], B, 30, 1, out, N, nout, status)

        wall, kern = timed(lib, indexed, a.iters, torch)
        leg("f4 FindLeafNode", "descriptors/s", (B + 1) * N, wall, kern, "bow.leaves", (B + 1) * N * (32 + 4))
        leg("a15 IndexedMatch", "frame pairs/s", B, wall, kern, "match.indexed", B * N * (32 + 4) * 2 + B * N * 16)
    if "remap" in legs:
        cal = Calibration.make(910.0, 905.0, 652.5, 349.0, [0.9, -0.3, 0.0007, 0.0002, 0.02, 1.2, -0.2, 0.05])
        u = image.Undistorter(cal, W, H)
        src = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
        orb.synth_frames_device(src, B, W, H, 0, synth.FRAME_SEED)
        dst = torch.empty_like(src)

        def remap():
            u.batch_device(src, W, W * H, dst, W, W * H, B)

        wall, kern = timed(lib, remap, a.iters, torch)
        # compulsory: frame in + frame out per frame, the shared map (8 B/px) once per launch
        leg("f3 UndistortImage", "frames/s", B, wall, kern, "image.remap", B * W * H * (1 + 1) + W * H * 8)
    if "kpundist" in legs:
        dcal = Calibration.make(910.0, 905.0, 652.5, 349.0, [-0.28, 0.07, 0.001, -0.0005, 0.01])
        ucal = Calibration.make(910.0, 905.0, 640.0, 360.0)
        kpw = kp.clone()

        def kpundist():
            orb.undistort_keypoints_batch_device(dcal, ucal, kpw[1:], N, cnt[1:], B)

        wall, kern = timed(lib, kpundist, a.iters, torch)
        leg("a12 UndistortKeypoints", "frames/s", B, wall, kern, "orb.undistort", B * N * 28 * 2)

    if "pose" in legs:
        from mageslam_amd import bundler

        pb = synth.pose_batch(problems=2048, obs=600, seed=synth.BA_SEED + 1)
        K, E = len(pb.pos), int(pb.obs_start[-1])
        T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x, dt)).cuda()  # noqa: E731
        args_in = (T(pb.pos, np.float32), T(pb.r9, np.float32), T(pb.intr, np.float32),
                   T(pb.obs_start.astype(np.int32), np.int32), T(pb.points, np.float32), T(pb.uv, np.float32),
                   T(pb.info, np.float32))
        outs = (torch.empty((K, 3), dtype=torch.float32, device="cuda"),
                torch.empty((K, 9), dtype=torch.float32, device="cuda"),
                torch.empty((K, 7), dtype=torch.float64, device="cuda"), torch.empty(E, dtype=torch.uint8, device="cuda"),
                torch.empty(K, dtype=torch.float32, device="cuda"), torch.empty((K, 2), dtype=torch.int32, device="cuda"))

        def pose():
            bundler.pose_batch_device(K, *args_in, 3, 4.0, 36.0, *outs)

        wall, kern = timed(lib, pose, a.iters, torch)
        # bench.py run_pose: observations (point 12 + uv 8 + info 4 + flag 1), pose in / out per problem
        leg("f2 pose-only BA (batched)", "problems/s", K, wall, kern, "ba.pose_batch", E * 25 + K * (64 + 116))
    if "train" in legs:
        tcnt = cnt[:15].cpu().numpy()
        tdesc = np.concatenate([desc[i, : tcnt[i]].cpu().numpy() for i in range(15)])

        def train():
            bow.OnlineBowTree.CreateTree(tdesc).close()

        wall, kern = timed(lib, train, a.iters, torch)
        ka = kern.get("bow.km_assign", (0, 0.0))
        ku = kern.get("bow.km_update", (0, 0.0))
        out = {"row": "f4 CreateTree", "value": 1.0 / wall, "unit": "trees/s", "wall_ms_per_tree": wall * 1e3,
               "descriptors": int(len(tdesc)),
               "kernel_ms_per_tree": (ka[0] * ka[1] + ku[0] * ku[1]) / a.iters,
               "kernels": {k: {"launches": n, "avg_ms": v} for k, (n, v) in kern.items()}}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
