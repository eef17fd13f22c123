"""Concurrent callers of the synchronous host-buffer entry points.

The reference calls these paths from several threads at once: both stereo frames'
OrbFeatureDetector::Process (UndistortKeypoints) run in parallel (ImageAnalyzer.cpp:160-216),
and the tracking / mapping / loop-closure threads each run matchers and BundlerLib instances
(BundlerLib.h:20-66 is used from four threads).  Every thread here runs
mage_radius_match, mage_hamming_match, mage_ba_pose_batch and mage_undistort_keypoints with its
own input sizes, many times, and must get exactly the single-threaded results.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from mageslam_amd import bundler, matcher, orb, synth

pytestmark = pytest.mark.gpu

THREADS = 6
ROUNDS = 8


def _work_items():
    det = orb.OrbDetector(nfeatures=2000)
    frames = [synth.frame(t, 640, 480) for t in range(THREADS + 1)]
    feats = [det.DetectAndCompute(f) for f in frames]
    det.close()
    from mageslam_amd._lib import Calibration

    cd = Calibration.make(500.0, 505.0, 320.0, 240.0, (-0.12, 0.03, 1e-4, -2e-4, 0.0))
    cu = Calibration.make(490.0, 490.0, 321.0, 239.0)
    items = []
    for i in range(THREADS):
        (kq, dq), (kt, dt) = feats[i + 1], feats[i]
        nq = 400 + 250 * i  # different sizes per thread: the scratch of one must not fit another
        nt = 2000 - 150 * i
        items.append(dict(
            kq=kq[:nq], dq=dq[:nq], kt=kt[:nt], dt=dt[:nt], radius=4.0 + 2.0 * i,
            pb=synth.pose_batch(problems=8 + 40 * i, obs=120 + 60 * i, seed=100 + i), cd=cd, cu=cu))
    return items


def _run(it):
    r = matcher.RadiusMatch(it["kq"], it["dq"], it["kt"], it["dt"], it["radius"], maxHammingDist=40,
                            minHammingDifference=1)
    m = matcher.Match(it["dq"], it["dt"], maxHammingDist=40, minHammingDifference=1)
    p = bundler.OptimizeCameraPoses(it["pb"], 3, 36.0, 4.0)
    u = orb.UndistortKeypoints(it["kq"], it["cd"], it["cu"])
    return (r.tobytes(), m.tobytes(), p["qt7"].tobytes(), p["outlier"].tobytes(), u.tobytes())


def test_concurrent_host_entry_points_match_single_thread(gpu):
    items = _work_items()
    expect = [_run(it) for it in items]
    assert all(len(e[0]) > 0 and len(e[1]) > 0 for e in expect)

    def worker(i):
        bad = 0
        for _ in range(ROUNDS):
            bad += _run(items[i]) != expect[i]
        return bad

    with cf.ThreadPoolExecutor(THREADS) as ex:
        assert list(ex.map(worker, range(THREADS))) == [0] * THREADS


def test_match_batch_device_threads_share_one_stream(gpu):
    """Several host threads launch mage_hamming_match_batch_device on ONE stream with growing pair
    counts: each growth of the per-stream scratch must never free a buffer another thread is about
    to launch on (capi.cpp stream_scratch, keyed per thread)."""
    import torch

    det = orb.OrbDetector(nfeatures=2000)
    feats = [det.DetectAndCompute(synth.frame(t, 640, 480)) for t in range(9)]
    det.close()
    N = 2000
    desc = torch.zeros((9, N, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(9, dtype=torch.int32, device="cuda")
    for i, (_, d) in enumerate(feats):
        desc[i, :len(d)] = torch.from_numpy(d)
        cnt[i] = len(d)
    shared = torch.cuda.Stream()

    def run(pairs, stream):
        out = torch.zeros((pairs, N * 16), dtype=torch.uint8, device="cuda")
        nm = torch.zeros(pairs, dtype=torch.int32, device="cuda")
        matcher.match_batch_device(desc[1:1 + pairs], N * 32, cnt[1:1 + pairs], desc[:pairs], N * 32, cnt[:pairs],
                                   pairs, 30, 1, out, N, nm, stream=stream)
        return out, nm

    expect = {}
    for p in range(1, 9):
        out, nm = run(p, None)
        torch.cuda.synchronize()
        expect[p] = (out.cpu(), nm.cpu())

    def worker(w):
        bad = 0
        for r in range(ROUNDS):
            p = 1 + (w + r) % 8  # every thread walks its own growing / shrinking pair counts
            with torch.cuda.stream(shared):
                out, nm = run(p, shared.cuda_stream)
            shared.synchronize()
            bad += not (torch.equal(out.cpu(), expect[p][0]) and torch.equal(nm.cpu(), expect[p][1]))
        return bad

    with cf.ThreadPoolExecutor(THREADS) as ex:
        assert list(ex.map(worker, range(THREADS))) == [0] * THREADS


def test_thread_scratch_released_on_thread_exit(gpu):
    """Short-lived threads (one per call) do not accumulate device memory."""
    import torch

    it = _work_items()[THREADS - 1]
    _run(it)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(12):
        with cf.ThreadPoolExecutor(1) as ex:
            ex.submit(_run, it).result()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free0 - free1 < 64 << 20, (free0, free1)
