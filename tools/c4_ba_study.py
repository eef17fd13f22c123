"""C4 local-BA accuracy study on the CPU oracle (development tool, not the product).

  python tools/c4_ba_study.py extract            # oracle ORB over the 1000-frame C4 sequence -> /tmp/c4_feats.npz
  python tools/c4_ba_study.py run MODE[,MODE...] # one oracle tracking run per mode (~60 s each), RMSE vs ground truth

Modes (combine with '+'): noba (local BA off), ba (the C4 composition: ring of 4 keyframes, the
covisibility window of GetMapPointsAndDistantKeyframes — the new keyframe and the ring keyframes
sharing >= theta points with it free, ThreadSafeMap.cpp:888-957), free1 / free2 / free3 (the newest
N keyframes free instead: ba_free_keyframes; free2 was the round-4/5 rule), lm6 / lm8
(local_map_keyframes), minobs (only points with >= 2 observations in the window), anch (only points
observed by a fixed keyframe), norefine (refinement counts not incremented after a window), steps3 /
steps10 (3x / 10x the LM steps per window), nopoints (the window's poses written back, its points
not), noposes (points written back, poses not), depth2 / depth5 (new map points at a depth off by
2 % / 5 % rms: TrackerSettings.map_point_depth_noise, the error a triangulated point would carry
instead of the exact plane depth).  Output: one line per mode, pose RMSE (translation, rotation)
over the 1000 frames against the synthetic ground truth; profiles/r5_c4_ba_study.md and
profiles/r6_c4_ba_study.md hold runs.
"""
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mageslam_amd import synth, tracking  # noqa: E402

T = 1000
FEATS = Path("/tmp/c4_feats.npz")


def sequence():
    return synth.scene_sequence(T, 1280, 720, step=0.03, origin=synth.rank_origin(0))


def extract():
    from oracle import oracle as O

    seq = sequence()
    s = O.default_settings(2000)

    def one(i):
        f = synth.scene_frames(seq, i, 1)[0]
        _, kp, d = O.orb_detect(np.ascontiguousarray(f), s)
        return kp, d

    t0 = time.time()
    with ThreadPoolExecutor(8) as ex:
        feats = list(ex.map(one, range(T)))
    np.savez(FEATS, **{f"kp{i}": k for i, (k, _) in enumerate(feats)}, **{f"d{i}": d for i, (_, d) in enumerate(feats)})
    print(f"extract {time.time() - t0:.0f} s -> {FEATS}")


def _filter(w, keep):
    newidx = np.cumsum(keep) - 1
    okobs = keep[w.pt]
    w.points = w.points[keep]
    w.point_src = [p for p, k in zip(w.point_src, keep) if k]
    w.uv, w.cam, w.info = w.uv[okobs], w.cam[okobs], w.info[okobs]
    w.pt = newidx[w.pt[okobs]].astype(np.uint32)
    w.obs_src = [o for o, k in zip(w.obs_src, okobs) if k]
    return w


def run(mode):
    from oracle.tracking_backend import OracleBackend

    opts = set(mode.split("+"))
    z = np.load(FEATS)
    feats = [(z[f"kp{i}"], z[f"d{i}"]) for i in range(T)]
    seq = sequence()
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    gt = tracking.TrackResult(poses=[tracking.Pose(seq.R[i], seq.t[i]) for i in range(T)])
    kw = dict(width=1280, height=720, local_ba="noba" not in opts)
    for n in (1, 2, 3):
        if f"free{n}" in opts:
            kw["ba_free_keyframes"] = n
    if "depth2" in opts or "depth5" in opts:
        kw["map_point_depth_noise"] = 0.02 if "depth2" in opts else 0.05
    if "lm6" in opts:
        kw["local_map_keyframes"] = 6
    if "lm8" in opts:
        kw["local_map_keyframes"] = 8
    build, apply = tracking.build_ba_window, tracking.apply_ba_window

    def build_w(ring, K_, s, theta=None):
        w, theta = build(ring, K_, s, theta)
        if w is None:
            return w, theta
        keep = np.ones(len(w.points), bool)
        if "minobs" in opts:
            keep &= np.bincount(w.pt, minlength=len(w.points)) >= 2
        if "anch" in opts:
            seen = np.zeros(len(w.points), bool)
            seen[w.pt[w.fixed[w.cam] == 1]] = True
            keep &= seen
        if "steps3" in opts:
            w.huber_widths = w.huber_widths * 3
        if "steps10" in opts:
            w.huber_widths = w.huber_widths * 10
        return _filter(w, keep), theta

    def apply_w(ring, w, outl, pos, r9, pts, s):
        saved = [k.refine.copy() for k in ring] if "norefine" in opts else None
        if "noposes" in opts:
            pos, r9 = w.pos.copy(), w.rot_colmajor.copy()
        if "nopoints" in opts:
            pts = w.points.copy()
        apply(ring, w, outl, pos, r9, pts, s)
        if saved is not None:
            for k, r in zip(ring, saved):
                k.refine[:] = r

    tracking.build_ba_window, tracking.apply_ba_window = build_w, apply_w
    try:
        t0 = time.time()
        r = tracking.track(feats, K, p0, synth.SCENE_PLANE_Z, OracleBackend(2000), tracking.TrackerSettings(**kw))
    finally:
        tracking.build_ba_window, tracking.apply_ba_window = build, apply
    rt, rr = tracking.pose_rmse(r, gt)
    nout = sum(n for _, n in r.ba_outliers)
    n600 = sum(n for f, n in r.ba_outliers if f < 600)
    print(f"| {mode} | {rt:.5f} | {rr:.6f} | {len(r.keyframes)} | {len(r.ba_outliers)} | {nout} ({n600} in the first 600 "
          f"frames) | {time.time() - t0:.0f} s |", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "extract":
        extract()
    else:
        print("| mode | translation RMSE | rotation RMSE | keyframes | BA windows | BA outliers | time |")
        print("|---|---|---|---|---|---|---|")
        for m in sys.argv[2].split(","):
            run(m)
