"""Where a local-BA window on the reference schedule spends its time (development probe, GPU).

  python tools/ba_schedule_probe.py [windows]

Per window (bench.py ba_reference_window): set_graph + SetCurrentLambda, then 10 x (StepBundleAdjustment
at the decaying threshold + GetPose / GetPoint).  Prints the wall time of each phase (host clock,
synchronous calls) per window, the median over the windows, and the per-kernel dispatch times of one window.
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch  # noqa: F401  (HIP runtime through torch, as the bench)

    from mageslam_amd import _lib, bundler, synth

    W = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    g = synth.ba_graph()
    b = bundler.BundlerLib(device=0)
    lam = None
    acc = {}

    win = {}

    def tick(name, t0):
        t1 = time.perf_counter()
        win[name] = win.get(name, 0.0) + (t1 - t0)
        return t1

    lib = _lib.load()
    for w in range(W + 4):
        if w == 2:
            acc.clear()
        if w == W + 1:
            lib.mage_profile_reset()
            lib.mage_profile_enable(1)
        t = time.perf_counter()
        b.set_graph(g)
        if lam is not None:
            b.SetCurrentLambda(lam)
        t = tick("set_graph (host arrays)", t)
        L = _lib.load()
        c, o = b._cams, b._obs
        ptr = _lib.ptr
        _lib.check(L.mage_ba_set_cameras(b._h, len(c["pos"]), ptr(c["pos"]), ptr(c["r9"]), ptr(c["intr"]), ptr(c["fixed"])))
        t = tick("  set_cameras", t)
        _lib.check(L.mage_ba_set_points(b._h, len(b._pts), ptr(b._pts)))
        t = tick("  set_points", t)
        _lib.check(L.mage_ba_set_observations(b._h, len(o["cam"]), ptr(o["uv"]), ptr(o["cam"]), ptr(o["pt"]), ptr(o["info"])))
        t = tick("  set_observations", t)
        b._uploaded.update(cams=True, pts=True, obs=True)
        b._upload()
        t = tick("  set_tethers", t)
        me = 7.25
        for k in range(10):
            _, out = b.step([1.8], me)
            t = tick("step 0 (upload + initialize + LM step)" if k == 0 else
                     ("step with removal" if len(out) else "step without removal"), t)
            win.setdefault("n_removal", 0.0)
            if k and len(out):
                win["n_removal"] += 1
            b.poses()
            b.points()
            t = tick("GetPose / GetPoint", t)
            me *= np.float32(0.95) ** 2
        lam = max(b.GetCurrentLambda(), 1e-3)
        for k, v in win.items():
            acc.setdefault(k, []).append(v)
        win.clear()
    lib.mage_profile_enable(0)
    kern = _lib.profile_report()
    n_rem = acc.pop("n_removal")
    out = {k: 1e3 * float(np.median(v)) for k, v in acc.items()}  # ms per window, median over windows
    out["removal steps per window"] = float(np.mean(n_rem))
    out["kernels_one_window_ms"] = {k: {"launches": c, "total_ms": ms} for k, (c, ms) in kern.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
