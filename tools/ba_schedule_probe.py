"""Where a local-BA window on the reference schedule spends its time (development probe, GPU).

  python tools/ba_schedule_probe.py [windows]

Per window (bench.py ba_reference_window): set_graph + SetCurrentLambda, then 10 x (StepBundleAdjustment
at the decaying threshold + GetPose / GetPoint).  Prints the wall time of each phase (host clock,
synchronous calls) averaged over the windows, and the per-kernel dispatch times of one window.
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

    def tick(name, t0):
        t1 = time.perf_counter()
        acc[name] = acc.get(name, 0.0) + (t1 - t0)
        return t1

    lib = _lib.load()
    for w in range(W + 2):
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
        me = 7.25
        for k in range(10):
            _, out = b.step([1.8], me)
            t = tick("step 0 (upload + initialize + LM step)" if k == 0 else
                     ("step with removal" if len(out) else "step without removal"), t)
            acc.setdefault("n_removal", 0.0)
            if k and len(out):
                acc["n_removal"] += 1
            b.poses()
            b.points()
            t = tick("GetPose / GetPoint", t)
            me *= np.float32(0.95) ** 2
        lam = max(b.GetCurrentLambda(), 1e-3)
    lib.mage_profile_enable(0)
    kern = _lib.profile_report()
    n_rem = acc.pop("n_removal")
    out = {k: 1e3 * v / W for k, v in acc.items()}
    out["removal steps per window"] = n_rem / W
    out["kernels_one_window_ms"] = {k: {"launches": c, "total_ms": ms} for k, (c, ms) in kern.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
