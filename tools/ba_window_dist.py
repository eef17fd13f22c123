"""Distribution of reference-schedule window times (bench.py ba_reference_window), one BundlerLib
on one GPU (development probe): mean, median and the windows above 3 ms with their index — a
doubling pattern there points at a buffer that keeps growing.

  python tools/ba_window_dist.py [windows]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    from mageslam_amd import bundler, synth

    W = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    g = synth.ba_graph()
    b = bundler.BundlerLib(device=0)
    lam = bench.ba_reference_window(b, g, None, 10, b.SetCurrentLambda, b.GetCurrentLambda)
    torch.cuda.synchronize()
    ts = []
    for _ in range(W):
        t0 = time.perf_counter()
        lam = bench.ba_reference_window(b, g, lam, 10, b.SetCurrentLambda, b.GetCurrentLambda)
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    print(json.dumps({"windows": W, "mean_ms": float(ts.mean()), "median_ms": float(np.median(ts)),
                      "calls_per_s_mean": 10e3 / float(ts.mean()),
                      "outliers": [(i, round(float(t), 2)) for i, t in enumerate(ts) if t > 3]}))


if __name__ == "__main__":
    main()
