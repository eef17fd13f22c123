"""Regenerates tests/golden/* from the CPU oracle (run in the build container).

These are regression fixtures of the oracle restatement (no reference fixtures exist for this
path: SURVEY.md §4), plus the SHA-256 of the BRIEF tables extracted from the reference by
tools/extract_patterns.py.
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from mageslam_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

G = ROOT / "tests" / "golden"


def main():
    G.mkdir(parents=True, exist_ok=True)
    lines = []
    for patch in (15, 31):
        data = (ROOT / "mageslam_amd" / "data" / f"bit_pattern_{patch}_rotated.bin").read_bytes()
        lines.append(f"{hashlib.sha256(data).hexdigest()} bit_pattern_{patch}_rotated.bin")
    (G / "pattern_tables.sha256").write_text("\n".join(lines) + "\n")

    f0 = synth.frame(0, 640, 480)
    f1 = synth.frame(1, 640, 480)
    st, kp0, d0 = O.orb_detect(f0, O.default_settings(2000))
    st1, kp1, d1 = O.orb_detect(f1, O.default_settings(2000))
    np.savez_compressed(G / "orb_vga_t0.npz", frame_sha256=hashlib.sha256(f0.tobytes()).hexdigest(),
                        kp_xyr=np.stack([kp0["x"], kp0["y"], kp0["response"]], 1), desc=d0)
    m = O.match(d1, d0, max_distance=30, min_difference=1)
    np.savez_compressed(G / "match_vga_t1_t0.npz", desc_a=d1, desc_b=d0,
                        matches=np.stack([m["query_idx"], m["train_idx"], m["distance"].astype(np.int32)], 1))

    g = synth.ba_graph(cameras=12, points=400, obs_per_point=8, fixed_cameras=3, seed=1)
    b = O.BundlerOracle()
    b.set_graph(g)
    outs = []
    for it in range(3):
        _, o = b.step([1.8], 7.25 * 0.9025 ** it)
        outs.append(o)
    qt, xyz = b.state()
    np.savez_compressed(G / "ba_small.npz", qt=qt, xyz=xyz, outliers=np.concatenate(outs))
    print("golden fixtures written to", G)


if __name__ == "__main__":
    main()
