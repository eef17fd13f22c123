"""Candidate-gate probe (development tool): per-batch gate stats and orb.fast_nms time with the
gate as the detector sets it, forced off, and forced to fixed values (C2 batch)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from mageslam_amd import _lib, orb, synth  # noqa: E402

W, H, B, N = 1280, 720, 256, 2000
frames = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
kp = torch.zeros((B, N * 28), dtype=torch.uint8, device="cuda")
desc = torch.zeros((B, N, 32), dtype=torch.uint8, device="cuda")
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
L = _lib.load()
det = orb.OrbDetector(nfeatures=N)
for t0 in range(0, 4 * B, B):
    orb.synth_frames_device(frames, B, W, H, t0, synth.FRAME_SEED)
    det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
    torch.cuda.synchronize()
    print("batch", t0 // B, det.fast_gate_stats(), flush=True)
for forced in (None, 0, 40, 60, 80, 90, 100):
    L.mage_profile_reset()
    L.mage_profile_enable(1)
    for _ in range(5):
        if forced is not None:
            det.set_fast_gate(forced)
        det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
    torch.cuda.synchronize()
    rep = _lib.profile_report()
    L.mage_profile_enable(0)
    st = det.fast_gate_stats()
    print(f"gate {forced}: " + "  ".join(f"{k} {v[1] / v[0]:.4f}" for k, v in sorted(rep.items())), st, flush=True)
