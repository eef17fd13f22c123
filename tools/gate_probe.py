"""FAST candidate-gate sensitivity on the C2 stream (development probe, GPU).

  python tools/gate_probe.py [gate,gate,...]

For the C2 workload (256-frame batches of the 1280x720 pan sequence, 2000 features) prints the
gate the detector derives by itself (7/8 of the batch's smallest `lower`, orb.hip select_frame),
then for each forced gate: orb.fast_nms / select / redo kernel times, the frames that took the
exact path again, and the whole extraction step (host clock around synchronised batches).
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from mageslam_amd import _lib, orb, synth
    W, H, B, N = 1280, 720, 256, 2000
    gates = [int(g) for g in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 70, 82, 86, 88, 90, 92, 94]
    frames = torch.empty((4, B, H, W), dtype=torch.uint8, device="cuda")
    for s in range(4):
        orb.synth_frames_device(frames[s], B, W, H, s * B, synth.FRAME_SEED)
    kp = torch.zeros((B, N * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, N, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    L = _lib.load()
    det = orb.OrbDetector(nfeatures=N)
    for s in range(8):
        det.detect_and_compute_batch_device(frames[s % 4], W, H, kp, desc, cnt, N)
        print("natural", s, det.fast_gate_stats(), flush=True)
    ref = desc.clone()
    for g in gates:
        redo = 0
        L.mage_profile_reset()
        L.mage_profile_enable(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(8):
            det.set_fast_gate(g)
            det.detect_and_compute_batch_device(frames[s % 4], W, H, kp, desc, cnt, N)
            redo += det.fast_gate_stats()["last_redo"]
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        L.mage_profile_enable(0)
        rep = _lib.profile_report()
        ms = {k: v[1] / max(v[0], 1) for k, v in rep.items()}
        same = bool(torch.equal(desc, ref))
        print(f"gate {g:3d}: fast_nms {ms.get('orb.fast_nms', 0):.4f} select {ms.get('orb.select', 0):.4f} "
              f"fast_redo {ms.get('orb.fast_redo', 0):.4f} select_redo {ms.get('orb.select_redo', 0):.4f} "
              f"describe {ms.get('orb.describe', 0):.4f} ms; redo frames {redo}/{8 * B}; "
              f"step {el / 8 * 1e3:.3f} ms (incl. stats syncs); same output {same}", flush=True)
    det.close()


if __name__ == "__main__":
    main()
