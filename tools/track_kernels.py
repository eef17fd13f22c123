"""Per-kernel time of the device-resident C4 loop (development probe, GPU):
python tools/track_kernels.py [frames]  -> JSON: wall ms per frame of mage_track_sequence_device and
the per-kernel launches / total ms over the sequence (dispatch timestamps)."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from mageslam_amd import _lib, orb, synth, tracking

    T = int(sys.argv[1]) if len(sys.argv) > 1 else 240
    seq = synth.scene_sequence(T, 1280, 720)
    cams = torch.from_numpy(seq.cams()).cuda()
    frames = torch.empty((T, 720, 1280), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().mage_synth_scene_device(_lib.ptr(frames), T, 1280, 720, 1280 * 720, _lib.ptr(cams), seq.fx,
                                                   seq.fy, seq.cx, seq.cy, synth.SCENE_PLANE_Z, synth.SCENE_TEXEL_SCALE,
                                                   synth.SCENE_TEXEL_OFFSET, synth.FRAME_SEED, None))
    K = (seq.fx, seq.fy, seq.cx, seq.cy)
    p0 = tracking.Pose(seq.R[0], seq.t[0])
    det = orb.OrbDetector(nfeatures=2000)
    kp = torch.zeros((T, 2000 * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((T, 2000, 32), dtype=torch.uint8, device="cuda")
    n = torch.zeros(T, dtype=torch.int32, device="cuda")
    for b0 in range(0, T, 64):
        det.detect_and_compute_batch_device(frames[b0:b0 + 64], 1280, 720, kp[b0:b0 + 64], desc[b0:b0 + 64],
                                            n[b0:b0 + 64], 2000)
    torch.cuda.synchronize()
    out = {}
    for nk in (4, 0):
        s = tracking.TrackerSettings(local_map_keyframes=nk)
        tracking.track_native_device(kp, desc, 2000, n, T, K, p0, synth.SCENE_PLANE_Z, settings=s)
        t0 = time.perf_counter()
        r = tracking.track_native_device(kp, desc, 2000, n, T, K, p0, synth.SCENE_PLANE_Z, settings=s)
        wall = (time.perf_counter() - t0) / T * 1e3
        lib = _lib.load()
        lib.mage_profile_reset()
        lib.mage_profile_enable(1)
        tracking.track_native_device(kp, desc, 2000, n, T, K, p0, synth.SCENE_PLANE_Z, settings=s)
        torch.cuda.synchronize()
        lib.mage_profile_enable(0)
        kern = _lib.profile_report()
        out[f"local_map_keyframes={nk}"] = {
            "ms_per_frame": wall, "keyframes": len(r.keyframes), "mean_inliers": sum(r.inliers[1:]) / (T - 1),
            "kernels_us_per_frame": {k: round(1e3 * ms / (T - 1), 2) for k, (c, ms) in sorted(kern.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
