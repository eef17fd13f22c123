"""Timing ablation of fast_nms_kernel (development tool, not part of the product).

  python tools/ablate_fast.py build     # compile variants into abl/f<N>/libmage_hot.so (CPU)
  python tools/ablate_fast.py run       # time orb.fast_nms of each variant on the GPU (C2 batch)

MAGE_FAST_ABLATE bits: 1 no blur, 2 no NMS / emission, 4 no score, 8 no tile load, 16 NMS without
emission, 32 keep the skipped stages' inputs alive.  "a:w:s:k" also sets __launch_bounds__ min waves per EU (w), MAGE_FAST_SCHED (s) and MAGE_DESC_KPW (k).
"""
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
# variant "a" or "a:w" (ablation bits a, __launch_bounds__ min waves per EU w)
VARIANTS = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "17", "35", "39", "47"]
# MAGE_ABLATE_GATE=<g>: force the candidate gate of every timed batch
GATE = int(os.environ["MAGE_ABLATE_GATE"]) if os.environ.get("MAGE_ABLATE_GATE") else None


def build():
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    from abl import variant_source

    src, _ = variant_source("orb.hip")  # the product source + tools/patches/orb_variants.patch
    objs = [p for p in (B.OBJ).glob("*.o") if not p.name.startswith("orb")]
    for v in VARIANTS:
        out = ROOT / "abl" / ("f" + v.replace(":", "w"))
        out.mkdir(parents=True, exist_ok=True)
        obj = out / "orb.o"
        a, w, sch, kpw = (v.split(":") + ["", "", ""])[:4]
        subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                        f"-DMAGE_FAST_ABLATE={a}", f"-DMAGE_FAST_WAVES_PER_EU={w or 5}", f"-DMAGE_FAST_SCHED={sch or 0}", f"-DMAGE_DESC_KPW={kpw or 4}",
                        "-c", str(src),
                        "-o", str(obj)], check=True)
        subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out / "libmage_hot.so"),
                        str(obj), *map(str, objs)], check=True)
        print("built", out)
    src.unlink()


def run():
    import torch
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib, orb, synth
    W, H, B, N = 1280, 720, 256, 2000
    frames = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
    kp = torch.zeros((B, N * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, N, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    for v in VARIANTS:
        L = C.CDLL(str(ROOT / "abl" / ("f" + v.replace(":", "w")) / "libmage_hot.so"))
        _lib._declare(L)
        _lib._lib = L
        orb.synth_frames_device(frames, B, W, H, 0, synth.FRAME_SEED)
        det = orb.OrbDetector(nfeatures=N)
        for _ in range(3):
            det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
        torch.cuda.synchronize()
        L.mage_profile_reset()
        L.mage_profile_enable(1)
        for _ in range(10):
            if GATE is not None:  # ablations without emission never set a gate themselves
                det.set_fast_gate(GATE)
            det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
        torch.cuda.synchronize()
        rep = _lib.profile_report()
        L.mage_profile_enable(0)
        c, ms = rep.get("orb.fast_nms", (1, float("nan")))
        print(f"variant {v:>5}: fast_nms {ms / c:.4f} ms  select {rep.get('orb.select', (1, 0))[1] / 10:.4f} ms  "
              f"describe {rep.get('orb.describe', (1, 0))[1] / 10:.4f} ms  mean keypoints {cnt.float().mean().item():.0f}", flush=True)
        det.close()


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
