"""Per-phase timing of fast_nms_kernel from s_memtime stamps (development tool, not the product).

  python tools/fast_stamps.py build   # abl/fst/libmage_hot.so with -DMAGE_FAST_STAMPS=1 (CPU)
  python tools/fast_stamps.py run     # C2 batches (gate forced to 89) on the GPU

Each wave of the tiles of frames 0..14 stamps s_memtime at the phase boundaries of fast_tile's
gated path; the table is the mean over waves of each phase's cycles (the wave's own elapsed time,
which includes the cycles its SIMD spent on other waves) and the share of the wave's lifetime.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "abl" / "fst"
NAMES = ["load + barrier", "gate", "listing", "dense barrier", "exact scoring", "scores barrier", "xor tile",
         "nms + emission", "pre-blur barrier", "blur", "final barrier", "output"]


def build():
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    objs = [p for p in B.OBJ.glob("*.o") if not p.name.startswith("orb")]
    OUT.mkdir(parents=True, exist_ok=True)
    subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                    "-DMAGE_FAST_STAMPS=1", "-c", str(B.CSRC / "orb.hip"), "-o", str(OUT / "orb.o")], check=True)
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(OUT / "libmage_hot.so"),
                    str(OUT / "orb.o"), *map(str, objs)], check=True)
    print("built", OUT)


def run():
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib, orb, synth
    L = C.CDLL(str(OUT / "libmage_hot.so"))
    _lib._declare(L)
    _lib._lib = L
    W, H, B, N = 1280, 720, 256, 2000
    frames = torch.empty((B, H, W), dtype=torch.uint8, device="cuda")
    kp = torch.zeros((B, N * 28), dtype=torch.uint8, device="cuda")
    desc = torch.zeros((B, N, 32), dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    orb.synth_frames_device(frames, B, W, H, 0, synth.FRAME_SEED)
    det = orb.OrbDetector(nfeatures=N)
    st = np.zeros((4096, 2, 16), np.uint64)
    acc = []
    for it in range(6):
        det.set_fast_gate(89)
        det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
        torch.cuda.synchronize()
        L.mage_debug_fast_stamps(st.ctypes.data_as(C.c_void_p))
        if it >= 2:
            s = st[:, :, :13].reshape(-1, 13).astype(np.int64)
            ok = (s[:, 0] > 0) & np.all(np.diff(s, axis=1) >= 0, axis=1)
            acc.append(np.diff(s[ok], axis=1))
    d = np.concatenate(acc)
    m = d.mean(0)
    tot = m.sum()
    print(f"waves {len(d)}, mean lifetime {tot:.0f} cycles")
    for n, v in zip(NAMES, m):
        print(f"  {n:18s} {v:8.0f} cycles  {100 * v / tot:5.1f} %")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
