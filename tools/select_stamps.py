"""Per-phase timing of select_kernel from s_memtime stamps (development tool, not the product).

  python tools/select_stamps.py build   # abl/sel/libmage_hot.so with -DMAGE_SELECT_STAMPS=1 (CPU)
  python tools/select_stamps.py run     # C2 batches on the GPU, mean cycles per phase over frames

Phases (stamps 0..10): tile scan | histogram | cut | retained items | bbox + cell zero | cell
count + scan | cell scatter | ring search | sort | output.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "abl" / "sel"
NAMES = ["tiles", "hist", "cut", "items", "bbox", "cellcount", "scatter", "ring", "sort", "output"]


def build():
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    objs = [p for p in B.OBJ.glob("*.o") if not p.name.startswith("orb")]
    OUT.mkdir(parents=True, exist_ok=True)
    subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                    "-DMAGE_SELECT_STAMPS=1", "-c", str(B.CSRC / "orb.hip"), "-o", str(OUT / "orb.o")], check=True)
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
    st = np.zeros((1024, 16), np.uint64)
    acc, sub = [], []
    for it in range(6):
        det.detect_and_compute_batch_device(frames, W, H, kp, desc, cnt, N)
        torch.cuda.synchronize()
        L.mage_debug_select_stamps(st.ctypes.data_as(C.c_void_p))
        if it >= 2:
            s = st[:B, :11].astype(np.int64)
            acc.append(np.diff(s, axis=1))
            x = st[:B].astype(np.int64)
            sub.append(np.stack([x[:, 11] - x[:, 8], x[:, 12] - x[:, 11], x[:, 13] - x[:, 12], x[:, 9] - x[:, 13]], 1))
            print("start spread (cycles):", int(s[:, 0].max() - s[:, 0].min()), " end-start mean:",
                  int((s[:, 10] - s[:, 0]).mean()), flush=True)
    d = np.concatenate(acc).mean(0)
    tot = d.sum()
    for n, v in zip(NAMES, d):
        print(f"{n:>10}: {v:9.0f} cycles  {100 * v / tot:5.1f} %")
    for n, v in zip(["mhist", "mscan", "compact", "bitonic"], np.concatenate(sub).mean(0)):
        print(f"{n:>10}: {v:9.0f} cycles  (inside sort)")
    print(f"{'total':>10}: {tot:9.0f} cycles ({tot / 100e6 * 1e3:.3f} ms at the 100 MHz s_memtime? see note)")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
