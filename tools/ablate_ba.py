"""Timing ablation of the BA dense solve (development tool, not part of the product).

  python tools/ablate_ba.py build   # variants of ba.hip (MAGE_CHOL_ABLATE) into abl/ba<N>/ (CPU)
  python tools/ablate_ba.py run     # per-kernel times of the C3 graph for each variant (GPU)

MAGE_CHOL_ABLATE: 0 full, 2 trivial diagonal-block factorisation (time of the serial block factor),
3 = 0 + per-phase s_memtime cycle counts of wave 0 printed by the kernel.
The variant library is loaded by this script alone; the product loader is untouched.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
VARIANTS = [0, 2, 3]


def build():
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    objs = [p for p in B.OBJ.glob("*.o") if not p.name.startswith("ba.")]
    for v in VARIANTS:
        out = ROOT / "abl" / f"ba{v}"
        out.mkdir(parents=True, exist_ok=True)
        subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                        f"-DMAGE_CHOL_ABLATE={v}", "-c", str(B.CSRC / "ba.hip"), "-o", str(out / "ba.o")], check=True)
        subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out / "libmage_hot.so"),
                        str(out / "ba.o"), *map(str, objs)], check=True)
        print("built", out)


def run():
    import torch  # noqa: F401  (HIP runtime init through torch, as the bench does)
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib, bundler, synth
    g = synth.ba_graph()
    for v in VARIANTS:
        lib = C.CDLL(str(ROOT / "abl" / f"ba{v}" / "libmage_hot.so"))
        _lib._declare(lib)
        _lib._lib = lib  # this process only: route the mirror classes to the variant
        b = bundler.BundlerLib(device=0)
        b.set_graph(g)
        for _ in range(3):
            b.step([1.8], 7.25)
        lib.mage_profile_reset()
        lib.mage_profile_enable(1)
        for _ in range(1 if v == 3 else 20):
            b.step([1.8], 7.25)
        lib.mage_profile_enable(0)
        rep = _lib.profile_report()
        print(f"variant {v}: " + ", ".join(f"{k} {ms / max(c, 1):.4f} ms" for k, (c, ms) in sorted(rep.items())), flush=True)
        del b


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
