"""Timing ablation of the BA kernels (development tool, not part of the product).

  python tools/ablate_ba.py build [V1 V2 ...]   # variants of ba.hip into abl/ba_<i>/ (CPU)
  python tools/ablate_ba.py run   [V1 V2 ...]   # per-kernel times of the C3 graph per variant (GPU)
  python tools/ablate_ba.py libs  name[,name]   # the same for abl/<name>/libmage_hot.so (tools/abl.py build)

A variant is a '+'-joined list of NAME=VALUE preprocessor definitions ("0" = the product build),
e.g. MAGE_CHOL_ABLATE=3.  Switches in ba.hip:
MAGE_CHOL_ABLATE (0 full, 2 trivial diagonal-block factorisation, 3 per-phase s_memtime cycles of
wave 0 printed by the kernel, 4 per-step barrier timestamps of every wave; 5 the same per segment of
chol_lead), MAGE_CHOL_LEAD (1 chol_lead, 0 chol_tiles).  The variant library is loaded by this script alone; the product
loader is untouched.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
VARIANTS = sys.argv[2:] or ["0", "MAGE_CHOL_ABLATE=2", "MAGE_CHOL_ABLATE=3"]


def defines(v):
    return [] if v == "0" else ["-D" + d for d in v.split("+")]


def build():
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    from abl import variant_source

    src, _ = variant_source("ba.hip")  # the product source + tools/patches/ba_variants.patch
    objs = [p for p in B.OBJ.glob("*.o") if not p.name.startswith("ba.")]
    for i, v in enumerate(VARIANTS):
        out = ROOT / "abl" / f"ba_{i}"
        out.mkdir(parents=True, exist_ok=True)
        subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                        *defines(v), "-c", str(src), "-o", str(out / "ba.o")], check=True)
        subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out / "libmage_hot.so"),
                        str(out / "ba.o"), *map(str, objs)], check=True)
        (out / "variant.txt").write_text(v)
        print("built", out, v)
    src.unlink()


def run(libs=None):
    import torch  # noqa: F401  (HIP runtime init through torch, as the bench does)
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib, bundler, synth
    g = synth.ba_graph()
    for i, v in enumerate(libs or VARIANTS):
        if libs:
            d = ROOT / "abl" / v
        else:
            d = ROOT / "abl" / f"ba_{i}"
            assert (d / "variant.txt").read_text() == v, f"abl/ba_{i} was built for another variant"
        lib = C.CDLL(str(d / "libmage_hot.so"))
        _lib._declare(lib)
        _lib._lib = lib  # this process only: route the mirror classes to the variant
        b = bundler.BundlerLib(device=0)
        b.set_graph(g)
        for _ in range(3):
            b.step([1.8], 7.25)
        lib.mage_profile_reset()
        lib.mage_profile_enable(1)
        n = 1 if any(f"MAGE_CHOL_ABLATE={i}" in v for i in (3, 4, 5)) else 20
        for _ in range(n):
            b.step([1.8], 7.25)
        lib.mage_profile_enable(0)
        rep = _lib.profile_report()
        tot = sum(ms for c, ms in rep.values()) / n
        print(f"variant {v}: total {tot:.4f} ms/it | " + ", ".join(f"{k[3:]} {ms / max(c, 1):.4f}" for k, (c, ms) in sorted(rep.items())), flush=True)
        del b


if __name__ == "__main__":
    if sys.argv[1] == "libs":
        run(sys.argv[2].split(","))
    else:
        {"build": build, "run": run}[sys.argv[1]]()
