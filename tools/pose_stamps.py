"""Per-phase timing of one pose-only BA problem (pose_ba_kernel, the tracker's single-problem
launch) from s_memtime stamps (development tool, not the product).

  python tools/pose_stamps.py build [name [-DX=Y ...]]  # abl/<name, pose>/libmage_hot.so, -DMAGE_POSE_STAMPS=1
  python tools/pose_stamps.py run [name ...]            # one problem per launch at E = 600 / 1200 / 2000

Stamps: 0 start | 1 initial pose + staging | 2 edge loop done | 3 reduction done | 9 trial solve
done | 4 exp map done | 5 trial decided | 6 post-pass edges | 7 post-pass reduction | 8 end.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def build(name="pose", *defs):
    out = ROOT / "abl" / name
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    objs = [p for p in B.OBJ.glob("*.o") if not p.name.startswith("pose")]
    out.mkdir(parents=True, exist_ok=True)
    subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                    "-DMAGE_POSE_STAMPS=1", *defs, "-c", str(B.CSRC / "pose.hip"), "-o", str(out / "pose.o")],
                   check=True)
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out / "libmage_hot.so"),
                    str(out / "pose.o"), *map(str, objs)], check=True)
    print("built", out)


def run(*names):
    for name in names or ("pose",):
        print(f"== {name}")
        run_one(ROOT / "abl" / name)


def run_one(OUT):
    import numpy as np
    import torch  # noqa: F401  (HIP runtime through torch first)
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib, bundler, synth
    L = C.CDLL(str(OUT / "libmage_hot.so"))
    _lib._declare(L)
    _lib._lib = L
    names = {2: "edges", 3: "reduce", 9: "solve", 4: "exp map", 5: "decide", 6: "post edges", 7: "post reduce", 8: "outputs"}
    st = np.zeros(256, np.uint64)
    for E in (600, 1200, 2000):
        pb = synth.pose_batch(problems=1, obs=E, vary=False)
        per = {}
        tot, nrep = [], 0
        for rep in range(30):
            out = bundler.OptimizeCameraPoses(pb, 3, 36.0, 4.0)
            L.mage_debug_pose_stamps(st.ctypes.data_as(C.c_void_p))
            if rep < 5:
                continue
            n = int(st[255])
            ids = (st[:n] >> np.uint64(56)).astype(int)
            t = (st[:n] & np.uint64((1 << 56) - 1)).astype(np.int64)
            tot.append(int(t[-1] - t[0]))
            nrep += 1
            for k in range(1, n):
                per.setdefault(int(ids[k]), []).append(int(t[k] - t[k - 1]))
        print(f"E = {E}: iterations / trials {out['stats'][0].tolist()}, total {np.mean(tot):.0f} cycles "
              f"(stamps in order: {ids.tolist()})")
        for k in sorted(per):
            v = np.array(per[k])
            print(f"  -> {k} {names.get(k, ''):>12}: {len(v) / nrep:4.1f} per launch x {v.mean():7.0f} cycles "
                  f"= {len(v) / nrep * v.mean():8.0f}")


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]](*sys.argv[2:])
