"""Timing ablation of the matcher tile body (development tool, not part of the product).

  python tools/ablate_match.py build     # compile variants into abl/v<N>/libmage_hot.so (CPU)
  python tools/ablate_match.py run       # time each variant on the GPU (random descriptors)

MAGE_MATCH_ABLATE: 0 full, 1 no column top-2, 2 no row top-2, 4 MFMA + one max only,
5 = 4 without stage fills, 6 = 5 without stage barriers.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
VARIANTS = [0, 1, 2, 4, 5, 6]


def build():
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import build as B
    B.build()
    from abl import variant_source

    src, _ = variant_source("match.hip")  # the product source + tools/patches/match_variants.patch
    objs = [p for p in (B.OBJ).glob("*.o") if not p.name.startswith("match")]
    for v in VARIANTS:
        out = ROOT / "abl" / f"v{v}"
        out.mkdir(parents=True, exist_ok=True)
        obj = out / "match.o"
        subprocess.run([B.hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", *B.COMMON,
                        f"-DMAGE_MATCH_ABLATE={v}", "-c", str(src), "-o", str(obj)], check=True)
        subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out / "libmage_hot.so"),
                        str(obj), *map(str, objs)], check=True)
        print("built", out)
    src.unlink()


def run():
    import torch
    sys.path.insert(0, str(ROOT))
    from mageslam_amd import _lib
    pairs, n = 256, 2000
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.randint(0, 256, (pairs, n, 32), dtype=torch.uint8, device="cuda", generator=g)
    B = torch.randint(0, 256, (pairs, n, 32), dtype=torch.uint8, device="cuda", generator=g)
    nA = torch.full((pairs,), n, dtype=torch.int32, device="cuda")
    out = torch.empty((pairs, n, 4), dtype=torch.int32, device="cuda")
    cnt = torch.empty((pairs,), dtype=torch.int32, device="cuda")
    for v in VARIANTS:
        lib = C.CDLL(str(ROOT / "abl" / f"v{v}" / "libmage_hot.so"))
        f = lib.mage_hamming_match_batch_device
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_uint32,
                      C.c_int32, C.c_int32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        st = torch.cuda.current_stream().cuda_stream

        def call():
            r = f(A.data_ptr(), n * 32, nA.data_ptr(), B.data_ptr(), n * 32, nA.data_ptr(), pairs, 30, 5,
                  out.data_ptr(), n, cnt.data_ptr(), st)
            assert r == 0, r
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        torch.cuda.synchronize()
        print(f"variant {v}: {e0.elapsed_time(e1) / 20:.4f} ms  matches/pair {cnt.float().mean().item():.1f}", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
