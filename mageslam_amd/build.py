"""Builds libmage_hot.so (HIP for gfx950 + host C++) in-tree under mageslam_amd/_lib/.

hipcc cross-compiles without a GPU; the resulting .so travels to the GPU box with the repo
snapshot.  `python -m mageslam_amd.build` or __graft_entry__.build() runs this.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OUT = PKG / "_lib"
OBJ = OUT / "obj"
LIB = OUT / "libmage_hot.so"
ARCH = os.environ.get("MAGE_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["orb.hip", "match.hip", "radius.hip", "localmap.hip", "bow.hip", "ba.hip", "pose.hip", "image.hip", "track.hip"]
CXX_SOURCES = ["capi.cpp", "tables.cpp", "track.cpp"]

COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          f"-I{PKG.parent / 'include'}"]


def kernel_sources_sha() -> str:
    """SHA-256 (first 16 hex digits) of the HIP / C++ sources and headers the library is built
    from: ties committed profiler counters (profiles/pmc_summary.json) to the kernels they measured."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.hpp")) + list(CSRC.glob("*.cpp"))):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def kernel_file_shas() -> dict:
    """Per-file SHA-256 (first 16 hex digits) of the same sources: a committed counter summary stays
    valid for a kernel while the files that kernel is built from are unchanged."""
    import hashlib

    return {f.name: hashlib.sha256(f.read_bytes()).hexdigest()[:16]
            for f in sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.hpp")) + list(CSRC.glob("*.cpp")))}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm 7.2 expected at /opt/rocm)")


def _compile(src: Path, obj: Path) -> tuple[Path, str]:
    cc = hipcc()
    if src.suffix == ".hip":
        cmd = [cc, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *COMMON, "-c",
               str(src), "-o", str(obj)]
    else:
        cmd = [cc, "-x", "c++", *COMMON, "-I/opt/rocm/include", f'-DMAGE_DATA_DIR={PKG / "data"}', "-D__HIP_PLATFORM_AMD__",
               "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj, res.stderr


def _stale(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(verbose: bool = False, force: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.hpp")) + [PKG.parent / "include" / "mage_hot.h"]
    data = list((PKG / "data").glob("*.bin"))
    jobs = []
    objs = []
    for name in HIP_SOURCES + CXX_SOURCES:
        src = CSRC / name
        obj = OBJ / (name + ".o")
        objs.append(obj)
        deps = [src, *headers] + (data if name == "tables.cpp" else [])
        if force or _stale(obj, deps):
            jobs.append((src, obj))
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            for obj, warn in ex.map(lambda a: _compile(*a), jobs):
                if verbose and warn.strip():
                    print(warn, file=sys.stderr)
    if force or _stale(LIB, objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs),
               "-Wl,--no-undefined"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
