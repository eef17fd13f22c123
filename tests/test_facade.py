"""The C++ facades compile against include/ and drive libmage_hot.so like the reference's callers."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "cpp" / "facade_demo.cpp"


def build_demo(tmp_path_factory=None):
    from mageslam_amd import build

    lib = build.build()
    out = ROOT / "mageslam_amd" / "_lib" / "facade_demo"
    if not out.exists() or out.stat().st_mtime < max(SRC.stat().st_mtime, lib.stat().st_mtime,
                                                       (ROOT / "include" / "mage" / "mage.hpp").stat().st_mtime):
        subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", f"-I{ROOT / 'include'}", str(SRC), "-o", str(out),
                        f"-L{lib.parent}", "-lmage_hot", f"-Wl,-rpath,{lib.parent}"], check=True)
    return out


def run_demo(tmp_path, img):
    exe = build_demo()
    raw = tmp_path / "img.raw"
    img.tofile(raw)
    outf = tmp_path / "out.bin"
    r = subprocess.run([str(exe), str(raw), str(img.shape[1]), str(img.shape[0]), str(outf)],
                       capture_output=True, text=True)
    return r, outf


def test_facade_compiles_and_reports_no_device(tmp_path):
    import torch

    from mageslam_amd import synth

    r, _ = run_demo(tmp_path, synth.frame(0, 320, 240))
    if torch.cuda.is_available():
        assert r.returncode == 0, r.stderr
    else:
        assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)


@pytest.mark.gpu
def test_facade_matches_python_api(gpu, tmp_path):
    from mageslam_amd import orb, synth

    img = synth.frame(5, 640, 480)
    r, outf = run_demo(tmp_path, img)
    assert r.returncode == 0, r.stderr
    data = outf.read_bytes()
    n = int(np.frombuffer(data[:4], np.uint32)[0])
    kp = np.frombuffer(data[4:4 + 28 * n], np.uint8)
    desc = np.frombuffer(data[4 + 28 * n:4 + 60 * n], np.uint8).reshape(n, 32)
    nm = int(np.frombuffer(data[4 + 60 * n:8 + 60 * n], np.uint32)[0])
    ms = float(np.frombuffer(data[8 + 60 * n:12 + 60 * n], np.float32)[0])
    pk, pd = orb.OrbDetector(nfeatures=2000).DetectAndCompute(img)
    assert n == len(pk) and np.array_equal(kp, pk.view(np.uint8).reshape(-1)) and np.array_equal(desc, pd)
    assert nm == n  # self-match keeps every distinct descriptor
    assert ms < 1e-3  # noiseless observations converge
    nr = int(np.frombuffer(data[12 + 60 * n:16 + 60 * n], np.uint32)[0])
    from mageslam_amd import matcher

    assert nr == len(matcher.RadiusMatch(pk, pd, pk, pd, 2.0))
    ni = int(np.frombuffer(data[16 + 60 * n:20 + 60 * n], np.uint32)[0])
    from mageslam_amd import bow

    nodes = pd[:7]
    tree = bow.OnlineBowTree(nodes, np.array([0, 3, 6, 6, 6, 6, 6, 6], np.uint32), np.arange(1, 7, dtype=np.uint32))
    assert ni == len(bow.IndexedMatch(tree, pd, pd))
    nt = int(np.frombuffer(data[20 + 60 * n:24 + 60 * n], np.uint32)[0])
    assert nt == len(bow.IndexedMatch(bow.OnlineBowTree.CreateTree(pd), pd, pd))
    nl = int(np.frombuffer(data[24 + 60 * n:28 + 60 * n], np.uint32)[0])
    lres = np.frombuffer(data[28 + 60 * n:28 + 64 * n], np.int32)
    pos = np.stack([pk["x"], pk["y"]], 1)
    res, _ = matcher.LocalMapMatch(pos, pk["octave"], pd, pk, pd, np.ones(n, bool), 2.0, 30, 1)
    assert nl == int((res >= 0).sum()) and np.array_equal(lres, res)


def test_bundler_step_argument_reuse(monkeypatch):
    """StepBundleAdjustment reuses its huber array and outlier buffer across calls (no GPU: the
    library call is stubbed): a changed huber schedule must reach the library, and the outliers
    the library reports are appended in order."""
    import ctypes as C

    from mageslam_amd import bundler

    seen = []

    class Lib:
        def mage_ba_step(self, h, hw, nhw, maxerr, out, cap, n_ref, ms_ref):
            arr = (C.c_float * nhw).from_address(hw.value)
            seen.append((list(arr), maxerr))
            outs = (C.c_uint32 * cap).from_address(out.value)
            k = len(seen)  # call k reports k outliers: 10, 11, ...
            for i in range(k):
                outs[i] = 10 + i
            C.cast(n_ref, C.POINTER(C.c_uint32))[0] = k
            C.cast(ms_ref, C.POINTER(C.c_float))[0] = 0.5 * k
            return 0

    monkeypatch.setattr(bundler._lib, "load", lambda: Lib())
    b = bundler.BundlerLib.__new__(bundler.BundlerLib)
    b._obs = {"cam": np.zeros(16, np.uint32)}
    b._upload = lambda: None
    b._h = C.c_void_p(0)
    o1, o2, o3 = [], [], []
    assert b.StepBundleAdjustment([1.8], 7.25, o1) == 0.5
    assert b.StepBundleAdjustment([1.8], 7.25, o2) == 1.0
    assert b.StepBundleAdjustment(np.array([4.0, 0.9], np.float32), 20.25, o3) == 1.5
    assert [s[0] for s in seen] == [[np.float32(1.8)], [np.float32(1.8)], [4.0, np.float32(0.9)]]
    assert [s[1] for s in seen] == [7.25, 7.25, 20.25]
    assert o1 == [10] and o2 == [10, 11] and o3 == [10, 11, 12]
