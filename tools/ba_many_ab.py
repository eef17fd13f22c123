"""A/B of the many-windows BA rate (bench.py run_ba_many's fixed schedule) between library builds,
in one process per build on the same GPU (development tool).

  python tools/ba_many_ab.py LIB [LIB ...]     # e.g. mageslam_amd/_lib/libmage_hot.so abl/old/libmage_hot.so

Each library is loaded in a child process that routes the Python BundlerLib mirror to it; only the
BundlerLib entry points are declared, so builds from other rounds (other exports) load as well.
"""
import ctypes as C
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(lib_path: str, threads: int, seconds: float, single: bool):
    import torch  # noqa: F401

    sys.path.insert(0, str(ROOT))
    from concurrent.futures import ThreadPoolExecutor

    from mageslam_amd import _lib, bundler, synth

    lib = C.CDLL(lib_path)

    class Tolerant:  # _declare over the symbols this build has
        def __init__(self, l):
            self.l = l

        def __getattr__(self, name):
            try:
                return getattr(self.l, name)
            except AttributeError:
                return type("Missing", (), {})()

    _lib._declare(Tolerant(lib))
    _lib._lib = lib
    g = synth.ba_graph()

    def round_(b, steps):
        b.set_graph(g)
        b.step([1.8], 7.25)
        t0 = time.perf_counter()
        for _ in range(steps):
            b.step([1.8], 7.25)
        return time.perf_counter() - t0

    n = 1 if single else threads
    libs = [bundler.BundlerLib(device=0) for _ in range(n)]
    for b in libs:
        round_(b, 1)

    def work(w):
        el, k = 0.0, 0
        while el < seconds:
            el += round_(libs[w], 10)
            k += 10
        return k / el

    with ThreadPoolExecutor(n) as ex:
        rates = list(ex.map(work, range(n)))
    print(json.dumps({"lib": lib_path, "windows": n, "iters_per_s": sum(rates)}), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), float(sys.argv[4]), sys.argv[5] == "1")
        return
    for lib in sys.argv[1:]:
        for single in ("1", "0"):
            r = subprocess.run([sys.executable, __file__, "--child", str(Path(lib).resolve()), "16", "3", single],
                               capture_output=True, text=True, timeout=300)
            print(r.stdout.strip() or r.stderr[-800:], flush=True)


if __name__ == "__main__":
    main()
