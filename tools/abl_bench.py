"""bench.py against a variant library built by tools/abl.py (development tool, not the product):
python tools/abl_bench.py <variant> [bench.py arguments...]"""
import ctypes as C
import runpy
import sys
from pathlib import Path

import torch  # noqa: F401,E402  (the HIP runtime through torch first, as bench.py and tools/abl.py do)

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from mageslam_amd import _lib  # noqa: E402

lib = C.CDLL(str(ROOT / "abl" / sys.argv[1] / "libmage_hot.so"))
_lib._declare(lib)
_lib._lib = lib
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")
