"""The C-ABI library builds, loads without a GPU and exports every symbol include/mage_hot.h
declares; no compute calls are made here."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    text = (ROOT / "include" / "mage_hot.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mage_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_surface():
    syms = declared_symbols()
    for s in ("mage_orb_detect_and_compute", "mage_hamming_match", "mage_ba_step", "mage_ba_create"):
        assert s in syms


def test_library_exports_all_declared_symbols():
    from mageslam_amd import _lib
    from mageslam_amd import build

    build.build()
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared_symbols())


def test_version_and_error_without_gpu():
    from mageslam_amd import _lib

    lib = _lib.load()
    assert b"gfx950" in lib.mage_version()
    assert isinstance(lib.mage_last_error(), bytes)


def test_device_code_is_gfx950():
    import subprocess

    from mageslam_amd import build

    lib = build.build()
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    if "gfx" not in text:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in text


def test_cpu_only_reports_device_error():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mageslam_amd import _lib, orb

    with pytest.raises(_lib.MageError) as e:
        orb.OrbDetector()
    assert e.value.status == _lib.MAGE_EDEVICE


def test_struct_layouts():
    from mageslam_amd import _lib

    assert ctypes.sizeof(_lib.KeyPoint) == 28 == _lib.KP_DTYPE.itemsize
    assert _lib.DM_DTYPE.itemsize == 16
    assert ctypes.sizeof(_lib.OrbSettingsC) == 56
