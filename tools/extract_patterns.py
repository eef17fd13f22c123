"""Extract the pre-rotated BRIEF sampling tables from the reference as binary data.

The reference keeps two tables of signed bytes, `bit_pattern_31_rotated` and
`bit_pattern_15_rotated` (30 rotations x 256 bit-tests x 4 int8 = 30,720 B each), at
/root/reference/Core/MAGESLAM/Source/Image/OpenCVModified.cpp:74-138.  They are data
(sampling coordinates), not code; the descriptor kernels and the oracle need the exact
values to be bit-exact.  This script is run only in the build container (where
/root/reference exists) and writes the tables to mageslam_amd/data/*.bin, which are
committed and travel to the GPU box.
"""
import re
import sys
from pathlib import Path

SRC = Path("/root/reference/Core/MAGESLAM/Source/Image/OpenCVModified.cpp")
OUT = Path(__file__).resolve().parent.parent / "mageslam_amd" / "data"


def extract(text: str, name: str) -> bytes:
    m = re.search(r"signed char\s+" + name + r"\[[^\]]*\]\s*=\s*\{(.*?)\};", text, re.S)
    if not m:
        raise SystemExit(f"table {name} not found")
    vals = [int(v) for v in re.findall(r"-?\d+", m.group(1))]
    if len(vals) != 30 * 1024:
        raise SystemExit(f"{name}: expected 30720 values, got {len(vals)}")
    return bytes((v + 256) % 256 for v in vals)


def main() -> None:
    text = SRC.read_text(encoding="utf-8", errors="replace")
    OUT.mkdir(parents=True, exist_ok=True)
    for patch in (15, 31):
        data = extract(text, f"bit_pattern_{patch}_rotated")
        (OUT / f"bit_pattern_{patch}_rotated.bin").write_bytes(data)
        print(f"wrote bit_pattern_{patch}_rotated.bin ({len(data)} B)")


if __name__ == "__main__":
    sys.exit(main())
