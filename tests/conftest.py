import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def gpu():
    """Skip cleanly only when there is no GPU at all; on a GPU box a missing or broken HIP
    library is a failure, not a skip (no silent fallback)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mageslam_amd import _lib

    lib = _lib.load()
    return lib
