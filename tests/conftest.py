import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi

    oracle_ffi.load()
    return oracle_ffi


@pytest.fixture(scope="session")
def gsc_lib():
    import soundchunks_amd

    return soundchunks_amd.load()
