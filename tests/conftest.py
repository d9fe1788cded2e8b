import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
ORACLE = os.path.join(REPO, "oracle")
if ORACLE not in sys.path:
    sys.path.insert(0, ORACLE)

import avtubes  # noqa: E402,F401  (registers the `avt_amd` package from audio-visual-tubes_amd/)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
