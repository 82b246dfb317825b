import os
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import plo_amd  # noqa: E402

plo_amd.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    lib = ROOT / "oracle" / "liboracle_imls.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
