import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def _ensure_built():
    so = os.path.join(ROOT, "ugo_amd", "libugofec.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "ugo_amd", "csrc")])
    ora = os.path.join(ROOT, "oracle", "librs_oracle.so")
    if not os.path.exists(ora):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def gpu():
    """Fails loudly (never skips) when a GPU test runs without a GPU."""
    import torch

    assert torch.cuda.is_available(), "gpu-marked test needs a GPU (run with -m 'not gpu' on CPU hosts)"
    name = torch.cuda.get_device_properties(0).gcnArchName
    assert name.startswith("gfx950"), name
    return torch.device("cuda:0")
