import os
import sys

import pytest

# Load torch (and the HIP runtime it ships) before the engine library: a
# process must resolve one HIP runtime, and the GPU tests that use torch
# tensors (multi-server) need torch's to be the one.
import torch  # noqa: E402

if torch.cuda.is_available():  # initialise torch's HIP context first, too
    torch.cuda.init()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ORACLE = os.path.join(ROOT, "oracle")
if ORACLE not in sys.path:
    sys.path.insert(0, ORACLE)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def oracle_lib():
    import pyoracle
    return pyoracle.lib()
