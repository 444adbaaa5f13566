import os
import sys

# before torch / the HIP runtime initialise: hipGraph replay correctness (pldepth_amd/__init__.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import pytest  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpldepth_hip.so)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "sampler_golden.npz"))


@pytest.fixture(scope="session")
def cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device (run with -m 'not gpu' on CPU)"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)
