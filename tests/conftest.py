import os
import sys

import pytest

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


@pytest.fixture(scope="module")
def fixed_schedules():
    """Whole-model parity tests run the library's built-in conv schedules (the cost model's
    choice), not timing-based autotuning: the tuner may pick another tile, split-K order or even
    the exact-fp32 kernel for a shape from one run to the next, and gradients 50+ training-mode
    BNs deep move by several times the fp32 restatement's own error under such reorderings. Each
    schedule's arithmetic has its own per-op test (test_kernels_gpu.py::test_conv_every_schedule)."""
    from pldepth_amd import kernels as K
    saved = (K.AUTOTUNE, dict(K._TILE_CACHE))
    K.AUTOTUNE = False
    K._TILE_CACHE.clear()
    yield
    K.AUTOTUNE = saved[0]
    K._TILE_CACHE.clear()
    K._TILE_CACHE.update(saved[1])


@pytest.fixture
def bench_schedules():
    """The bench's persisted conv schedule table (kernels.DEFAULT_SCHEDULES, written by
    `bench.py --tune`) with timing-based tuning off: a test using it runs exactly the schedules
    bench.py's timed steps run (bench.py loads the same table by default). Yields the table's
    sha1; restores the previous tuning state afterwards."""
    from pldepth_amd import kernels as K
    saved = (K.AUTOTUNE, dict(K._TILE_CACHE))
    n, sha = K.use_schedule_table()
    assert n > 0, "the schedule table holds no entry for this GPU arch"
    yield sha
    K.AUTOTUNE = saved[0]
    K._TILE_CACHE.clear()
    K._TILE_CACHE.update(saved[1])
