import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)  # a GPU test must never pass on a fallback
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def reference_raft():
    """The unmodified reference RAFT class (read-only import), or skip."""
    core = os.path.join(REFERENCE, "core")
    if not os.path.isdir(core):
        pytest.skip("reference not mounted")
    if core not in sys.path:
        sys.path.insert(0, core)
    import warnings
    warnings.filterwarnings("ignore")
    from raft import RAFT as RefRAFT  # noqa
    return RefRAFT
