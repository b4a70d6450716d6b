import os
import sys

import pytest

# the GPU tests move frontier units through torch tensors: torch's HIP runtime must be the
# process's (quorum_intersection_amd._capi.lib)
os.environ.setdefault("QI_TORCH_RUNTIME", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    # GPU tests fail loudly on a box without a device; skip them only where no HIP
    # device exists AND the run did not select them explicitly with -m gpu.
    markexpr = config.getoption("-m") or ""
    if "gpu" in markexpr and "not gpu" not in markexpr:
        return
    try:
        import torch  # noqa: F401  (device_count does not initialise HIP on this image)
        have = torch.cuda.device_count() > 0
    except Exception:
        have = False
    if not have:
        skip = pytest.mark.skip(reason="no HIP device")
        for it in items:
            if "gpu" in it.keywords:
                it.add_marker(skip)
