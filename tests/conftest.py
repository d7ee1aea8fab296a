"""pytest configuration: `gpu` marks tests that need an MI355X (run with -m gpu).

CPU tests (-m "not gpu") cover the oracle against the golden fixtures, the
host logic, and that the C-ABI libraries load and export every declared
symbol -- no device compute."""
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "large: multi-GiB GPU case")


@pytest.fixture(scope="session")
def gpu():
    """torch on cuda:0; the in-tree libthrs.so must load (no fallback)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    import tinyhipradixsort_amd as T
    T.lib()  # raises ImportError if libthrs.so is missing: never silently skipped
    torch.cuda.set_device(0)
    return torch
