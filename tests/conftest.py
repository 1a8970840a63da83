import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _gpu_selected(config):
    """True when the run explicitly selects the GPU tests (``-m gpu``, not ``-m "not gpu"``)."""
    expr = (config.getoption("markexpr") or "").replace("(", " ").replace(")", " ").split()
    return any(w == "gpu" and (i == 0 or expr[i - 1] != "not") for i, w in enumerate(expr))


@pytest.fixture(scope="session")
def dev(request):
    """cuda:0.  Under ``-m gpu`` a missing device (or a broken HIP runtime) FAILS the test instead of
    skipping it, so a GPU run can never read green-with-skips; an unfiltered CPU run still skips."""
    import torch
    if not torch.cuda.is_available():
        if _gpu_selected(request.config):
            pytest.fail("-m gpu selected but no GPU is visible (torch.cuda.is_available() is False)")
        pytest.skip("no GPU")
    return torch.device("cuda:0")
