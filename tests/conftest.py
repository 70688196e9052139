import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) — run with -m gpu")


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def sub_state(z, prefix):
    """Collect '<prefix>param.<key>' arrays of a golden npz into a torch state_dict."""
    import torch
    pre = prefix + "param."
    return {k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)}


def sub_grads(z, prefix):
    import torch
    pre = prefix + "grad."
    return {k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)}


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
