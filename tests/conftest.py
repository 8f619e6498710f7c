import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libbeast_hip.so")


def load_npz(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


CONFIGS = {
    "k1": dict(num_dof=7, gripper_indices=None, gripper_zero_order=False),
    "k2": dict(num_dof=14, gripper_indices=None, gripper_zero_order=False),
    "k3": dict(num_dof=14, gripper_indices=[6, 13], gripper_zero_order=True),
}


@pytest.fixture(scope="session")
def golden():
    return {k: load_npz(f"bspline_{k}.npz") for k in CONFIGS}


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    from beast_tokenizer_amd import _lib
    _lib.load()
    return torch.device("cuda", 0)


@pytest.fixture(params=["specialised", "generic"])
def kernel_mode(request):
    """Run a parity test on the shape-specialised kernels and on the runtime-shape ones."""
    from beast_tokenizer_amd import _lib
    lib = _lib.load()
    lib.beast_set_option(_lib.OPT_GENERIC_KERNELS, 1 if request.param == "generic" else 0)
    yield request.param
    lib.beast_set_option(_lib.OPT_GENERIC_KERNELS, 0)
