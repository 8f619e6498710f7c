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


KERNEL_MODES = {"specialised": (0, 0), "specialised_w4": (0, 4), "specialised_w7": (0, 7),
                "specialised_w8": (0, 8), "generic": (1, 0)}


def set_kernel_mode(mode):
    """(runtime-shape kernels?, forced workgroup width) for the encode / reconstruct launches."""
    from beast_tokenizer_amd import _lib
    lib = _lib.load()
    generic, waves = KERNEL_MODES[mode]
    lib.beast_set_option(_lib.OPT_GENERIC_KERNELS, generic)
    lib.beast_set_option(_lib.OPT_BLOCK_WAVES, waves)


@pytest.fixture(params=["specialised", "specialised_w4", "specialised_w7", "specialised_w8", "generic"])
def kernel_mode(request):
    """Run a parity test on the shape-specialised kernels (the width the batch size picks,
    the 4-wave width large batches use, the 7-wave one-pass encode and the 8-wave per-trajectory
    encode forced at any batch) and on the runtime-shape ones."""
    set_kernel_mode(request.param)
    yield request.param
    set_kernel_mode("specialised")
