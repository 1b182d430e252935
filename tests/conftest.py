import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
# every render backward in the tests is followed by a read of the device fault
# word (hn_device_faults): a failed internal wait fails the test that caused it
os.environ.setdefault("HN_CHECK_FAULTS", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def pcg_table(seed, log2T, n_levels=16):
    """Regenerate a fixture's hash table from its seed (make_golden.make_embedder)."""
    g = np.random.Generator(np.random.PCG64(int(seed)))
    return (g.random((n_levels, 2 ** int(log2T), 2), dtype=np.float32) * 2 - 1) * 0.5


@pytest.fixture(scope="session")
def oracle():
    from oracle import hashnerf_oracle
    return hashnerf_oracle


@pytest.fixture(scope="session")
def hn():
    import hn_loader
    return hn_loader.load()
