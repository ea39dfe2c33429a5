import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "pixeltable-yolox_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG_ROOT, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: slow CPU test")


def pytest_collection_modifyitems(config, items):
    # GPU tests are selected explicitly with `-m gpu`; without a GPU they would only
    # fail on the missing device, so skip them when none is visible.
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name: str):
        if name not in cache:
            with np.load(os.path.join(GOLDEN, name)) as z:
                cache[name] = {k: np.array(z[k]) for k in z.files}
        return cache[name]

    return load


@pytest.fixture(scope="session")
def oracle():
    """The CPU oracle (test infrastructure); builds its C part on first use."""
    lib = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    from oracle import reference_cpu
    return reference_cpu
