import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
# the product packages (lit_gpt, generate) live under lit-gpt_amd/, mirroring the reference's repo root
for p in (str(REPO / "lit-gpt_amd"), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture
def golden():
    import numpy as np

    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)

    return load


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _skip_gpu_without_device(request):
    if request.node.get_closest_marker("gpu") is not None and not gpu_available():
        pytest.skip("no GPU in this container")


@pytest.fixture(autouse=True)
def restore_default_dtype():
    import torch

    yield
    torch.set_default_dtype(torch.float32)


os.environ.setdefault("OMP_NUM_THREADS", "8")
