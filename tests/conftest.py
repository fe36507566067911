import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture(autouse=True)
def _reset_sghmc_path(request):
    """GPU tests share one hmcx context per device: a test that picks an SGHMC path (1 kernels, 2 the
    2-D persistent kernel, 3 row space) must not leave it for the next test."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    nat = sys.modules.get("dropout_hamiltonian_montecarlo_amd._native")
    if nat is None:
        return
    for ctx in list(getattr(nat, "_ctxs", {}).values()):
        ctx.set_sghmc_path(0)
