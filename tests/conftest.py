import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lgm_amd import build as B
    B.build()
    return torch.device("cuda:0")


def pytest_sessionfinish(session, exitstatus):
    """Write the gradient-precision records of this session's GPU parity tests (tests/render_cases.PRECISION)."""
    try:
        from tests.render_cases import PRECISION
    except Exception:
        return
    if PRECISION:
        import json
        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "grad_precision.json"), "w") as f:
            json.dump(PRECISION, f, indent=1)
