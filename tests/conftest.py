import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the gpurun box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _reset_state():
    """Borg singletons leak across tests otherwise (reference test_utils/testing.py:650-660)."""
    yield
    from accelerate_hpc_test_amd.state import AcceleratorState, GradientState, PartialState

    AcceleratorState._reset_state(True)
    GradientState._reset_state()
