import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)
# arms the runtime's fault-injecting test hooks (PX_DEBUG_SET_THROW, _FAIL_REC, _POISON): they
# still act only while a test sets their own variable
os.environ["PX_TEST_HOOKS"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from _oracle import Oracle
    return Oracle()


@pytest.fixture
def store_factory():
    """px.Store instances closed at teardown (GPU tests only).  torch probes the device
    first: once the HIP library has initialised the runtime, a later first call to
    torch.cuda.is_available() in the same process reports False and would skip the
    GPU tests that follow."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pixiu_amd as px
    made = []

    def make(**kw):
        st = px.Store(**kw)
        made.append(st)
        return st

    yield make
    for st in made:
        st.close()
