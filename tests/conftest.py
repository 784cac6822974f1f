import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(autouse=True)
def _fresh_graph():
    """Every test starts with an empty variable store / train-op registry."""
    from mdtf.train import variables as V
    from mdtf.train import step as S
    from mdtf.cluster import server
    V.reset_default_graph()
    S.reset()
    server._set_current(None)
    yield
    V.reset_default_graph()
    S.reset()
    server._set_current(None)
