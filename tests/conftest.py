import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Under pytest-xdist (-n N) every worker and every process a test spawns would otherwise size its thread pool to
# the whole machine: N workers x (2-4 ranks) x cpu_count threads.  Give each worker its share of the CPUs (the
# env is inherited by spawned ranks and launched cluster tasks), so the multi-process tests keep their timing.
if os.environ.get("PYTEST_XDIST_WORKER"):
    _share = max(1, (os.cpu_count() or 1) // max(1, int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1"))))
    os.environ["OMP_NUM_THREADS"] = str(_share)
    import torch
    torch.set_num_threads(_share)


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
