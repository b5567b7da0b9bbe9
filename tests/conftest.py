import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # Under pytest-xdist every worker would start os.cpu_count() intra-op threads; the
    # oversubscribed OpenMP pools made the oracle tests ~90x slower (12 s serial, 1092 s
    # with -n 4). Split the cores between the workers instead.
    workers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "0") or 0)
    if workers > 1:
        import torch
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // workers))


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
