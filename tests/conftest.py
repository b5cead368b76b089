import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cosmos-sdk-rootchain_amd")
WORKLOAD = os.path.join(REPO, "tools", "workload")      # txkit: test / bench signing tooling, not the product
for p in (REPO, PKG, WORKLOAD):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
