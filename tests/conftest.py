import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: longer-running test")


@pytest.fixture(scope="session")
def oracle():
    import reflow_oracle
    reflow_oracle.lib()
    return reflow_oracle
