import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cmodel():
    from zbot_amd import compile_model

    return compile_model()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O

    O.build()
    return O
