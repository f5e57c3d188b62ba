import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: full-size workloads")


@pytest.fixture(scope="session", autouse=True)
def native_build():
    """Make sure every native artefact is current (make is a no-op when it is)."""
    import __graft_entry__ as g
    g.build_native()
    yield


@pytest.fixture(scope="session")
def ref_available():
    import scenario_lib as S
    return os.path.exists(S.REF_LIB)
