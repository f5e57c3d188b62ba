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
    """Make sure every native artefact is current (make is a no-op when it is).

    On the GPU box (GRAFT_REPO_ROOT set) the snapshot carries the libraries
    built here but not their object files, so make would rebuild them there
    (and a rebuilt library is no longer the one the committed PMC capture
    measured: bench.py's traffic_build_matches).  There the tests use the
    shipped libraries as they are, and build only what is missing."""
    import __graft_entry__ as g
    shipped = [os.path.join(ROOT, "siamese_amd", "libsiamese_amd.so"),
               os.path.join(ROOT, "tests", "hostsim", "libsiamese_hostsim.so"),
               os.path.join(ROOT, "harness", "libscenario.so")]
    if not (os.environ.get("GRAFT_REPO_ROOT") and all(os.path.exists(p) for p in shipped)):
        g.build_native()
    yield


@pytest.fixture(scope="session")
def ref_available():
    import scenario_lib as S
    return os.path.exists(S.REF_LIB)
