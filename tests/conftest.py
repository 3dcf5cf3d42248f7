import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def engine():
    """One device context for the whole GPU session (one process on the card)."""
    from parfastaai_amd import _capi
    e = _capi.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def diag_engine():
    """A context of the diagnostics build (libpfaai_hip_diag.so): the only
    library that reads the A/B switches (PFAAI_ROWS_KERNEL, PFAAI_PL_WINDOWS,
    ...), so the tests that force a kernel variant use it."""
    from parfastaai_amd import _capi
    e = _capi.Engine(0, lib_path=_capi.DIAG_LIB_PATH)
    yield e
    e.close()
