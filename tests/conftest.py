"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)
GOLDEN = os.path.join(TESTS, "golden")
# a host fault inside libedsbwt.so prints its native frames before Python's faulthandler dump
# (engine.hip segv_trace; read when the library loads, so set before any test imports it)
os.environ.setdefault("EDSBWT_SEGV_TRACE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libedsbwt.so)")


@pytest.fixture(scope="session")
def oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # noqa: E402  (test infrastructure only)
    orc.build()
    return orc


@pytest.fixture(scope="session")
def edsbwt():
    return importlib.import_module("eds-bwt_amd")
