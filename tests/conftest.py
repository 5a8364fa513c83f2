import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def libmxp():
    """Build (if stale) and load libmxp.so."""
    from istio_amd import build
    build.build()
    from istio_amd.engine import load_library
    return load_library()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "ilt_tests.json")) as f:
        return json.load(f)
