import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FIXTURES = os.path.join(ROOT, "tests", "golden", "reference_fixtures")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


def fixture(name: str) -> str:
    p = os.path.join(FIXTURES, name)
    if os.path.exists(p):
        return p
    if os.path.exists(p + ".gz"):
        return p + ".gz"
    raise FileNotFoundError(p)


@pytest.fixture(scope="session")
def gpu_ctx():
    from guacamole_amd import native
    ctx = native.Context(0)
    yield ctx
    ctx.close()
