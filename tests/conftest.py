import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture
def engine_factory():
    """Engines made by one test, closed when it ends: a session-long handle keeps its device arena (the full-size
    tests hold tens of GB each), so later tests would run out of HBM."""
    from accord_amd import engine

    made = []

    def make(**kw):
        e = engine.DepsEngine(**kw)
        made.append(e)
        return e

    yield make
    for e in made:
        e.close()
