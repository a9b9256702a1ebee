import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "cover_kat.json")) as f:
        return json.load(f)


def augment(cases, symmetric):
    """cover_test.go:31-58 runTest: swapped pairs when symmetric, plus the empty case."""
    out = [tuple(c) for c in cases]
    if symmetric:
        out += [(b, a, r) for (a, b, r) in out]
    out.append(([], [], []))
    return out
