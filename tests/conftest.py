import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")

# The oracle works on 81 x 81 (at most 729 x 729) matrices: threaded BLAS only thrashes
# there (a 16-thread OpenBLAS made one smooth-JP oracle point ~20x slower).
try:
    from threadpoolctl import threadpool_limits
    _BLAS_LIMIT = threadpool_limits(1)
except ImportError:                                       # pragma: no cover
    _BLAS_LIMIT = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


@pytest.fixture(scope="session")
def physics_golden():
    with open(os.path.join(GOLDEN, "physics_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def evolution_golden():
    with open(os.path.join(GOLDEN, "evolution_golden.json")) as f:
        return {e["name"]: e for e in json.load(f)}


def states_from_fixture(entry):
    return {k: np.asarray(v[0]) + 1j * np.asarray(v[1]) for k, v in entry["states"].items()}
