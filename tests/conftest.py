"""pytest configuration: the `gpu` marker and shared fixtures.

-m "not gpu" runs here (no GPU): oracle vs golden vectors, host logic, C-ABI exports.
-m gpu runs on the MI355X box: the HIP path against the oracle and the golden vectors.
"""

import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def golden_index():
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return json.load(f)


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))
