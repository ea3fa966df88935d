import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950); run with -m gpu on the GPU box")
    config.addinivalue_line("markers", "slow: multi-second test")


def _h(s):
    return np.frombuffer(bytes.fromhex(s), np.uint8) if s is not None else None


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ref_tables():
    with open(os.path.join(GOLDEN, "gf256_tables.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    from oracle.oracle import Oracle, build

    build()
    return Oracle()


hexarr = _h
