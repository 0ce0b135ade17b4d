import gzip
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers",
                            "gpu: needs an MI355X (runs through libgpeval.so)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


def load_golden(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as fh:
        return json.load(fh)


def decode_fitness(v):
    if v is None or isinstance(v, int):
        return v
    return float.fromhex(v)


@pytest.fixture(scope="session")
def golden():
    return load_golden
