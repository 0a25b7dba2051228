import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def load_fixture(name):
    p = os.path.join(GOLDEN, name)
    if p.endswith(".gz"):
        with gzip.open(p, "rb") as f:
            return json.loads(f.read())
    with open(p) as f:
        return json.load(f)


def fixture_names():
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".json") or f.endswith(".json.gz"))


@pytest.fixture(scope="session")
def golden_fixtures():
    return {n: load_fixture(n) for n in fixture_names()}
