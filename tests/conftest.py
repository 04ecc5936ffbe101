import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-file-storage_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")
EXAMPLES = os.path.join(ROOT, "tests", "golden", "examples")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def example_bytes():
    return {n: open(os.path.join(EXAMPLES, n), "rb").read() for n in os.listdir(EXAMPLES)}


@pytest.fixture(scope="session")
def engine():
    import dfs_amd
    eng = dfs_amd.FragmentEngine(0)
    yield eng
    eng.close()
