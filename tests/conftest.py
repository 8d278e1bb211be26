"""pytest configuration: `gpu` marker, import paths, shared fixtures."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dependable-data-storage-csd2017_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")


def _load_keys():
    raw = json.load(open(os.path.join(GOLDEN, "keys.json")))
    out = {}
    for name, v in raw.items():
        if isinstance(v, dict):
            out[name] = {k: (int(x, 16) if k != "x509_hex" else x) for k, x in v.items()}
        else:
            out[name] = v
    return out


@pytest.fixture(scope="session")
def keys():
    return _load_keys()


@pytest.fixture(scope="session")
def vectors():
    return json.load(open(os.path.join(GOLDEN, "vectors.json")))


@pytest.fixture(scope="session")
def eng():
    import ddshe
    e = ddshe.Engine(0)
    yield e
    e.close()
