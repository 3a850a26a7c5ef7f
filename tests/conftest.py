"""Test configuration: paths, the `gpu` marker and shared fixtures.

`-m "not gpu"` runs on the build container (no GPU): the oracle against the
reference's golden vectors, the host logic (sampler, driver, multi-rank
exchange over gloo) and the C-ABI library's exports.  `-m gpu` runs on an
MI355X and compares the HIP path, called through the C-ABI, with the oracle
and the golden fixtures.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpi-hungarian-method_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP path")


def load_npz_cases(name):
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    return z, meta


@pytest.fixture(scope="session")
def lsap_cases():
    return load_npz_cases("lsap_cases.npz")


@pytest.fixture(scope="session")
def santa_blocks():
    return load_npz_cases("santa_blocks.npz")


@pytest.fixture(scope="session")
def santa_triplets():
    return load_npz_cases("santa_triplets.npz")


@pytest.fixture(scope="session")
def full_data():
    """The seeded full-size synthetic instance the Santa fixtures were made on."""
    from santa_hip import data as D
    return D.synthetic(2017)


def golden_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)
