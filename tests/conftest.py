"""Shared fixtures. `-m gpu` tests need a gfx950 device; `-m "not gpu"` tests run anywhere."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) through the HIP library")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def built_lib():
    from oxen_amd import build

    return build.build()


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def cuda(built_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible (the -m gpu suite runs on the MI355X box)")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def ctx(cuda):
    from oxen_amd import _capi

    c = _capi.Context(0)
    yield c
    c.close()
