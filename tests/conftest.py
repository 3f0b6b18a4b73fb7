"""Shared pytest configuration: the `gpu` marker and repo-root imports."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
TESTS = os.path.join(REPO, "tests")
if REPO not in sys.path:
    sys.path.insert(0, REPO)
if TESTS not in sys.path:
    sys.path.append(TESTS)  # test helper modules (superpoint_weights, scenes)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP kernels")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
