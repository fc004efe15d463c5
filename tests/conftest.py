"""Shared fixtures.  ``-m gpu`` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def engine_mod():
    import prmi355x as P
    if not os.path.exists(P.LIB_PATH):
        P.build()
    return P
