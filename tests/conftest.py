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

# The build's placement search (large graphs only) is a matter of speed, not of results: the
# tests give it a short budget so the scale-26 / scale-28 cases do not pay seconds per build
# (test_placement_search_changes_no_bits sets its own).
os.environ.setdefault("PR_PLACE_BUDGET_MS", "300")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O
    O.build()
    return O


def _gpu_host() -> bool:
    return os.path.exists("/dev/kfd")


@pytest.fixture(scope="session")
def engine_mod():
    """The engine library, checked against the checked-out sources: the id baked into it
    (pr_build_id) must equal the hash of csrc/ + include/ + Makefile.  On a CPU-only host a
    stale or missing library is rebuilt before anything loads it (make is incremental); on a
    GPU box the library travels prebuilt, so a mismatch fails the session instead of testing
    some other binary as HEAD."""
    import prmi355x as P
    import source_hash as S
    want = S.source_hash()
    if S.library_build_id(P.LIB_PATH) != want:
        if _gpu_host() or P._lib is not None:
            pytest.fail(f"stale or missing {P.LIB_PATH}: built from "
                        f"{S.library_build_id(P.LIB_PATH)}, sources are {want}")
        P.build()
    assert S.library_build_id(P.LIB_PATH) == want
    assert P.build_id() == want
    return P
