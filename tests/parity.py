"""Comparison helpers shared by the parity tests.

Bars (north_star / SURVEY.md 8c):
  * defined set (pages present in the final ``ranks`` RDD) identical;
  * per page |rank_gpu - rank_oracle| <= RTOL * rank_oracle, RTOL = 1e-9;
  * top-K ordering identical modulo ties: the K rank values agree position by position
    within RTOL, and every listed page's oracle rank matches its listed rank.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

RTOL = 1e-9


def assert_ranks_close(got: np.ndarray, exp: np.ndarray, rtol: float = RTOL) -> float:
    got = np.asarray(got, np.float64)
    exp = np.asarray(exp, np.float64)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    dg, de = got > 0, exp > 0
    bad = np.nonzero(dg != de)[0]
    assert bad.size == 0, f"defined set differs at {bad[:10]} (gpu {got[bad[:10]]}, oracle {exp[bad[:10]]})"
    if not de.any():
        return 0.0
    rel = np.abs(got[de] - exp[de]) / exp[de]
    worst = float(rel.max())
    assert worst <= rtol, f"max relative error {worst:.3e} > {rtol:.0e}"
    return worst


def parse_top_page(text: bytes) -> List[Tuple[bytes, float]]:
    rows = []
    for line in text.split(b"\n"):
        if not line:
            continue
        t, r = line.rsplit(b"\t", 1)
        rows.append((t, float(r)))
    return rows


def assert_top_rows_match(got: Sequence[Tuple[bytes, float]], exp_all: Dict[bytes, float],
                          exp_sorted: Sequence[float], k: int, rtol: float = RTOL):
    """got: (title, rank) rows from the engine.  exp_all: title -> oracle rank (max over the
    page ids carrying that title).  exp_sorted: oracle ranks of all rows, descending."""
    kk = min(k, len(exp_sorted))
    assert len(got) == kk, (len(got), kk)
    titles = [t for t, _ in got]
    assert len(set(titles)) == len(titles) or len(set(exp_all)) < len(exp_sorted)
    for i, (t, r) in enumerate(got):
        assert abs(r - exp_sorted[i]) <= rtol * exp_sorted[i], (i, r, exp_sorted[i])
        assert t in exp_all, t
        assert abs(exp_all[t] - r) <= rtol * r, (t, exp_all[t], r)


def assert_same_order_mod_ties(got: Sequence[Tuple[bytes, float]],
                               exp: Sequence[Tuple[bytes, float]], rtol: float = RTOL,
                               tie_rtol: float = 1e-12):
    """Row-by-row rank agreement, and identical title sets inside every run of equal
    oracle ranks (the last run may be cut by take(k), so it is only rank-checked)."""
    assert len(got) == len(exp), (len(got), len(exp))
    for (_t, r), (_et, er) in zip(got, exp):
        assert abs(r - er) <= rtol * er, (r, er)
    i = 0
    while i < len(exp):
        j = i + 1
        while j < len(exp) and abs(exp[j][1] - exp[i][1]) <= tie_rtol * exp[i][1]:
            j += 1
        if j < len(exp):
            assert sorted(t for t, _ in got[i:j]) == sorted(t for t, _ in exp[i:j]), (i, j)
        i = j
