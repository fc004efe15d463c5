"""Normalized ranks and checkpoint / resume (the reference has neither:
PageRank.java:78,:143 fix r^0 = 1.0 and base 0.15, :92 always runs 10 rounds from scratch).

Resume is checked bit for bit: T1 rounds, then T2 more from the T1 ranks (pr_set_ranks or a
checkpoint file in a fresh context), equals T1 + T2 uninterrupted rounds -- the seed's
x = r/outdeg and exact dangling mass are the engine's own."""
import numpy as np
import pytest

import graphgen as G
import parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


@pytest.fixture(scope="module")
def O(oracle_mod):
    return oracle_mod


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


@pytest.mark.parametrize("T", [0, 1, 10])
def test_normalized_matches_oracle(P, O, T):
    g = O.Graph.from_rmat(14, 16, 9)
    eng = P.Engine(flags=P.PR_F_NORMALIZED)
    eng.generate_rmat(14, 16, 9)
    eng.run(T)
    exp = g.run(T, normalized=True)["ranks"]
    parity.assert_ranks_close(eng.ranks(), exp)
    plain = g.run(T)["ranks"]                    # linear: normalized = plain / N_tot
    n_tot = eng.info()["n_tot"]
    assert np.allclose(exp * n_tot, plain, rtol=1e-12, atol=0)


def test_normalized_text_and_tracked(P, O):
    a, m = G.wiki_text(seed=4, pages=3000, arcs_target=30000)
    g = O.Graph.from_text(a, m)
    eng = P.Engine(flags=P.PR_F_NORMALIZED)
    eng.ingest_buffers(a, m)
    st = eng.run(100, 1e-10)
    res = g.run(100, tol=1e-10, normalized=True)
    assert abs(st["iterations"] - res["iterations"]) <= 1
    if st["iterations"] == res["iterations"]:
        parity.assert_ranks_close(eng.ranks(), res["ranks"])
    assert 0.0 < st["rank_sum"] <= 1.0 + 1e-9


@pytest.mark.parametrize("flags", [0, "normalized"])
def test_resume_is_bit_identical(P, O, flags, tmp_path):
    f = P.PR_F_NORMALIZED if flags else 0
    full = P.Engine(flags=f)
    full.generate_rmat(15, 16, 10)
    full.run(12)
    r12 = full.ranks()
    part = P.Engine(flags=f)
    part.generate_rmat(15, 16, 10)
    part.run(5)
    r5 = part.ranks()
    part.set_ranks(r5, 5)
    part.run(7)
    assert np.array_equal(bits(part.ranks()), bits(r12))
    # through a checkpoint file, in a fresh context (tracked mode on the resumed part)
    part.run(0)                      # a seeded context that runs no round reports the seed
    assert np.array_equal(bits(part.ranks()), bits(r5))
    part.set_ranks(None)
    part.run(5)
    part.checkpoint_save(str(tmp_path / "ck"))
    fresh = P.Engine(flags=f)
    fresh.generate_rmat(15, 16, 10)
    fresh.checkpoint_load(str(tmp_path / "ck"))
    fresh.run(7, 1e-300)             # tol > 0: tracked residual path, stops at 7 anyway
    assert np.array_equal(bits(fresh.ranks()), bits(r12))
    # and against the oracle resumed from the same ranks
    g = O.Graph.from_rmat(15, 16, 10)
    exp = g.run(7, normalized=bool(f), r_init=r5)["ranks"]
    parity.assert_ranks_close(fresh.ranks(), exp)
    # a checkpoint of the resumed run counts all 12 rounds
    fresh.checkpoint_save(str(tmp_path / "ck12"))
    again = P.Engine(flags=f)
    again.generate_rmat(15, 16, 10)
    again.checkpoint_load(str(tmp_path / "ck12"))
    again.run(3)
    full.run(15)
    assert np.array_equal(bits(again.ranks()), bits(full.ranks()))


def test_resume_rank_group(P):
    grp = P.LocalGroup(3)
    grp.each("generate_rmat", 14, 16, 12)
    grp.run(9)
    r9 = grp.members[0].ranks()
    grp.run(4)
    r4 = grp.members[0].ranks()
    grp.each("set_ranks", r4, 4)
    grp.run(5)
    assert np.array_equal(bits(grp.members[0].ranks()), bits(r9))
    grp.close()


def test_resume_errors(P, tmp_path):
    eng = P.Engine()
    eng.generate_rmat(12, 8, 13)
    eng.run(3)
    r = eng.ranks()
    _o, indeg, _w = eng.degrees()
    bad = r.copy()
    bad[np.flatnonzero(indeg == 0)[0]] = 1.0       # no in-link: no rank after round 1
    with pytest.raises(P.PageRankError):
        eng.set_ranks(bad, 3)
    with pytest.raises(P.PageRankError):
        eng.set_ranks(r[:-1], 3)                    # wrong length
    with pytest.raises(P.PageRankError):
        eng.set_ranks(r, 0)                         # round 0 is r^0
    eng.checkpoint_save(str(tmp_path / "ck"))
    other = P.Engine()
    other.generate_rmat(12, 8, 14)                  # another graph
    with pytest.raises(P.PageRankError):
        other.checkpoint_load(str(tmp_path / "ck"))
    norm = P.Engine(flags=P.PR_F_NORMALIZED)
    norm.generate_rmat(12, 8, 13)
    with pytest.raises(P.PageRankError):
        norm.checkpoint_load(str(tmp_path / "ck"))  # normalization differs
    (tmp_path / "junk").write_bytes(b"not a checkpoint")
    with pytest.raises(P.PageRankError):
        eng.checkpoint_load(str(tmp_path / "junk"))


def test_resume_keeps_failure_round(P):
    """The reference dies at the round whose reduce sees an empty danglingMap; after a seed
    the failing round keeps its global number."""
    arcs, mapping = b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n"
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    with pytest.raises(P.UnsupportedOperationException, match="iteration 2"):
        eng.run(5)
    eng.run(1)
    eng.set_ranks(eng.ranks(), 1)
    with pytest.raises(P.UnsupportedOperationException, match="iteration 2"):
        eng.run(5)


def test_resume_keeps_failure_round_in_a_rank_group(P):
    """pr_run_group reports the failing round with the seed's rounds added, and a
    seeded group does not re-check round 1's dangling mass."""
    arcs, mapping = b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n"
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    eng.run(1)
    r1 = eng.ranks()
    grp = P.LocalGroup(2)
    grp.each("ingest_buffers", arcs, mapping)
    with pytest.raises(P.UnsupportedOperationException, match="iteration 2"):
        grp.run(5)
    grp.each("set_ranks", r1, 1)
    with pytest.raises(P.UnsupportedOperationException, match="iteration 2"):
        grp.run(5)
    grp.members[1].set_ranks(None)          # members seeded differently: refused
    with pytest.raises(P.PageRankError, match="seeded differently"):
        grp.run(1)
    grp.close()
