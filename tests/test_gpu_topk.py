"""Device top-K (PageRank.java:167-189: ranks.join(mappings) -> sortByKey(false) -> take(k)).

The engine selects the top-K candidates on the device (weighted radix select over the rank
bits, dev_topk_candidates) and orders only those on the host.  The expected lists here are
built from the engine's own final ranks (pr_get_ranks) by a full sort over every mapping
pair, so the comparison is exact: same pairs, same order, same rank bits.  Rank parity
against the oracle is covered by test_gpu_parity.py.
"""
import numpy as np
import pytest

import graphgen as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


def expected_pairs(ranks, pairs):
    """pairs: list of (pair index, page, title bytes).  Order of pr_topk: rank descending,
    then title bytes, then page (Spark leaves ties unordered)."""
    rows = [(-ranks[v], t, v, i) for i, v, t in pairs if ranks[v] > 0]
    rows.sort()
    return [(i, v, -nr) for nr, _t, v, i in rows]


def rmat_pairs(n):
    return [(v, v, b"v%d" % v) for v in range(n)]


def mapw_pairs(mapw):
    out, i = [], 0
    for v, w in enumerate(mapw):
        for j in range(int(w)):
            out.append((i, v, b"v%d" % v + (b"#%d" % j if j else b"")))
            i += 1
    return out


def check(top, exp, k):
    assert len(top) == min(k, len(exp))
    for (gp, gv, gr), (ep, ev, er) in zip(top, exp):
        assert (gp, gv) == (ep, ev)
        assert np.float64(gr).view(np.uint64) == np.float64(er).view(np.uint64)


def test_topk_rmat_every_k(P):
    """Scale 17: k from 1 to past the number of defined pages, across the CAP boundary of the
    selection (the boundary digit holds more than 65536 pages for large k)."""
    eng = P.Engine()
    eng.generate_rmat(17, 16, 7)
    eng.run(10)
    r = eng.ranks()
    exp = expected_pairs(r, rmat_pairs(len(r)))
    for k in (1, 2, 100, 1000, 65536, 70000, len(exp) - 1, len(exp), len(exp) + 5):
        check(eng.topk(k), exp, k)
    eng.close()


def test_topk_ties_and_weights(P):
    """Exactly tied ranks (a hub's spokes all rank alike) with k cutting through the tie
    group, pages mapped 0, 1 or 3 times (unmapped pages never appear, a page mapped w times
    fills w rows)."""
    n = 4000
    hub_out = np.arange(1, 3001, dtype=np.uint32)               # 0 -> 1..3000
    back = hub_out[:2000]                                       # 1..2000 link back to 0,
    src = np.concatenate([np.zeros(3000, np.uint32), back,      # 2001..3000 are dangling
                          np.arange(3001, 4000, dtype=np.uint32)])
    dst = np.concatenate([hub_out, np.zeros(2000, np.uint32),
                          (np.arange(3001, 4000, dtype=np.uint32) % 50) + 1])
    rng = np.random.default_rng(3)
    mapw = rng.choice(np.array([0, 1, 1, 1, 3], np.uint32), n)
    mapw[0] = 1
    eng = P.Engine()
    eng.load_edges(src, dst, n, mapw, int(mapw.sum()))
    eng.run(10)
    r = eng.ranks()
    assert len(np.unique(r[51:3001])) == 1                       # one big tie group
    exp = expected_pairs(r, mapw_pairs(mapw))
    for k in (1, 3, 50, 51, 52, 100, 1234, len(exp), len(exp) + 1):
        check(eng.topk(k), exp, k)
    eng.close()


def test_topk_text_graph(P):
    """Text ingest: ids with several titles, arc-only ids outside the mapping."""
    arcs, mapping = G.wiki_text(seed=9, pages=3000, arcs_target=30000)
    ids = [ln.split(b"\t")[0] for ln in mapping.splitlines()[:40]]
    mapping += b"".join(b"%s\tAlt title %d\n" % (x, j) for j, x in enumerate(ids))
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    eng.run(10)
    r = eng.ranks()
    npairs = int(eng.info()["n_pairs"])
    pairs = [(i,) + eng.pair(i) for i in range(npairs)]
    assert len({v for _i, v, _t in pairs}) < npairs            # some ids carry 2 titles
    exp = expected_pairs(r, pairs)
    for k in (1, 100, 999, len(exp) + 3):
        check(eng.topk(k), exp, k)
    eng.close()


@pytest.mark.parametrize("p", [2, 3])
def test_topk_rank_group(P, p):
    """p ranks: each selects over its own pages, the union is ordered on the host."""
    grp = P.LocalGroup(p)
    grp.each("generate_rmat", 15, 16, 8)
    grp.run(10)
    r = grp.members[0].ranks()
    exp = expected_pairs(r, rmat_pairs(len(r)))
    for k in (1, 100, 5000, len(exp) + 1):
        check(grp.members[0].topk(k), exp, k)
    grp.close()


def test_topk_zero_rounds(P):
    """T = 0: every source ranks 1.0 (PageRank.java:76-83), one tie group ordered by title."""
    eng = P.Engine()
    eng.generate_rmat(12, 8, 4)
    eng.run(0)
    r = eng.ranks()
    exp = expected_pairs(r, rmat_pairs(len(r)))
    for k in (10, len(exp)):
        check(eng.topk(k), exp, k)
    eng.close()
