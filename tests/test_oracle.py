"""Pin the oracle (CPU, no GPU): Appendix-B known answers, literal-vs-dense equivalence,
golden fixtures, exact summation, R-MAT generator properties.

Parity status: the reference job cannot run here and ships no outputs ("parity unpinned"
against Spark itself); these tests pin the two independent restatements to the
hand-checked Appendix-B answers and to each other, bit for bit.
"""
import gzip
import json
import math
import os
import random

import numpy as np
import pytest

import graphgen as G
import pagerank_literal as L

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT_ARCS = b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n1\t2\n2\t5\n"
KAT_MAP = b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n6\tF\n"


def test_appendix_b_by_hand():
    # T=1 by hand: a = 2/6; v1 = 0.15 + (1 + 1/3)*0.85, etc.
    a = 2.0 / 6.0
    r, _m, n = L.run_literal(KAT_ARCS, KAT_MAP, 1)
    assert n == 6
    assert r[b"1"] == 0.15 + (1.0 + a) * 0.85
    assert r[b"3"] == 0.15 + ((0.5 + 0.5 + 1.0) + a) * 0.85
    assert r[b"2"] == r[b"5"] == 0.15 + (0.5 + a) * 0.85
    assert set(r) == {b"1", b"2", b"3", b"5"}       # 4 (no in-links) and 6 vanish


@pytest.mark.parametrize("T,exp", [
    (1, {"1": "1.2833333333333332", "2": "0.8583333333333333", "3": "2.1333333333333333",
         "5": "0.8583333333333333"}),
    (2, {"1": "2.0849305555555557", "2": "0.8170138888888888", "3": "1.1818055555555553",
         "5": "0.6363888888888889"}),
    (10, {"1": "1.1158728630277965", "2": "0.7143307284984738", "3": "1.022884836250992",
          "5": "0.5361910468455172"}),
])
def test_appendix_b_table(oracle_mod, T, exp):
    r, _m, _n = L.run_literal(KAT_ARCS, KAT_MAP, T)
    assert {k.decode(): repr(v) for k, v in r.items()} == exp
    g = oracle_mod.Graph.from_text(KAT_ARCS, KAT_MAP)
    rr = g.run(T)["ranks"]
    ids = g.ids()
    assert {ids[v].decode(): repr(float(rr[v])) for v in range(g.n) if rr[v] > 0} == exp


def test_appendix_b_top_page_order():
    assert L.main_literal(KAT_ARCS, KAT_MAP, 2) == (
        b"A\t2.0849305555555557\nC\t1.1818055555555553\nB\t0.8170138888888888\n"
        b"E\t0.6363888888888889\n")


def test_appendix_b_crashes(oracle_mod):
    with pytest.raises(L.EmptyCollection):
        L.run_literal(b"1\t2\n2\t1\n", b"1\tA\n2\tB\n", 10)
    with pytest.raises(L.EmptyCollection):
        L.run_literal(b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n", 2)
    L.run_literal(b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n", 1)
    g = oracle_mod.Graph.from_text(b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n")
    with pytest.raises(oracle_mod.OracleError) as e:
        g.run(2)
    assert e.value.code == oracle_mod.ORC_E_EMPTY_DANGLING and e.value.line == 2


@pytest.mark.parametrize("line,ok", [
    (b"a\tb", True), (b"a\tb\tc", True), (b"\tb", True), (b"a\t\tb", True),
    (b"a", False), (b"a\t", False), (b"a\t\t", False), (b"\t", False), (b"", False),
])
def test_java_split_rules(oracle_mod, line, ok):
    if ok:
        L.parse_pair(line)
    else:
        with pytest.raises(L.ArrayIndexOutOfBounds):
            L.parse_pair(line)
    g = oracle_mod.Graph.from_text(line + b"\n", b"a\tT\n")
    assert (g.err == 0) == ok


def test_hadoop_lines():
    assert L.hadoop_lines(b"a\r\nb\rc\nd") == [b"a", b"b", b"c", b"d"]
    assert L.hadoop_lines(b"a\n\nb\n") == [b"a", b"", b"b"]
    assert L.hadoop_lines(b"") == []


def test_literal_vs_dense_fuzz(oracle_mod):
    ok = crash = 0
    for seed in range(1500):
        a, m = G.random_small_text(seed)
        T = seed % 13
        lerr = None
        try:
            lit = L.run_literal(a, m, T)
        except L.SparkJobError as e:
            lerr = {"ArrayIndexOutOfBounds": -2, "EmptyCollection": -3}[type(e).__name__]
        g = oracle_mod.Graph.from_text(a, m)
        cerr = g.err or None
        res = None
        if not cerr:
            try:
                res = g.run(T)
            except oracle_mod.OracleError as e:
                cerr = e.code
        assert lerr == cerr, (seed, lerr, cerr)
        if lerr:
            crash += 1
            continue
        ranks, _maps, ntot = lit
        ids = g.ids()
        dense = {ids[v]: float(res["ranks"][v]) for v in range(g.n) if res["ranks"][v] > 0}
        assert dense == ranks and ntot == g.n_tot, seed     # bit-exact
        ok += 1
    assert ok > 300 and crash > 300


def test_golden_config1(oracle_mod):
    arcs = gzip.decompress(open(os.path.join(GOLDEN, "cfg1_arcs.txt.gz"), "rb").read())
    mapping = gzip.decompress(open(os.path.join(GOLDEN, "cfg1_mapping.txt.gz"), "rb").read())
    exp = json.load(open(os.path.join(GOLDEN, "cfg1_expected.json")))
    g = oracle_mod.Graph.from_text(arcs, mapping)
    assert (g.n, g.raw_edges, g.nnz, g.n_tot) == (exp["n_vertices"], exp["raw_edges"],
                                                  exp["nnz"], exp["n_tot"])
    assert [str(x) for x in g.edge_digest()] == exp["edge_digest"]
    r = g.run(exp["iterations"])["ranks"]
    ids = g.ids()
    got = {ids[v].decode("utf-8", "surrogateescape"): repr(float(r[v])) for v in range(g.n) if r[v] > 0}
    assert got == exp["ranks"]
    assert L.main_literal(arcs, mapping, 10).decode() == exp["topPage"]


def test_golden_kat_file():
    kat = json.load(open(os.path.join(GOLDEN, "kat_expected.json")))
    for T, e in kat["rounds"].items():
        assert L.main_literal(kat["arcs"].encode(), kat["mapping"].encode(), int(T)).decode() == e["topPage"]


def test_exact_sum_is_correctly_rounded(oracle_mod):
    rng = random.Random(5)
    for _ in range(200):
        n = rng.randint(1, 400)
        v = [rng.choice([rng.uniform(0, 1), 10 ** rng.uniform(-20, 12), 1e-30, 2.0 ** 60])
             for _ in range(n)]
        w = [rng.randint(0, 5) for _ in range(n)]
        got = oracle_mod.exact_dot(np.array(v), np.array(w, np.uint32))
        exp = math.fsum(x * k for x, k in zip(v, w) for _ in [0]) if all(
            (x * k) == math.fsum([x] * k) for x, k in zip(v, w)) else None
        if exp is not None:
            assert got == exp
        assert got == math.fsum([x for x, k in zip(v, w) for _ in range(k)])


def test_rmat_generator_properties(oracle_mod):
    s, d = oracle_mod.rmat_edges(16, 4, 7)
    assert s.max() < (1 << 16) and d.max() < (1 << 16)
    # quadrant frequencies at the top level: a=.57, b=.19, c=.19, d=.05
    top_s, top_d = s >> 15, d >> 15
    f = np.bincount(top_s * 2 + top_d, minlength=4) / len(s)
    assert np.allclose(f, [0.57, 0.19, 0.19, 0.05], atol=0.01)
    s2, d2 = oracle_mod.rmat_edges(16, 4, 7, first=1000, count=10)
    assert np.array_equal(s2, s[1000:1010]) and np.array_equal(d2, d[1000:1010])


def test_java_double_to_string():
    cases = {1.0: "1.0", 0.15: "0.15", 2.1333333333333333: "2.1333333333333333",
             1e7: "1.0E7", 1.2345e7: "1.2345E7", 0.001: "0.001", 1e-4: "1.0E-4",
             123456.789: "123456.789", 9999999.999: "9999999.999", 100.0: "100.0",
             1.5e300: "1.5E300", 0.0: "0.0"}
    for v, s in cases.items():
        assert L.java_double_to_string(v) == s


def test_oracle_normalized_and_resume(oracle_mod):
    """The oracle's extra options: normalized = plain / N_tot up to
    rounding; T1 rounds then T2 from those ranks == T1 + T2 rounds, bit for bit."""
    import numpy as np
    O = oracle_mod
    g = O.Graph.from_rmat(12, 16, 5)
    plain = g.run(10)["ranks"]
    norm = g.run(10, normalized=True)["ranks"]
    assert np.allclose(norm * g.n_tot, plain, rtol=1e-12, atol=0)
    r4 = g.run(4)["ranks"]
    r10 = g.run(6, r_init=r4)["ranks"]
    assert np.array_equal(r10.view(np.uint64), plain.view(np.uint64))


def test_parallel_edge_sort_builds_the_same_csr(oracle_mod):
    """R-MAT scale 18 (4.2M raw arcs) takes the oracle's parallel MSD+LSD sort path (used for
    the scale 24-28 config tests): the CSR equals a numpy sort + unique of the same arcs."""
    O = oracle_mod
    s, d = O.rmat_edges(18, 16, 11)
    assert len(s) >= 1 << 22
    g = O.Graph.from_rmat(18, 16, 11)
    keys = np.unique((d.astype(np.uint64) << np.uint64(32)) | s.astype(np.uint64))
    rp, col = g.csr()
    assert g.nnz == len(keys)
    assert np.array_equal(col, (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    indeg = np.bincount((keys >> np.uint64(32)).astype(np.int64), minlength=g.n)
    assert np.array_equal(np.diff(rp.astype(np.int64)), indeg)
