"""Parity of the HIP engine (through the C ABI) against the oracle -- needs an MI355X.

Each case mirrors what the reference job does with the same input (PageRank.java:21-204):
the ranks after N rounds, the defined set, the top-K page list, the crash behaviour, and
the bit-exact edge set / degrees of the graph build.
"""
import gzip
import json
import os

import numpy as np
import pytest

import graphgen as G
import parity

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


@pytest.fixture(scope="module")
def O(oracle_mod):
    return oracle_mod


def text_case(P, O, arcs, mapping, T, tol=0.0, k=100):
    """Run both sides on the same text input; return (engine ranks, oracle ranks, eng)."""
    g = O.Graph.from_text(arcs, mapping)
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    info = eng.info()
    assert info["n_vertices"] == g.n and info["nnz"] == g.nnz and info["n_tot"] == g.n_tot
    # dense ids are assigned in the same first-appearance order on both sides
    for v in range(min(g.n, 64)):
        assert eng.id_string(v) == g.id_bytes(v)
    st = eng.run(T, tol)
    res = g.run(T, tol=tol)
    return eng.ranks(), res["ranks"], eng, g, st, res


def test_appendix_b_known_answers(P, O):
    kat = json.load(open(os.path.join(GOLDEN, "kat_expected.json")))
    arcs, mapping = kat["arcs"].encode(), kat["mapping"].encode()
    for T, exp in kat["rounds"].items():
        eng = P.Engine()
        eng.ingest_buffers(arcs, mapping)
        eng.run(int(T))
        r = eng.ranks()
        got = {eng.id_string(v).decode(): float(r[v]) for v in range(len(r)) if r[v] > 0}
        assert set(got) == set(exp["ranks"]), (T, got)
        for k, v in exp["ranks"].items():
            assert abs(got[k] - float(v)) <= 1e-15 * float(v), (T, k, got[k], v)
        eng.close()


def test_appendix_b_crash_cases(P):
    # empty dangling RDD in round 1 (reduce at PageRank.java:125)
    eng = P.Engine()
    eng.ingest_buffers(b"1\t2\n2\t1\n", b"1\tA\n2\tB\n")
    with pytest.raises(P.UnsupportedOperationException):
        eng.run(10)
    # vertex 5's entry vanishes after round 1 -> crash in round 2
    eng = P.Engine()
    eng.ingest_buffers(b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n")
    st = P.Stats()
    rc = P.lib().pr_run(eng._h, 10, 0.0, st)
    assert rc == P.PR_E_EMPTY_DANGLING and st.failed_iteration == 2
    eng.run(1)  # one round is fine
    # malformed lines (AIOOBE at :40 / :49)
    for a, m in ((b"1\t2\n3\n", b"1\tA\n"), (b"1\t2\n", b"1\tA\n2\t\n"), (b"1\t\t\n", b"1\tA\n")):
        with pytest.raises(P.ArrayIndexOutOfBoundsException):
            P.Engine().ingest_buffers(a, m)


def test_zero_rounds_is_initial_ranks(P):
    eng = P.Engine()
    eng.ingest_buffers(b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n")
    eng.run(0)
    r = eng.ranks()
    assert list(r) == [1.0, 1.0, 1.0, 1.0, 0.0]


def test_fuzz_small_graphs(P, O):
    n_ok = n_crash = 0
    worst = 0.0
    for seed in range(400):
        arcs, mapping = G.random_small_text(seed)
        T = seed % 13
        g = O.Graph.from_text(arcs, mapping)
        exp_err = g.err
        exp = None
        if not exp_err:
            try:
                exp = g.run(T)["ranks"]
            except O.OracleError as e:
                exp_err = e.code
        eng = P.Engine()
        try:
            eng.ingest_buffers(arcs, mapping)
            eng.run(T)
            got = eng.ranks()
        except P.PageRankError as e:
            assert e.code == exp_err, (seed, e.code, exp_err, str(e))
            n_crash += 1
            continue
        finally:
            eng.close()
        assert not exp_err, (seed, exp_err)
        worst = max(worst, parity.assert_ranks_close(got, exp))
        n_ok += 1
    assert n_ok > 100 and n_crash > 50
    print(f"fuzz: {n_ok} runs, {n_crash} crashes, worst rel err {worst:.2e}")


def test_config1_golden(P, O, tmp_path):
    arcs = gzip.decompress(open(os.path.join(GOLDEN, "cfg1_arcs.txt.gz"), "rb").read())
    mapping = gzip.decompress(open(os.path.join(GOLDEN, "cfg1_mapping.txt.gz"), "rb").read())
    exp = json.load(open(os.path.join(GOLDEN, "cfg1_expected.json")))
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    info = eng.info()
    assert info["nnz"] == exp["nnz"] and info["n_tot"] == exp["n_tot"]
    assert info["dangling_entries"] == exp["dangling_entries"]
    assert [str(x) for x in eng.edge_digest()] == exp["edge_digest"]
    eng.run(exp["iterations"])
    r = eng.ranks()
    ids = [eng.id_string(v).decode("utf-8", "surrogateescape") for v in range(len(r))]
    got = {ids[v]: float(r[v]) for v in range(len(r)) if r[v] > 0}
    assert set(got) == set(exp["ranks"])
    worst = max(abs(got[k] - float(v)) / float(v) for k, v in exp["ranks"].items())
    assert worst <= parity.RTOL, worst
    out = tmp_path / "topPage"
    eng.write_top_page(str(out))
    rows = parity.parse_top_page(out.read_bytes())
    exp_rows = parity.parse_top_page(exp["topPage"].encode())
    assert len(rows) == 100
    parity.assert_same_order_mod_ties(rows, exp_rows)


def test_degrees_and_digest_text(P, O):
    arcs, mapping = G.wiki_text(seed=7, pages=3000, arcs_target=30000)
    g = O.Graph.from_text(arcs, mapping)
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    o, i, w = eng.degrees()
    eo, ei, ew = g.degrees()
    assert np.array_equal(o, eo) and np.array_equal(i, ei) and np.array_equal(w, ew)
    assert eng.edge_digest() == g.edge_digest()


@pytest.mark.parametrize("scale,ef,seed,T", [(12, 16, 3, 10), (16, 8, 4, 10), (20, 5, 2, 20)])
def test_rmat_device_generator_and_ranks(P, O, scale, ef, seed, T):
    g = O.Graph.from_rmat(scale, ef, seed)
    eng = P.Engine()
    eng.generate_rmat(scale, ef, seed)
    info = eng.info()
    assert info["nnz"] == g.nnz and info["n_vertices"] == g.n
    assert eng.edge_digest() == g.edge_digest()           # bit-exact edge set
    o, i, w = eng.degrees()
    eo, ei, ew = g.degrees()
    assert np.array_equal(o, eo) and np.array_equal(i, ei) and np.array_equal(w, ew)
    st = eng.run(T)
    worst = parity.assert_ranks_close(eng.ranks(), g.run(T)["ranks"])
    print(f"rmat s{scale} ef{ef}: nnz={g.nnz} worst rel {worst:.2e} {st['ms_per_iter']:.3f} ms/round")


def test_load_edges_matches_generator(P, O):
    s, d = O.rmat_edges(14, 8, 9)
    a = P.Engine()
    a.load_edges(s, d, 1 << 14)
    b = P.Engine()
    b.generate_rmat(14, 8, 9)
    assert a.edge_digest() == b.edge_digest()
    a.run(10)
    b.run(10)
    assert np.array_equal(a.ranks(), b.ranks())


def test_deterministic_bits(P):
    eng = P.Engine()
    eng.generate_rmat(16, 16, 5)
    eng.run(10)
    r1 = eng.ranks()
    eng.run(10)
    r2 = eng.ranks()
    assert np.array_equal(r1.view(np.uint64), r2.view(np.uint64))


@pytest.mark.parametrize("tiny", [False, True])
def test_lean_stream_bit_identical(P, O, monkeypatch, tiny):
    """The lean stream instruction stream (PR_LEAN=1: fma-form piece sums, DPP-masked scans,
    SDWA LDS addresses) computes the same sums in the same order as the earlier form: ranks
    bit-identical."""
    if tiny:   # every stream path: several LDS blocks, L2 waves, split segments
        for k, v in (("PR_HOTLDS", "256"), ("PR_NLDS", "6"), ("PR_QH", "1024"), ("PR_SEG", "512")):
            monkeypatch.setenv(k, v)
    out = []
    for lean in ("0", "1"):
        monkeypatch.setenv("PR_LEAN", lean)
        eng = P.Engine()
        eng.generate_rmat(16, 16, 31)
        eng.run(8)
        out.append(eng.ranks())
        eng.close()
    for o in out[1:]:
        assert np.array_equal(out[0].view(np.uint64), o.view(np.uint64))
    parity.assert_ranks_close(out[-1], O.Graph.from_rmat(16, 16, 31).run(8)["ranks"])


@pytest.mark.parametrize("p", [1, 3])
def test_row_offset_layouts_bit_identical(P, O, monkeypatch, p):
    """The 10-bit packed row offsets of the row launch (3 per dword, one 12-byte load per
    step) and the earlier 8 x u16 layout (PR_ROFF16=1) feed the same adds: ranks
    bit-identical, with heavy blocks and at several ranks."""
    monkeypatch.setenv("PR_HDEG", "40")
    out = []
    for lay in ("1", "0"):
        monkeypatch.setenv("PR_ROFF16", lay)
        if p == 1:
            eng = P.Engine()
            eng.generate_rmat(17, 16, 35)
            eng.run(6)
            out.append(eng.ranks())
            eng.close()
        else:
            grp = P.LocalGroup(p)
            grp.each("generate_rmat", 17, 16, 35)
            grp.run(6)
            out.append(grp.members[0].ranks())
            grp.close()
    assert np.array_equal(out[0].view(np.uint64), out[1].view(np.uint64))
    parity.assert_ranks_close(out[1], O.Graph.from_rmat(17, 16, 35).run(6)["ranks"])


@pytest.mark.parametrize("p,tiny", [(4, False), (8, False), (2, True), (4, True)])
def test_sparse_exchange_bit_identical(P, O, monkeypatch, p, tiny):
    """The sparse x' exchange (PR_SPARSE_X: only the entries a peer's edges reference travel,
    packed per (chunk, peer)) leaves every rank the same x values to gather: ranks bit-identical
    to the dense exchange, and the oracle's."""
    if tiny:
        for k, v in (("PR_HOTLDS", "256"), ("PR_NLDS", "6"), ("PR_QH", "1024"), ("PR_SEG", "512")):
            monkeypatch.setenv(k, v)
    out = []
    for sx in ("0", "1"):
        monkeypatch.setenv("PR_SPARSE_X", sx)
        grp = P.LocalGroup(p)
        grp.each("generate_rmat", 16, 16, 37)
        grp.run(9)
        out.append(grp.members[0].ranks())
        grp.close()
    assert np.array_equal(out[0].view(np.uint64), out[1].view(np.uint64))
    parity.assert_ranks_close(out[1], O.Graph.from_rmat(16, 16, 37).run(9)["ranks"])


@pytest.mark.parametrize("p,tiny,dyn", [(1, False, ("0", "8", "1")), (1, True, ("30", "3", "1")),
                                        (1, True, ("0", "1", "0")), (2, True, ("50", "2", "1")),
                                        (4, False, ("30", "8", "1"))])
def test_dynamic_task_claims_bit_identical(P, O, monkeypatch, p, tiny, dyn):
    """Which wave runs a task is decided at run time in the late LDS phases and (PR_DYNL2) for
    the L2 group -- slice-wide counters instead of fixed shares (PR_DYNTAIL percent of the
    phases stay fixed, PR_DYNG tasks per claim).  A task's pieces and their places do not depend
    on who runs it: ranks bit-identical to fixed shares, and the oracle's."""
    if tiny:
        for k, v in (("PR_HOTLDS", "256"), ("PR_NLDS", "6"), ("PR_QH", "1024"), ("PR_SEG", "512")):
            monkeypatch.setenv(k, v)
    scale = 16 if tiny else 20
    out = []
    for tail, g, l2 in (("100", "4", "0"), dyn):
        monkeypatch.setenv("PR_DYNTAIL", tail)
        monkeypatch.setenv("PR_DYNG", g)
        monkeypatch.setenv("PR_DYNL2", l2)
        if p == 1:
            eng = P.Engine()
            eng.generate_rmat(scale, 16, 47)
            eng.run(7)
            eng.run(7)               # a second run: the counters start from zero again
            out.append(eng.ranks())
            eng.close()
        else:
            grp = P.LocalGroup(p)
            grp.each("generate_rmat", scale, 16, 47)
            grp.run(7)
            out.append(grp.members[0].ranks())
            grp.close()
    assert np.array_equal(out[0].view(np.uint64), out[1].view(np.uint64))
    parity.assert_ranks_close(out[1], O.Graph.from_rmat(scale, 16, 47).run(7)["ranks"])


@pytest.mark.parametrize("p,scale,ef", [(8, 9, 2), (5, 11, 4), (7, 12, 8), (6, 8, 1)])
def test_sparse_exchange_small_graphs(P, O, p, scale, ef):
    """Sparse exchange corner cases: many (chunk, peer) lists empty (tiny graphs at 8 ranks),
    and rank counts that do not divide 8 (plain x layout): ranks vs the oracle."""
    exp = O.Graph.from_rmat(scale, ef, 41).run(7)["ranks"]
    grp = P.LocalGroup(p)
    grp.each("generate_rmat", scale, ef, 41)
    grp.run(7)
    got = grp.members[0].ranks()
    grp.close()
    parity.assert_ranks_close(got, exp)


def test_convergence_mode(P, O):
    g = O.Graph.from_rmat(14, 16, 3)
    eng = P.Engine()
    eng.generate_rmat(14, 16, 3)
    st = eng.run(200, 1e-8)
    res = g.run(200, tol=1e-8)
    assert abs(st["iterations"] - res["iterations"]) <= 1
    assert st["residual"] <= 1e-8
    if st["iterations"] == res["iterations"]:
        parity.assert_ranks_close(eng.ranks(), res["ranks"])


def test_in_memory_mapping_weights(P, O):
    rng = np.random.default_rng(11)
    n, m = 5000, 40000
    s = rng.integers(0, n, m).astype(np.uint32)
    d = (rng.zipf(1.5, m) % n).astype(np.uint32)
    mapw = rng.integers(0, 3, n).astype(np.uint32)   # 0 = unmapped, 2 = two titles
    g = O.Graph.from_edges(s, d, n, mapw, n_tot=int(mapw.sum()) + 7)
    eng = P.Engine()
    eng.load_edges(s, d, n, mapw, int(mapw.sum()) + 7)
    eng.run(15)
    parity.assert_ranks_close(eng.ranks(), g.run(15)["ranks"])
    top = eng.topk(50)
    r = g.run(15)["ranks"]
    exp_sorted = np.sort(np.repeat(r, mapw)[np.repeat(r, mapw) > 0])[::-1]
    for i, (_pair, v, rk) in enumerate(top):
        assert abs(rk - exp_sorted[i]) <= parity.RTOL * exp_sorted[i]
        assert abs(r[v] - rk) <= parity.RTOL * rk


def test_pagerank_main_cli_contract(P, O, tmp_path):
    arcs, mapping = G.wiki_text(seed=3, pages=2000, arcs_target=20000)
    (tmp_path / "a").write_bytes(arcs)
    (tmp_path / "m").write_bytes(mapping)
    out = tmp_path / "topPage"
    P.PageRank.main([str(tmp_path / "a"), str(tmp_path / "m"), "10"], out=str(out))
    import pagerank_literal as L
    exp = L.main_literal(arcs, mapping, 10)
    got_rows = parity.parse_top_page(out.read_bytes())
    exp_rows = parity.parse_top_page(exp)
    parity.assert_same_order_mod_ties(got_rows, exp_rows)
    # the C++ CLI writes the same file
    import subprocess
    cli = os.path.join(os.path.dirname(P.LIB_PATH), "pagerank")
    out2 = tmp_path / "topPage2"
    subprocess.run([cli, str(tmp_path / "a"), str(tmp_path / "m"), "10", "--out", str(out2)],
                   check=True, timeout=120)
    assert out2.read_bytes() == out.read_bytes()


# ---- multi-rank layout on one GPU: single-process rank group (copies replace RCCL) -------
@pytest.mark.parametrize("p", [2, 3, 4, 8])
def test_rank_group_matches_single(P, O, p):
    """p ranks (rows dealt in 16-row chunks, x exchanged every round) against one rank and
    the oracle.  Each rank's stream cuts rows into pieces at its own task boundaries, so the
    summation order (and the last bits) may differ from p = 1; the defined set may not."""
    ref = P.Engine()
    ref.generate_rmat(15, 16, 6)
    ref.run(10)
    r1 = ref.ranks()
    grp = P.LocalGroup(p)
    grp.each("generate_rmat", 15, 16, 6)
    info = [m.info() for m in grp.members]
    assert sum(i["local_nnz"] for i in info) == info[0]["nnz"]
    assert sum(i["local_rows"] for i in info) == info[0]["n_rows"]
    grp.run(10)
    rp = grp.members[p - 1].ranks()
    assert parity.assert_ranks_close(rp, r1, rtol=1e-12) <= 1e-12
    exp = O.Graph.from_rmat(15, 16, 6).run(10)["ranks"]
    parity.assert_ranks_close(rp, exp)
    grp.run(10)   # deterministic for a fixed rank count
    assert np.array_equal(rp.view(np.uint64), grp.members[0].ranks().view(np.uint64))
    top_ref = [(str(v).encode(), r) for _, v, r in ref.topk(100)]
    top_grp = [(str(v).encode(), r) for _, v, r in grp.members[0].topk(100)]
    parity.assert_same_order_mod_ties(top_grp, top_ref, rtol=1e-12)
    grp.close()


def test_rank_group_text_and_errors(P, O):
    arcs, mapping = G.wiki_text(seed=5, pages=3000, arcs_target=30000)
    g = O.Graph.from_text(arcs, mapping)
    grp = P.LocalGroup(3)
    grp.each("ingest_buffers", arcs, mapping)
    grp.run(10)
    parity.assert_ranks_close(grp.members[1].ranks(), g.run(10)["ranks"])
    st = grp.run(100, 1e-10)                       # tracked residual across ranks
    res = g.run(100, tol=1e-10)
    assert abs(st["iterations"] - res["iterations"]) <= 1
    bad = P.LocalGroup(2)
    bad.each("ingest_buffers", b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n")
    with pytest.raises(P.UnsupportedOperationException, match="iteration 2"):
        bad.run(5)


# ---- the stream layout at small scale: tiny LDS blocks / segments force every code path ----
@pytest.fixture
def tiny_blocks(monkeypatch):
    """LDS blocks of 256 x entries, a 1024-entry L2-hot range and 512-entry cold segments:
    small graphs then use LDS groups (16-bit columns), the L2 group, cold segments and
    group padding, which the default sizes only reach at scale >= 18."""
    for k, v in (("PR_HOTLDS", "256"), ("PR_NLDS", "6"), ("PR_QH", "1024"), ("PR_SEG", "512")):
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("scale,ef,seed,l2w", [(14, 16, 21, 0), (16, 8, 22, 0), (14, 16, 23, 4),
                                             (16, 8, 24, 7)])
def test_stream_layout_tiny_blocks(P, O, tiny_blocks, monkeypatch, scale, ef, seed, l2w):
    """l2w > 0: dedicated L2-group waves beside the LDS-phase waves (PR_L2W)."""
    monkeypatch.setenv("PR_L2W", str(l2w))
    g = O.Graph.from_rmat(scale, ef, seed)
    exp = g.run(10)["ranks"]
    eng = P.Engine()
    eng.generate_rmat(scale, ef, seed)
    eng.run(10)
    parity.assert_ranks_close(eng.ranks(), exp)
    for p in (2, 3):   # slice-major (p | 8) and plain x layouts
        grp = P.LocalGroup(p)
        grp.each("generate_rmat", scale, ef, seed)
        grp.run(10)
        parity.assert_ranks_close(grp.members[0].ranks(), exp)
        grp.close()


@pytest.mark.parametrize("hdeg,rbh", [(3, 64), (40, 256), (1, 1024)])
def test_heavy_row_blocks(P, O, monkeypatch, hdeg, rbh):
    """The highest in-degree rows go to smaller row-launch blocks (PR_HDEG / PR_RBH): ranks
    match the oracle for p = 1 and a 3-rank group, and the exported CSR is the same graph."""
    monkeypatch.setenv("PR_HDEG", str(hdeg))
    monkeypatch.setenv("PR_RBH", str(rbh))
    g = O.Graph.from_rmat(15, 16, 9)
    exp = g.run(10)["ranks"]
    eng = P.Engine()
    eng.generate_rmat(15, 16, 9)
    eng.run(10)
    parity.assert_ranks_close(eng.ranks(), exp)
    rp, col, od, dw = eng.export_csr()
    indeg = np.diff(rp.astype(np.int64))
    assert np.all(indeg >= 0) and int(rp[-1]) == len(col) == eng.info()["nnz"]
    assert np.array_equal(np.sort(indeg), np.sort(g.degrees()[1].astype(np.int64)))
    eng.close()
    grp = P.LocalGroup(3)
    grp.each("generate_rmat", 15, 16, 9)
    grp.run(10)
    parity.assert_ranks_close(grp.members[0].ranks(), exp)
    grp.close()


def test_export_csr_is_the_same_graph(P, O):
    """pr_export_csr rebuilds the pull CSR from the streams (internal ids): the oracle run on
    it gives the engine's rank multiset, and its degrees match the edge set."""
    eng = P.Engine()
    eng.generate_rmat(15, 16, 7)
    eng.run(10)
    got = np.sort(eng.ranks())
    rp, col, od, dw = eng.export_csr()
    n = len(od)
    assert int(rp[-1]) == eng.info()["nnz"] == len(col)
    assert np.all(np.diff(rp.astype(np.int64)) >= 0)
    indeg = np.diff(rp.astype(np.int64))
    g = O.Graph.from_rmat(15, 16, 7)
    eo, ei, ew = g.degrees()
    assert np.array_equal(np.sort(indeg), np.sort(ei.astype(np.int64)))
    assert np.array_equal(np.bincount(col, minlength=n), od.astype(np.int64))
    for r in range(0, n, max(1, n // 97)):          # sources ascending inside each row
        seg = col[rp[r]:rp[r + 1]]
        assert np.all(np.diff(seg.astype(np.int64)) > 0)
    res = O.pagerank_csr(rp, col, od, dw, int(eng.info()["n_tot"]), 10, exact=True)
    parity.assert_ranks_close(got, np.sort(res["ranks"]))


def test_rank_sum_checksum_scale22(P):
    """Size-independent property at a large graph: the exact rank sum the engine accumulates
    in tracked mode (integer superaccumulator, one rounding) equals the correctly rounded
    exact sum of the ranks it returns."""
    import math
    eng = P.Engine()
    eng.generate_rmat(22, 16, 8)
    st = eng.run(10, 1e-300)           # tol > 0: tracked mode, all 10 rounds run
    assert st["iterations"] == 10
    r = eng.ranks()
    assert st["rank_sum"] == math.fsum(r.tolist())
    d = r > 0
    assert d.sum() > 0 and np.all(r[d] >= 0.15)


def test_placement_search_changes_no_bits(P, monkeypatch):
    """The build may move the per-piece sums to another allocation when the stream launch runs
    faster there (dev_tune_placement; large graphs only unless PR_PLACE_MIN_MB says otherwise).
    Where the array lives changes no sum: ranks with the search on and off are bit-identical,
    and the graph info reports what the search timed."""
    monkeypatch.setenv("PR_PLACE_MIN_MB", "1")
    monkeypatch.setenv("PR_PLACE_BUDGET_MS", "400")
    out = []
    for on in ("1", "0"):
        monkeypatch.setenv("PR_PLACE", on)
        eng = P.Engine(device=0)
        eng.generate_rmat(20, 16, 11)
        info = eng.info()
        eng.run(6)
        out.append((eng.ranks(), info))
        eng.close()
    assert np.array_equal(out[0][0].view(np.uint64), out[1][0].view(np.uint64))
    assert out[0][1]["place_ms_first"] > 0 and out[0][1]["place_ms_best"] <= out[0][1]["place_ms_first"]
    assert out[1][1]["place_ms_first"] == 0 and out[1][1]["place_tried"] == 0
