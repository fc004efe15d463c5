"""Device text ingest (ingest.hip) against the oracle's parser and the
host parser (PageRank.java:26-60, Appendix A.1 rules): dense ids in first-appearance
order, the raw arcs (degrees + edge-set digest), distinct (id, title) pairs in order, N_tot,
and the first malformed line with its number."""
import numpy as np
import pytest

import graphgen as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


@pytest.fixture(scope="module")
def O(oracle_mod):
    return oracle_mod


def same_graph(eng, g, all_ids=True):
    info = eng.info()
    assert (info["n_vertices"], info["raw_edges"], info["n_tot"]) == (g.n, g.raw_edges, g.n_tot)
    pairs = g.pairs()
    assert info["n_pairs"] == len(pairs)
    if all_ids:
        assert [eng.id_string(v) for v in range(g.n)] == g.ids()
        assert [eng.pair(i) for i in range(len(pairs))] == pairs
    else:
        rng = np.random.default_rng(0)
        for v in rng.integers(0, g.n, 2000):
            assert eng.id_string(int(v)) == g.id_bytes(int(v))
        for i in rng.integers(0, len(pairs), 2000):
            assert eng.pair(int(i)) == pairs[int(i)]
    o, i, w = eng.degrees()
    eo, ei, ew = g.degrees()
    assert np.array_equal(o, eo) and np.array_equal(i, ei) and np.array_equal(w, ew)
    assert eng.edge_digest() == g.edge_digest()


def test_fuzz_small_inputs(P, O):
    """CRLF / lone CR terminators, empty ids, extra columns, duplicate arcs and pairs, ids
    outside the mapping, missing final newline, malformed lines (same line number as the
    host parser and the oracle)."""
    for seed in range(300):
        a, m = G.random_small_text(seed)
        g = O.Graph.from_text(a, m)
        eng = P.Engine()
        if g.err:
            host = P.Engine(device=P.PR_DEVICE_NONE)
            with pytest.raises(P.ArrayIndexOutOfBoundsException) as xh:
                host.ingest_buffers(a, m)
            with pytest.raises(P.ArrayIndexOutOfBoundsException) as xd:
                eng.ingest_buffers(a, m)
            assert str(xd.value) == str(xh.value)
            host.close()
        else:
            eng.ingest_buffers(a, m)
            same_graph(eng, g)
        eng.close()


@pytest.mark.parametrize("arcs,mapping", [
    (b"a\tb\r\nb\ta\rc\ta", b"a\tA\r\nb\tB\rc\tC"),            # CRLF, lone CR, no final newline
    (b"a\t\tb\nb\ta\n", b"a\tA\nb\tB\n\tE\n"),                 # a\t\tb -> value "" ; key ""
    (b"a\tb\textra\tmore\nb\ta\n", b"a\tA\tx\na\tA\tx\na\tA\n"),  # extra fields; N_tot counts lines
    (b"a\tb\r\n\r\n", b"a\tA\n"),                              # empty line -> malformed (line 2)
    (b"a\tb\n", b"a\tA\nb\t\t\n"),                             # "b\t\t" -> malformed (mapping 2)
    (b"a\t\t\nb\tc\n", b"a\tA\nbad\n"),                        # arcs error wins over mapping
    (b"", b"a\tA\n"),                                          # no arcs at all
    (b"a\tb\n" * 5, b""),                                      # no mapping at all
    (b"a\tb\r", b"a\tA\r\r\n"),                                # "\r" then "\r\n": empty line 2
])
def test_edge_cases_match_host(P, O, arcs, mapping):
    host = P.Engine(device=P.PR_DEVICE_NONE)
    eng = P.Engine()
    try:
        host.ingest_buffers(arcs, mapping)
    except P.ArrayIndexOutOfBoundsException as xh:
        with pytest.raises(P.ArrayIndexOutOfBoundsException) as xd:
            eng.ingest_buffers(arcs, mapping)
        assert str(xd.value) == str(xh)
        return
    eng.ingest_buffers(arcs, mapping)
    hi, di = host.info(), eng.info()
    for k in ("n_vertices", "raw_edges", "n_tot", "n_pairs"):
        assert hi[k] == di[k], k
    assert [eng.id_string(v) for v in range(int(di["n_vertices"]))] == \
        [host.id_string(v) for v in range(int(hi["n_vertices"]))]
    assert [eng.pair(i) for i in range(int(di["n_pairs"]))] == \
        [host.pair(i) for i in range(int(hi["n_pairs"]))]
    g = O.Graph.from_text(arcs, mapping)
    if not g.err:
        same_graph(eng, g)


def test_large_input(P, O):
    """2M arc lines, 200k pages (ids hashed on the device; hub destinations hammer one slot)."""
    a, m = G.big_text(seed=1, pages=200_000, arcs=2_000_000)
    g = O.Graph.from_text(a, m)
    eng = P.Engine()
    eng.ingest_buffers(a, m)
    same_graph(eng, g, all_ids=False)


def test_wiki_config1_ranks(P, O):
    """The config-1 stand-in through the device ingest and 10 rounds (ranks vs the oracle)."""
    import parity
    a, m = G.wiki_text(seed=1)
    g = O.Graph.from_text(a, m)
    eng = P.Engine()
    eng.ingest_buffers(a, m)
    same_graph(eng, g, all_ids=False)
    eng.run(10)
    parity.assert_ranks_close(eng.ranks(), g.run(10)["ranks"])


def test_oversized_text_falls_back_to_host_parser(engine_mod, oracle_mod, monkeypatch):
    """a text input too large for the device ingest (2^30 id tokens; lowered here
    with PR_INGEST_MAX_TOKENS) is parsed on the host instead of failing; the graph and the
    ranks are the same as through the device path."""
    P, O = engine_mod, oracle_mod
    arcs, mapping = G.wiki_text(seed=9, pages=2000, arcs_target=15000)
    ref = P.Engine()
    ref.ingest_buffers(arcs, mapping)
    assert ref.info()["ingest_flags"] == 0
    monkeypatch.setenv("PR_INGEST_MAX_TOKENS", "1000")
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    info = eng.info()
    assert info["ingest_flags"] == 1
    g = O.Graph.from_text(arcs, mapping)
    assert (info["n_vertices"], info["nnz"], info["n_tot"]) == (g.n, g.nnz, g.n_tot)
    assert eng.edge_digest() == ref.edge_digest() == g.edge_digest()
    ref.run(10)
    eng.run(10)
    assert np.array_equal(eng.ranks(), ref.ranks())
    with pytest.raises(P.ArrayIndexOutOfBoundsException):   # the host path keeps the AIOOBE
        P.Engine().ingest_buffers(arcs + b"bad line\n", mapping)
