"""Full rank dump: every page of the final ranks RDD, by id, one
`id \\t title \\t Double.toString(rank)` line per mapping pair -- the rows of
ranks.join(mappings) (PageRank.java:168) before sortByKey/take (:187-189) -- against the
oracle on config 1 (through the C ABI and through the CLI's --dump)."""
import gzip
import os
import subprocess

import numpy as np
import pytest

import graphgen as G
import parity

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def expected_dump(g, ranks):
    by_id = {}
    for v, t in g.pairs():
        by_id.setdefault(v, []).append(t)
    rows = []
    for v in range(g.n):
        if ranks[v] > 0:
            for t in by_id.get(v, [b""]):
                rows.append((g.id_bytes(v), t, float(ranks[v])))
    return rows


def parse_dump(data: bytes):
    rows = []
    for line in data.split(b"\n")[:-1]:
        i, t, r = line.split(b"\t")
        rows.append((i, t, r))
    return rows


def check(rows, exp, P):
    assert len(rows) == len(exp)
    for (i, t, r), (ei, et, er) in zip(rows, exp):
        assert (i, t) == (ei, et)
        assert abs(float(r) - er) <= parity.RTOL * er
        assert r == P.format_double(float(r)).encode()     # Java Double.toString layout


def test_rank_dump_config1(engine_mod, oracle_mod, tmp_path):
    P, O = engine_mod, oracle_mod
    arcs = gzip.decompress(open(os.path.join(GOLDEN, "cfg1_arcs.txt.gz"), "rb").read())
    mapping = gzip.decompress(open(os.path.join(GOLDEN, "cfg1_mapping.txt.gz"), "rb").read())
    g = O.Graph.from_text(arcs, mapping)
    exp = expected_dump(g, g.run(10)["ranks"])
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    eng.run(10)
    out = tmp_path / "dump"
    eng.write_rank_dump(str(out))
    check(parse_dump(out.read_bytes()), exp, P)
    # the CLI writes the same dump beside ./topPage
    (tmp_path / "a").write_bytes(arcs)
    (tmp_path / "m").write_bytes(mapping)
    cli = os.path.join(os.path.dirname(P.LIB_PATH), "pagerank")
    subprocess.run([cli, str(tmp_path / "a"), str(tmp_path / "m"), "10", "--out",
                    str(tmp_path / "top"), "--dump", str(tmp_path / "dump2")], check=True, timeout=120)
    assert (tmp_path / "dump2").read_bytes() == out.read_bytes()


def test_rank_dump_multi_title_and_unmapped(engine_mod, oracle_mod, tmp_path):
    """In-memory graph with pages mapped 0, 1 or 2 times: two lines for a two-title page, one
    line with an empty title for a ranked page outside the mapping."""
    P, O = engine_mod, oracle_mod
    rng = np.random.default_rng(5)
    n, m = 3000, 20000
    s = rng.integers(0, n // 2, m).astype(np.uint32)          # pages >= n/2 are dangling
    d = np.where(rng.random(m) < 0.5, rng.zipf(1.6, m) % n, rng.integers(0, n, m)).astype(np.uint32)
    mapw = rng.integers(0, 3, n).astype(np.uint32)
    g = O.Graph.from_edges(s, d, n, mapw, n_tot=int(mapw.sum()))
    r = g.run(8)["ranks"]
    eng = P.Engine()
    eng.load_edges(s, d, n, mapw, int(mapw.sum()))
    eng.run(8)
    eng.write_rank_dump(str(tmp_path / "d"))
    rows = parse_dump((tmp_path / "d").read_bytes())
    exp = []
    for v in range(n):
        if r[v] > 0:
            titles = [b"v%d" % v + (b"#%d" % j if j else b"") for j in range(mapw[v])] or [b""]
            exp += [(b"%d" % v, t, float(r[v])) for t in titles]
    check(rows, exp, P)
    assert any(t == b"" for _i, t, _r in rows) and any(b"#1" in t for _i, t, _r in rows)
