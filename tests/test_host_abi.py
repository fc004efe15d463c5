"""C-ABI library on CPU: it loads, exports every symbol include/prmi355x.h declares, and its
host-side ingest (PageRank.java:26-60 text rules) agrees with the oracle.  No device work:
contexts are created with PR_DEVICE_NONE (host-only), and device calls must refuse loudly.
"""
import ctypes
import random
import struct
import subprocess

import numpy as np
import pytest

import graphgen as G
import pagerank_literal as L


def test_library_exports_every_declared_symbol(engine_mod):
    lib = ctypes.CDLL(engine_mod.LIB_PATH)
    names = engine_mod.declared_symbols()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", engine_mod.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(names) <= exported


def test_host_only_context_refuses_device_calls(engine_mod):
    P = engine_mod
    e = P.Engine(device=P.PR_DEVICE_NONE)
    e.ingest_buffers(b"1\t2\n", b"1\tA\n2\tB\n")
    with pytest.raises(P.PageRankError) as x:
        e.run(1)
    assert x.value.code == P.PR_E_NODEV
    with pytest.raises(P.PageRankError):
        e.degrees()


def test_host_ingest_matches_oracle(engine_mod, oracle_mod):
    P = engine_mod
    for seed in range(300):
        a, m = G.random_small_text(seed)
        g = oracle_mod.Graph.from_text(a, m)
        e = P.Engine(device=P.PR_DEVICE_NONE)
        if g.err:
            with pytest.raises(P.ArrayIndexOutOfBoundsException):
                e.ingest_buffers(a, m)
            continue
        e.ingest_buffers(a, m)
        info = e.info()
        assert (info["n_vertices"], info["raw_edges"], info["n_tot"]) == (g.n, g.raw_edges, g.n_tot)
        assert [e.id_string(v) for v in range(g.n)] == g.ids()
        pairs = g.pairs()
        assert info["n_pairs"] == len(pairs)
        assert [e.pair(i) for i in range(len(pairs))] == pairs


def test_host_ingest_config1(engine_mod, oracle_mod):
    P = engine_mod
    a, m = G.wiki_text(seed=1)
    g = oracle_mod.Graph.from_text(a, m)
    e = P.Engine(device=P.PR_DEVICE_NONE)
    e.ingest_buffers(a, m)
    info = e.info()
    assert (info["n_vertices"], info["raw_edges"], info["n_tot"], info["n_pairs"]) == \
        (g.n, g.raw_edges, g.n_tot, len(g.pairs()))


def test_parse_error_line_numbers(engine_mod):
    P = engine_mod
    e = P.Engine(device=P.PR_DEVICE_NONE)
    with pytest.raises(P.ArrayIndexOutOfBoundsException, match="arcs line 3"):
        e.ingest_buffers(b"1\t2\r\n2\t3\r\nbad\r\n", b"1\tA\n")
    with pytest.raises(P.ArrayIndexOutOfBoundsException, match="mapping line 2"):
        e.ingest_buffers(b"1\t2\n", b"1\tA\n\n2\tB\n")


def test_format_double_matches_java_layout(engine_mod):
    rng = random.Random(3)
    for _ in range(50000):
        v = rng.choice([rng.uniform(0, 10), rng.uniform(0, 1e8), 10 ** rng.uniform(-6, 15),
                        struct.unpack("d", struct.pack("Q", rng.getrandbits(62)))[0]])
        if v != v or v in (float("inf"),):
            continue
        assert engine_mod.format_double(v) == L.java_double_to_string(v), v


def test_missing_library_fails_loudly(engine_mod, monkeypatch, tmp_path):
    P = engine_mod
    monkeypatch.setattr(P, "_lib", None)
    monkeypatch.setattr(P, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="not built"):
        P.Engine()


def test_library_emits_roctx_ranges(engine_mod):
    """Build phases, ingest, runs and rounds are roctx ranges (rocprofv3 --marker-trace;
    profiles/r02/marker_stats.csv holds a traced bench run)."""
    out = subprocess.run(["nm", "-D", engine_mod.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    und = {ln.split()[-1] for ln in out.splitlines() if " U " in ln}
    assert {"roctxRangePushA", "roctxRangePop"} <= und
