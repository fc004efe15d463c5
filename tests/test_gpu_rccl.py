"""The real multi-process RCCL path: 2 processes on 2 GPUs run the text job with
rows dealt over the ranks and the chunked ncclSend/ncclRecv exchange of x' per round, then
the collective outputs.  Compared with a single-rank run of the same files: ranks within
1e-12 (pieces are cut at rank-specific task boundaries), the same top-k lists for k in
{1, 37, 100, 1000} modulo exact-tie groups (PageRank.java:167-189), the same topPage rows
(:192-204), and a
checkpoint written by the 2-rank world that a single-rank context resumes from.  Skipped on a
box with fewer than 2 GPUs (the driver's GPU tier has one; its 8-GPU bench runs the same
exchange)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import graphgen as G
import parity

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _gpus() -> int:
    import torch  # device_count does not initialise HIP on this image
    return torch.cuda.device_count()


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.skipif(_gpus() < 2, reason="needs 2 GPUs (RCCL rejects two ranks on one device)")
@pytest.mark.parametrize("sparse,tiny", [("0", False), ("1", False), ("1", True), ("0", True)])
def test_rccl_two_ranks_match_one_rank(engine_mod, oracle_mod, tmp_path, monkeypatch, sparse, tiny):
    """sparse = 1 forces the sparse x' exchange (its RCCL count check, packed send/recv); tiny
    = a stream geometry with LDS blocks on this small graph, so the ranks run the overlapped
    schedule (cut stream launch, hot-first exchange plan) over RCCL."""
    P, O = engine_mod, oracle_mod
    monkeypatch.setenv("PR_SPARSE_X", sparse)
    if tiny:
        for k, v in (("PR_HOTLDS", "256"), ("PR_NLDS", "6"), ("PR_QH", "1024"), ("PR_SEG", "512")):
            monkeypatch.setenv(k, v)
    a, m = G.wiki_text(seed=3, pages=20_000, arcs_target=200_000)
    (tmp_path / "arcs").write_bytes(a)
    (tmp_path / "map").write_bytes(m)
    out = str(tmp_path / "w2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(HERE, "rccl_worker.py"), out, str(tmp_path / "arcs"), str(tmp_path / "map")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = np.load(out + ".ranks.npy")
    res = json.load(open(out + ".json"))

    one = P.Engine(device=0)
    one.ingest_buffers(a, m)
    one.run(10)
    r1 = one.ranks()
    parity.assert_ranks_close(got, r1, rtol=1e-12)
    parity.assert_ranks_close(got, O.Graph.from_text(a, m).run(10)["ranks"])
    key = lambda pair, v: b"%d:%d" % (pair, v)  # noqa: E731
    for k, lst in res["topk"].items():
        exp = one.topk(int(k))
        parity.assert_same_order_mod_ties([(key(x[0], x[1]), x[2]) for x in lst],
                                          [(key(e[0], e[1]), e[2]) for e in exp], rtol=1e-12)
    one.write_top_page(str(tmp_path / "one.topPage"))
    parity.assert_same_order_mod_ties(parity.parse_top_page(open(out + ".topPage", "rb").read()),
                                      parity.parse_top_page(open(tmp_path / "one.topPage", "rb").read()),
                                      rtol=1e-12)
    # the 2-rank checkpoint resumes in a single-rank context
    two_more = P.Engine(device=0)
    two_more.ingest_buffers(a, m)
    two_more.checkpoint_load(out + ".ckpt")
    two_more.run(2)
    one.run(12)
    parity.assert_ranks_close(two_more.ranks(), one.ranks(), rtol=1e-12)
