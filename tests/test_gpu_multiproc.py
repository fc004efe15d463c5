"""The multi-process path on one GPU: p processes, one engine context per
rank (n_ranks = p, rows dealt in 16-row chunks), every round's x slot and exact dangling
record exchanged over a torch.distributed gloo world through the caller-staged exchange
(pr_comm_init_external / pr_ext_*).  This runs the per-rank contexts, their layouts and the
round protocol of a multi-GPU job -- everything but RCCL itself, which needs several GPUs --
and compares the assembled ranks with one rank and with the oracle."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import parity

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_world(p, tmp_path, scale, ef, seed, rounds, tol=0.0):
    port = free_port()
    out = str(tmp_path / f"w{p}")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mp_ext_worker.py"), str(r),
                               str(p), str(port), out, str(scale), str(ef), str(seed),
                               str(rounds), repr(tol)], env=env)
             for r in range(p)]
    rcs = [pr.wait(timeout=240) for pr in procs]
    assert rcs == [0] * p, rcs
    return np.load(out + ".npy"), json.load(open(out + ".json"))


@pytest.mark.parametrize("p", [2, 4])
def test_external_exchange_world_matches_one_rank(engine_mod, oracle_mod, tmp_path, p):
    P, O = engine_mod, oracle_mod
    ref = P.Engine(device=0)
    ref.generate_rmat(15, 16, 6)
    ref.run(10)
    r1 = ref.ranks()
    ref.close()
    rp, info = run_world(p, tmp_path, 15, 16, 6, 10)
    assert info["sum_local_nnz"] == info["nnz"] and info["sum_local_rows"] == info["n_rows"]
    assert info["iterations"] == 10
    parity.assert_ranks_close(rp, r1, rtol=1e-12)
    parity.assert_ranks_close(rp, O.Graph.from_rmat(15, 16, 6).run(10)["ranks"])


def test_external_exchange_tracked_convergence(engine_mod, oracle_mod, tmp_path):
    """tol > 0: the exact residual is combined from the p records; the world stops on the
    same round as the oracle."""
    O = oracle_mod
    rp, info = run_world(2, tmp_path, 14, 16, 3, 200, 1e-8)
    res = O.Graph.from_rmat(14, 16, 3).run(200, tol=1e-8)
    assert abs(info["iterations"] - res["iterations"]) <= 1
    assert info["residual"] <= 1e-8
    if info["iterations"] == res["iterations"]:
        parity.assert_ranks_close(rp, res["ranks"])
