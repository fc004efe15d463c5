"""World-size-2 CPU rehearsal (gloo) of the engine's multi-GPU protocol.

Two gloo ranks on the CPU run the round protocol of a 2-GPU job -- rows dealt to ranks, every
rank's new contribution values written into its own slot of x, the slots all-gathered in place,
the exact dangling records combined in any order -- with the layout taken from the engine
itself: owner rank, local row and x position of every vertex come from ``pr_layout_map``, the
host build of the very functions the kernels use (engine.hip owner_of / local_of / xpos), not
from a model of them.  The arithmetic of a round is numpy (there is no GPU here).  Checks:
(1) both ranks derive the same x layout and it is collision-free, (2) local rows are dense and
a rank's class-A rows land exactly in its own slot, (3) every edge and row is owned by exactly
one rank, (4) the assembled ranks are bit-identical to the same protocol at p = 1 and match
the oracle within 1e-9.  The device side of the same protocol runs in tests/test_gpu_multiproc.py
(gloo worlds of 2 and 4 processes on one GPU) and tests/test_gpu_parity.py (rank groups); the
RCCL transport needs one GPU per rank (tests/test_gpu_rccl.py).
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SCALE, EF, SEED, ROUNDS = 12, 16, 3, 10


def internal_order(src, dst, n, mapw):
    outd = np.bincount(src, minlength=n)
    ind = np.bincount(dst, minlength=n)
    cls = np.where(ind > 0, np.where(outd > 0, 0, 1), np.where(outd > 0, 2, 3))
    perm = np.lexsort((np.arange(n), -ind, cls))          # (class, indeg desc, id)
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n)
    counts = np.bincount(cls, minlength=4)
    dang_w = np.where(outd == 0, mapw, 0)
    return perm, inv, counts, outd, ind, dang_w


def protocol(rank, p, src, dst, n, mapw, n_tot, allgather, gather_records):
    import prmi355x as P
    perm, inv, (nA, nB, nC, _nD), outd, ind, dang_w = internal_order(src, dst, n, mapw)
    R = nA + nB
    # the engine's own deal and x layout (host build of the kernels' layout functions)
    allrows = np.arange(R)
    owner, local, _xp, dims = P.layout_map(p, rank, nA, nB, nC, allrows)
    maxA, X = dims["max_a"], dims["x_len"]
    cols_all = np.concatenate([np.arange(nA), np.arange(R, R + nC)])
    _o, _l, xp_cols, _d = P.layout_map(p, rank, nA, nB, nC, cols_all)
    xpos = np.full(n, -1, np.int64)
    xpos[cols_all] = xp_cols.astype(np.int64)
    assert len(np.unique(xp_cols)) == len(cols_all) and xp_cols.max() < X     # collision-free
    assert np.all(xpos[:nA] < p * maxA) and np.all(xpos[R:R + nC] >= p * maxA)  # slots, then C

    own = allrows[owner == rank]                            # internal rows of this rank
    assert len(own) == dims["local_rows"] and int((own < nA).sum()) == dims["local_a"]
    assert np.array_equal(local[owner == rank], np.arange(len(own)))   # local rows are dense
    kd, ks = inv[dst], inv[src]
    mine = owner[kd] == rank
    order = np.lexsort((ks[mine], local[kd[mine]]))        # (local row, internal source)
    lrow = local[kd[mine]][order].astype(np.int64)
    lsrc = ks[mine][order]
    col = xpos[lsrc]
    rp = np.zeros(len(own) + 1, np.int64)
    np.add.at(rp, lrow + 1, 1)
    rp = np.cumsum(rp)
    x = np.zeros(X)
    x[xpos[cols_all]] = 1.0 / outd[perm[cols_all]]
    r_loc = np.zeros(len(own))
    w_own = dang_w[perm[own]]
    a = float(dang_w.sum()) / n_tot
    isA = own < nA
    slot_of = xpos[own[isA]] - rank * maxA                   # own class-A rows: inside own slot
    assert slot_of.min(initial=0) >= 0 and slot_of.max(initial=0) < maxA
    for _t in range(ROUNDS):
        c = np.array([math.fsum(x[col[rp[l]:rp[l + 1]]]) for l in range(len(own))])
        r_loc = np.where(c > 0, 0.15 + (c + a) * 0.85, 0.0)
        slot = np.zeros(maxA)
        slot[slot_of] = r_loc[isA] / outd[perm[own[isA]]]
        xn = np.zeros(X)
        xn[:p * maxA] = allgather(slot)                   # in-place all-gather of slots
        x = xn
        recs = gather_records([(float(r), int(w)) for r, w in zip(r_loc, w_own) if w and r > 0])
        assert recs, "empty collection"
        a = math.fsum(r * w for r, w in recs) / n_tot      # exact, order-free combine
    full = np.zeros(n)
    full[perm[own]] = r_loc
    return full, (len(own), len(lsrc)), xp_cols


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for d in ("page-rank-and-tfidf-using-apache-spark_amd", "oracle"):
        if os.path.join(root, d) not in sys.path:
            sys.path.insert(0, os.path.join(root, d))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    s, d = O.rmat_edges(SCALE, EF, SEED)
    k = np.unique((d.astype(np.uint64) << np.uint64(32)) | s.astype(np.uint64))
    dst = (k >> np.uint64(32)).astype(np.int64)
    src = (k & np.uint64(0xFFFFFFFF)).astype(np.int64)
    n = 1 << SCALE
    mapw = np.ones(n, np.int64)

    def allgather(slot):
        parts = [torch.zeros(len(slot), dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(slot))
        return torch.cat(parts).numpy()

    def gather_records(recs):
        out = [None] * world
        dist.all_gather_object(out, recs)
        return [r for part in out for r in part]

    full, owned, xp_cols = protocol(rank, world, src, dst, n, mapw, n, allgather, gather_records)
    # every rank derives the same x layout
    lay = [None] * world
    dist.all_gather_object(lay, xp_cols.tobytes())
    assert all(b == lay[0] for b in lay)
    t = torch.from_numpy(full)
    dist.all_reduce(t)                                    # one nonzero per page: exact
    if rank == 0:
        q.put((t.numpy().copy(), owned))
    own = [None] * world
    dist.all_gather_object(own, owned)
    if rank == 0:
        q.put(own)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_two_rank_protocol_matches_single_rank_and_oracle(oracle_mod, engine_mod):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    full2, _ = q.get(timeout=300)
    owned = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    # the same protocol at p = 1 (no communication)
    O = oracle_mod
    s, d = O.rmat_edges(SCALE, EF, SEED)
    k = np.unique((d.astype(np.uint64) << np.uint64(32)) | s.astype(np.uint64))
    dst = (k >> np.uint64(32)).astype(np.int64)
    src = (k & np.uint64(0xFFFFFFFF)).astype(np.int64)
    n = 1 << SCALE
    full1, own1, _xp = protocol(0, 1, src, dst, n, np.ones(n, np.int64), n,
                                lambda sl: sl, lambda recs: recs)
    assert np.array_equal(full1.view(np.uint64), full2.view(np.uint64))
    assert sum(o[0] for o in owned) == own1[0] and sum(o[1] for o in owned) == own1[1] == len(k)
    exp = O.Graph.from_rmat(SCALE, EF, SEED).run(ROUNDS)["ranks"]
    d_ = exp > 0
    assert np.array_equal(full2 > 0, d_)
    assert np.max(np.abs(full2[d_] - exp[d_]) / exp[d_]) <= 1e-9
