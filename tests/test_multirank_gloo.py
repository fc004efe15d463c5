"""World-size-2 CPU rehearsal (gloo) of the engine's multi-GPU protocol.

The engine deals internal rows to ranks in chunks of 16 (chunk c = k // 16 goes to rank
c % p), writes each rank's new contribution values into its own contiguous slot of x
(A-row k at owner(k)*maxA + local(k), C-vertex k at p*maxA + (k - R), maxA a multiple of
16), all-gathers the slots in place, and
sums the per-rank exact dangling records in any order.  This test replays that protocol
with numpy on two gloo ranks and checks: (1) the assembled ranks are bit-identical to the
same protocol at p = 1, (2) they match the oracle within 1e-9, (3) every edge and row is
owned by exactly one rank.  The real RCCL path runs on the driver's 8-GPU node; the same
layout is exercised on one GPU by tests/test_gpu_parity.py::test_rank_group_*.
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
    perm, inv, (nA, nB, nC, _nD), outd, ind, dang_w = internal_order(src, dst, n, mapw)
    R = nA + nB
    CH = 16

    def owner(k):
        return (k // CH) % p

    def local(k):
        return ((k // CH) // p) * CH + k % CH

    # slice-major x (p divides 8): rank slot -> slice region (chunk % 8) -> chunk order
    NS = 8
    SL = CH * -(-(-(-nA // CH)) // NS)
    SLC = CH * -(-(-(-nC // CH)) // NS)
    maxA = (NS // p) * SL
    X = p * maxA + NS * SLC

    def xpos(k):
        c = k // CH
        kc = k - R
        cc = kc // CH
        a = ((c % NS) % p) * maxA + ((c % NS) // p) * SL + (c // NS) * CH + k % CH
        b = p * maxA + (cc % NS) * SLC + (cc // NS) * CH + kc % CH
        return np.where(k < nA, a, b)

    def xslot(l):                                           # local row -> offset in own slot
        c = (l // CH) * p + rank
        return ((c % NS) // p) * SL + (c // NS) * CH + l % CH

    allrows = np.arange(R)
    own = allrows[owner(allrows) == rank]                   # internal rows of this rank
    assert np.array_equal(local(own), np.arange(len(own)))  # local rows are dense
    kd, ks = inv[dst], inv[src]
    mine = owner(kd) == rank
    order = np.lexsort((ks[mine], local(kd[mine])))        # (local row, internal source)
    lrow = local(kd[mine])[order]
    lsrc = ks[mine][order]
    col = xpos(lsrc)
    rp = np.zeros(len(own) + 1, np.int64)
    np.add.at(rp, lrow + 1, 1)
    rp = np.cumsum(rp)
    x = np.zeros(X)
    cols_all = np.concatenate([np.arange(nA), np.arange(R, R + nC)])
    x[xpos(cols_all)] = 1.0 / outd[perm[cols_all]]
    r_loc = np.zeros(len(own))
    w_own = dang_w[perm[own]]
    a = float(dang_w.sum()) / n_tot
    for _t in range(ROUNDS):
        c = np.array([math.fsum(x[col[rp[l]:rp[l + 1]]]) for l in range(len(own))])
        r_loc = np.where(c > 0, 0.15 + (c + a) * 0.85, 0.0)
        slot = np.zeros(maxA)
        isA = own < nA
        slot[xslot(np.nonzero(isA)[0])] = r_loc[isA] / outd[perm[own[isA]]]
        assert np.array_equal(rank * maxA + xslot(np.nonzero(isA)[0]), xpos(own[isA]))
        xn = np.zeros(X)
        xn[:p * maxA] = allgather(slot)                   # in-place all-gather of slots
        x = xn
        recs = gather_records([(float(r), int(w)) for r, w in zip(r_loc, w_own) if w and r > 0])
        assert recs, "empty collection"
        a = math.fsum(r * w for r, w in recs) / n_tot      # exact, order-free combine
    full = np.zeros(n)
    full[perm[own]] = r_loc
    return full, (len(own), len(lsrc))


def _worker(rank, world, port, q):
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

    full, owned = protocol(rank, world, src, dst, n, mapw, n, allgather, gather_records)
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


def test_two_rank_protocol_matches_single_rank_and_oracle(oracle_mod):
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
    full1, own1 = protocol(0, 1, src, dst, n, np.ones(n, np.int64), n,
                           lambda sl: sl, lambda recs: recs)
    assert np.array_equal(full1.view(np.uint64), full2.view(np.uint64))
    assert sum(o[0] for o in owned) == own1[0] and sum(o[1] for o in owned) == own1[1] == len(k)
    exp = O.Graph.from_rmat(SCALE, EF, SEED).run(ROUNDS)["ranks"]
    d_ = exp > 0
    assert np.array_equal(full2 > 0, d_)
    assert np.max(np.abs(full2[d_] - exp[d_]) / exp[d_]) <= 1e-9
