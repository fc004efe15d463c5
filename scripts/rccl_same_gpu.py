#!/usr/bin/env python3
"""Multi-process RCCL path of the engine (needs one GPU per rank: RCCL rejects two ranks on
one device with "Duplicate GPU detected").  Launch: python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 --master-port 29511 scripts/rccl_same_gpu.py
Checks the ranks agree with a single-rank run of the same graph (1e-12 relative; the pieces
are cut at rank-specific task boundaries, so the last bits may differ)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd"))
import numpy as np
import prmi355x as P
P.lib()  # bind ROCm's HIP/RCCL before torch loads its own
import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
dev = int(os.environ.get("LOCAL_RANK", "0"))
eng = P.Engine(device=dev, n_ranks=world, rank=rank)
uid = P.comm_unique_id() if rank == 0 else bytes(128)
t = torch.tensor(list(uid), dtype=torch.uint8)
dist.broadcast(t, 0)
eng.comm_init(bytes(t.tolist()))
eng.generate_rmat(16, 16, 6)
st = eng.run(10)
r = eng.ranks()
top = eng.topk(20)
if rank == 0:
    ref = P.Engine(device=dev)
    ref.generate_rmat(16, 16, 6)
    ref.run(10)
    r1 = ref.ranks()
    d = r1 > 0
    same_set = np.array_equal(r > 0, d)
    rel = float(np.max(np.abs(r[d] - r1[d]) / r1[d])) if d.any() else 0.0
    print(f"RCCL world={world}: defined set equal: {same_set}; max rel diff vs single rank {rel:.2e}; "
          f"{st['ms_per_iter']:.3f} ms/round", flush=True)
    assert same_set and rel <= 1e-12
dist.barrier()
eng.close()
dist.destroy_process_group()
