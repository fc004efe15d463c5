#!/usr/bin/env python3
"""What sharding costs in compute: the scale-26 graph dealt over p ranks that all live on ONE
GPU (LocalGroup: device copies replace RCCL).  The p ranks' launches share the card, so the
round time is the sum of the p shares; if it stays near the p = 1 time, a rank's compute at
p GPUs is ~1/p of the single-GPU round and only the exchange separates strong scaling from
linear.  usage: python scripts/group_split.py [scale] [p ...]   (PRMI_SEED: R-MAT seed, 4)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd"))
import prmi355x as P  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
ps = [int(a) for a in sys.argv[2:]] or [1, 2, 4, 8]
seed = int(os.environ.get("PRMI_SEED", "4"))
for p in ps:
    g = P.LocalGroup(p)
    g.each("generate_rmat", scale, 16, seed)
    nnz = sum(int(m.info()["local_nnz"]) for m in g.members)
    g.run(2)
    st = g.run(10)
    print(f"scale {scale} p={p}: {st['ms_per_iter']:.3f} ms/round for all {p} shares on one GPU "
          f"(local nnz total {nnz}), SpMV kernels {st['ms_spmv_kernel']:.3f} ms", flush=True)
    g.close()
