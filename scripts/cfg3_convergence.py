#!/usr/bin/env python3
"""R-MAT scale 24, edge factor 16, seed 3, run to relative L1
residual sum|r'-r| / sum r' <= 1e-8 on one MI355X; the oracle (exact sums, C) runs the same
convergence on the host and the ranks are compared (defined set exact, <= 1e-9 relative)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import prmi355x as P  # noqa: E402
import oracle as O  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
eng = P.Engine()
t = time.perf_counter()
eng.generate_rmat(scale, 16, 3)
info = eng.info()
print(f"scale {scale}: n={int(info['n_vertices'])} nnz={int(info['nnz'])} build {time.perf_counter() - t:.2f} s")
st = eng.run(200, 1e-8)
print(f"engine: {st['iterations']} rounds to residual {st['residual']:.3e}, "
      f"{st['ms_per_iter']:.3f} ms/round, {st['gteps']:.1f} GTEPS, rank sum {st['rank_sum']:.6f}")
r = eng.ranks()
O.build()
t = time.perf_counter()
g = O.Graph.from_rmat(scale, 16, 3)
res = g.run(200, tol=1e-8, threads=16)
print(f"oracle (exact sums, 16 threads): {res['iterations']} rounds, residual {res['residual']:.3e}, "
      f"{time.perf_counter() - t:.1f} s")
e = res["ranks"]
same = np.array_equal(r > 0, e > 0)
d = e > 0
rel = float(np.max(np.abs(r[d] - e[d]) / e[d])) if d.any() else 0.0
print(f"defined set identical: {same}; max relative difference {rel:.2e} "
      f"(rounds {st['iterations']} vs {res['iterations']})")
