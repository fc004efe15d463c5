#!/usr/bin/env python3
"""Time text ingest (PageRank.java:26-60) on a large fixed-width wiki-style input: the host
parser (PR_DEVICE_NONE context) against the device ingest (ingest.hip).
usage: scripts/ingest_time.py [arcs=20000000] [pages=2000000]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import graphgen as G  # noqa: E402
import prmi355x as P  # noqa: E402

arcs = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
pages = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
a, m = G.big_text(seed=1, pages=pages, arcs=arcs)
print(f"input: {arcs} arc lines ({len(a) / 1e6:.0f} MB), {pages} pages ({len(m) / 1e6:.0f} MB)")
modes = [("host", P.PR_DEVICE_NONE)]
if "--host-only" not in sys.argv:
    modes.append(("device", 0))
for name, dev in modes:
    for rep in range(2):
        e = P.Engine(device=dev)
        t = time.perf_counter()
        e.ingest_buffers(a, m)
        wall = 1e3 * (time.perf_counter() - t)
        i = e.info()
        print(f"{name:6s} rep {rep}: ingest {i['ms_ingest']:9.1f} ms (call {wall:9.1f} ms)  "
              f"n={int(i['n_vertices'])} raw={int(i['raw_edges'])} pairs={int(i['n_pairs'])} "
              f"n_tot={int(i['n_tot'])}")
        e.close()
