#!/usr/bin/env python3
"""Time the TF-IDF job (Spark.java) on a synthetic Wikipedia-style dump: device ingest
(clean + count + df) and the "cloud" lookup, against the literal CPU restatement
(oracle/tfidf_literal.py, single thread) on a bounded sample of the same dump.
usage: scripts/tfidf_time.py [docs=200000] [words_per_doc=300]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("page-rank-and-tfidf-using-apache-spark_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import graphgen as G  # noqa: E402
import prmi355x as P  # noqa: E402
import tfidf_literal as T  # noqa: E402

docs = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
wpd = int(sys.argv[2]) if len(sys.argv) > 2 else 300
data = G.tfidf_dump(1, docs=docs, words_per_doc=wpd)
mb = len(data) / 1e6
print(f"dump: {docs} docs, {mb:.1f} MB")
eng = P.Engine()
for rep in range(3):
    t = time.perf_counter()
    eng.tfidf_ingest(data)
    dt = time.perf_counter() - t
    t = time.perf_counter()
    rows = eng.tfidf_lookup(b"cloud", 100)
    dl = time.perf_counter() - t
    info = eng.tfidf_info()
    print(f"device rep {rep}: ingest {1e3 * dt:8.1f} ms ({mb / dt / 1e3:.2f} GB/s incl. H2D), "
          f"lookup {1e3 * dl:6.2f} ms; {info}")
sample = data[: len(data) // 20]
sample = sample[: sample.rfind(b"\n") + 1]
t = time.perf_counter()
T.lookup(sample, b"cloud")
dc = time.perf_counter() - t
print(f"cpu literal oracle (1 thread) on {len(sample) / 1e6:.1f} MB: {dc:.2f} s "
      f"({len(sample) / 1e6 / dc:.1f} MB/s)")
