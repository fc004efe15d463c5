#!/usr/bin/env python3
"""What the build-time placement search finds for ONE rank of a p-rank world (the rank built alone on
the GPU, externally exchanged context): prints the search's timings.  usage: rank_alone_placement.py P"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "page-rank-and-tfidf-using-apache-spark_amd"))
import prmi355x as P
p = int(sys.argv[1])
eng = P.Engine(device=0, n_ranks=p, rank=0)
eng.comm_init_external()
eng.generate_rmat(26, 16, 4)
i = eng.info()
print("p", p, "placement tried", i["place_tried"], "first %.4f kept %.4f ms" % (i["place_ms_first"], i["place_ms_best"]), flush=True)
eng.close()
