"""Regenerate the committed golden fixtures (run from the repo root:
``python tests/golden/make_golden.py``).

The reference job (PageRank.java, Spark 1.x) cannot run in this image and ships no outputs,
so the expected values come from the literal-RDD restatement ``oracle/pagerank_literal.py``
(exact sums) and are cross-checked against the dense C restatement before being written.
Inputs are synthetic (seeded); nothing here reads /root/reference.

Files:
  cfg1_arcs.txt.gz / cfg1_mapping.txt.gz   config-1 inputs (10k pages, ~100k links, seed 1)
  cfg1_expected.json                       N_tot, distinct arcs, degrees digest, every
                                           defined page's rank (repr, 17 sig. digits) after 10
                                           rounds, and the exact ./topPage bytes
  kat_expected.json                        SURVEY.md Appendix B known answers, T = 0,1,2,10
"""
import gzip
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import graphgen  # noqa: E402
import oracle as O  # noqa: E402
import pagerank_literal as L  # noqa: E402

KAT_ARCS = b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n1\t2\n2\t5\n"
KAT_MAP = b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n6\tF\n"


def ranks_by_id(graph, ranks):
    ids = graph.ids()
    return {ids[v].decode("utf-8", "surrogateescape"): repr(float(ranks[v]))
            for v in range(graph.n) if ranks[v] > 0}


def check_agree(arcs, mapping, T):
    lit, _m, _n = L.run_literal(arcs, mapping, T)
    g = O.Graph.from_text(arcs, mapping)
    r = g.run(T)["ranks"]
    dense = ranks_by_id(g, r)
    lit_s = {k.decode("utf-8", "surrogateescape"): repr(v) for k, v in lit.items()}
    assert dense == lit_s, "literal and dense oracles disagree"
    return g, lit_s


def main():
    # ---- Appendix B ----
    kat = {"arcs": KAT_ARCS.decode(), "mapping": KAT_MAP.decode(), "rounds": {}}
    for T in (0, 1, 2, 10):
        _g, lit = check_agree(KAT_ARCS, KAT_MAP, T)
        kat["rounds"][str(T)] = {"ranks": lit,
                                 "topPage": L.main_literal(KAT_ARCS, KAT_MAP, T).decode()}
    with open(os.path.join(HERE, "kat_expected.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)

    # ---- config 1 ----
    arcs, mapping = graphgen.wiki_text(seed=1)
    for name, data in (("cfg1_arcs.txt.gz", arcs), ("cfg1_mapping.txt.gz", mapping)):
        with open(os.path.join(HERE, name), "wb") as f:
            f.write(gzip.compress(data, mtime=0))
    g, lit = check_agree(arcs, mapping, 10)
    o, i, w = g.degrees()
    exp = {
        "iterations": 10,
        "n_vertices": g.n, "raw_edges": g.raw_edges, "nnz": g.nnz, "n_tot": g.n_tot,
        "dangling_entries": int(w.sum()),
        "outdeg_sha256": hashlib.sha256(o.tobytes()).hexdigest(),
        "indeg_sha256": hashlib.sha256(i.tobytes()).hexdigest(),
        "edge_digest": [str(x) for x in g.edge_digest()],
        "ranks": lit,
        "topPage": L.main_literal(arcs, mapping, 10).decode(),
    }
    with open(os.path.join(HERE, "cfg1_expected.json"), "w") as f:
        json.dump(exp, f, indent=0, sort_keys=True, ensure_ascii=False)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
