"""Seeded generators of reference-format inputs (arcs + mapping text) for the tests.

Formats follow PageRank.java:26-51: arcs lines ``src\\tdst``, mapping lines ``id\\ttitle``.
"""
from __future__ import annotations

import random
from typing import List, Tuple

import numpy as np


def random_small_text(seed: int, max_v: int = 12, max_e: int = 30) -> Tuple[bytes, bytes]:
    """Tiny adversarial graphs: duplicate arcs, self-loops, arcs to unmapped ids, ids with
    two titles, extra columns, CRLF / CR terminators, empty ids, missing final newline."""
    rng = random.Random(seed)
    nv = rng.randint(1, max_v)
    ids = [str(rng.randint(0, 3 * nv)) for _ in range(nv)]
    if rng.random() < 0.2:
        ids.append("")                       # "\tb" -> key "" (PageRank.java:39)
    if rng.random() < 0.2:
        ids.append("007")                    # exact string ids: "007" != "7"
    ne = rng.randint(0, max_e)
    arcs: List[str] = []
    if rng.random() < 0.7:
        # a 2-cycle feeding a mapped dangling page keeps danglingMap non-empty every round
        arcs += ["cyc1\tcyc2", "cyc2\tcyc1", "cyc1\tdz"]
        ids += ["cyc1", "cyc2", "dz"]
    for _ in range(ne):
        s, d = rng.choice(ids), rng.choice(ids)
        if rng.random() < 0.1:
            d = "x" + str(rng.randint(0, 5))   # destination absent from the mapping
        line = f"{s}\t{d}"
        if rng.random() < 0.08:
            line += "\textra"                  # extra columns are ignored
        arcs.append(line)
        if rng.random() < 0.15:
            arcs.append(line)                  # duplicate arc
    maps: List[str] = ["dz\tDangling Z"] if "dz" in ids else []
    for v in sorted(set(ids) - {"dz"}, key=lambda z: rng.random()):
        if rng.random() < 0.85:
            maps.append(f"{v}\tT{v}")
        if rng.random() < 0.1:
            maps.append(f"{v}\tAlt {v}")       # second title -> dangling weight 2
        if rng.random() < 0.05:
            maps.append(f"{v}\tT{v}\tjunk")    # same pair, distinct raw line (N_tot counts it)
    if maps and rng.random() < 0.1:
        maps.append(maps[0])                   # duplicate raw line
    terms = ["\n", "\r\n", "\r"]

    def join(lines: List[str]) -> bytes:
        if not lines:
            return b""
        out = ""
        for i, ln in enumerate(lines):
            out += ln + (rng.choice(terms) if rng.random() < 0.2 else "\n")
        if rng.random() < 0.2:
            out = out.rstrip("\r\n")
        return out.encode()

    return join(arcs), join(maps)


def wiki_text(seed: int = 1, pages: int = 10_000, arcs_target: int = 100_000,
              dangling_frac: float = 0.3, dup_frac: float = 0.01,
              unmapped_frac: float = 0.005) -> Tuple[bytes, bytes]:
    """Config-1 stand-in: wiki-style ids (random 7-digit strings), titles
    with spaces / commas / UTF-8, Zipf out-degrees, ~1% duplicate arc lines, ~0.5% arcs to
    unmapped ids, ~30% dangling pages that still receive in-links."""
    rng = np.random.default_rng(seed)
    ids = rng.choice(np.arange(1_000_000, 10_000_000), size=pages, replace=False)
    ids = [str(int(x)) for x in ids]
    words = ["Cloud", "Strife", "St.", "Paul, Minnesota", "Zürich", "naïve", "東京", "Data",
             "(film)", "List of", "Apache", "Spark", "page", "rank"]
    titles = []
    for i in range(pages):
        k = int(rng.integers(1, 4))
        titles.append(" ".join(words[int(j)] for j in rng.integers(0, len(words), k)) + f" {i}")
    n_src = int(pages * (1.0 - dangling_frac))
    # Zipf-like out-degree over the sources, scaled to the arc target
    w = 1.0 / np.arange(1, n_src + 1) ** 0.9
    deg = np.maximum(1, np.round(w / w.sum() * arcs_target)).astype(np.int64)
    order = rng.permutation(n_src)
    pop = 1.0 / np.arange(1, pages + 1) ** 0.7          # popularity of destinations
    pop /= pop.sum()
    perm = rng.permutation(pages)
    lines: List[str] = []
    for si in range(n_src):
        s = ids[order[si]]
        dsts = perm[rng.choice(pages, size=int(deg[si]), p=pop)]
        for d in dsts:
            if rng.random() < unmapped_frac:
                lines.append(f"{s}\t{int(rng.integers(10_000_000, 20_000_000))}")
            else:
                lines.append(f"{s}\t{ids[int(d)]}")
    ndup = int(len(lines) * dup_frac)
    for j in rng.integers(0, len(lines), ndup):
        lines.append(lines[int(j)])
    lines = [lines[int(j)] for j in rng.permutation(len(lines))]
    arcs = ("\n".join(lines) + "\n").encode()
    maps = ("\n".join(f"{ids[i]}\t{titles[i]}" for i in range(pages)) + "\n").encode()
    return arcs, maps


def rmat_text(scale: int, edge_factor: int, seed: int) -> Tuple[bytes, bytes]:
    """Config-2 stand-in: R-MAT edges (same Philox generator as the engine) written as
    decimal-id text; mapping = every id 0..2^scale-1 with title ``v<id>``."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import oracle as O
    s, d = O.rmat_edges(scale, edge_factor, seed)
    arcs = "".join(f"{a}\t{b}\n" for a, b in zip(s.tolist(), d.tolist())).encode()
    maps = "".join(f"{i}\tv{i}\n" for i in range(1 << scale)).encode()
    return arcs, maps


def big_text(seed: int, pages: int, arcs: int) -> Tuple[bytes, bytes]:
    """Large fixed-width wiki-style input built with numpy (ingest scale tests / timing):
    7-digit ids, Zipf-skewed destinations, one title per page plus a second title on 1% of
    pages, ~2% duplicate arc lines, ~1% arcs to ids outside the mapping."""
    rng = np.random.default_rng(seed)
    ids = rng.permutation(9_000_000)[:pages + pages // 50] + 1_000_000
    mapped, unmapped = ids[:pages], ids[pages:]

    def digits(v):
        out = np.empty((len(v), 7), np.uint8)
        x = v.copy()
        for c in range(6, -1, -1):
            out[:, c] = 48 + x % 10
            x //= 10
        return out

    src = mapped[rng.integers(0, pages, arcs)]
    dst = mapped[np.minimum(rng.zipf(1.3, arcs) - 1, pages - 1)]
    stray = rng.random(arcs) < 0.01
    dst[stray] = unmapped[rng.integers(0, len(unmapped), int(stray.sum()))]
    dup = rng.random(arcs) < 0.02
    src[1:][dup[1:]] = src[:-1][dup[1:]]
    dst[1:][dup[1:]] = dst[:-1][dup[1:]]
    a = np.empty((arcs, 16), np.uint8)
    a[:, 0:7], a[:, 7], a[:, 8:15], a[:, 15] = digits(src), 9, digits(dst), 10
    m1 = np.empty((pages, 22), np.uint8)      # "ddddddd\tPage ddddddd\n"
    m1[:, 0:7], m1[:, 7], m1[:, 8:13], m1[:, 13:20] = digits(mapped), 9, list(b"Page "), digits(mapped)
    m1[:, 20], m1[:, 21] = ord("x"), 10
    two = mapped[rng.random(pages) < 0.01]
    m2 = np.empty((len(two), 22), np.uint8)
    m2[:, 0:7], m2[:, 7], m2[:, 8:13], m2[:, 13:20] = digits(two), 9, list(b"Alt  "), digits(two)
    m2[:, 20], m2[:, 21] = ord("y"), 10
    return a.tobytes(), m1.tobytes() + m2.tobytes()


def tfidf_dump(seed: int, docs: int = 2000, words_per_doc: int = 60) -> bytes:
    """Stand-in for the Wikipedia dump Spark.java:26 reads (absent from the reference):
    `id \\t title \\t date \\t text` lines with HTML tags, literal backslash-n sequences,
    digits, punctuation, mixed case, titles with commas and repeated titles, some empty
    texts and extra columns; "cloud" is common."""
    rng = random.Random(seed)
    vocab = ["cloud", "Cloud", "CLOUD", "computing", "storm", "rain", "sky", "data", "the",
             "of", "and", "strife", "oort", "st", "server", "alpha", "beta", "gamma"] + \
            ["w" + "".join(chr(97 + (i // 26 ** q) % 26) for q in range(3)) for i in range(3000)]
    extra = ["<ref name=x>", "</ref>", "<b>", "</b>", "\\n", "\\n\\n", "1999", "3rd", "--",
             "(", ")", "e.g.", "&amp;", "<", ">", "x<y", "a\\b", "\\", "n"]
    titles = ["Page %d" % i for i in range(docs)]
    for i in range(0, docs, 17):
        titles[i] = "St. Cloud, Place %d" % (i % 5)          # truncated at ',' -> "St. Cloud"
    for i in range(3, docs, 41):
        titles[i] = titles[i - 1]                             # repeated titles merge
    lines = []
    for i in range(docs):
        toks = []
        for _ in range(rng.randint(0, words_per_doc)):
            r = rng.random()
            if r < 0.12:
                toks.append(rng.choice(extra))
            elif r < 0.2:
                toks.append(rng.choice(["cloud", "Cloud"]))
            else:
                toks.append(rng.choice(vocab))
        sep = rng.choice([" ", "  ", ", ", ".", " - "])
        text = sep.join(toks)
        if rng.random() < 0.05:
            text = ""
        if rng.random() < 0.1:
            text = " " + text
        cols = [str(100000 + i), titles[i], "2015-0%d" % rng.randint(1, 9), text]
        if rng.random() < 0.05 or not text:   # an empty text needs a later field to exist
            cols.append("extra column")
        lines.append("\t".join(cols))
    term = rng.choice(["\n", "\r\n"])
    return (term.join(lines) + (term if rng.random() < 0.8 else "")).encode()
