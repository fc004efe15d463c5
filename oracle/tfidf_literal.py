"""TEST INFRASTRUCTURE ONLY -- literal restatement of the reference's TF-IDF job (Spark.java).

Part of ``oracle/``: only ``tests/`` may import it, and only as a checker.

PARITY STATUS: pinned only by the reference's own output artifact ``tfidf`` (the dataset it
was computed on is not in the repository): the IDF is ``Math.log(titleCount / dword)`` with
Long / Integer *integer* division (every value of ``tfidf:2-100`` is an integer multiple of
ln 86 for titleCount = 1117712), and ``Double.toString`` formatting of ``tf * IDF``
(``tests/test_tfidf_oracle.py`` reproduces rows of the artifact).  Everything else is
restated from Spark.java line by line.

Byte model (shared with the engine): lines, fields and words are raw bytes.  The
reference decodes UTF-8 and lowercases with Java's ``String.toLowerCase``; non-ASCII
characters are turned into spaces by ``[^a-zA-Z]`` either way, except the few that Java
lowercases *to* ASCII letters (U+0130, U+212A): inputs containing those differ.  Titles
are compared (sort ties, Spark.java:155) by their ASCII-lowercased bytes.
"""
from __future__ import annotations

import math
import re
from collections import defaultdict
from typing import Dict, List, Tuple

from pagerank_literal import ArrayIndexOutOfBounds, hadoop_lines, java_double_to_string


def java_split_literal(s: bytes, sep: bytes) -> List[bytes]:
    """``String.split(sep)`` for a one-character literal separator: no match -> [s]; else
    every field, then trailing empty fields dropped (a leading empty field stays)."""
    if sep not in s:
        return [s]
    parts = s.split(sep)
    while parts and parts[-1] == b"":
        parts.pop()
    return parts


def java_split_ws(s: bytes) -> List[bytes]:
    """``text.split("\\\\s+")`` (Spark.java:43): a leading run of whitespace yields a leading
    empty word; trailing empty fields are dropped; no match -> [s] (so "" -> [""])."""
    if not re.search(rb"\s+", s):
        return [s]
    parts = re.split(rb"\s+", s)
    while parts and parts[-1] == b"":
        parts.pop()
    return parts


def clean(text: bytes) -> bytes:
    """Spark.java:38-42, in program order."""
    t = re.sub(rb"<[^>]*>", b" ", text)      # replaceAll("\\<[^>]*>", " "): \< is a literal <
    t = t.replace(b"\\n", b" ")              # replace("\\n", " "): backslash + n, literally
    t = t.lower()                            # toLowerCase() (ASCII in the byte model)
    t = re.sub(rb"[0-9]", b" ", t)
    t = re.sub(rb"[^a-zA-Z]", b" ", t)
    t = re.sub(rb"\s+", b" ", t)
    return t


def doc_words(line: bytes, lineno: int) -> Tuple[bytes, List[bytes]]:
    """Spark.java:35-47 for one line: (title, words)."""
    cols = java_split_literal(line, b"\t")
    if len(cols) < 4:
        raise ArrayIndexOutOfBounds(f"{1 if len(cols) < 2 else 3} (line {lineno})")
    return cols[1], java_split_ws(clean(cols[3]))


def run(data: bytes):
    """The job up to the join (Spark.java:26-131): returns (titleCount, counts, df) with
    counts[(word, title)] = tf and df[word] = documents (distinct titles) holding word."""
    lines = hadoop_lines(data)
    # :50-56 titles.distinct().count() runs first: a line without columns[1] dies there
    for i, s in enumerate(lines, 1):
        if len(java_split_literal(s, b"\t")) < 2:
            raise ArrayIndexOutOfBounds(f"1 (line {i})")
    titles = set()
    counts: Dict[Tuple[bytes, bytes], int] = defaultdict(int)
    first_line: Dict[Tuple[bytes, bytes], int] = {}
    for i, s in enumerate(lines, 1):
        title, words = doc_words(s, i)
        titles.add(title)
        for w in words:
            counts[(w, title)] += 1                     # :57-71 (word + "," + title, 1) sums
            first_line.setdefault((w, title), i)
    # :75-131 split(",") of the key: a title with no byte other than ',' leaves too few fields
    bad = None
    for (w, t), i in first_line.items():
        fields = java_split_literal(w + b"," + t, b",")
        if len(fields) < 2 and (bad is None or i < bad[0]):
            bad = (i, len(fields))
    if bad is not None:
        raise ArrayIndexOutOfBounds(f"{bad[1]} (line {bad[0]})")
    df: Dict[bytes, int] = defaultdict(int)
    for (w, _t) in counts:
        df[w] += 1
    return len(titles), counts, df


def lookup(data: bytes, word: bytes = b"cloud", k: int = 100):
    """Spark.java:120-162: rows (title', tfidf) for `word`, sorted by tfidf descending, ties
    by lowercased title' (then the full title: Spark's order is unspecified there)."""
    n, counts, df = run(data)
    rows = []
    for (w, t), tf in counts.items():
        if w != word:
            continue
        t1 = java_split_literal(w + b"," + t, b",")[1]   # :106 the title up to its first ','
        idf = math.log(n // df[w])                        # :130 Long / Integer, then ln
        rows.append((tf * idf, t1, t))
    rows.sort(key=lambda r: (-r[0], r[1].lower(), r[2]))
    return n, [(t1, v) for v, t1, _t in rows[:k]]


def output(data: bytes, word: bytes = b"cloud", k: int = 100) -> bytes:
    """The ./output file (Spark.java:164-171)."""
    n, rows = lookup(data, word, k)
    out = [b"total docs are %d\n" % n]
    for t1, v in rows:
        out.append(t1 + b"\t" + java_double_to_string(v).encode() + b"\n")
    return b"".join(out)
