"""TEST INFRASTRUCTURE ONLY -- literal-RDD restatement of PageRank.java (the oracle).

This module is part of ``oracle/``: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as a checker.  It is never on
the product path.

PARITY STATUS: *parity unpinned*.  The reference (``/root/reference/PageRank.java``, Spark
1.x Java) ships no tests, no golden vectors and no recorded ``topPage`` output, and it cannot
be run in this image (no JVM, no Spark -- SURVEY.md section 8c).  This restatement is pinned
instead by (a) the hand-checked known-answer tests of SURVEY.md Appendix B and (b) bit-exact
agreement with the independent dense C restatement ``oracle/pagerank_oracle.c`` on
thousands of random graphs (``tests/test_oracle.py``).

What it does: replays every Spark operator of ``PageRank.main`` (PageRank.java:21-204) with
Python dicts / lists, in program order, so that the behaviour -- including the reference's
non-standard semantics (non-normalised ranks, the shrinking defined set, per-title dangling
multiplicity, ``totalVertices`` = distinct mapping *lines*, and the crash on an empty
dangling RDD) -- is reproduced literally.  Floating-point sums whose order Spark leaves
unspecified (``reduce`` at :125, ``reduceByKey(Sum)`` at :139) are taken *exactly*
(``math.fsum``: the correctly rounded value of the exact sum), which is the order-free
answer every Spark run approximates.
"""
from __future__ import annotations

import math
from decimal import Decimal
from typing import Dict, Iterable, List, Sequence, Tuple


class SparkJobError(Exception):
    """Base for the exceptions the reference job dies with."""


class ArrayIndexOutOfBounds(SparkJobError):
    """``parts[1]`` on a line with fewer than two tab-separated fields
    (PageRank.java:40 arcs, :49 mapping) -> java.lang.ArrayIndexOutOfBoundsException."""


class EmptyCollection(SparkJobError):
    """``danglingMap.values().reduce(...)`` on an empty RDD (PageRank.java:125)
    -> java.lang.UnsupportedOperationException("empty collection") [Spark 1.x]."""


# ----------------------------------------------------------------------------------------
# Java / Hadoop text rules
# ----------------------------------------------------------------------------------------

def hadoop_lines(data: bytes) -> List[bytes]:
    """Split a file the way Hadoop ``TextInputFormat`` does for ``spark.textFile``
    (PageRank.java:26-30): terminators are ``\\n``, ``\\r`` and ``\\r\\n``; a final line
    without a terminator is still a line; nothing follows the last terminator."""
    out: List[bytes] = []
    i, n, start = 0, len(data), 0
    while i < n:
        c = data[i]
        if c == 0x0A or c == 0x0D:
            out.append(data[start:i])
            if c == 0x0D and i + 1 < n and data[i + 1] == 0x0A:
                i += 1
            start = i + 1
        i += 1
    if start < n:
        out.append(data[start:n])
    return out


def java_split_tab(line: bytes) -> List[bytes]:
    """``String.split("\\t")`` (PageRank.java:39,47): split on every tab, then drop
    *trailing* empty fields (a leading empty field is kept)."""
    parts = line.split(b"\t")
    while parts and parts[-1] == b"":
        parts.pop()
    return parts


def parse_pair(line: bytes) -> Tuple[bytes, bytes]:
    """``new Tuple2(parts[0], parts[1])`` (PageRank.java:40,49)."""
    parts = java_split_tab(line)
    if len(parts) < 2:
        raise ArrayIndexOutOfBounds(f"line {line!r} has {len(parts)} field(s)")
    return parts[0], parts[1]


def java_double_to_string(v: float) -> str:
    """``Double.toString`` as printed by ``page + "\\t" + rank`` (PageRank.java:197).

    JDK >= 19 layout and digit choice (shortest decimal that round-trips):
    plain notation with at least one fractional digit for 1e-3 <= |v| < 1e7, otherwise
    ``d.dddE[-]n``.  Python's ``repr`` yields the same shortest digit string."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Infinity" if v > 0 else "-Infinity"
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    sign = "-" if v < 0 else ""
    a = abs(v)
    t = Decimal(repr(a)).normalize().as_tuple()
    digits = "".join(str(d) for d in t.digits)
    # value = 0.d1d2...dn * 10^e10  (scientific exponent = e10 - 1)
    e10 = len(digits) + t.exponent
    if 1e-3 <= a < 1e7:
        if e10 <= 0:
            s = "0." + "0" * (-e10) + digits
        elif e10 >= len(digits):
            s = digits + "0" * (e10 - len(digits)) + ".0"
        else:
            s = digits[:e10] + "." + digits[e10:]
        return sign + s
    mant = digits[0] + "." + (digits[1:] if len(digits) > 1 else "0")
    return f"{sign}{mant}E{e10 - 1}"


# ----------------------------------------------------------------------------------------
# The job, operator by operator
# ----------------------------------------------------------------------------------------

def run_literal(arcs: bytes, mapping: bytes, iterations: int = 10):
    """Replay PageRank.main (PageRank.java:21-189) on in-memory file contents.

    Returns ``(ranks, mappings_pairs, total_vertices)`` where ``ranks`` is the final
    ``ranks`` RDD as a dict id(bytes) -> float.  Raises ``ArrayIndexOutOfBounds`` or
    ``EmptyCollection`` exactly where the reference job would die."""
    arc_lines = hadoop_lines(arcs)
    map_lines = hadoop_lines(mapping)

    # :60 ``mappingFile.distinct().count()`` is the first action: raw lines, no parse.
    total_vertices = len(set(map_lines))

    # :35-42  mapToPair(split) -> distinct -> groupByKey -> cache
    arc_pairs = [parse_pair(s) for s in arc_lines]
    distinct_arcs = list(dict.fromkeys(arc_pairs))            # distinct(), any order
    adjacency: Dict[bytes, List[bytes]] = {}
    for s, d in distinct_arcs:                                # groupByKey()
        adjacency.setdefault(s, []).append(d)

    # :43-51  mappings = mapToPair(split) -> distinct
    mappings = list(dict.fromkeys(parse_pair(s) for s in map_lines))

    # :56  dangling = mappings.subtractByKey(adjacencyList).keys()   (multiset)
    dangling = [k for (k, _v) in mappings if k not in adjacency]
    # :64-73  danglingMap = (id, 1.0)
    dangling_map: List[Tuple[bytes, float]] = [(k, 1.0) for k in dangling]
    # :76-83  ranks = adjacencyList.mapValues(1.0)
    ranks: Dict[bytes, float] = {k: 1.0 for k in adjacency}

    for _current in range(iterations):                        # :92
        # :94-117  adjacencyList.join(ranks).values().flatMapToPair(...)
        contribs: List[Tuple[bytes, float]] = []
        for src, dsts in adjacency.items():
            if src not in ranks:                              # inner join drops it
                continue
            r = ranks[src]
            url_count = len(dsts)                             # :103-108
            for n in dsts:                                    # :111-114
                contribs.append((n, r / url_count))
        # :121-138  reduce over danglingMap.values(); empty -> crash
        if not dangling_map:
            raise EmptyCollection("empty collection")
        dsum = math.fsum(v for _k, v in dangling_map)
        addthis = dsum / float(total_vertices)                # :135 (long -> double)
        # :139  reduceByKey(new Sum())   (exact sum per key)
        grouped: Dict[bytes, List[float]] = {}
        for k, v in contribs:
            grouped.setdefault(k, []).append(v)
        # :140-145  0.15 + (sum + addthis) * 0.85   (Java: no fused multiply-add)
        ranks = {k: 0.15 + (math.fsum(vs) + addthis) * 0.85 for k, vs in grouped.items()}
        # :146-160  danglingMap.join(ranks) keeps the new rank; missing ids drop out
        dangling_map = [(k, ranks[k]) for (k, _old) in dangling_map if k in ranks]

    return ranks, mappings, total_vertices


def top_pages(ranks: Dict[bytes, float], mappings: Sequence[Tuple[bytes, bytes]],
              k: int = 100) -> List[Tuple[bytes, float]]:
    """:167-189  ranks.join(mappings) -> (rank,(id,title)) -> sortByKey(false) -> take(k).

    Spark leaves the order of equal ranks unspecified; here ties are broken by
    (title, id) ascending so the oracle is deterministic -- comparisons against it must
    treat equal-rank runs as groups."""
    rows = [(ranks[i], t, i) for (i, t) in mappings if i in ranks]
    rows.sort(key=lambda r: (-r[0], r[1], r[2]))
    return [(t, r) for (r, t, _i) in rows[:k]]


def format_top_page(rows: Iterable[Tuple[bytes, float]]) -> bytes:
    """:192-197  ``page + "\\t" + rank + "\\n"`` per row."""
    return b"".join(t + b"\t" + java_double_to_string(r).encode() + b"\n" for t, r in rows)


def main_literal(arcs: bytes, mapping: bytes, iterations: int = 10, k: int = 100) -> bytes:
    """Whole job: returns the bytes the reference writes to ``./topPage``."""
    ranks, mappings, _n = run_literal(arcs, mapping, iterations)
    return format_top_page(top_pages(ranks, mappings, k))
