"""The TF-IDF oracle (oracle/tfidf_literal.py) pinned against the reference's own output
artifact (tests/golden/tfidf_reference_output.txt = the reference's `tfidf` file: Spark.java
run on the course's Wikipedia dump, which the repository does not hold), plus the
Spark.java text rules on hand-made documents.  CPU only."""
import math
import os

import pytest

import tfidf_literal as T
from pagerank_literal import ArrayIndexOutOfBounds, java_double_to_string

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "tfidf_reference_output.txt")


def test_reference_artifact_is_integer_division_idf():
    """Every row of the artifact is Double.toString(tf * Math.log(titleCount / df)) with
    Long / Integer integer division: titleCount = 1117712 and floor(N / df) = 86 here."""
    lines = open(GOLDEN, "rb").read().decode().splitlines()
    n = int(lines[0].split()[-1])
    assert lines[0] == f"total docs are {n}" and n == 1117712
    idf = math.log(n // 12996)                       # any df in (N/87, N/86] gives 86
    assert n // 12996 == 86 and idf != math.log(n / 12996)
    rows = [ln.rsplit("\t", 1) for ln in lines[1:]]
    assert len(rows) == 99
    prev = None
    for title, s in rows:
        tf = round(float(s) / idf)
        assert java_double_to_string(tf * idf) == s, (title, s)
        assert prev is None or float(s) <= prev       # sorted by tfidf descending
        prev = float(s)
    # titles with commas are cut at the first one (key.split(",")[1], Spark.java:106)
    assert sum(1 for t, _ in rows if t == "St. Cloud") == 2
    assert all("," not in t for t, _ in rows)


def test_text_cleaning_rules():
    c = T.clean
    assert c(b"a<b>c") == b"a c"
    assert c(b"x<ref name=y>Cloud</ref>z") == b"x cloud z"
    assert c(b"a<b<c>d") == b"a d"                     # <[^>]*> from the first '<'
    assert c(b"a>b<c") == b"a b c"                      # unmatched brackets are just non-letters
    assert c(b"foo\\nbar") == b"foo bar"               # literal backslash-n
    assert c(b"foo\\<i>nbar") == b"foo nbar"           # tag removal runs before the \\n rule
    assert c(b"R2D2 3rd") == b"r d rd"
    assert T.java_split_ws(b" a b") == [b"", b"a", b"b"]
    assert T.java_split_ws(b"a b ") == [b"a", b"b"]
    assert T.java_split_ws(b"") == [b""]
    assert T.java_split_ws(b" ") == []


def test_job_counts_and_errors():
    data = (b"1\tA\tx\tcloud Cloud <b>cloud</b> sky\n"
            b"2\tB, Inc\tx\tthe cloud\n"
            b"3\tA\tx\tsky\n"                         # same title as line 1: one document
            b"4\tC\tx\t\n"                            # trailing empty fields: no columns[3]
            ).replace(b"4\tC\tx\t\n", b"4\tC\tx\t\tmore\n")  # columns[3] = "" -> word ""
    n, counts, df = T.run(data)
    assert n == 3
    assert counts[(b"cloud", b"A")] == 3 and counts[(b"sky", b"A")] == 2
    assert counts[(b"", b"C")] == 1
    assert df[b"cloud"] == 2
    n, rows = T.lookup(data)
    assert rows[0] == (b"A", 3 * math.log(3 // 2)) and rows[1][0] == b"B"
    with pytest.raises(ArrayIndexOutOfBounds, match="1 .line 2"):
        T.run(b"1\tA\tx\ty\nlonely\n")
    with pytest.raises(ArrayIndexOutOfBounds, match="3 .line 1"):
        T.run(b"1\tA\tx\t\t\n2\tB\tx\ty\n")
    with pytest.raises(ArrayIndexOutOfBounds, match="1 .line 2"):
        T.run(b"1\tA\tx\ty\n2\t,,\tx\tword\n")        # title of commas only
    assert T.output(b"1\tA\tx\tsky\n").startswith(b"total docs are 1\n")
