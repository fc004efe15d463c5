"""The TF-IDF job on the device (tfidf.hip; Spark.java:22-173) against the
literal oracle (oracle/tfidf_literal.py, itself pinned by the reference's `tfidf` output
artifact in test_tfidf_oracle.py): the ./output file byte for byte, lookups of many words,
counts, and the reference's crash lines."""
import math

import pytest

import graphgen as G
import tfidf_literal as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


def check_dump(P, data, words=(b"cloud", b"sky", b"the", b"w7", b"", b"zzz", b"Cloud"),
               tmp_path=None):
    eng = P.Engine()
    eng.tfidf_ingest(data)
    n, counts, df = T.run(data)
    info = eng.tfidf_info()
    assert info["docs"] == n
    assert info["words"] == len(df)
    assert info["pairs"] == len(counts)
    assert info["tokens"] == sum(counts.values())
    for w in words:
        _n, exp = T.lookup(data, w, k=10 ** 9)
        got = eng.tfidf_lookup(w, 10 ** 6)
        assert [t.split(b",")[0] for t, _ in got] == [t for t, _ in exp]
        assert [v for _, v in got] == [v for _, v in exp]   # same IEEE values
    if tmp_path is not None:
        out = tmp_path / "output"
        eng.tfidf_write_output(None, str(out))
        assert out.read_bytes() == T.output(data)
    eng.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_synthetic_dump(P, seed, tmp_path):
    check_dump(P, G.tfidf_dump(seed, docs=1500), tmp_path=tmp_path)


def test_hand_made_rules(P, tmp_path):
    data = (b"1\tA\tx\tcloud Cloud <b>cloud</b> sky\n"
            b"2\tB, Inc\tx\tthe cloud\\ncloud\n"
            b"3\tA\tx\tsky<unclosed cloud\n"
            b"4\tC\tx\t\tmore\n"
            b"5\t,lead\tx\t <i>cloud</i>\r\n"
            b"6\tD\tx\t\\<b>ncloud x<y>cloud\r"
            b"7\tE\tx\t123 !!! \n"
            b"8\tF\tx\tCLOUD")
    check_dump(P, data, words=(b"cloud", b"sky", b"", b"n", b"ncloud", b"unclosed", b"more"),
               tmp_path=tmp_path)


def test_large_documents(P, tmp_path):
    """Texts much longer than a wave's 64-byte chunk (tags and escapes across chunks)."""
    import random
    rng = random.Random(5)
    lines = []
    for i in range(300):
        parts = []
        for _ in range(rng.randint(0, 3000)):
            parts.append(rng.choice(["cloud", "<a href=\"x\">", "</a>", "\\n", "sky", "Data9",
                                     "rain", "<", ">", "storm", "n"]))
        lines.append(b"%d\tT%d\tx\t%s" % (i, i % 97, " ".join(parts).encode()))
    check_dump(P, b"\n".join(lines) + b"\n", tmp_path=tmp_path)


@pytest.mark.parametrize("data", [
    b"1\tA\tx\ty\nlonely\n",              # no columns[1]: the titles job dies first
    b"1\tA\tx\t\t\n2\tB\tx\ty\n",          # trailing empty fields: no columns[3]
    b"1\tA\tx\ty\n2\tB\tx\n\nfoo\n",       # line 2 has no columns[3], line 3 no columns[1]
    b"1\tA\tx\ty\n2\t,,\tx\tword\n",       # a title of commas only (Spark.java:106)
    b"1\tA\tx\ty\n2\t\tx\t\tz\n",          # an empty title: its first key splits to [""]
])
def test_crash_lines(P, data):
    with pytest.raises(T.ArrayIndexOutOfBounds) as xo:
        T.run(data)
    eng = P.Engine()
    with pytest.raises(P.ArrayIndexOutOfBoundsException) as xe:
        eng.tfidf_ingest(data)
    assert str(xo.value) in str(xe.value)


def test_idf_is_integer_division(P):
    """3 documents, "a" in 2 of them: Math.log(3 / 2) with Long / Integer = ln(1) = 0."""
    eng = P.Engine()
    eng.tfidf_ingest(b"1\tX\t-\ta a b\n2\tY\t-\ta\n3\tZ\t-\tb b b c\n")
    assert eng.tfidf_lookup(b"a") == [(b"X", 0.0), (b"Y", 0.0)]
    assert eng.tfidf_lookup(b"c") == [(b"Z", math.log(3))]
    assert eng.tfidf_lookup(b"b") == [(b"X", 0.0), (b"Z", 0.0)]   # ties: by title


def test_tfidf_cli_contract(P, tmp_path):
    """`_build/tfidf DUMP --out PATH` (Spark.main's file contract) writes the oracle's file;
    a malformed dump exits 1 with the Java exception on stderr."""
    import os
    import subprocess
    cli = os.path.join(os.path.dirname(P.LIB_PATH), "tfidf")
    data = G.tfidf_dump(7, docs=800)
    (tmp_path / "data").write_bytes(data)
    subprocess.run([cli, str(tmp_path / "data"), "--out", str(tmp_path / "output")],
                   check=True, timeout=120)
    assert (tmp_path / "output").read_bytes() == T.output(data)
    (tmp_path / "bad").write_bytes(b"1\tA\tx\ty\nlonely\n")
    r = subprocess.run([cli, str(tmp_path / "bad"), "--out", str(tmp_path / "o2")],
                       capture_output=True, timeout=120)
    assert r.returncode == 1 and b"ArrayIndexOutOfBoundsException: 1" in r.stderr
    assert not (tmp_path / "o2").exists()
