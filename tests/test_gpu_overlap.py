"""The overlapped exchange of the multi-rank round loop -- needs an MI355X.

With more than one rank the next round's stream launch is cut in two (PR_XOVERLAP, on by
default): the part that reads only the hot prefix of x starts when chunk 0 of the exchange has
landed, the cold-segment tasks and the row launch wait for everything.  The cut changes when
work starts, not what is summed in which order: ranks must be bit-identical to the uncut
schedule (PR_XOVERLAP=0) -- with the sparse and the dense exchange, with tiny stream geometries
(several cold segments per slice, task boundaries inside the hot range), with an injected
transfer delay that makes the parts really run apart, and in tracked mode.  This is the
reduceByKey shuffle of PageRank.java:139 overlapped with the next round's flatMapToPair (:94-117).
"""
import numpy as np
import pytest

import parity

pytestmark = pytest.mark.gpu

TINY = (("PR_HOTLDS", "256"), ("PR_NLDS", "6"), ("PR_QH", "1024"), ("PR_SEG", "512"))


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


@pytest.fixture(scope="module")
def O(oracle_mod):
    return oracle_mod


def group_ranks(P, p, scale, ef, seed, T, flags=0):
    grp = P.LocalGroup(p, flags=flags)
    grp.each("generate_rmat", scale, ef, seed)
    st = grp.run(T)
    r = grp.members[p - 1].ranks()
    grp.close()
    return r, st


@pytest.mark.parametrize("p,tiny,sx,delay", [(2, False, "1", 0), (4, False, "1", 0), (8, False, "1", 0),
                                             (8, False, "0", 0), (2, True, "1", 0), (4, True, "0", 0),
                                             (8, True, "1", 0), (4, True, "1", 300), (8, False, "1", 200)])
def test_overlapped_schedule_bit_identical(P, O, monkeypatch, p, tiny, sx, delay):
    if tiny:
        for k, v in TINY:
            monkeypatch.setenv(k, v)
    monkeypatch.setenv("PR_SPARSE_X", sx)
    if delay:
        monkeypatch.setenv("PR_XDELAY_US", str(delay))
    scale = 16 if tiny else 19     # (untuned geometry: LDS blocks need ~2^19 vertices)
    out = []
    for ov in ("0", "1"):
        monkeypatch.setenv("PR_XOVERLAP", ov)
        out.append(group_ranks(P, p, scale, 16, 43, 8)[0])
    assert np.array_equal(out[0].view(np.uint64), out[1].view(np.uint64))
    parity.assert_ranks_close(out[1], O.Graph.from_rmat(scale, 16, 43).run(8)["ranks"])


@pytest.mark.parametrize("p,tiny,delay", [(4, True, 0), (8, False, 0), (2, True, 200)])
def test_pack_stream_bit_identical(P, monkeypatch, p, tiny, delay):
    """The sparse exchange packs a chunk's send buffers on the comm stream, ahead of the chunk's
    sends (PR_PACKCOMM=1, the default), or on the compute stream behind the chunk's rows (0):
    the same ranks, bit for bit, with and without the overlapped schedule."""
    if tiny:
        for k, v in TINY:
            monkeypatch.setenv(k, v)
    if delay:
        monkeypatch.setenv("PR_XDELAY_US", str(delay))
    scale = 16 if tiny else 19
    out = []
    for pk, ov in (("0", "1"), ("1", "1"), ("1", "0")):
        monkeypatch.setenv("PR_PACKCOMM", pk)
        monkeypatch.setenv("PR_XOVERLAP", ov)
        out.append(group_ranks(P, p, scale, 16, 47, 8)[0])
    assert np.array_equal(out[0].view(np.uint64), out[1].view(np.uint64))
    assert np.array_equal(out[0].view(np.uint64), out[2].view(np.uint64))


def test_overlapped_schedule_tracked_and_crash_round(P, O, monkeypatch):
    """Tracked mode (exact residual and rank sum through the overlapped rounds) and the round of
    the empty-collection crash (PageRank.java:125) are those of the uncut schedule."""
    for k, v in TINY:
        monkeypatch.setenv(k, v)
    res = []
    for ov in ("0", "1"):
        monkeypatch.setenv("PR_XOVERLAP", ov)
        r, st = group_ranks(P, 4, 15, 16, 7, 12, flags=P.PR_F_TRACK_RESIDUAL)
        res.append((r, st["residual"], st["rank_sum"]))
    assert np.array_equal(res[0][0].view(np.uint64), res[1][0].view(np.uint64))
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2] and res[1][2] > 0
    # vertex 5's dangling entry vanishes after round 1: the job dies in round 2
    arcs, mapping = b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n"
    grp = P.LocalGroup(2)
    grp.each("ingest_buffers", arcs, mapping)
    with pytest.raises(P.UnsupportedOperationException) as e:
        grp.run(10)
    assert "iteration 2" in str(e.value)
    grp.close()
