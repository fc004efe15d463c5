"""pr_run_static (the allocation-free variant of pr_run) against pr_run -- needs an MI355X.

Both entry points run the same kernels in the same order, so the ranks must be bit-identical.
The static scratch is shared by every context on the GPU and keeps the last call's contents:
two calls in a row, the second on a smaller graph, must both match; so must tracked runs, a
crash round, and a call after the scratch was used by another context.  During the call the
device's free memory must not move (nothing is allocated or freed).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def P(engine_mod):
    return engine_mod


def _free_bytes(P):
    # hipMemGetInfo of the HIP runtime the engine itself is linked to (dlsym through the
    # engine's handle): loading a second copy of the runtime by path fails once another test
    # has brought torch's bundled ROCm libraries into the process
    fn = P.lib().hipMemGetInfo
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    free, total = C.c_size_t(0), C.c_size_t(0)
    assert fn(C.byref(free), C.byref(total)) == 0
    return free.value


def _pair(P, scale, ef, seed, T, tol=0.0, flags=0):
    """(ranks by pr_run, stats) on a fresh context of the same graph."""
    eng = P.Engine(flags=flags)
    eng.generate_rmat(scale, ef, seed)
    st = eng.run(T, tol)
    r = eng.ranks()
    eng.close()
    return r, st


def test_static_run_matches_run_two_calls_in_a_row(P):
    big, small = (14, 16, 3), (11, 8, 5)
    exp_big, _ = _pair(P, *big, 10)
    exp_small, _ = _pair(P, *small, 7)
    a, b = P.Engine(), P.Engine()
    a.generate_rmat(*big)
    b.generate_rmat(*small)
    a.run(1)
    b.run(1)                      # warm: every lazily created handle of the contexts exists
    free0 = _free_bytes(P)
    sa = a.run_static(10)
    sb = b.run_static(7)          # second call, smaller input, same scratch
    assert _free_bytes(P) == free0, "pr_run_static changed the device's free memory"
    assert sa["iterations"] == 10 and sb["iterations"] == 7
    ra, rb = a.ranks(), b.ranks()
    assert np.array_equal(ra.view(np.uint64), exp_big.view(np.uint64))
    assert np.array_equal(rb.view(np.uint64), exp_small.view(np.uint64))
    # and the big one again after the small one dirtied the scratch; then plain pr_run still
    # works on the same context (its own buffers were never touched)
    a.run_static(10)
    assert np.array_equal(a.ranks().view(np.uint64), exp_big.view(np.uint64))
    a.run(10)
    assert np.array_equal(a.ranks().view(np.uint64), exp_big.view(np.uint64))
    a.close()
    b.close()


def test_static_run_tracked_and_converging(P):
    exp, st = _pair(P, 13, 16, 9, 300, tol=1e-4)
    eng = P.Engine()
    eng.generate_rmat(13, 16, 9)
    got = eng.run_static(300, 1e-4)
    assert got["iterations"] == st["iterations"] and got["iterations"] < 300
    assert got["residual"] == st["residual"] and got["rank_sum"] == st["rank_sum"]
    assert np.array_equal(eng.ranks().view(np.uint64), exp.view(np.uint64))
    eng.close()


def test_static_run_crash_round_and_text_graph(P):
    arcs, mapping = b"1\t2\n1\t3\n2\t3\n3\t1\n4\t3\n", b"1\tA\n2\tB\n3\tC\n4\tD\n5\tE\n"
    eng = P.Engine()
    eng.ingest_buffers(arcs, mapping)
    st = P.Stats()
    rc = P.lib().pr_run_static(eng._h, 10, 0.0, st)
    assert rc == P.PR_E_EMPTY_DANGLING and st.failed_iteration == 2
    eng.run_static(1)
    r1 = eng.ranks()
    eng.run(1)
    assert np.array_equal(r1.view(np.uint64), eng.ranks().view(np.uint64))
    eng.run_static(0)
    assert list(eng.ranks()) == [1.0, 1.0, 1.0, 1.0, 0.0]
    eng.close()


def test_static_run_rejects_what_it_cannot_hold(P):
    eng = P.Engine()
    eng.generate_rmat(21, 16, 1)        # ~33 M edges: more piece sums than the scratch holds
    with pytest.raises(P.PageRankError) as e:
        eng.run_static(2)
    assert e.value.code == P.PR_E_ARG and "static scratch holds" in str(e.value)
    eng.run(2)                           # the allocating entry point takes it
    eng.close()
    grp = P.LocalGroup(2)
    grp.each("generate_rmat", 10, 8, 1)
    with pytest.raises(P.PageRankError) as e:
        grp.members[0].run_static(2)
    assert e.value.code == P.PR_E_ARG
    grp.close()
