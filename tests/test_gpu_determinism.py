"""The summation order of the row launch is a function of the layout alone -- needs an MI355X.

reduceByKey(Sum) (PageRank.java:139, :208-213) leaves the order of a page's adds open; the
engine's ranks are reproducible bit for bit only if its own order is fixed.  The one place
where the hardware, not the code, orders adds is the row launch's LDS double-add: lanes of one
instruction that hit the same row.  pr_selftest_sum_order issues that instruction form with
many lane / row / value patterns from 8192 waves on every compute unit, many launches each;
every copy of a pattern must carry the same bits.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_same_address_lds_adds_apply_in_one_fixed_order(engine_mod):
    eng = engine_mod.Engine()
    res = eng.selftest_sum_order(cases=96, launches=25)
    eng.close()
    assert res["copies"] == 96 * 25 * 8192
    assert res["differing"] == 0, res
    print(f"LDS add order: {res['copies']} accumulator sets identical per pattern; "
          f"{res['lane_order_cases']}/{res['cases']} patterns equal the ascending-lane serial sum")


def test_rounds_repeat_bit_for_bit_across_contexts_and_launch_histories(engine_mod):
    """Ten rounds on one graph from three contexts with different histories on the device
    (fresh; after another graph ran; after a rank group used the card): identical rank bits."""
    P = engine_mod
    def ten(scale=16):
        e = P.Engine()
        e.generate_rmat(scale, 16, 21)
        e.run(10)
        r = e.ranks()
        e.close()
        return r
    a = ten()
    other = P.Engine()
    other.generate_rmat(18, 16, 2)
    other.run(5)
    b = ten()
    other.close()
    grp = P.LocalGroup(4)
    grp.each("generate_rmat", 15, 16, 3)
    grp.run(3)
    c = ten()
    grp.close()
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
    assert np.array_equal(a.view(np.uint64), c.view(np.uint64))
