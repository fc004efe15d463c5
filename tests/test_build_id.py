"""The library under test is the one built from the checked-out sources:
pr_build_id() is the hash of csrc/ + include/ + Makefile baked in at build time."""
import pytest


def _check(P):
    import source_hash as S
    assert P.build_id() == S.source_hash() == S.library_build_id(P.LIB_PATH)
    assert len(P.build_id()) == 20


def test_library_is_built_from_these_sources(engine_mod):
    _check(engine_mod)


@pytest.mark.gpu
def test_gpu_box_library_is_built_from_these_sources(engine_mod):
    """Same check where the driver runs -m gpu: the .so that travelled to the box is HEAD's."""
    _check(engine_mod)
    e = engine_mod.Engine(device=0)       # and that library drives the device
    e.generate_rmat(8, 4, 1)
    e.run(2)
    assert (e.ranks() > 0).any()
