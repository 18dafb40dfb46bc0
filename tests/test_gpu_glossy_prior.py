"""GPU side of the glossy prior (pg_config.glossy_prior; tests/test_glossy_prior.py has the oracle
side): on an all-glossy scene the guided GPU render equals the unguided one bit for bit, and with the
learned fraction the guided GPU image of a mixed scene agrees with the unguided oracle."""
import numpy as np
import pytest

from test_glossy_prior import glossy_cornell

pytestmark = pytest.mark.gpu


def test_gpu_all_glossy_scene_is_not_guided(pg):
    from mitsuba_path_guiding_amd.integrator import Device
    sc = glossy_cornell(pg, 48, 48)
    films = []
    for guided in (True, False):
        d = Device(pg.capi.default_config(guiding=int(guided), s_tree_threshold=300.0, glossy_prior=1))
        d.upload(sc)
        off = 0
        if guided:
            for it in range(3):
                d.render_pass(2 ** it, off, True)
                off += 2 ** it
                d.splat_local()
                d.refit(it)
            assert d.stats()["dtree_nodes"] > 1
            d.reset_film()
        d.render_pass(16, 7)
        films.append(d.read_film())
        d.close()
    assert np.array_equal(films[0][0], films[1][0]) and np.array_equal(films[0][1], films[1][1])


def test_gpu_prior_learned_image_unbiased(pg, O):
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    from test_gpu_parity import _zstats
    S = pg.scenes
    sc = S.cornell(64, 64, short_material=S.material("roughconductor", conductor="Cu", alpha=0.05, distribution="ggx"),
                   tall_material=S.material("roughplastic", alpha=0.2, distribution="ggx",
                                            diffuse_reflectance=(0.5, 0.4, 0.3)))
    integ = GuidedPathTracer({"trainingIterations": 5, "sTreeThreshold": 400.0, "glossyPrior": True,
                              "bsdfSamplingFractionBound": "learned"})
    integ.preprocess(sc)
    rgbw, sq = integ.render(256)
    integ.postprocess()
    c = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(), 512)[:2]
    m1, m2, z = _zstats((rgbw, sq), c)
    assert (np.abs(z) < 5).mean() > 0.995
    assert abs(m1.mean() - m2.mean()) / m2.mean() < 0.01
