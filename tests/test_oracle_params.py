"""The oracle's handling of the integrator parameters, pinned to the semantics the reference's loop
defines (src/integrators/path/progressive_path.cpp:133-314, progressiveintegrator.cpp:274-277).  The GPU
side of every case is tests/test_gpu_params.py (same streams against this oracle).

  * maxDepth = 1: the loop adds emission at depth 1 and stops (:149,167-169,175): each sample is Le or 0;
  * hideEmitters with maxDepth = 1: nothing is ever added (:168);
  * maxDepth = 2 is direct lighting: NEE (:193-219) and the BSDF-sampled emitter hit (:276-284), MIS-
    weighted, estimate the same expectation with and without useNee (:280-282, the weight is 1 without);
  * maxComponentValue scales every sample down to the bound (:274-277), so no pixel mean exceeds it;
  * rrDepth only changes the estimator's variance, not its expectation (:296-306).
"""
import numpy as np

from test_volume import _mean_z, _zimg


def _render(pg, O, sc, spp, **kw):
    return O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(**kw), spp, nthreads=8)


def test_max_depth_one_is_emission_only(pg, O):
    sc = pg.scenes.cornell(24, 24)
    rgbw, sq, _ = _render(pg, O, sc, 16, max_depth=1)
    le = np.array([17.0, 12.0, 4.0])
    frac = rgbw[..., :3] / rgbw[..., 3:] / le  # fraction of samples that saw the light
    assert np.allclose(frac, frac[..., :1], atol=1e-6)  # every sample is 0 or exactly Le
    k = frac[..., 0] * 16
    assert np.allclose(k, np.round(k), atol=1e-4)
    assert 0 < (k > 0).mean() < 0.2  # the light covers a few pixels
    rgbw, _, _ = _render(pg, O, sc, 16, max_depth=1, hide_emitters=1)
    assert not rgbw[..., :3].any()


def test_direct_lighting_with_and_without_nee(pg, O):
    sc = pg.scenes.cornell(24, 24)
    a = _render(pg, O, sc, 256, max_depth=2)[:2]
    b = _render(pg, O, sc, 4096, max_depth=2, use_nee=0, seed=99)[:2]
    # per 4x4-pixel block (BSDF-sampled hits on the small light are rare per pixel, hence also the
    # larger spp without NEE: with few hits the sample variance underestimates the estimator's)
    blk = [tuple(x[..., c].reshape(6, 4, 6, 4).sum((1, 3)) for c in range(4)) for x in (a[0], a[1], b[0], b[1])]
    (ar, ag, ab, an), (sr, sg, sb, _), (br, bg, bb, bn), (tr, tg, tb, _) = blk
    ma, mb = (ar + ag + ab) / an / 3, (br + bg + bb) / bn / 3
    va = ((sr + sg + sb) / an / 3 - ma ** 2) / an
    vb = ((tr + tg + tb) / bn / 3 - mb ** 2) / bn
    z = (ma - mb) / np.sqrt(va + vb + 1e-12)
    assert (np.abs(z) < 5).all(), np.abs(z).max()
    assert abs(_mean_z(a, b)) < 5
    m1 = _zimg(a, b)[0]
    full = _render(pg, O, sc, 64)[0]
    assert m1.mean() < 0.9 * (full[..., :3] / full[..., 3:]).mean()  # indirect light is missing


def test_clamp_bounds_every_pixel(pg, O):
    sc = pg.scenes.cornell(24, 24)
    for bound in (0.25, 1.0):
        rgbw, _, _ = _render(pg, O, sc, 32, max_component_value=bound)
        assert (rgbw[..., :3] / rgbw[..., 3:]).max() <= bound * (1 + 1e-6)


def test_rr_depth_keeps_the_expectation(pg, O):
    sc = pg.scenes.cornell(24, 24)
    a = _render(pg, O, sc, 256, rr_depth=1)[:2]
    b = _render(pg, O, sc, 256, rr_depth=8, seed=5)[:2]
    assert abs(_mean_z(a, b)) < 5
