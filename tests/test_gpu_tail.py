"""The chunk-tail megakernel (k_tail, pg_config.tail_paths): once a chunk's live paths drop to the
threshold, one launch loops shade -> shadow any-hit -> closest hit per thread instead of one launch
pair and a count readback per bounce.  It runs the same per-path arithmetic in the same order, so
films, SD-trees and path statistics are bit-identical with the per-bounce launches -- off (< 0),
the default threshold and a threshold that sends every bounce after the first through k_tail."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COUNTED = ("segments", "escaped", "shadow_rays", "records")


def _guided(pg, sc, tail):
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    t = GuidedPathTracer({"trainingIterations": 4, "sTreeThreshold": 400.0, "tailPaths": tail})
    t.preprocess(sc)
    rgbw, sq = t.render(16)
    tree = t.dev.get_sdtree()
    st = t.postprocess()
    return rgbw, sq, tree, st


@pytest.mark.parametrize("scene", ["cornell", "envmap"])
def test_tail_launch_is_bit_identical(pg, scene):
    S = pg.scenes
    sc = S.cornell(96, 96) if scene == "cornell" else S.sky_courtyard(64, 48, env=S.sky_envmap(128, 64, sun_radiance=20.0))
    runs = {tail: _guided(pg, sc, tail) for tail in (-1, 0, 1 << 30)}
    off = runs[-1]
    assert off[3]["tail_launches"] == 0
    for tail in (0, 1 << 30):
        r = runs[tail]
        assert r[3]["tail_launches"] > 0, tail
        assert np.array_equal(r[0], off[0]) and np.array_equal(r[1], off[1]), tail
        assert np.array_equal(r[2], off[2]), tail
        for k in COUNTED:
            assert r[3][k] == off[3][k], (tail, k)
