"""A Mitsuba XML scene through the GPU path: the hand-written test scene of
test_mitsuba_xml.py (analytic shapes, a referenced roughplastic, named IOR, a constant environment,
a mirrored sensor) rendered by the plugin mirror, against the oracle on the same loaded scene
(per-pixel z-test |z| < 5 for >= 99.9 % of pixel channels, 1e-5 relative floor; mean within 0.5 %)."""
import numpy as np
import pytest

from test_mitsuba_xml import SCENE

pytestmark = pytest.mark.gpu


def test_xml_scene_gpu_vs_oracle(pg, O):
    out = pg.mitsuba_xml.load(SCENE, defines={"depth": -1}, sphere_res=(32, 16))
    sc = out.scene
    from mitsuba_path_guiding_amd.integrator import ProgressivePathTracer
    integ = ProgressivePathTracer(dict(out.integrator_props, samplesPerProgression=64))
    integ.preprocess(sc)
    rgbw, sq = integ.render(256)
    integ.postprocess()
    c = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(max_depth=-1), 256)[:2]
    c = (c[0][:, ::-1], c[1][:, ::-1])  # the sensor mirrors x: the plugin flips its read-out
    n1, n2 = np.maximum(rgbw[..., 3:4], 1), np.maximum(c[0][..., 3:4], 1)
    m1, m2 = rgbw[..., :3] / n1, c[0][..., :3] / n2
    v1 = np.maximum(sq[..., :3] / n1 - m1 ** 2, 0) / n1
    v2 = np.maximum(c[1][..., :3] / n2 - m2 ** 2, 0) / n2
    z = (m1 - m2) / np.sqrt(v1 + v2 + (1e-5 * m2) ** 2 + 1e-12)
    assert (np.abs(z) < 5).mean() > 0.999
    assert abs(m1.mean() - m2.mean()) / m2.mean() < 5e-3
