"""GPU: the guided integrator's inverse-variance combination of iteration images (sampleCombination
= "inversevar") against "discard" on the Cornell box: same final render, the combination adds the
31 training spp with weights that favour the better-guided iterations.  Checked: weights normalised
with the final image weighted most, the combined image unbiased against a 2048-spp oracle (mean
within 1 %), and its MSE against that reference not above the discard image's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_inverse_variance_combination(pg, O):
    sc = pg.scenes.cornell(64, 64)
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    imgs = {}
    for mode in ("discard", "inversevar"):
        g = GuidedPathTracer({"trainingIterations": 5, "sTreeThreshold": 400.0, "sampleCombination": mode})
        g.preprocess(sc)
        rgbw, _ = g.render(32)
        imgs[mode] = rgbw[..., :3] / np.maximum(rgbw[..., 3:4], 1)
        if mode == "inversevar":
            w = g.combination_weights
            assert len(w) == 6 and abs(sum(w) - 1) < 1e-6 and int(np.argmax(w)) == 5, w
            assert rgbw[..., 3].min() == 32 + 31
        g.postprocess()
    ref = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(seed=4242), 2048)[0]
    ref = ref[..., :3] / ref[..., 3:4]
    mse = {k: float(np.mean((v - ref) ** 2)) for k, v in imgs.items()}
    assert abs(imgs["inversevar"].mean() - ref.mean()) / ref.mean() < 0.01
    assert mse["inversevar"] <= mse["discard"], mse
