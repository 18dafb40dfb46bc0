"""Inverse-variance combination of the guided integrator's iteration images (SURVEY.md §8f f2,
GuidedPathTracer sampleCombination = "inversevar"), host-side math on synthetic films."""
import numpy as np


def test_inverse_variance_combination_math(pg):
    """combine_inverse_variance: weights are 1 / image variance, normalised; constant images combine
    to the same constant; a noisier image gets proportionally less weight."""
    from mitsuba_path_guiding_amd.integrator import combine_inverse_variance

    def film(mean, var_of_sample, n, shape=(8, 8)):
        rgbw = np.zeros(shape + (4,), np.float32)
        sq = np.zeros(shape + (4,), np.float32)
        rgbw[..., :3] = mean * n
        rgbw[..., 3] = n
        sq[..., :3] = (var_of_sample + mean * mean) * n
        return rgbw, sq

    class O:
        combination_weights = None

    o = O()
    a, b = film(1.0, 4.0, 16), film(1.0, 1.0, 16)  # b has a quarter of a's variance
    rgbw, sq = combine_inverse_variance([a, b], o)
    assert np.allclose(o.combination_weights, [0.2, 0.8])
    assert np.allclose(rgbw[..., :3] / rgbw[..., 3:4], 1.0)
    c = film(2.0, 1.0, 16)
    rgbw, _ = combine_inverse_variance([b, c], o)
    assert np.allclose(rgbw[..., :3] / rgbw[..., 3:4], 1.5) and rgbw[0, 0, 3] == 32
