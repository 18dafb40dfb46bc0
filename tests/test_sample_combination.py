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


def test_inverse_variance_weights_do_not_depend_on_the_shard(pg):
    """A tile shard holds only its pixels (the rest of its film is zero).  With the variance sums and
    pixel counts summed over ranks, every shard gets the single-rank weights and the union of the
    shards' combined images is the single-rank image."""
    from mitsuba_path_guiding_amd.integrator import combine_inverse_variance
    rng = np.random.default_rng(3)
    H, W = 16, 24

    def film(scale):
        n = rng.integers(4, 9, (H, W, 1)).astype(np.float32)
        x = rng.gamma(2.0, scale, (H, W, 3)).astype(np.float32)
        rgbw = np.concatenate([x * n, n], -1)
        sq = np.concatenate([(x * x + rng.random((H, W, 3)).astype(np.float32) * scale) * n, 0 * n], -1)
        return rgbw, sq

    films = [film(s) for s in (3.0, 1.0, 0.5)]

    class O:
        combination_weights = None

    full = O()
    ref, _ = combine_inverse_variance(films, full)
    tile = (np.arange(H)[:, None] // 8 + np.arange(W)[None, :] // 8) % 2  # two ranks, 8x8 tiles
    shards = [[(f[0] * (tile == r)[..., None], f[1] * (tile == r)[..., None]) for f in films] for r in (0, 1)]
    local = []
    for sh in shards:  # phase 1: each rank's local sums
        combine_inverse_variance(sh, O(), lambda x: local.append(x.copy()) or x)
    total = local[0] + local[1]
    out = np.zeros_like(ref)
    for r, sh in enumerate(shards):
        o = O()
        img, _ = combine_inverse_variance(sh, o, lambda x: total)
        assert np.allclose(o.combination_weights, full.combination_weights, rtol=1e-12)
        out += img * (tile == r)[..., None]
    assert np.allclose(out, ref, rtol=1e-6)
    # without the reduction a shard's weights differ from the single-rank ones
    o = O()
    combine_inverse_variance(shards[0], o)
    assert not np.allclose(o.combination_weights, full.combination_weights, rtol=1e-6)
