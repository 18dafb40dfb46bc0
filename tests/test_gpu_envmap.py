"""GPU parity of the environment emitter and the denoiser feature buffers,
through the C-ABI against the CPU oracle.

Tolerances: per-query fp32 results (sampled direction, pdf, value / pdf, radiance) within 1e-3
relative for >= 99.9 % of queries (device libm and FMA contraction); images per pixel |z| < 5 for
>= 99.9 % of pixel channels, with a 1e-5 relative floor under the spread (fp32 film sums), and the
image mean within 0.5 % (unguided) / 1 % (guided against the unguided oracle); the white furnace
within 0.5 % of its exact value; feature buffers: identical sample counts, albedo bit-exact and
normals within 1e-4 for >= 99.9 % of pixels (same camera jitter, same first hit).
"""
import numpy as np
import pytest

from test_envmap import _env_scene, _maps

pytestmark = pytest.mark.gpu


def make_dev(pg, scene, **cfg):
    from mitsuba_path_guiding_amd.integrator import Device
    d = Device(pg.capi.default_config(**cfg))
    d.upload(scene)
    return d


def _z(g, c):
    n1, n2 = np.maximum(g[0][..., 3:4], 1), np.maximum(c[0][..., 3:4], 1)
    m1, m2 = g[0][..., :3] / n1, c[0][..., :3] / n2
    v1 = np.maximum(g[1][..., :3] / n1 - m1 ** 2, 0) / n1
    v2 = np.maximum(c[1][..., :3] / n2 - m2 ** 2, 0) / n2
    return m1, m2, (m1 - m2) / np.sqrt(v1 + v2 + (1e-5 * m2) ** 2 + 1e-12)


@pytest.mark.parametrize("name", ["sky", "smooth"])
def test_envmap_query_parity(pg, O, name):
    sc = _env_scene(pg, _maps(pg)[name], to_world=pg.scenes.rot_x(40))
    dev = make_dev(pg, sc)
    osc = O.OracleScene(pg.capi, sc)
    rng = np.random.default_rng(5)
    u = rng.random((100_000, 2)).astype(np.float32)
    g, c = dev.envmap_query(0, u), osc.envmap_query(0, u)
    assert ((g[:, 3] > 0) == (c[:, 3] > 0)).mean() > 0.9999
    ok = (g[:, 3] > 0) & (c[:, 3] > 0)
    assert np.quantile(np.abs(g[ok, :3] - c[ok, :3]).max(1), 0.999) < 1e-4
    for a, b in ((g[ok, 3], c[ok, 3]), (g[ok, 4:7], c[ok, 4:7]), (g[ok, 7], c[ok, 7])):
        assert np.quantile(np.abs(a - b) / np.maximum(np.abs(b), 1e-6), 0.999) < 1e-3
    d = rng.normal(size=(100_000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gp, cp = dev.envmap_query(1, d), osc.envmap_query(1, d)
    assert np.quantile(np.abs(gp - cp) / np.maximum(cp, 1e-6), 0.999) < 1e-3
    ge, ce = dev.envmap_query(2, d), osc.envmap_query(2, d)
    assert np.quantile(np.abs(ge - ce) / np.maximum(np.abs(ce), 1e-6), 0.999) < 1e-3
    dev.close()


def test_envmap_white_furnace_gpu(pg, O):
    """Constant environment radiance 1 over a one-sided diffuse quad of albedo 0.5 (exact answer 0.5
    on the quad, 1 elsewhere), and the denoiser features of the same render."""
    sc = _env_scene(pg, np.ones((16, 32, 3), np.float32), albedo=0.5)
    dev = make_dev(pg, sc, aovs=1)
    dev.render_pass(256, 0)
    rgbw, sq = dev.read_film()
    alb, nrm = dev.read_aovs()
    m = rgbw[..., 0] / rgbw[..., 3]
    on = alb[..., 0] == 0.5 * alb[..., 3]
    off = alb[..., 0] == 0
    assert on.sum() > 200 and off.sum() > 100
    assert np.allclose(m[off], 1.0, atol=1e-5)
    assert np.allclose(nrm[off], [0, 0, -256, 0]) and np.allclose(nrm[on][:, 1], 256, rtol=1e-5)
    assert abs(m[on].mean() - 0.5) < 5e-3, m[on].mean()
    dev.close()


def test_image_parity_sky_unguided(pg, O):
    sc = pg.scenes.sky_courtyard(64, 48, env=pg.scenes.sky_envmap(128, 64, sun_radiance=20.0), area_light=True)
    spp = 256
    dev = make_dev(pg, sc)
    dev.render_pass(spp, 0)
    g = dev.read_film()
    dev.close()
    c = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(), spp)[:2]
    assert np.array_equal(g[0][..., 3], c[0][..., 3])
    m1, m2, z = _z(g, c)
    assert (np.abs(z) < 5).mean() > 0.999
    assert abs(m1.mean() - m2.mean()) / m2.mean() < 5e-3


def test_guided_sky_matches_unguided_oracle(pg, O):
    """Guided training + render under the envmap: training records carry escaped-path radiance, and
    the guided image converges to the unguided oracle's (guiding is unbiased)."""
    sc = pg.scenes.sky_courtyard(64, 48, env=pg.scenes.sky_envmap(128, 64, sun_radiance=20.0))
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    integ = GuidedPathTracer({"trainingIterations": 4, "sTreeThreshold": 400.0})
    integ.preprocess(sc)
    rgbw, sq = integ.render(256)
    st = integ.postprocess()
    assert st["records"] > 0 and st["stree_nodes"] > 1 and st["dtree_nodes"] > 100
    c = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(), 1024)[:2]
    m1, m2, z = _z((rgbw, sq), c)
    assert (np.abs(z) < 5).mean() > 0.995
    assert abs(m1.mean() - m2.mean()) / m2.mean() < 0.01


@pytest.mark.parametrize("scene", ["cornell", "sky"])
def test_aov_parity(pg, O, scene):
    S = pg.scenes
    sc = S.cornell(64, 64) if scene == "cornell" else S.sky_courtyard(64, 48)
    dev = make_dev(pg, sc, aovs=1)
    dev.render_pass(8, 0)
    dev.render_pass(8, 8)
    ga, gn = dev.read_aovs()
    ca, cn = O.OracleScene(pg.capi, sc).render_aovs(16)
    assert np.array_equal(ga[..., 3], ca[..., 3]) and (ga[..., 3] == 16).all()
    assert (np.abs(ga - ca).max(-1) <= 1e-6 * 16).mean() > 0.999
    assert (np.abs(gn - cn).max(-1) <= 1e-4 * 16).mean() > 0.999
    dev.reset_film()
    assert not dev.read_aovs()[0].any()
    dev.close()


def test_envmap_and_aov_errors(pg):
    from mitsuba_path_guiding_amd.integrator import Device, PGError
    with pytest.raises(PGError):
        Device(pg.capi.default_config(aovs=1, integrator=pg.capi.PG_INTEGRATOR_VOLPATH))
    sc = _env_scene(pg, np.ones((4, 8, 3), np.float32))
    d = Device(pg.capi.default_config(integrator=pg.capi.PG_INTEGRATOR_VOLPATH))
    with pytest.raises(PGError, match="environment"):
        d.upload(sc)
    d.close()
    d = make_dev(pg, sc)
    with pytest.raises(PGError, match="aovs"):
        d.read_aovs()
    d.close()
    black = _env_scene(pg, np.zeros((4, 8, 3), np.float32))
    d = Device(pg.capi.default_config())
    with pytest.raises(PGError, match="black"):
        d.upload(black)
    d.close()
    plain = pg.scenes.cornell(16, 16)
    d = make_dev(pg, plain)
    with pytest.raises(PGError, match="no environment"):
        d.envmap_query(1, np.zeros((1, 3), np.float32))
    d.close()
