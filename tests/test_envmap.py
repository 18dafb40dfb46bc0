"""Environment emitter (src/emitters/envmap.cpp) in the CPU oracle — SURVEY.md §8f f4.

* Emitter chi-square: the reference's test03_EmitterDirect protocol (src/tests/test_chisquare.cpp:
  344-389,577-620: sampleDirect from the origin vs pdfDirect, 10 theta x 20 phi bins, significance
  0.25 %) on the configuration of data/tests/test_emitter.xml (envmap rotated 40 degrees about x).
  The fixture's data/tests/envmap.exr is PIZ-compressed and no EXR decoder is available here, so the
  image is the seeded procedural sky of scenes.sky_envmap (HDR, with a sun disk) plus a smooth
  random map: parity of the image itself is unpinned, the sampling/pdf arithmetic is what the test
  checks.
* Half-precision texels (the MIP map's SpectrumHalf): a constant map evaluates to float16(value).
* White furnace under a constant environment: a one-sided diffuse quad of albedo rho seen from
  above reflects exactly rho (every reflected direction escapes), background pixels see the map.
* NEE-only / BSDF-only / MIS estimators agree on the sky courtyard (useNee on vs off).
"""
import numpy as np
import pytest

from test_oracle_bsdf import _chi2

THETA_BINS, PHI_BINS = 10, 20
SIGNIFICANCE = 0.0025


def _env_scene(pg, rgb, to_world=None, albedo=0.5, res=(32, 32)):
    S = pg.scenes
    s = S.Scene()
    m = s.add_material(S.material("diffuse", reflectance=(albedo, albedo, albedo)))
    V, F = S.quad((-1, 0, -1), (1, 0, -1), (1, 0, 1), (-1, 0, 1), facing=(0, 1, 0))
    s.add_mesh(V, F, material=m)
    s.set_envmap(rgb, to_world=to_world)
    s.set_camera((0, 3, -0.01), (0, 0, 0), (0, 0, 1), 50.0, *res)
    return s.finalize()


def _maps(pg):
    rng = np.random.default_rng(3)
    smooth = np.abs(np.cumsum(np.cumsum(rng.normal(size=(48, 96, 3)), 0), 1)).astype(np.float32)
    smooth /= smooth.max()
    return {"sky": pg.scenes.sky_envmap(128, 64, sun_radiance=50.0), "smooth": smooth + 0.02}


def _bins_pdf(osc, sub=24):
    th = (np.arange(THETA_BINS * sub) + 0.5) * (np.pi / THETA_BINS / sub)
    ph = (np.arange(PHI_BINS * sub) + 0.5) * (2 * np.pi / PHI_BINS / sub)
    T, P = np.meshgrid(th, ph, indexing="ij")
    d = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1).reshape(-1, 3).astype(np.float32)
    pdf = osc.envmap_query(1, d).reshape(T.shape) * np.sin(T) * (np.pi / THETA_BINS / sub) * (2 * np.pi / PHI_BINS / sub)
    return pdf.reshape(THETA_BINS, sub, PHI_BINS, sub).sum((1, 3))


@pytest.mark.parametrize("name", ["sky", "smooth"])
def test_envmap_chisquare(pg, O, name):
    rgb = _maps(pg)[name]
    sc = _env_scene(pg, rgb, to_world=pg.scenes.rot_x(40))  # test_emitter.xml: <rotate x="1" angle="40"/>
    osc = O.OracleScene(pg.capi, sc)
    n = 200_000
    u = np.random.default_rng(11).random((n, 2)).astype(np.float32)
    out = osc.envmap_query(0, u)
    ok = out[:, 3] > 0
    assert ok.mean() > 0.999
    d = out[ok, :3]
    th = np.arccos(np.clip(d[:, 2], -1, 1))
    ph = np.mod(np.arctan2(d[:, 1], d[:, 0]), 2 * np.pi)
    obs, _, _ = np.histogram2d(th, ph, bins=[np.linspace(0, np.pi, THETA_BINS + 1),
                                              np.linspace(0, 2 * np.pi, PHI_BINS + 1)])
    exp = _bins_pdf(osc)
    assert abs(exp.sum() - 1) < 2e-3  # the pdf integrates to one over the sphere
    p = _chi2(obs, exp * ok.sum())
    assert p > SIGNIFICANCE, p
    # the sampler's pdf is pdfDirect(d), and its weight is evalEnvironment(d) / pdf
    pdf = osc.envmap_query(1, d)
    assert np.quantile(np.abs(pdf - out[ok, 3]) / out[ok, 3], 0.999) < 1e-3
    val = osc.envmap_query(2, d) / pdf[:, None]
    assert np.quantile(np.abs(val - out[ok, 4:7]) / np.maximum(np.abs(out[ok, 4:7]), 1e-6), 0.999) < 1e-3


def test_envmap_half_texels_and_rotation(pg, O):
    for c in (0.1, 1.0 / 3.0, 7.77, 1234.567, 3e-6):
        sc = _env_scene(pg, np.full((8, 16, 3), c, np.float32))
        osc = O.OracleScene(pg.capi, sc)
        d = np.random.default_rng(0).normal(size=(64, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        v = osc.envmap_query(2, d)
        assert np.allclose(v, np.float32(np.float16(c)), rtol=2e-6, atol=0), (c, v[:2])
    # a map bright only around local +Y (theta < 10 deg) rotated by 90 deg about x looks along world +Z
    rgb = np.zeros((64, 128, 3), np.float32)
    rgb[:4] = 1.0
    rgb += 1e-4
    osc = O.OracleScene(pg.capi, _env_scene(pg, rgb, to_world=pg.scenes.rot_x(90)))
    v = osc.envmap_query(2, np.array([[0, 0, 1], [0, 1, 0]], np.float32))
    assert v[0, 0] > 0.5 and v[1, 0] < 1e-2


def test_envmap_white_furnace(pg, O):
    """Constant environment radiance 1 over a one-sided diffuse quad (albedo 0.5): every pixel on the
    quad has expectation exactly 0.5 (NEE + BSDF sampling with MIS), every other pixel sees 1."""
    sc = _env_scene(pg, np.ones((16, 32, 3), np.float32), albedo=0.5)
    osc = O.OracleScene(pg.capi, sc)
    rgbw, sq, _ = O.render(osc, pg.capi.default_config(), 256)
    m = rgbw[..., 0] / rgbw[..., 3]
    alb, _ = osc.render_aovs(256)
    on = alb[..., 0] == 0.5 * alb[..., 3]  # every sample of the pixel hit the quad
    off = alb[..., 0] == 0
    assert on.sum() > 200 and off.sum() > 100
    assert np.allclose(m[off], 1.0, atol=1e-5)
    n = rgbw[..., 3][on]
    var = (sq[..., 0][on] / n - m[on] ** 2) / n
    z = (m[on].mean() - 0.5) / np.sqrt(var.sum()) * len(n)
    assert abs(z) < 5 and abs(m[on].mean() - 0.5) < 5e-3, (m[on].mean(), z)


def test_envmap_nee_vs_bsdf_sampling(pg, O):
    """useNee = false (BSDF sampling only, the env is hit by escaping rays) and useNee = true (NEE +
    MIS) estimate the same image of the sky courtyard."""
    sc = pg.scenes.sky_courtyard(48, 36, env=pg.scenes.sky_envmap(128, 64, sun_radiance=20.0))
    osc = O.OracleScene(pg.capi, sc)
    a = O.render(osc, pg.capi.default_config(), 512)[:2]
    b = O.render(osc, pg.capi.default_config(use_nee=0, seed=99), 2048)[:2]
    ma, mb = a[0][..., :3] / a[0][..., 3:4], b[0][..., :3] / b[0][..., 3:4]
    assert abs(ma.mean() - mb.mean()) / ma.mean() < 0.02, (ma.mean(), mb.mean())
    va = np.maximum(a[1][..., :3] / a[0][..., 3:4] - ma ** 2, 0) / a[0][..., 3:4]
    vb = np.maximum(b[1][..., :3] / b[0][..., 3:4] - mb ** 2, 0) / b[0][..., 3:4]
    # fp32 film sums put a floor under the spread of near-constant sky pixels
    z = (ma - mb) / np.sqrt(va + vb + (1e-5 * ma) ** 2 + 1e-12)
    assert (np.abs(z) < 5).mean() > 0.999


def test_envmap_desc_plumbing(pg):
    """The Python mirror hands the pg_envmap to the C-ABI scene description."""
    sc = _env_scene(pg, np.ones((4, 8, 3), np.float32))
    d = sc.desc()
    assert bool(d.envmap) and d.envmap.contents.width == 8 and d.envmap.contents.height == 4

