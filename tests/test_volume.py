"""Volumetric path tracing: the CPU oracle's medium, phase function and
integrator restatement (oracle/orc_medium.h, oracle/orc_volpath.h) checked against the reference's
own test protocol and against closed forms.

  * HG phase function: the test_chisquare protocol (src/tests/test_chisquare.cpp:29-37,393-500) on
    the test_phase.xml entries hg g = 0.9 and g = -0.3, plus sample weight == eval / pdf.
  * Grid lookups: GridDataSource::lookupFloat (gridvolume.cpp:337-380) against an independent numpy
    trilinear restatement, including the x2 >= res rule on the upper faces.
  * Woodcock free flight / transmittance (heterogeneous.cpp:546-660) on a constant grid: the
    interaction distance is Exp(sigma) (KS test) and the 2-run delta-tracking estimator averages to
    exp(-sigma d).
  * The integrator: an absorbing slab in front of a light (pixel value = Le exp(-sigma d)); a
    furnace (camera inside a non-absorbing heterogeneous medium enclosed by unit emitters, so every
    pixel's expectation is exactly 1); the surface-only Cornell box through VolLi matches the
    surface path tracer; the lazy transmittance walk matches the reference's eager one.
No reference fixture pins full volumetric images (the reference ships none): beyond these closed
forms the integrator restatement is parity-unpinned, see DESIGN.md.
"""
import numpy as np
import pytest
from scipy import stats

from test_oracle_bsdf import _chi2

THETA_BINS, PHI_BINS = 10, 20


def _sph(T, P):
    return np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1)


@pytest.mark.parametrize("g", [0.9, -0.3])  # data/tests/test_phase.xml:11-20
def test_hg_chisquare(pg, O, g):
    rng = np.random.default_rng(7)
    n = 200_000
    level = 1 - (1 - 0.0025) ** (1.0 / 8)
    for j in range(4):
        wi = rng.normal(size=3)
        wi /= np.linalg.norm(wi)
        u = rng.random((n, 2)).astype(np.float32)
        out = O.hg_query(pg.capi, g, np.tile(wi, (n, 1)), u)
        wo = out[:, :3]
        assert np.allclose(np.linalg.norm(wo, axis=1), 1, atol=1e-5)
        th = np.arccos(np.clip(wo[:, 2], -1, 1))
        ph = np.mod(np.arctan2(wo[:, 1], wo[:, 0]), 2 * np.pi)
        sub = 30
        dth, dph = np.pi / THETA_BINS / sub, 2 * np.pi / PHI_BINS / sub
        T, P = np.meshgrid((np.arange(THETA_BINS * sub) + 0.5) * dth, (np.arange(PHI_BINS * sub) + 0.5) * dph,
                           indexing="ij")
        d = _sph(T, P).reshape(-1, 3).astype(np.float32)
        ev = O.hg_query(pg.capi, g, np.tile(wi, (len(d), 1)), np.zeros((len(d), 2), np.float32), d)[:, 4]
        exp = (ev.reshape(T.shape) * np.sin(T) * dth * dph).reshape(THETA_BINS, sub, PHI_BINS, sub).sum((1, 3))
        assert abs(exp.sum() - 1) < 2e-3  # the phase function integrates to one
        obs, _, _ = np.histogram2d(th, ph, bins=[np.linspace(0, np.pi, THETA_BINS + 1),
                                                 np.linspace(0, 2 * np.pi, PHI_BINS + 1)])
        assert _chi2(obs, exp * n) > level, (g, j)
        # weight 1 = eval / pdf: the returned pdf is eval at the sampled direction
        chk = O.hg_query(pg.capi, g, np.tile(wi, (1000, 1)), np.zeros((1000, 2), np.float32), wo[:1000])[:, 4]
        assert np.allclose(chk, out[:1000, 3], rtol=1e-5)


def _const_medium_scene(pg, density, scale, albedo=0.0, res=8, lo=(-1, -1, -1), hi=(1, 1, 1)):
    S = pg.scenes
    s = S.Scene()
    nullm = s.add_material(S.material("null"))
    dens = np.full((res, res, res), density, np.float32) if np.isscalar(density) else density
    m = s.add_medium(dens, lo, hi, scale, (albedo,) * 3, 0.0)
    V, F = S.box(lo, hi)
    s.add_mesh(V, F, material=nullm, interior=m)
    s.set_camera((0, 0, 5), (0, 0, 0), (0, 1, 0), 30.0, 8, 8)
    return s.finalize()


def test_grid_lookup_kat(pg, O):
    rng = np.random.default_rng(3)
    res = (5, 7, 6)  # x, y, z
    dens = rng.random((res[2], res[1], res[0])).astype(np.float32)
    sc = _const_medium_scene(pg, dens, 1.0, lo=(-1, -2, 0), hi=(2, 1, 3))
    osc = O.OracleScene(pg.capi, sc)
    lo, hi = np.array([-1, -2, 0], np.float32), np.array([2, 1, 3], np.float32)
    p = lo + (hi - lo) * rng.uniform(-0.1, 1.1, size=(20000, 3)).astype(np.float32)
    p[:50, 0] = hi[0]  # on the upper x face: x2 == res -> 0 (gridvolume.cpp:344-346)
    got = osc.medium_lookup(0, p)
    # independent restatement: world -> grid (res - 1) / extent, trilinear over the 8 corners
    s = (np.array(res, np.float32) - 1) / (hi - lo)
    gp = p * s + s * -lo
    i0 = np.floor(gp).astype(np.int64)
    f = gp - i0
    inside = np.all((i0 >= 0) & (i0 + 1 < np.array(res)), axis=1)
    want = np.zeros(len(p), np.float64)
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                w = np.where(dx, f[:, 0], 1 - f[:, 0]) * np.where(dy, f[:, 1], 1 - f[:, 1]) * \
                    np.where(dz, f[:, 2], 1 - f[:, 2])
                ii = np.clip(i0 + [dx, dy, dz], 0, np.array(res) - 1)
                want += w * dens[ii[:, 2], ii[:, 1], ii[:, 0]]
    want[~inside] = 0
    assert np.all(got[:50] == 0)
    assert np.allclose(got, want, atol=2e-6)
    assert inside.mean() > 0.5


def test_woodcock_free_flight_and_transmittance(pg, O):
    sigma = 3.0  # density 0.5 * scale 6
    sc = _const_medium_scene(pg, 0.5, 6.0)
    osc = O.OracleScene(pg.capi, sc)
    n = 40000
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = (-1.5, 0.1, 0.2)
    rays[:, 4:7] = (1, 0, 0)
    rays[:, 3] = 0.0
    rays[:, 7] = np.inf
    keys = np.stack([np.arange(n, dtype=np.uint32) * 7919 + 11, np.full(n, 3, np.uint32)], 1)
    out = osc.medium_sample(0, rays, keys)
    hit = out[:, 0] > 0.5
    # entry at t = 0.5; the box is 2 long: P(interaction) = 1 - exp(-2 sigma), distance ~ Exp(sigma)
    p = 1 - np.exp(-2 * sigma)
    assert abs(hit.mean() - p) < 5 * np.sqrt(p * (1 - p) / n)
    d = out[hit, 1] - 0.5
    trunc = stats.truncexpon(b=2 * sigma, scale=1 / sigma)
    assert stats.kstest(d, trunc.cdf).pvalue > 1e-3
    # draws: 2 per tentative collision (distance + acceptance), +1 for the final distance of a miss;
    # the majorant is scale * 1 = 6, so each tentative collision is accepted with probability 1/2
    k = out[:, 2]
    assert np.all(k[hit] % 2 == 0) and np.all(k[~hit] % 2 == 1)
    assert abs((k[hit] / 2).mean() - 2.0) < 0.1  # ~ Geometric(1/2) trials, truncated at the exit
    # 2-run delta-tracking transmittance over a 1.2-long segment inside the box
    rays[:, 0:3] = (-0.6, 0.1, 0.2)
    rays[:, 7] = 1.2
    tr = osc.medium_sample(0, rays, keys, transmittance=True)[:, 0]
    assert set(np.unique(tr)) <= {0.0, 0.5, 1.0}
    want = np.exp(-sigma * 1.2)
    se = np.sqrt(want * (1 - want) / (2 * n))
    assert abs(tr.mean() - want) < 5 * se
    # a ray missing the density box: transmittance 1 without any draw, no interaction
    miss = rays[:10].copy()
    miss[:, 0:3] = (-1.5, 3.0, 0.0)
    assert np.all(osc.medium_sample(0, miss, keys[:10], transmittance=True)[:, :2] == [1.0, 0.0])


def test_majorant_grid_matches_global(pg, O):
    """Delta tracking against the majorant grid (PG_MAJORANT_GRID) samples the same free-flight
    distribution and transmittance as the reference's single majorant, with fewer draws."""
    sc = pg.scenes.smoke(8, 8, res=40)
    osc = O.OracleScene(pg.capi, sc)
    rng = np.random.default_rng(5)
    n = 60000
    rays = np.zeros((n, 8), np.float32)
    o = rng.uniform(-1.4, 1.4, size=(n, 3))
    tgt = rng.uniform(-0.5, 0.5, size=(n, 3))
    d = tgt - o
    rays[:, 0:3] = o
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = np.inf
    keys = np.stack([np.arange(n, dtype=np.uint32), np.full(n, 9, np.uint32)], 1)
    a = osc.medium_sample(0, rays, keys)
    b = osc.medium_sample(0, rays, keys, grid=True)
    pa, pb = a[:, 0].mean(), b[:, 0].mean()
    se = np.sqrt(pa * (1 - pa) / n + pb * (1 - pb) / n)
    assert abs(pa - pb) < 5 * se
    ha, hb = a[:, 0] > 0.5, b[:, 0] > 0.5
    assert stats.ks_2samp(a[ha, 1], b[hb, 1]).pvalue > 1e-3
    # empty space is skipped: 16^3-voxel cells (pg_layout.h PG_MAJORANT_CELL) draw ~0.7x the global
    # majorant's numbers here (8^3 cells: ~0.5x, but twice the DDA steps)
    assert b[:, 2].mean() < 0.8 * a[:, 2].mean()
    ta = osc.medium_sample(0, rays, keys, transmittance=True)[:, 0]
    tb = osc.medium_sample(0, rays, keys, transmittance=True, grid=True)[:, 0]
    se = np.sqrt(ta.var() / n + tb.var() / n)
    assert abs(ta.mean() - tb.mean()) < 5 * se


def test_volpath_majorant_modes_agree(pg, O):
    sc = pg.scenes.smoke(24, 24, res=32)
    osc = O.OracleScene(pg.capi, sc)
    a = O.render(osc, _vol_cfg(pg, volume_majorant=pg.capi.PG_MAJORANT_GLOBAL), 128)[:2]
    b = O.render(osc, _vol_cfg(pg, seed=11), 128)[:2]
    m1, m2, z = _zimg(a, b)
    assert (np.abs(z) < 5).mean() > 0.995
    assert abs(_mean_z(a, b)) < 5


def _vol_cfg(pg, **kw):
    return pg.capi.default_config(integrator=pg.capi.PG_INTEGRATOR_VOLPATH, **kw)


def absorber_scene(pg, sigma, le=(4.0, 3.0, 2.0)):
    """Camera -> absorbing medium slab (null-bounded box, albedo 0) -> emitter quad filling the view."""
    S = pg.scenes
    s = S.Scene()
    nullm = s.add_material(S.material("null"))
    black = s.add_material(S.material("diffuse", reflectance=(0, 0, 0)))
    m = s.add_medium(np.ones((4, 4, 4), np.float32), (-2, -2, -0.5), (2, 2, 0.5), sigma, (0.0, 0.0, 0.0), 0.3)
    V, F = S.box((-2, -2, -0.5), (2, 2, 0.5))
    s.add_mesh(V, F, material=nullm, interior=m)
    V, F = S.quad((-3, -3, -2), (3, -3, -2), (3, 3, -2), (-3, 3, -2), facing=(0, 0, 1))
    s.add_mesh(V, F, material=black, radiance=le)
    s.set_camera((0, 0, 6), (0, 0, 0), (0, 1, 0), 2.0, 16, 16)
    return s.finalize()


def test_absorbing_slab(pg, O):
    sigma, le = 0.9, np.array([4.0, 3.0, 2.0])
    sc = absorber_scene(pg, sigma, tuple(le))
    spp = 64
    rgbw, sq, st = O.render(O.OracleScene(pg.capi, sc), _vol_cfg(pg), spp)
    img = rgbw[..., :3] / rgbw[..., 3:]
    # every path crosses 1.0 of medium (to within 1.6e-4 at this field of view): a camera sample
    # sees Le with probability exp(-sigma) and 0 otherwise
    p = np.exp(-sigma)
    frac = img.reshape(-1, 3) / le
    n = 16 * 16 * spp
    assert abs(frac.mean() - p) < 5 * np.sqrt(p * (1 - p) / n)
    assert st[0] == n


def furnace_scene(pg, res=24, seed=3):
    """Camera inside a closed box of unit inward-facing emitters (black BSDF) filled with a
    heterogeneous, non-absorbing (albedo 1) medium: radiance is 1 everywhere, for any density."""
    S = pg.scenes
    s = S.Scene()
    black = s.add_material(S.material("diffuse", reflectance=(0, 0, 0)))
    dens = S.fbm_density(res, seed)
    m = s.add_medium(dens, (-1, -1, -1), (1, 1, 1), 6.0, (1.0, 1.0, 1.0), 0.6)
    V, F = S.box((-1.2, -1.2, -1.2), (1.2, 1.2, 1.2), inward=True)
    for k in range(6):  # one emitter per wall
        s.add_mesh(V[4 * k:4 * k + 4], F[2 * k:2 * k + 2] - 4 * k, material=black, radiance=(1.0, 1.0, 1.0))
    s.set_camera((0.2, -0.1, 0.9), (0.0, 0.0, 0.0), (0, 1, 0), 70.0, 16, 16)
    s.camera_medium = m
    return s.finalize()


@pytest.mark.parametrize("eager", [False, True])
def test_furnace(pg, O, eager):
    sc = furnace_scene(pg)
    O.set_volpath_eager(pg.capi, eager)
    try:
        rgbw, sq, st = O.render(O.OracleScene(pg.capi, sc), _vol_cfg(pg), 64)
    finally:
        O.set_volpath_eager(pg.capi, False)
    n = rgbw[..., 3:]
    m = rgbw[..., :3].sum((0, 1)) / n.sum()
    var = (sq[..., :3].sum((0, 1)) / n.sum() - m ** 2) / n.sum()
    assert np.all(np.abs(m - 1) < 5 * np.sqrt(var) + 1e-3), (m, np.sqrt(var))
    assert st[1] > st[0] * 2  # paths scatter


def _zimg(a, b):
    n1, n2 = np.maximum(a[0][..., 3:], 1), np.maximum(b[0][..., 3:], 1)
    m1, m2 = a[0][..., :3] / n1, b[0][..., :3] / n2
    v1 = np.maximum(a[1][..., :3] / n1 - m1 ** 2, 0) / n1
    v2 = np.maximum(b[1][..., :3] / n2 - m2 ** 2, 0) / n2
    return m1, m2, (m1 - m2) / np.sqrt(v1 + v2 + 1e-12)


def _mean_z(a, b):
    """z-score of the difference of the two images' overall means (per-path variance from sumsq)."""
    def ms(x):
        n = x[0][..., 3].sum()
        m = x[0][..., :3].sum() / n / 3
        return m, (x[1][..., :3].sum() / n / 3 - m * m) / n
    (m1, v1), (m2, v2) = ms(a), ms(b)
    return (m1 - m2) / np.sqrt(v1 + v2)


def test_volpath_surface_only_matches_path(pg, O):
    """Without media VolLi's surface branch is the path tracer's Li (different random streams)."""
    sc = pg.scenes.cornell(24, 24)
    osc = O.OracleScene(pg.capi, sc)
    a = O.render(osc, pg.capi.default_config(), 256)[:2]
    b = O.render(osc, _vol_cfg(pg, seed=99), 256)[:2]
    m1, m2, z = _zimg(a, b)
    assert (np.abs(z) < 5).mean() > 0.998
    assert abs(m1.mean() - m2.mean()) / m2.mean() < 0.01


def test_lazy_walk_matches_eager_on_smoke(pg, O):
    sc = pg.scenes.smoke(24, 24, res=32)
    osc = O.OracleScene(pg.capi, sc)
    a = O.render(osc, _vol_cfg(pg), 128)[:2]
    O.set_volpath_eager(pg.capi, True)
    try:
        b = O.render(osc, _vol_cfg(pg, seed=5), 128)[:2]
    finally:
        O.set_volpath_eager(pg.capi, False)
    m1, m2, z = _zimg(a, b)
    assert (np.abs(z) < 5).mean() > 0.995
    assert abs(_mean_z(a, b)) < 5
