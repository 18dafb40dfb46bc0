"""Guided volumetric path tracing (config C5: SD-tree guiding at medium and surface vertices with
one-sample MIS against the HG phase function / BSDF, plus guided free-flight sampling), CPU oracle
(oracle/orc_volpath.h VolLi, GuidedAccept).

The reference has no guiding code or fixture, so the guided arithmetic is
PARITY UNPINNED.  What pins it here is unbiasedness: a guided render must converge to the unguided
(reference) volpath estimator.  Checked on
  * the furnace (closed unit-emitter box filled with a non-absorbing heterogeneous medium: every
    pixel's expectation is exactly 1) for every guiding mode, including a large distance-guiding
    weight, so any weighting error in the tracking shows up as a biased mean;
  * the C5 smoke scene at a small resolution: guided vs unguided per-pixel z-test and image mean.
"""
import numpy as np
import pytest

from test_volume import _mean_z, _vol_cfg, _zimg, furnace_scene


def train_oracle(pg, O, osc, cfg, iters=4, spp0=4):
    """SD-tree training with the oracle volpath (records at medium + surface vertices)."""
    tree = O.OracleSDTree(osc)
    off = 0
    for it in range(iters):
        spp = spp0 << it
        _, _, st = O.render(osc, cfg, spp, sample_offset=off, record=True, sdtree=tree)
        off += spp
        assert st[3] > 0  # records were written
        tree.splat_pending()
        tree.refit(it, cfg)
    return tree, off


def _gcfg(pg, **kw):
    kw.setdefault("s_tree_threshold", 400.0)
    return _vol_cfg(pg, guiding=1, **kw)


@pytest.mark.parametrize("beta", [0.0, 0.5, 0.9])
def test_guided_furnace(pg, O, beta):
    sc = furnace_scene(pg)
    osc = O.OracleScene(pg.capi, sc)
    cfg = _gcfg(pg, distance_guiding=beta)
    tree, off = train_oracle(pg, O, osc, cfg, iters=3)
    rgbw, sq, st = O.render(osc, cfg, 64, sample_offset=off, sdtree=tree)
    n = rgbw[..., 3:]
    m = rgbw[..., :3].sum((0, 1)) / n.sum()
    var = (sq[..., :3].sum((0, 1)) / n.sum() - m ** 2) / n.sum()
    assert np.all(np.abs(m - 1) < 5 * np.sqrt(var) + 1e-3), (beta, m, np.sqrt(var))


def test_guided_records_cover_medium(pg, O):
    """Training records come from medium vertices too: inside the smoke box most of them."""
    sc = pg.scenes.smoke(24, 24, res=32)
    osc = O.OracleScene(pg.capi, sc)
    cfg = _gcfg(pg)
    tree = O.OracleSDTree(osc)
    O.render(osc, cfg, 8, record=True, sdtree=tree)
    rec = tree.take_records(pg.capi).view(np.float32).reshape(-1, 8)
    pos = rec[:, :3]
    inside = np.all(np.abs(pos) < 0.999, axis=1)
    assert len(rec) > 1000 and inside.mean() > 0.3
    assert np.all(np.isfinite(rec[:, 4])) and np.all(rec[:, 5] > 0)  # radiance, wo_pdf


@pytest.mark.parametrize("beta", [0.0, 0.5])
def test_guided_smoke_matches_unguided(pg, O, beta):
    sc = pg.scenes.smoke(24, 24, res=32)
    osc = O.OracleScene(pg.capi, sc)
    cfg = _gcfg(pg, distance_guiding=beta)
    tree, off = train_oracle(pg, O, osc, cfg)
    a = O.render(osc, cfg, 256, sample_offset=off, sdtree=tree)[:2]
    b = O.render(osc, _vol_cfg(pg, seed=21), 256)[:2]
    m1, m2, z = _zimg(a, b)
    assert (np.abs(z) < 5).mean() > 0.995
    assert abs(_mean_z(a, b)) < 5
