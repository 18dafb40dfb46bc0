"""Glossy prior on the BSDF-sampling fraction (pg_config.glossy_prior; BSDF::getGlossySamplingRate,
bsdf.h:365-381, roughplastic.cpp:323-345): a vertex whose BSDF is all glossy (roughconductor,
roughdielectric) is not guided, a roughplastic vertex samples its BSDF with probability
r + (1 - r) alpha, and only r = 0 vertices feed the learned-fraction statistics.  Oracle side; the
GPU side is tests/test_gpu_glossy_prior.py.  Parity unpinned against the reference (it has no guiding)."""
import numpy as np


def glossy_cornell(pg, w=32, h=32):
    """The Cornell box with every surface (the emitter's too) a rough conductor: with the prior no
    vertex is guided, so a guided render must equal the unguided one bit for bit."""
    S = pg.scenes
    sc = S.cornell(w, h)
    for i in range(len(sc.materials)):
        sc.materials[i] = S.material("roughconductor", conductor="Al", alpha=0.3, distribution="ggx")
    return sc.finalize()  # rebuild the descriptor's material array


def trained_tree(pg, O, osc, cfg, iters=3):
    tree = O.OracleSDTree(osc)
    off = 0
    for it in range(iters):
        O.render(osc, cfg, 2 ** it, off, record=True, sdtree=tree)
        off += 2 ** it
        tree.splat_pending()
        tree.refit(it, cfg)
    return tree, off


def test_all_glossy_scene_is_not_guided(pg, O):
    sc = glossy_cornell(pg)
    osc = O.OracleScene(pg.capi, sc)
    train = pg.capi.default_config(guiding=1, s_tree_threshold=300.0)
    tree, off = trained_tree(pg, O, osc, train)
    on = pg.capi.default_config(guiding=1, s_tree_threshold=300.0, glossy_prior=1)
    g = O.render(osc, on, 16, off, sdtree=tree)[:2]
    u = O.render(osc, pg.capi.default_config(), 16, off)[:2]
    assert np.array_equal(g[0], u[0]) and np.array_equal(g[1], u[1])
    off_prior = O.render(osc, train, 16, off, sdtree=tree)[:2]
    assert not np.array_equal(off_prior[0], u[0])  # without the prior these vertices are guided


def test_prior_render_unbiased_and_stats_exclude_glossy(pg, O):
    S = pg.scenes
    sc = S.cornell(32, 32, short_material=S.material("roughconductor", conductor="Cu", alpha=0.05, distribution="ggx"),
                   tall_material=S.material("roughplastic", alpha=0.2, distribution="ggx",
                                            diffuse_reflectance=(0.5, 0.4, 0.3)))
    osc = O.OracleScene(pg.capi, sc)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=300.0, glossy_prior=1,
                                 bsdf_fraction_bound=pg.capi.PG_FRACTION_LEARNED)
    tree, off = trained_tree(pg, O, osc, cfg)
    g = O.render(osc, cfg, 256, off, sdtree=tree)[:2]
    u = O.render(osc, pg.capi.default_config(), 256, 0)[:2]
    mg = g[0][..., :3].sum() / g[0][..., 3].sum()
    mu = u[0][..., :3].sum() / u[0][..., 3].sum()
    assert abs(mg / mu - 1) < 0.01
    # records of a recording pass: with the prior fewer of them carry p_guide (glossy / roughplastic
    # vertices are excluded from the learned statistics)
    counts = []
    for prior in (0, 1):
        c2 = pg.capi.default_config(guiding=1, s_tree_threshold=300.0, glossy_prior=prior,
                                    bsdf_fraction_bound=pg.capi.PG_FRACTION_LEARNED)
        O.render(osc, c2, 4, off, record=True, sdtree=tree)
        recs = np.frombuffer(tree.take_records(pg.capi).tobytes(), np.float32).reshape(-1, 8)
        counts.append(((recs[:, 7] >= 0).sum(), len(recs)))
    (g0, n0), (g1, n1) = counts
    assert n0 > 1000 and n1 > 1000
    assert g1 / n1 < g0 / n0 - 0.05, counts
