"""SD-tree oracle checks (PARITY UNPINNED against the reference — the snapshot has no guiding code;
these pin the restatement of Mueller et al. 2017 to its own mathematical properties and to the
committed golden vectors, which the GPU path must then reproduce bit for bit)."""
import os

import numpy as np
from scipy import stats

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _trained(pg, O, iters=3, res=32, thr=400.0):
    sc = pg.scenes.cornell(res, res)
    osc = O.OracleScene(pg.capi, sc)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=thr, bsdf_fraction_bound=pg.capi.PG_FRACTION_FIXED)
    tree = O.OracleSDTree(osc)
    for it in range(iters):
        O.render(osc, cfg, 2 ** it, 2 ** it - 1, record=True, sdtree=tree, nthreads=1)
        tree.splat_pending()
        tree.refit(it, cfg)
    return sc, osc, tree


def test_golden_vectors(pg, O):
    z = np.load(os.path.join(GOLDEN, "sdtree_cornell.npz"))
    sc, osc, tree = _trained(pg, O)
    assert np.array_equal(tree.serialize(), z["blob"])
    assert np.array_equal(tree.pdf(z["pos"], z["dir"]), z["pdf"])
    d, p = tree.sample(z["pos"], z["u"])
    assert np.array_equal(p, z["sample_pdf"])
    assert np.array_equal(d, z["sample_dir"])


def test_serialize_roundtrip(pg, O):
    z = np.load(os.path.join(GOLDEN, "sdtree_cornell.npz"))
    sc = pg.scenes.cornell(32, 32)
    t2 = O.OracleSDTree(O.OracleScene(pg.capi, sc))
    t2.deserialize(z["blob"])
    assert np.array_equal(t2.serialize(), z["blob"])
    assert np.array_equal(t2.pdf(z["pos"], z["dir"]), z["pdf"])


def test_pdf_normalized_and_sampling_matches(pg, O):
    """Each D-tree's pdf integrates to 1 over the sphere; sampled directions follow it (chi-square
    over a 16x16 grid of the canonical square, where pdf is piecewise constant per quadtree leaf)."""
    sc, osc, tree = _trained(pg, O)
    lo, hi = sc.bounds()
    rng = np.random.default_rng(9)
    for k in range(4):
        p = (lo + (hi - lo) * rng.random(3)).astype(np.float32)
        n = 256
        uu = (np.arange(n) + 0.5) / n
        U, V = np.meshgrid(uu, uu, indexing="ij")
        cos_t = 2 * U - 1
        phi = 2 * np.pi * V
        s = np.sqrt(1 - cos_t ** 2)
        d = np.stack([s * np.cos(phi), s * np.sin(phi), cos_t], -1).reshape(-1, 3).astype(np.float32)
        pdf = tree.pdf(np.tile(p, (len(d), 1)), d)
        integral = pdf.sum() * 4 * np.pi / len(d)  # the canonical map has constant Jacobian 4 pi
        assert abs(integral - 1) < 2e-3, integral
        m = 200_000
        dirs, spdf = tree.sample(np.tile(p, (m, 1)), rng.random((m, 2)).astype(np.float32))
        assert np.all(spdf > 0)
        cu = (dirs[:, 2] + 1) / 2
        cv = np.mod(np.arctan2(dirs[:, 1], dirs[:, 0]), 2 * np.pi) / (2 * np.pi)
        obs, _, _ = np.histogram2d(cu, cv, bins=16, range=[[0, 1], [0, 1]])
        exp = pdf.reshape(16, 16, 16, 16).transpose(0, 2, 1, 3).reshape(16, 16, -1).sum(-1)
        exp = exp * 4 * np.pi / len(d) * m
        keep = exp > 5
        chi = ((obs[keep] - exp[keep]) ** 2 / exp[keep]).sum()
        assert stats.chi2.sf(chi, keep.sum() - 1) > 1e-4
        # the sampler's pdf equals the evaluated pdf of the sampled direction
        ev = tree.pdf(np.tile(p, (m, 1)), dirs)
        assert (np.abs(ev - spdf) <= 1e-4 * spdf).mean() > 0.999


def test_refinement_rules(pg, O):
    """S-tree splits only where record counts exceed c*sqrt(2^k); refit is deterministic and
    independent of record order (fixed-point splat)."""
    sc = pg.scenes.cornell(32, 32)
    osc = O.OracleScene(pg.capi, sc)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=1e9)
    t = O.OracleSDTree(osc)
    O.render(osc, cfg, 1, 0, record=True, sdtree=t, nthreads=1)
    recs = t.take_records(pg.capi)
    t.splat_bytes(recs)
    t.refit(0, cfg)
    blob = t.serialize()
    hdr = blob[:64].view(np.uint32)
    assert hdr[0] == 0x44534750 and hdr[2] == 1
    assert hdr[12] == 1  # huge threshold -> the S-tree stays a single leaf
    # shuffled records -> identical tree
    t2 = O.OracleSDTree(osc)
    r = recs.reshape(-1, 32)[np.random.default_rng(1).permutation(len(recs) // 32)].ravel()
    t2.splat_bytes(r)
    t2.refit(0, cfg)
    assert np.array_equal(t2.serialize(), blob)
    # small threshold -> the S-tree refines
    cfg2 = pg.capi.default_config(guiding=1, s_tree_threshold=50.0)
    t3 = O.OracleSDTree(osc)
    t3.splat_bytes(recs)
    t3.refit(0, cfg2)
    assert t3.serialize()[:64].view(np.uint32)[12] > 1


def test_fraction_bound_modes_unbiased(pg, O):
    """Every pg_config.bsdf_fraction_bound mode picks alpha per vertex independently of the sampled
    direction, so the guided image keeps the unguided expectation (per-pixel means pooled over the
    image; independent of the tree's quality)."""
    sc, osc, tree = _trained(pg, O)
    ref, rsq, _ = O.render(osc, pg.capi.default_config(), 512, 1 << 20, nthreads=8)
    n = ref[..., 3:4]
    m_ref = ref[..., :3].sum() / n.sum()
    var_ref = (rsq[..., :3].sum() / n.sum() - (ref[..., :3] / n) ** 2).clip(0).mean()
    for mode in (pg.capi.PG_FRACTION_FIXED, pg.capi.PG_FRACTION_ALBEDO, pg.capi.PG_FRACTION_THROUGHPUT):
        cfg = pg.capi.default_config(guiding=1, bsdf_fraction_bound=mode)
        g, gsq, _ = O.render(osc, cfg, 256, 7, sdtree=tree, nthreads=8)
        m = g[..., :3].sum() / g[..., 3].sum()
        assert abs(m - m_ref) / m_ref < 0.01, (mode, m, m_ref)
