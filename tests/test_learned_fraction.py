"""Learned BSDF-sampling fraction per S-tree leaf (pg_config.bsdf_fraction_bound = PG_FRACTION_LEARNED,
after Mueller 2019's learned selection probability).  Parity unpinned against the
reference (it has no guiding code): these tests pin the oracle's restatement to the optimum it must
find, and tests/test_gpu_learned_fraction.py pins the GPU to the oracle bit for bit.

The cross-entropy objective sum_j w_j log2 q_a(w_j) over records drawn from a mixture q0 is maximised,
for records that fall either where only the BSDF samples (p_guide = 0) or only the guide samples
(p_bsdf = 0), at a* = F_bsdf / (F_bsdf + F_guide) -- the classic mixture-weight optimum."""
import numpy as np
import pytest

CANDIDATES = 0.05 + 0.1 * np.arange(10, dtype=np.float32)


def learned_cfg(pg, **kw):
    return pg.capi.default_config(guiding=1, s_tree_threshold=1e9, bsdf_fraction_bound=pg.capi.PG_FRACTION_LEARNED,
                                  **kw)


def synthetic_records(capi, pos, n_each, f_bsdf, f_guide, q0=0.5, radiance=1.0):
    """n_each records with p_guide = 0 (contribution f_bsdf) and n_each with p_bsdf = 0 (f_guide), all
    drawn with a0 = 0.5 so that q0 = 0.5: w = F / q0."""
    recs = (capi.pg_record * (2 * n_each))()
    for i in range(2 * n_each):
        r = recs[i]
        r.pos[0], r.pos[1], r.pos[2] = pos
        r.dir = (i * 2654435761) & 0xFFFFFFFF
        r.radiance = radiance
        r.wo_pdf = q0
        guide = i >= n_each
        r.product = (f_guide if guide else f_bsdf) / q0
        r.weight = 1.0 if guide else 0.0  # p_guide
    return np.frombuffer(recs, np.uint8).copy()


def tree_alphas(blob):
    """Per-D-tree learned fraction from the wire format (meta word 6)."""
    ns, nd = np.frombuffer(blob[48:56].tobytes(), np.uint32)
    meta = np.frombuffer(blob[64 + 8 * int(ns): 64 + 8 * int(ns) + 32 * int(nd)].tobytes(), np.uint32).reshape(-1, 8)
    return meta[:, 6].copy().view(np.float32)


@pytest.mark.parametrize("f_bsdf,f_guide", [(0.3, 0.7), (0.9, 0.1), (0.5, 0.5), (0.02, 0.98)])
def test_oracle_learns_mixture_optimum(pg, O, f_bsdf, f_guide):
    sc = pg.scenes.cornell(16, 16)
    tree = O.OracleSDTree(O.OracleScene(pg.capi, sc))
    cfg = learned_cfg(pg)
    lo, hi = sc.bounds()
    recs = synthetic_records(pg.capi, tuple(((lo + hi) / 2).tolist()), 200, f_bsdf, f_guide)
    tree.configure(cfg)
    tree.splat_bytes(recs)
    tree.refit(0, cfg)
    a = tree_alphas(tree.serialize())
    assert len(a) == 1
    obj = f_bsdf * np.log2(CANDIDATES) + f_guide * np.log2(1 - CANDIDATES)
    best = CANDIDATES[np.flatnonzero(obj >= obj.max() - 1e-6).max()]
    assert a[0] == np.float32(best), (a[0], best)


def test_too_few_records_keep_the_default(pg, O):
    sc = pg.scenes.cornell(16, 16)
    tree = O.OracleSDTree(O.OracleScene(pg.capi, sc))
    cfg = learned_cfg(pg)
    lo, hi = sc.bounds()
    tree.configure(cfg)
    tree.splat_bytes(synthetic_records(pg.capi, tuple(((lo + hi) / 2).tolist()), 31, 0.1, 0.9))  # 62 < 64
    tree.refit(0, cfg)
    assert tree_alphas(tree.serialize())[0] == 0.0  # not learned: the device uses bsdfSamplingFraction
    # fixed mode ignores the statistics altogether
    t2 = O.OracleSDTree(O.OracleScene(pg.capi, sc))
    fixed = pg.capi.default_config(guiding=1, s_tree_threshold=1e9)
    t2.configure(fixed)
    t2.splat_bytes(synthetic_records(pg.capi, tuple(((lo + hi) / 2).tolist()), 200, 0.1, 0.9))
    t2.refit(0, fixed)
    assert tree_alphas(t2.serialize())[0] == 0.0


def test_learned_training_is_unbiased_and_learns(pg, O):
    """A learned-fraction guided render of the Cornell box: every leaf that saw enough guided records
    holds a candidate fraction, and the guided image agrees with the unguided one (any per-leaf
    fraction fixed before the direction is sampled is unbiased)."""
    sc = pg.scenes.cornell(32, 32)
    osc = O.OracleScene(pg.capi, sc)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=300.0, bsdf_fraction_bound=pg.capi.PG_FRACTION_LEARNED)
    tree = O.OracleSDTree(osc)
    off = 0
    for it in range(4):
        O.render(osc, cfg, 2 ** it, off, record=True, sdtree=tree)
        off += 2 ** it
        tree.splat_pending()
        tree.refit(it, cfg)
    a = tree_alphas(tree.serialize())
    learned = a[a > 0]
    assert len(learned) > 0.5 * len(a)
    assert np.isin(learned, CANDIDATES).all()
    g = O.render(osc, cfg, 256, off, sdtree=tree)[:2]
    u = O.render(osc, pg.capi.default_config(), 256, 0)[:2]
    mg = g[0][..., :3].sum() / g[0][..., 3].sum()
    mu = u[0][..., :3].sum() / u[0][..., 3].sum()
    assert abs(mg / mu - 1) < 0.01
