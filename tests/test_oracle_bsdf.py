"""Oracle BSDF checks, following the reference's test_chisquare protocol
(src/tests/test_chisquare.cpp:29-37,393-500 with data/tests/test_bsdf.xml): for each BSDF and a set
of incident directions, sample the BSDF, histogram the outgoing directions in 10 theta x 20 phi bins,
compare against the pdf integrated over each bin with a chi-square test at significance 0.25 %
(Sidak-corrected over all tests), and check that every sample weight equals eval/pdf within 1e-2
(ERROR_REQ for single precision).  Delta lobes are checked for their discrete probabilities.

The test_bsdf.xml entries covered are those of the configs' BSDF set (diffuse, twosided, conductor,
dielectric water/air, roughdielectric beckmann/ggx alpha .3, roughconductor beckmann alpha .3, an
anisotropic rough conductor (GGX 0.1/0.3 in place of the unsupported Ashikhmin-Shirley), plastic,
roughplastic beckmann alpha .7 plus a GGX one).
"""
import numpy as np
import pytest
from scipy import stats

THETA_BINS, PHI_BINS = 10, 20
N_SAMPLES = 120_000
N_WI = 4
SIGNIFICANCE = 0.0025


def materials(S):
    return [
        ("diffuse", S.material("diffuse", reflectance=(0.5, 0.5, 0.5)), False),
        ("twosided_diffuse", S.material("diffuse", reflectance=(0.5, 0.5, 0.5), twosided=True), True),
        ("plastic", S.material("plastic", diffuse_reflectance=(0.5, 0.5, 0.5)), False),
        ("roughconductor_beckmann", S.material("roughconductor", conductor="Cu", alpha=0.3), False),
        ("roughconductor_ggx_aniso", S.material("roughconductor", conductor="Au", alpha_u=0.1, alpha_v=0.3,
                                                distribution="ggx"), False),
        ("roughconductor_ggx_all", S.material("roughconductor", conductor="Al", alpha=0.3, distribution="ggx",
                                              sample_visible=False), False),
        ("roughdielectric_beckmann", S.material("roughdielectric", int_ior=1.5, ext_ior=1.0, alpha=0.3), True),
        ("roughdielectric_ggx", S.material("roughdielectric", int_ior=1.5, ext_ior=1.0, alpha=0.3,
                                           distribution="ggx"), True),
        ("roughplastic_beckmann", S.material("roughplastic", alpha=0.7), False),  # test_bsdf.xml:133-136
        ("roughplastic_ggx", S.material("roughplastic", alpha=0.2, distribution="ggx",
                                        diffuse_reflectance=(0.5, 0.3, 0.2)), False),
    ]


def _bins_pdf(O, capi, mat, wi, sub=30):
    """pdf integrated over each (theta, phi) bin by a sub x sub midpoint rule (solid angle); sub=10
    under-resolves glossy lobes of alpha ~0.2 (false rejections), 30 does not."""
    th_edges = np.linspace(0, np.pi, THETA_BINS + 1)
    ph_edges = np.linspace(0, 2 * np.pi, PHI_BINS + 1)
    dth = np.pi / THETA_BINS / sub
    dph = 2 * np.pi / PHI_BINS / sub
    th = (np.arange(THETA_BINS * sub) + 0.5) * dth
    ph = (np.arange(PHI_BINS * sub) + 0.5) * dph
    T, P = np.meshgrid(th, ph, indexing="ij")
    d = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1).reshape(-1, 3)
    out = O.bsdf_query(capi, mat, np.tile(wi, (len(d), 1)), np.zeros((len(d), 3), np.float32), d)
    # integrate over the BSDF's support: roughdielectric.cpp's pdf() (:358-418) only checks the
    # incident side's masking, so it reports density where eval() is 0 and sample() never goes
    support = out[:, 8:11].sum(1) > 0
    pdf = (out[:, 11] * support).reshape(T.shape) * np.sin(T) * dth * dph
    return pdf.reshape(THETA_BINS, sub, PHI_BINS, sub).sum((1, 3)), th_edges, ph_edges


def _chi2(obs, exp):
    obs, exp = obs.ravel(), exp.ravel()
    order = np.argsort(exp)
    obs, exp = obs[order], exp[order]
    # pool the smallest expected bins until every pooled bin expects >= 5 samples
    po, pe = [], []
    ao = ae = 0.0
    for o, e in zip(obs, exp):
        ao += o
        ae += e
        if ae >= 5:
            po.append(ao)
            pe.append(ae)
            ao = ae = 0.0
    if ae > 0 or ao > 0:
        if pe:
            po[-1] += ao
            pe[-1] += ae
        else:
            po.append(ao)
            pe.append(ae)
    po, pe = np.array(po), np.array(pe)
    if len(po) < 2:
        return 1.0
    chi = np.sum((po - pe) ** 2 / pe)
    return float(stats.chi2.sf(chi, len(po) - 1))


@pytest.mark.parametrize("idx", range(10))
def test_chisquare(pg, O, idx):
    name, mat, both_sides = materials(pg.scenes)[idx]
    rng = np.random.default_rng(100 + idx)
    n_tests = 8 * N_WI
    level = 1 - (1 - SIGNIFICANCE) ** (1.0 / n_tests)
    for j in range(N_WI):
        wi = rng.normal(size=3)
        wi /= np.linalg.norm(wi)
        if not both_sides or j % 2 == 0:
            wi[2] = abs(wi[2]) + 0.05
            wi /= np.linalg.norm(wi)
        else:
            wi[2] = -abs(wi[2]) - 0.05
            wi /= np.linalg.norm(wi)
        u = rng.random((N_SAMPLES, 3)).astype(np.float32)
        out = O.bsdf_query(pg.capi, mat, np.tile(wi, (N_SAMPLES, 1)), u, None)
        typ = out[:, 7].astype(np.int64)
        smooth = (typ != 0) & ((typ & pg.capi.EDelta) == 0)
        wo = out[smooth, :3]
        th = np.arccos(np.clip(wo[:, 2], -1, 1))
        ph = np.mod(np.arctan2(wo[:, 1], wo[:, 0]), 2 * np.pi)
        exp_frac, te, pe = _bins_pdf(O, pg.capi, mat, wi.astype(np.float32))
        obs, _, _ = np.histogram2d(th, ph, bins=[te, pe])
        p = _chi2(obs, exp_frac * N_SAMPLES)
        assert p > level, (name, j, p)
        # sample weight == eval / pdf (relative 1e-2, single precision ERROR_REQ)
        chk = O.bsdf_query(pg.capi, mat, np.tile(wi, (len(wo), 1)), np.zeros((len(wo), 3), np.float32), wo)
        ev, pdf = chk[:, 8:11], chk[:, 11]
        wt = out[smooth, 4:7]
        ok = pdf > 1e-3
        rel = np.abs(wt[ok] - ev[ok] / pdf[ok, None]) / np.maximum(np.abs(ev[ok] / pdf[ok, None]), 1e-6)
        assert np.quantile(rel, 0.999) < 1e-2, (name, j)
        # the sampler's own pdf equals pdf(wi, wo)
        sp = out[smooth, 3]
        relp = np.abs(sp[ok] - pdf[ok]) / pdf[ok]
        assert np.quantile(relp, 0.999) < 1e-2, (name, j)


def test_delta_probabilities(pg, O):
    """Discrete lobes: dielectric (water/air) reflects with probability F(cos theta_i); plastic picks
    its specular lobe with the documented probability; conductors reflect into the mirror direction."""
    S = pg.scenes
    water = S.material("dielectric", int_ior=1.333, ext_ior=1.000277)
    rng = np.random.default_rng(7)
    n = 200_000
    for cos_i in (0.95, 0.5, 0.1, -0.6):
        wi = np.array([np.sqrt(1 - cos_i ** 2), 0.0, cos_i], np.float32)
        out = O.bsdf_query(pg.capi, water, np.tile(wi, (n, 1)), rng.random((n, 3)).astype(np.float32))
        refl = (out[:, 7].astype(int) & pg.capi.EDeltaReflection) != 0
        eta = 1.333 / 1.000277
        # fresnelDielectricExt restated in numpy
        sc = 1 / eta if cos_i > 0 else eta
        ct2 = 1 - (1 - cos_i ** 2) * sc * sc
        if ct2 <= 0:
            F = 1.0
        else:
            ci, ct = abs(cos_i), np.sqrt(ct2)
            Rs = (ci - eta * ct) / (ci + eta * ct)
            Rp = (eta * ci - ct) / (eta * ci + ct)
            F = 0.5 * (Rs * Rs + Rp * Rp)
        assert abs(refl.mean() - F) < 5 * np.sqrt(F * (1 - F) / n) + 1e-4
        wo = out[refl, :3]
        assert np.allclose(wo, [-wi[0], -wi[1], wi[2]], atol=1e-6)
    cu = S.material("conductor", conductor="Cu")
    wi = np.array([0.6, 0.0, 0.8], np.float32)
    out = O.bsdf_query(pg.capi, cu, np.tile(wi, (10, 1)), rng.random((10, 3)).astype(np.float32))
    assert np.allclose(out[:, :3], [-0.6, 0.0, 0.8], atol=1e-6)
    assert np.all(out[:, 4:7] > 0) and np.all(out[:, 4:7] < 1)


def test_material_types(pg, O):
    """EBSDFType bits per model (include/mitsuba/render/bsdf.h:224-262, plugin configure())."""
    S, c = pg.scenes, pg.capi
    assert O.material_type(c, S.material("diffuse")) == c.EDiffuseReflection | c.EFrontSide
    assert O.material_type(c, S.material("diffuse", twosided=True)) == c.EDiffuseReflection | c.EFrontSide | c.EBackSide
    assert O.material_type(c, S.material("dielectric")) == c.EDelta | c.EFrontSide | c.EBackSide
    assert O.material_type(c, S.material("roughconductor")) == c.EGlossyReflection | c.EFrontSide
    assert O.material_type(c, S.material("plastic")) == c.EDeltaReflection | c.EDiffuseReflection | c.EFrontSide
    assert O.material_type(c, S.material("roughplastic", alpha=0.3)) == (c.EGlossyReflection | c.EDiffuseReflection
                                                                           | c.EFrontSide)
