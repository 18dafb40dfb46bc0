"""GPU parity of the integrator's own parameters (SURVEY.md §8b's XML properties): the HIP path against
the CPU oracle on the same counter-RNG streams, with every parameter the radiance loop branches on
taken off its default.

    maxDepth            progressive_path.cpp:149,175       pg_kernels.hip k_shade (depth exit), k_rays
    rrDepth             progressive_path.cpp:296-306       pg_kernels.hip k_shade (RR)
    strictNormals       progressive_path.cpp:176-177,206-207,237
    hideEmitters        progressive_path.cpp:153-154,168,257
    maxComponentValue   progressiveintegrator.cpp:274-277  pg_kernels.hip k_film
    useNee              progressive_path.cpp:193,280-282

and the volumetric loop's equivalents (progressive_volpath.cpp:98-374; pg_volpath.hip volMedium /
volSurface / volRR, oracle/orc_volpath.h).

Both sides draw the same numbers for the same (pixel, sample, dimension), so a pixel's mean differs only
where fp32 rounding flips a branch of some path.  Bar: equal per-pixel sample counts, and at least
99.9 % of pixels whose means agree to 1e-3 relative (the measured figure is printed).  Scenes: Cornell
(diffuse) and the ajar door (rough conductor, glass) for the surface path, the smoke grid and the
reference's test_bidir_2 slab for the volumetric path, a coarse smooth-shaded sphere scene for
strictNormals (shading normals up to ~25 degrees off the facets), and the sky courtyard for
hideEmitters with an environment emitter.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share

# one parameter off its default per case, plus two combinations
CASES = {
    "maxDepth1": dict(max_depth=1),
    "maxDepth2": dict(max_depth=2),
    "maxDepth4": dict(max_depth=4),
    "rrDepth1": dict(rr_depth=1),
    "rrDepth2": dict(rr_depth=2),
    "clamp0.5": dict(max_component_value=0.5),
    "clamp2": dict(max_component_value=2.0),
    "noNee": dict(use_nee=0),
    "hideEmitters": dict(hide_emitters=1),
    "hide+maxDepth2": dict(hide_emitters=1, max_depth=2),
    "strict": dict(strict_normals=1),
    "strict+rr1+noNee": dict(strict_normals=1, rr_depth=1, use_nee=0),
}


def smooth_spheres(pg, width=48, height=48):
    """An open box (diffuse walls, one area light) holding coarse uv-spheres with the exact sphere
    normals as shading normals: at 8 x 4 facets the shading normal is up to ~25 degrees off the
    geometric one, so strictNormals' three tests (progressive_path.cpp:176,206,237) decide often."""
    S = pg.scenes
    s = S.Scene()
    white = s.add_material(S.material("diffuse", reflectance=(0.7, 0.7, 0.7)))
    red = s.add_material(S.material("diffuse", reflectance=(0.6, 0.1, 0.1)))
    gold = s.add_material(S.material("roughconductor", conductor="Au", alpha=0.25, distribution="ggx"))
    plastic = s.add_material(S.material("roughplastic", alpha=0.3, distribution="ggx",
                                         diffuse_reflectance=(0.2, 0.4, 0.6)))
    glass = s.add_material(S.material("dielectric", int_ior=1.5, ext_ior=1.0))
    lm = s.add_material(S.material("diffuse", reflectance=(0, 0, 0)))
    for a, b, c, d, m in (((-2, 0, -2), (2, 0, -2), (2, 0, 2), (-2, 0, 2), white),      # floor
                          ((-2, 0, 2), (2, 0, 2), (2, 3, 2), (-2, 3, 2), white),         # back
                          ((-2, 0, -2), (-2, 0, 2), (-2, 3, 2), (-2, 3, -2), red),       # left
                          ((2, 0, -2), (2, 3, -2), (2, 3, 2), (2, 0, 2), white),         # right
                          ((-2, 3, -2), (-2, 3, 2), (2, 3, 2), (2, 3, -2), white)):      # ceiling
        ctr = np.mean([a, b, c, d], 0)
        V, F = S.quad(a, b, c, d, facing=np.array([0.0, 1.5, 0.0]) - ctr)
        s.add_mesh(V, F, material=m)
    V, F = S.quad((-0.5, 2.95, -0.5), (0.5, 2.95, -0.5), (0.5, 2.95, 0.5), (-0.5, 2.95, 0.5), facing=(0, -1, 0))
    s.add_mesh(V, F, material=lm, radiance=(10.0, 9.0, 7.0))
    for ctr, r, m in (((-0.9, 0.6, 0.3), 0.6, white), ((0.8, 0.5, 0.6), 0.5, gold),
                      ((0.1, 0.45, -0.8), 0.45, plastic), ((1.0, 1.6, -0.6), 0.35, glass)):
        V, F, N = S.uv_sphere(ctr, r, 8, 4)
        s.add_mesh(V, F, N, material=m)
    s.set_camera((0.0, 1.5, -5.5), (0.0, 1.2, 0.0), (0, 1, 0), 55.0, width, height)
    return s.finalize()


def _scene(pg, name):
    S = pg.scenes
    if name == "cornell":
        return S.cornell(48, 48), 32
    if name == "ajar":
        return S.ajar_door(96, 54), 16
    if name == "spheres":
        return smooth_spheres(pg), 32
    if name == "sky":
        return S.sky_courtyard(48, 36, env=S.sky_envmap(64, 32, sun_radiance=20.0)), 16
    if name == "smoke":
        return S.smoke(40, 40, res=48), 32
    if name == "bidir_2":
        from test_bidir_pin import bidir_scene
        return bidir_scene(pg, "bidir_2")[0], 64
    raise KeyError(name)


def _means(film):
    rgbw, sq = film
    n = np.maximum(rgbw[..., 3:4], 1)
    return rgbw[..., :3] / n


def same_stream_parity(pg, O, scene_name, params, volpath=False, guided_tree=None):
    """Render on the GPU and in the oracle with one configuration; returns (fraction of pixels within
    1e-3 relative, image-mean relative difference, GPU film)."""
    from mitsuba_path_guiding_amd.integrator import Device
    sc, spp = _scene(pg, scene_name)
    kw = dict(params)
    if volpath:
        kw["integrator"] = pg.capi.PG_INTEGRATOR_VOLPATH
    if guided_tree is not None:
        kw.update(guiding=1, s_tree_threshold=400.0)
    cfg = pg.capi.default_config(**kw)
    dev = Device(cfg)
    dev.upload(sc)
    off = 0
    osc = O.OracleScene(pg.capi, sc)
    tree = None
    if guided_tree is not None:
        blob, off = guided_tree
        dev.put_sdtree(blob)
        tree = O.OracleSDTree(osc)
        tree.deserialize(blob)
    dev.render_pass(spp, off)
    g = dev.read_film()
    dev.close()
    c = O.render(osc, cfg, spp, off, sdtree=tree, nthreads=THREADS)[:2]
    np.testing.assert_array_equal(g[0][..., 3], c[0][..., 3])  # same accepted samples per pixel
    mg, mc = _means(g), _means(c)
    close = np.abs(mg - mc).max(-1) <= 1e-3 * np.maximum(np.abs(mc).max(-1), 1e-3)
    denom = max(float(mc.mean()), 1e-12)
    return float(close.mean()), float(abs(mg.mean() - mc.mean()) / denom), (g, mc)


# (scene, case) pairs on which the parameter leaves the image unchanged (checked with the oracle): the
# ajar door's and the smoke's emitters are never seen directly, and no sample of the bidir_2 slab
# exceeds either clamp
INERT = {("ajar", "hideEmitters"), ("smoke", "hideEmitters"), ("bidir_2", "hideEmitters"),
         ("bidir_2", "clamp0.5"), ("bidir_2", "clamp2")}
_baseline = {}


def assert_parameter_took_effect(pg, scene_name, case, film, volpath=False):
    """The case's GPU film differs from the default configuration's (the parameter reached the kernels)."""
    from mitsuba_path_guiding_amd.integrator import Device
    key = (scene_name, volpath)
    if key not in _baseline:
        sc, spp = _scene(pg, scene_name)
        dev = Device(pg.capi.default_config(**({"integrator": pg.capi.PG_INTEGRATOR_VOLPATH} if volpath else {})))
        dev.upload(sc)
        dev.render_pass(spp, 0)
        _baseline[key] = dev.read_film()[0]
        dev.close()
    same = np.array_equal(film[0], _baseline[key])
    assert same == ((scene_name, case) in INERT), (scene_name, case, same)


def _check(tag, frac, rel, bar=0.999):
    print(f"{tag}: pixels within 1e-3 {frac:.5f}, image-mean rel diff {rel:.2e}")
    assert frac >= bar, (tag, frac)
    assert rel < 2e-3, (tag, rel)


SURFACE = [(s, c) for s in ("cornell", "ajar") for c in CASES if not c.startswith("strict")] + \
          [("spheres", c) for c in CASES] + [("sky", "hideEmitters"), ("sky", "hide+maxDepth2"), ("sky", "maxDepth2")]


@pytest.mark.parametrize("scene_name,case", SURFACE)
def test_surface_params_same_streams(pg, O, scene_name, case):
    frac, rel, (g, mc) = same_stream_parity(pg, O, scene_name, CASES[case])
    _check(f"path {scene_name} {case}", frac, rel)
    assert_parameter_took_effect(pg, scene_name, case, g)
    p = CASES[case]
    if p.get("max_component_value") is not None:
        # the clamp bounds every accepted sample, hence every pixel mean (progressiveintegrator.cpp:274-277)
        assert _means(g).max() <= p["max_component_value"] * (1 + 1e-6)
    if p.get("hide_emitters") and p.get("max_depth") == 1:
        assert not g[0][..., :3].any()


VOLUME = [(s, c) for s in ("smoke", "bidir_2") for c in CASES if not c.startswith("strict")] + \
         [("spheres", c) for c in CASES if c.startswith("strict")]


@pytest.mark.parametrize("scene_name,case", VOLUME)
def test_volpath_params_same_streams(pg, O, scene_name, case):
    frac, rel, (g, mc) = same_stream_parity(pg, O, scene_name, CASES[case], volpath=True)
    _check(f"volpath {scene_name} {case}", frac, rel)
    assert_parameter_took_effect(pg, scene_name, case, g, volpath=True)
    p = CASES[case]
    if p.get("max_component_value") is not None:
        assert _means(g).max() <= p["max_component_value"] * (1 + 1e-6)


@pytest.fixture(scope="module")
def sphere_tree(pg):
    """An SD-tree trained on the GPU for the sphere scene (default parameters), injected on both sides."""
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    integ = GuidedPathTracer({"trainingIterations": 3, "sTreeThreshold": 400.0})
    integ.preprocess(smooth_spheres(pg))
    integ.train()
    blob = integ.dev.get_sdtree()
    integ.postprocess()
    return blob, 7


@pytest.mark.parametrize("case", ["maxDepth4", "rrDepth1", "clamp2", "noNee", "strict", "strict+rr1+noNee"])
def test_guided_params_same_tree(pg, O, sphere_tree, case):
    """The guided shading instantiations (CAN_GUIDE: one-sample MIS with the SD-tree) under the same
    parameters, one tree on both sides."""
    frac, rel, _ = same_stream_parity(pg, O, "spheres", CASES[case], guided_tree=sphere_tree)
    _check(f"guided spheres {case}", frac, rel)
