"""GPU parity of the volumetric path (pg_volpath.hip) against the CPU oracle (oracle/orc_volpath.h).

Unit level, same inputs and the same counter-RNG draws on both sides: HG sample/eval, grid lookups,
Woodcock free flight and transmittance estimates (identical draw counts for >= 99.9 % of rays; free-flight
distances within 1e-6 relative: the tracking loops' device logf rounds differently from the reference's
double-precision fastlog on 39 % of arguments, an ulp per step; measured 100 % equal draw counts and
<= 3.2e-7, and bit-identical results with PG_TRACK_FASTLOG=1, profiles/r05x_fastlog/).  Image level: per-pixel
z-test and overall-mean z-test on the furnace (expectation exactly 1), the absorbing slab (closed
form) and the C5 smoke scene class at a reduced grid and resolution.
"""
import numpy as np
import pytest

from test_volume import _mean_z, _vol_cfg, _zimg, absorber_scene, furnace_scene

pytestmark = pytest.mark.gpu


def make_dev(pg, scene, **cfg):
    from mitsuba_path_guiding_amd.integrator import Device
    d = Device(_vol_cfg(pg, **cfg))
    d.upload(scene)
    return d


def test_phase_and_medium_units(pg, O):
    sc = pg.scenes.smoke(16, 16, res=48)
    dev = make_dev(pg, sc)
    osc = O.OracleScene(pg.capi, sc)
    rng = np.random.default_rng(1)
    n = 100_000
    wi = rng.normal(size=(n, 3)).astype(np.float32)
    wi /= np.linalg.norm(wi, axis=1, keepdims=True)
    u = rng.random((n, 2)).astype(np.float32)
    wog = rng.normal(size=(n, 3)).astype(np.float32)
    wog /= np.linalg.norm(wog, axis=1, keepdims=True)
    g = dev.phase_query(0, wi, u, wog)
    c = O.hg_query(pg.capi, 0.8, wi, u, wog)
    print(f"hg: direction max |diff| {np.abs(g[:, :3] - c[:, :3]).max():.3g}, bit-equal rows "
          f"{np.all(g == c, axis=1).mean():.5f}, pdf/eval max rel "
          f"{(np.abs(g[:, 3:] - c[:, 3:]) / np.maximum(np.abs(c[:, 3:]), 1e-6)).max():.3g}")
    assert np.quantile(np.abs(g[:, :3] - c[:, :3]), 0.999) < 1e-4
    assert np.quantile(np.abs(g[:, 3:] - c[:, 3:]) / np.maximum(np.abs(c[:, 3:]), 1e-6), 0.999) < 1e-4
    # grid lookups
    p = rng.uniform(-1.1, 1.1, size=(n, 3)).astype(np.float32)
    lg, lc = dev.medium_lookup(0, p), osc.medium_lookup(0, p)
    print(f"lookups: bit-equal {np.mean(lg == lc):.5f}, max |diff| {np.abs(lg - lc).max():.3g}")
    assert np.allclose(lg, lc, atol=1e-6)
    # Woodcock free flight / transmittance with the same draws
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-1.5, 1.5, size=(n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = rng.uniform(0.5, 4.0, size=n)
    keys = rng.integers(0, 2 ** 32, size=(n, 2), dtype=np.uint32)
    for tr, grid in ((False, False), (True, False), (False, True), (True, True)):
        gg = dev.medium_sample(0, rays, keys, transmittance=tr, grid=grid)
        cc = osc.medium_sample(0, rays, keys, transmittance=tr, grid=grid)
        col = 1 if tr else 2
        same = gg[:, col] == cc[:, col]
        print(f"tracking tr={tr} grid={grid}: same lookups {same.mean():.5f}, bit-equal results "
              f"{np.all(gg[:, :3] == cc[:, :3], axis=1).mean():.5f}")
        assert same.mean() > 0.999, (tr, grid, same.mean())
        assert np.array_equal(gg[same, 0], cc[same, 0])
        if not tr:
            hit = same & (cc[:, 0] > 0.5)
            assert np.quantile(np.abs(gg[hit, 1] - cc[hit, 1]) / np.abs(cc[hit, 1]).clip(1e-3), 0.999) < 1e-6
    dev.close()


def _film(dev):
    rgbw, sq = dev.read_film()
    return rgbw, sq


def test_furnace_gpu(pg):
    sc = furnace_scene(pg)
    dev = make_dev(pg, sc)
    spp = 256
    dev.render_pass(spp, 0)
    rgbw, sq = _film(dev)
    st = dev.stats()
    dev.close()
    n = rgbw[..., 3:].sum()
    m = rgbw[..., :3].sum((0, 1)) / n
    se = np.sqrt((sq[..., :3].sum((0, 1)) / n - m ** 2) / n)
    assert np.all(np.abs(m - 1) < 5 * se + 1e-3), (m, se)
    assert st["paths"] == 16 * 16 * spp and st["segments"] > 2 * st["paths"]


def test_absorbing_slab_gpu(pg):
    sigma, le = 0.9, np.array([4.0, 3.0, 2.0])
    dev = make_dev(pg, absorber_scene(pg, sigma, tuple(le)))
    spp = 256
    dev.render_pass(spp, 0)
    rgbw, _ = _film(dev)
    dev.close()
    frac = (rgbw[..., :3] / rgbw[..., 3:]).reshape(-1, 3) / le
    p, n = np.exp(-sigma), 16 * 16 * spp
    assert abs(frac.mean() - p) < 5 * np.sqrt(p * (1 - p) / n)


def test_smoke_image_parity(pg, O):
    sc = pg.scenes.smoke(48, 48, res=64)
    spp = 64
    dev = make_dev(pg, sc)
    dev.render_pass(spp // 2, 0)
    dev.render_pass(spp // 2, spp // 2)  # two progressions accumulate like one pass
    g = _film(dev)
    dev.close()
    c = O.render(O.OracleScene(pg.capi, sc), _vol_cfg(pg), spp)[:2]
    assert np.array_equal(g[0][..., 3], c[0][..., 3])
    m1, m2, z = _zimg(g, c)
    assert (np.abs(z) < 5).mean() > 0.999
    assert abs(_mean_z(g, c)) < 5
    # same counter streams on both sides: most pixels agree to fp32 noise, not just statistically
    close = np.abs(m1 - m2) <= 1e-3 * np.maximum(np.abs(m2), 1e-3)
    print(f"c5 smoke same streams: pixels within 1e-3 {close.mean():.4f}")
    assert close.mean() > 0.99, close.mean()  # measured 1.0000 (profiles/r05x_fastlog/)


def test_smoke_image_parity_global_majorant(pg, O):
    """The reference's single-majorant tracking on the GPU against the oracle (same streams)."""
    sc = pg.scenes.smoke(32, 32, res=48)
    spp = 64
    cfg = dict(volume_majorant=pg.capi.PG_MAJORANT_GLOBAL)
    dev = make_dev(pg, sc, **cfg)
    dev.render_pass(spp, 0)
    g = _film(dev)
    dev.close()
    c = O.render(O.OracleScene(pg.capi, sc), _vol_cfg(pg, **cfg), spp)[:2]
    m1, m2, z = _zimg(g, c)
    assert (np.abs(z) < 5).mean() > 0.999
    assert abs(_mean_z(g, c)) < 5


def test_volpath_surface_scene_matches_path_gpu(pg, O):
    """No media: the volpath kernel on the Cornell box against the oracle's surface path tracer."""
    sc = pg.scenes.cornell(32, 32)
    dev = make_dev(pg, sc)
    dev.render_pass(128, 0)
    g = _film(dev)
    dev.close()
    c = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(), 128)[:2]
    m1, m2, z = _zimg(g, c)
    assert (np.abs(z) < 5).mean() > 0.998
    assert abs(_mean_z(g, c)) < 5


def test_volpath_config_errors(pg):
    from mitsuba_path_guiding_amd.integrator import Device, PGError
    with pytest.raises(PGError):
        Device(pg.capi.default_config(integrator=pg.capi.PG_INTEGRATOR_VOLPATH, guiding=1, distance_guiding=1.0))
    with pytest.raises(PGError):
        Device(pg.capi.default_config(integrator=7))
    sc = pg.scenes.smoke(8, 8, res=8)
    sc._densities[0][0, 0, 0] = 1.5  # outside [0, 1] (heterogeneous.cpp:236-239)
    d = Device(_vol_cfg(pg))
    with pytest.raises(PGError):
        d.upload(sc)
    d.close()


# ---- guided volpath (GuidedVolumetricPathTracer; oracle/orc_volpath.h, PARITY UNPINNED vs the
# reference, which has no guiding: pinned here by unbiasedness and by the oracle on injected trees)

def _guided(pg, sc, beta, iters=4, spp=128, **props):
    from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer
    p = {"trainingIterations": iters, "sTreeThreshold": 400.0, "distanceGuiding": beta}
    p.update(props)
    integ = GuidedVolumetricPathTracer(p)
    integ.preprocess(sc)
    rgbw, sq = integ.render(spp)
    tree = integ.dev.get_sdtree()
    st = integ.postprocess()
    return (rgbw, sq), st, tree


@pytest.mark.parametrize("beta", [0.0, 0.5, 0.9])
def test_guided_volpath_furnace_gpu(pg, beta):
    (rgbw, sq), st, _ = _guided(pg, furnace_scene(pg), beta, iters=3, spp=128)
    n = rgbw[..., 3:].sum()
    m = rgbw[..., :3].sum((0, 1)) / n
    se = np.sqrt((sq[..., :3].sum((0, 1)) / n - m ** 2) / n)
    assert np.all(np.abs(m - 1) < 5 * se + 1e-3), (beta, m, se)
    assert st["records"] > 0 and st["stree_nodes"] > 1


def test_guided_smoke_gpu_matches_unguided_oracle(pg, O):
    sc = pg.scenes.smoke(32, 32, res=48)
    g, st, _ = _guided(pg, sc, 0.5, iters=4, spp=256)
    c = O.render(O.OracleScene(pg.capi, sc), _vol_cfg(pg, seed=77), 256)[:2]
    m1, m2, z = _zimg(g, c)
    assert (np.abs(z) < 5).mean() > 0.995
    assert abs(_mean_z(g, c)) < 5


@pytest.mark.parametrize("beta", [0.0, 0.5])
def test_guided_volpath_same_tree_parity(pg, O, beta):
    """One SD-tree (trained by the oracle) injected on both sides, the same counter streams: the
    guided GPU render and its training records against the oracle's."""
    sc = pg.scenes.smoke(32, 32, res=48)
    osc = O.OracleScene(pg.capi, sc)
    cfg = _vol_cfg(pg, guiding=1, s_tree_threshold=400.0, distance_guiding=beta)
    from test_volume_guided import train_oracle
    otree, off = train_oracle(pg, O, osc, cfg, iters=3)
    blob = otree.serialize()
    dev = make_dev(pg, sc, guiding=1, s_tree_threshold=400.0, distance_guiding=beta)
    dev.put_sdtree(blob)
    assert np.array_equal(dev.get_sdtree(), blob)
    spp = 64
    dev.render_pass(spp, off, record=True)
    g = _film(dev)
    nrec_gpu = dev.record_count()
    recs = dev.get_records()
    dev.close()
    c = O.render(osc, cfg, spp, sample_offset=off, record=True, sdtree=otree)
    nrec_cpu = int(c[2][3])
    m1, m2, z = _zimg(g, c[:2])
    assert (np.abs(z) < 5).mean() > 0.999
    assert abs(_mean_z(g, c[:2])) < 5
    close = np.abs(m1 - m2) <= 1e-3 * np.maximum(np.abs(m2), 1e-3)
    print(f"c5 guided same tree beta {beta}: pixels within 1e-3 {close.mean():.4f}, records {nrec_gpu} / {nrec_cpu}")
    assert close.mean() > 0.99, close.mean()  # measured 1.0000 / 1.0000 (profiles/r05x_fastlog/)
    assert abs(nrec_gpu - nrec_cpu) <= 0.001 * nrec_cpu, (nrec_gpu, nrec_cpu)  # measured equal
    r = np.frombuffer(recs.tobytes(), np.float32).reshape(-1, 8)
    assert np.all(np.isfinite(r[:, [0, 1, 2, 4, 5]])) and np.all(r[:, 5] > 0)


def test_diffuse_null_surface_kernels_bit_identical(pg, monkeypatch):
    """A scene whose materials are all diffuse or null runs the surface launches compiled for those two
    models only (VolDev::models, k_vvertex KIND 3, k_vtail): the same arithmetic for every material it
    has, so the guided job's film, tree and records are bit-identical to the generic kernels'."""
    from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer
    sc = pg.scenes.smoke(64, 64, res=48)
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PG_VOL_MODELS", flag)
        t = GuidedVolumetricPathTracer({"trainingIterations": 3, "samplesPerProgression": 8})
        t.preprocess(sc)
        rgbw, sq = t.render(16)
        out.append((rgbw, sq, t.dev.get_sdtree()))
        t.postprocess()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)


def test_volpath_refill_threshold_bit_identical(pg, monkeypatch):
    """k_volpath refills a wave's idle lanes in batches (VolDev.refill_min, PG_VOL_REFILL): every
    work item draws from its own stream and writes its own slots, so films and trees must not depend
    on when lanes are refilled."""
    from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer
    sc = pg.scenes.smoke(96, 96, res=48)
    out = []
    monkeypatch.setenv("PG_VOL_WAVEFRONT", "0")  # the megakernel (the wavefront has no lane refill)
    for r in ("1", "24", "64"):
        monkeypatch.setenv("PG_VOL_REFILL", r)
        t = GuidedVolumetricPathTracer({"trainingIterations": 3, "samplesPerProgression": 8})
        t.preprocess(sc)
        rgbw, sq = t.render(8)
        out.append((rgbw, sq, t.dev.get_sdtree()))
        t.postprocess()
    for o in out[1:]:
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])
        assert np.array_equal(o[2], out[0][2])


@pytest.mark.parametrize("case", ["guided", "plain_global", "guided_exact_chunked", "delta_surfaces"])
def test_volpath_wavefront_equals_megakernel(pg, monkeypatch, case):
    """The volumetric wavefront (k_vcam / k_vflight / k_vvertex / k_vtail, PG_VOL_WAVEFRONT) runs the
    megakernel's volFlight / volMedium / volSurface on the same random streams, each path in its own
    slot: films, sums of squares, training records (through the trees) and path counters must be the
    megakernel's bit for bit -- whether every iteration runs as launches (tail threshold 0), the
    default tail threshold, or the tail kernel takes the whole chunk after the camera rays; with one,
    two or three (default) lanes of chunks in flight (films in chunk order), with the flight queues
    sorted by cell (PG_VOL_SORT), and whether the interactions' transmittance walks run inline at the end of
    each interaction (the default, pg_host.cpp volNeeStage) or as a stage of their own (PG_VOL_NEE_STAGE=1:
    k_vvertex<NEE_STAGE> writes the deferred-walk records, k_vnee walks them, either on a second stream
    overlapping the next iteration's free flights (PG_VOL_NEE_OVERLAP, default with the stage) or on the
    lane's stream (PG_VOL_NEE_OVERLAP=0)), and the medium and surface interactions as two launches (default)
    or one (PG_VOL_SPLIT_VERTEX=0): the walks draw from their own sub-streams and add to L in a fixed order
    (oracle/orc_volpath.h subStream)."""
    from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer, ProgressiveVolumetricPathTracer
    sc = pg.scenes.smoke(96, 96, res=48)
    props = {"trainingIterations": 3, "samplesPerProgression": 8}
    if case == "delta_surfaces":  # C3's smooth and rough conductors and dielectrics: the split surface queues
        sc = pg.scenes.ajar_door(96, 54)
    if case == "plain_global":
        Tracer, props = ProgressiveVolumetricPathTracer, {"samplesPerProgression": 8}
    else:
        Tracer = GuidedVolumetricPathTracer
    if case == "guided_exact_chunked":
        props.update({"exactMis": True, "maxPathsInFlight": 4096 + 512})
    out = []
    # (wavefront, tail threshold, lanes, flight sort, NEE stage, split vertex launches, NEE stage overlap)
    runs = (("0", None, None, None, None, None, None), ("1", "0", None, None, None, None, None),
            ("1", None, None, None, None, None, None), ("1", str(1 << 30), None, None, None, None, None),
            ("1", None, "1", None, None, None, None), ("1", "0", "3", "1", None, None, None),
            ("1", "0", "2", None, None, "0", None),
            ("1", "0", None, None, "1", None, "1"), ("1", None, None, None, "1", None, "0"),
            ("1", "0", "2", None, "1", "0", "0"))
    for wf, tail, lanes, sort, nee, split, overlap in runs:
        monkeypatch.setenv("PG_VOL_WAVEFRONT", wf)
        for var, val in (("PG_VOL_TAIL_PATHS", tail), ("PG_VOL_LANES", lanes), ("PG_VOL_SORT", sort),
                         ("PG_VOL_NEE_STAGE", nee), ("PG_VOL_SPLIT_VERTEX", split), ("PG_VOL_NEE_OVERLAP", overlap)):
            if val is None:
                monkeypatch.delenv(var, raising=False)
            else:
                monkeypatch.setenv(var, val)
        t = Tracer(dict(props))
        if case == "plain_global":  # the reference's single majorant (heterogeneous.cpp:589-660)
            t.cfg.volume_majorant = pg.capi.PG_MAJORANT_GLOBAL
        t.preprocess(sc)
        rgbw, sq = t.render(8)
        st = t.dev.stats()
        out.append((rgbw, sq, t.dev.get_sdtree() if t.guided else None,
                    (st["paths"], st["segments"], st["shadow_rays"], st["density_lookups"], st["records"])))
        t.postprocess()
    base = out[0]
    assert base[3][0] > 0 and (base[3][3] > 0 or case == "delta_surfaces")
    for o in out[1:]:
        assert np.array_equal(o[0], base[0]) and np.array_equal(o[1], base[1])
        if base[2] is not None:
            assert np.array_equal(o[2], base[2])
        assert o[3] == base[3], (o[3], base[3])


def test_volpath_wavefront_tile_shard(pg):
    """C5's multi-GPU form (image tiles sharded over ranks, building statistics all-
    reduced before each refit) on the volumetric wavefront, emulated with two shard contexts on one
    GPU: every training iteration's summed statistics give the single-rank tree bit for bit, and the
    two ranks' final films add up to the single-rank film bit for bit (the random streams are keyed by
    the global pixel)."""
    sc = pg.scenes.smoke(96, 96, res=48)
    cfg = dict(guiding=1, s_tree_threshold=300.0)
    full = make_dev(pg, sc, **cfg)
    parts = [make_dev(pg, sc, rank=r, world_size=2, **cfg) for r in range(2)]
    off = 0
    for it in range(3):
        full.render_pass(2 ** it, off, True)
        full.splat_local()
        full.refit(it)
        for d in parts:
            d.render_pass(2 ** it, off, True)
            d.splat_local()
        total = parts[0].get_tree_stats() + parts[1].get_tree_stats()
        for d in parts:
            d.put_tree_stats(total)
            d.refit(it)
        off += 2 ** it
    t = full.get_sdtree()
    assert all(np.array_equal(d.get_sdtree(), t) for d in parts)
    for d in parts + [full]:
        d.reset_film()
        d.render_pass(8, off)
    f = full.read_film()[0]
    p0, p1 = parts[0].read_film()[0], parts[1].read_film()[0]
    assert np.array_equal(p0 + p1, f)
    assert ((p0[..., 3] > 0) ^ (p1[..., 3] > 0)).all()
    for d in parts + [full]:
        d.close()
