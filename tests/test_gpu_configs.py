"""GPU parity at the workloads the headline metric is quoted on:
the HIP path through the C-ABI against the CPU oracle, with one SD-tree on both sides and the same
counter-RNG streams, so that per-pixel agreement is far tighter than a Monte-Carlo tolerance.

  C3  guided ajar door at the full 1280x720: the GPU trains the whole job (5 iterations), the
      oracle renders a block of tiles of the final pass with the GPU's tree
      (progressive_path.cpp:133-314, progressiveintegrator.cpp:222-282);
  C4  guided kitchen class (~1 M triangles, 5 emitters) on a 4-rank tile shard: four shard contexts
      train with the pg_get/put_tree_stats all-reduce and must hold the single-rank tree bit for
      bit; the union of their final renders against the oracle with that tree;
  C5  guided volumetric path tracer on the 256^3 smoke grid.
Plus the chunk scheduler: tiny max_paths_in_flight (pixel-range chunks, many rounds of lanes) gives
the default chunking's film and SD-tree bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share


def _md5(a):
    import hashlib
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()[:12]


def make_dev(pg, scene, **cfg):
    from mitsuba_path_guiding_amd.integrator import Device
    d = Device(pg.capi.default_config(**cfg))
    d.upload(scene)
    return d


def tiles_of(scene, ntiles, T=32):
    W, H = scene.width, scene.height
    tiles = [[y * W + x for y in range(ty, min(ty + T, H)) for x in range(tx, min(tx + T, W))]
             for ty in range(0, H, T) for tx in range(0, W, T)]
    mid = len(tiles) // 2
    return np.array([p for i in range(ntiles) for p in tiles[(mid + i) % len(tiles)]], np.uint32)


def means(film):
    rgbw, sq = film
    n = np.maximum(rgbw[..., 3:4], 1)
    m = rgbw[..., :3] / n
    v = np.maximum(sq[..., :3] / n - m * m, 0) / n
    return m, v


def pixel_parity(g, c, pix):
    """(z over the pixels, fraction of pixels whose means differ by more than 1e-3 relative)"""
    mg, vg = means(g)
    mc, vc = means(c)
    mg, vg, mc, vc = (a.reshape(-1, 3)[pix] for a in (mg, vg, mc, vc))
    z = (mg - mc) / np.sqrt(vg + vc + 1e-12)
    rel = np.abs(mg - mc).max(-1) / np.maximum(mc.max(-1), 1e-3)
    return z, float((rel > 1e-3).mean())


def test_c3_guided_full_resolution(pg, O):
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    sc = pg.scenes.ajar_door(1280, 720)
    integ = GuidedPathTracer({"trainingIterations": 5})
    integ.preprocess(sc)
    integ.train()
    blob = integ.dev.get_sdtree()
    st = integ.dev.stats()
    assert st["stree_nodes"] > 1000 and st["records"] > 10_000_000
    spp, off = 64, 31
    integ.dev.reset_film()
    integ.dev.render_pass(spp, off)
    g = integ.dev.read_film()
    cfg = integ.cfg
    integ.postprocess()
    osc = O.OracleScene(pg.capi, sc)
    tree = O.OracleSDTree(osc)
    tree.deserialize(blob)
    pix = tiles_of(sc, 32)
    c = O.render(osc, cfg, spp, off, sdtree=tree, pixels=pix, nthreads=THREADS)[:2]
    assert np.array_equal(g[0].reshape(-1, 4)[pix, 3], c[0].reshape(-1, 4)[pix, 3])
    z, diverged = pixel_parity(g, c, pix)
    print(f"c3 guided: |z|<5 {(np.abs(z) < 5).mean():.6f} diverged {diverged:.6f} tree {_md5(blob)} film {_md5(g[0])}")
    assert (np.abs(z) < 5).mean() > 0.999
    # paths whose fp32 libm/FMA rounding flips a branch diverge; the fraction depends on the trained
    # tree (5.2e-4 and 1.13e-3 measured for two trees of this job)
    assert diverged < 2e-3, diverged
    # same-tree relative RMSE of the GPU image against the oracle's: a diverged path moves
    # a single-sample glint, so the full figure is set by the few pixels that hold one (0.03-0.15 at 1024
    # spp, tools/diverge_c3.py); without the worst 0.1 % of pixels it is bounded tightly
    mg, mc = means(g)[0].reshape(-1, 3)[pix].astype(np.float64), means(c)[0].reshape(-1, 3)[pix].astype(np.float64)
    se = ((mg - mc) ** 2).sum(1)
    keep = np.argsort(se)[: len(se) - len(se) // 1000]
    rel_full = float(np.sqrt(se.mean() / 3) / np.sqrt((mc ** 2).mean()))
    rel_trim = float(np.sqrt(se[keep].mean() / 3) / np.sqrt((mc[keep] ** 2).mean()))
    print(f"c3 same-tree relative RMSE {rel_full:.5f}, without the worst 0.1 % of pixels {rel_trim:.5f}")
    assert rel_trim < 0.01, rel_trim
    # round 5: the kernels round as the oracle does (no FP contraction, ties on the original triangle
    # id), so single-sample glints no longer set the full figure
    assert rel_full < 0.1, rel_full


def test_c4_guided_four_rank_shard(pg, O):
    sc = pg.scenes.kitchen(192, 108)
    cfg = dict(guiding=1, s_tree_threshold=2000.0)
    full = make_dev(pg, sc, **cfg)
    shards = [make_dev(pg, sc, rank=r, world_size=4, **cfg) for r in range(4)]
    off = 0
    for it in range(4):
        full.render_pass(2 ** it, off, True)
        full.splat_local()
        full.refit(it)
        for d in shards:
            d.render_pass(2 ** it, off, True)
            d.splat_local()
        total = sum(d.get_tree_stats() for d in shards)  # the all-reduce of the postprogression exchange
        for d in shards:
            d.put_tree_stats(total)
            d.refit(it)
        off += 2 ** it
    blob = full.get_sdtree()
    assert all(np.array_equal(d.get_sdtree(), blob) for d in shards)
    assert full.stats()["stree_nodes"] > 1
    spp = 16
    films = []
    for d in shards:
        d.reset_film()
        d.render_pass(spp, off)
        films.append(d.read_film())
    g = (sum(f[0] for f in films), sum(f[1] for f in films))
    assert (g[0][..., 3] > 0).all() and g[0][..., 3].max() <= spp  # the shards tile the image exactly once
    ocfg = pg.capi.default_config(**cfg)
    osc = O.OracleScene(pg.capi, sc)
    tree = O.OracleSDTree(osc)
    tree.deserialize(blob)
    c = O.render(osc, ocfg, spp, off, sdtree=tree, nthreads=THREADS)[:2]
    assert (g[0][..., 3] == c[0][..., 3]).mean() > 0.999
    z, diverged = pixel_parity(g, c, np.arange(sc.width * sc.height))
    assert (np.abs(z) < 5).mean() > 0.999
    # same tree and streams; ~1 M triangles with many shared edges and glass/plastic clutter.  Until
    # round 4 edge ties went by BVH order on the GPU and by original index in the oracle, and the kernels
    # contracted the BSDF arithmetic to FMAs: 2.6 % of pixels diverged at 16 spp.  Both now match the
    # oracle (pg_trace.h acceptHit, Makefile FPC=off)
    print(f"c4 kitchen: diverged {diverged:.6f}")
    assert diverged < 0.01, diverged
    for d in shards + [full]:
        d.close()


def test_c5_guided_volpath_256_grid(pg, O):
    from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer
    sc = pg.scenes.smoke(64, 64, res=256)
    integ = GuidedVolumetricPathTracer({"trainingIterations": 3, "sTreeThreshold": 400.0})
    integ.preprocess(sc)
    integ.train()
    blob = integ.dev.get_sdtree()
    spp, off = 32, 7
    integ.dev.reset_film()
    integ.dev.render_pass(spp, off, True)
    g = integ.dev.read_film()
    nrec_gpu = integ.dev.record_count()
    cfg = integ.cfg
    integ.postprocess()
    osc = O.OracleScene(pg.capi, sc)
    tree = O.OracleSDTree(osc)
    tree.deserialize(blob)
    c = O.render(osc, cfg, spp, off, record=True, sdtree=tree, nthreads=THREADS)
    nrec_cpu = int(c[2][3])
    mg, _ = means(g)
    mc, _ = means(c[:2])
    z, _ = pixel_parity(g, c[:2], np.arange(64 * 64))
    assert (np.abs(z) < 5).mean() > 0.999
    close = np.abs(mg - mc).max(-1) <= 1e-3 * np.maximum(mc.max(-1), 1e-3)
    print(f"c5 guided 256^3 same tree: |z|<5 {(np.abs(z) < 5).mean():.5f}, pixels within 1e-3 {close.mean():.5f}, "
          f"records {nrec_gpu} / {nrec_cpu}")
    # same tree and streams on both sides: measured 1.00000 (and equal record counts, gpurun_out/r06b)
    assert close.mean() >= 0.999, close.mean()
    assert abs(nrec_gpu - nrec_cpu) <= 0.001 * nrec_cpu, (nrec_gpu, nrec_cpu)


@pytest.mark.parametrize("paths", [1024, 4096])
def test_small_chunks_bitexact(pg, paths):
    """max_paths_in_flight far below the pass: pixel-range chunks (1024) or one layer per chunk
    (4096), many rounds of three lanes, record-buffer growth with lanes in flight.  Films are
    committed in chunk order and splats are integer, so film and SD-tree equal the default's."""
    sc = pg.scenes.cornell(64, 64)
    out = []
    for cap in (0, paths):
        d = make_dev(pg, sc, guiding=1, s_tree_threshold=300.0, max_paths_in_flight=cap)
        off = 0
        for it in range(3):
            d.render_pass(2 ** it, off, True)
            d.splat_local()
            d.refit(it)
            off += 2 ** it
        d.reset_film()
        d.render_pass(8, off, True)
        out.append((d.read_film()[0], d.get_sdtree(), d.record_count(), d.stats()["paths"]))
        d.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2] and out[0][3] == out[1][3]


def test_max_render_time(pg):
    """maxRenderTime (renderTime, progressiveintegrator.cpp:117-168): whole progressions until the
    budget is spent.  The film is then exactly the fixed-spp film of the same sample count (every
    pixel holds the same number of samples), and the budget is kept to within a progression."""
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer, ProgressivePathTracer
    sc = pg.scenes.cornell(128, 128)
    budget = 0.4
    t = ProgressivePathTracer({"maxRenderTime": budget, "samplesPerProgression": 4})
    t.preprocess(sc)
    t.render(1)  # warm-up (kernel loading)
    t.dev.reset_film()
    t.sample_offset = 0
    rgbw, sq = t.render(1)
    n = t.rendered_spp
    assert n >= 8 and n % 4 == 0, n
    assert budget <= t.render_seconds < budget + 0.25, t.render_seconds
    ref = ProgressivePathTracer({"samplesPerProgression": n})
    ref.preprocess(sc)
    r = ref.render(n)
    assert np.array_equal(r[0], rgbw) and np.array_equal(r[1], sq)
    assert (rgbw[..., 3] == n).mean() > 0.999
    for x in (t, ref):
        x.postprocess()
    # guided: the budget covers training + final render
    g = GuidedPathTracer({"trainingIterations": 3, "sTreeThreshold": 400.0, "maxRenderTime": budget})
    g.preprocess(sc)
    g.render(1)
    g.reset()
    rgbw, _ = g.render(1)
    assert g.rendered_spp > 0 and g.render_seconds < budget + 0.25
    assert (rgbw[..., 3] == g.rendered_spp).mean() > 0.999
    g.postprocess()


def test_training_independent_of_lanes_and_runs(pg, monkeypatch):
    """Paths are pure functions of (pixel, sample): guided kitchen training gives the same sorted
    records, films and trees for 1 and 3 lanes in flight, again on a fresh context (closest-hit
    ties resolved independently of traversal order; DESIGN.md §4 Determinism), and with the fused
    per-bounce launches or separate ones."""
    sc = pg.scenes.kitchen(128, 72)

    def train(lanes, timing=0):
        d = make_dev(pg, sc, guiding=1, s_tree_threshold=1500.0, path_lanes=lanes, kernel_timing=timing)
        off, out = 0, []
        for it in range(4):
            d.render_pass(2 ** it, off, True)
            rec = d.get_records().reshape(-1, 32)
            out.append((_md5(rec[np.lexsort(rec.T[::-1])]), _md5(d.read_film()[0])))
            d.splat_local()
            d.refit(it)
            off += 2 ** it
        out.append(_md5(d.get_sdtree()))
        d.close()
        return out

    a = train(3)
    assert train(1) == a
    assert train(3) == a
    # per-launch timing times the fused launches a render runs (k_shade_all + k_rays)
    assert train(3, timing=1) == a
    # the unfused per-class k_shade launches and separate k_shadow / k_trace launches (the path an
    # environment-lit scene takes for shading): same paths
    monkeypatch.setenv("PG_NO_SHADE_FUSION", "1")
    monkeypatch.setenv("PG_NO_RAYS_FUSION", "1")
    assert train(3) == a
    assert train(1, timing=1) == a
