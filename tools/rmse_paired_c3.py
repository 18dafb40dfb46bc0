"""SURVEY.md §8c(3) / north_star "per-pixel RMSE within 1 % of CPU at 1024 spp", resolved statistically.

The GPU trains the C3 guided job and renders its 1024-spp final pass; the CPU oracle renders the same
final pass with the GPU's tree and the same random streams on a growing set of 32x32 tiles (centre
outwards).  Both images are compared with the committed ground truths (the 65,536-spp GPU image and,
where it covers the tiles, the 8192-spp CPU oracle tiles).  For each sample size the paired RMSE ratio
RMSE_gpu / RMSE_cpu and its jackknife standard error over the tiles are reported; the criterion is met
when the ratio is within 1.01 and the standard error below 0.01.  GPU box only.

  python tools/rmse_paired_c3.py OUT.json [--tiles 256] [--threads 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def ratio_se(se_g, se_c):
    """RMSE ratio over tiles and its jackknife standard error (leave one tile out)"""
    n = len(se_g)
    r = float(np.sqrt(se_g.sum() / se_c.sum()))
    jk = np.sqrt((se_g.sum() - se_g) / (se_c.sum() - se_c))
    return r, float(np.sqrt((n - 1) / n * ((jk - jk.mean()) ** 2).sum()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--tiles", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--spp", type=int, default=1024)
    a = ap.parse_args()
    import pgload
    pg = pgload.load()
    import bench
    import oracle_py as O  # checker
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    scene = pg.scenes.ajar_door(1280, 720)
    integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": a.spp, **bench.BENCH_GUIDING}, device=0)
    integ.preprocess(scene)
    integ.reset()
    final, _ = integ.render(a.spp)
    blob = integ.dev.get_sdtree()
    cfg = integ.cfg
    integ.postprocess()
    W, H, T = scene.width, scene.height, 32
    tiles = [[y * W + x for y in range(ty, min(ty + T, H)) for x in range(tx, min(tx + T, W))]
             for ty in range(0, H, T) for tx in range(0, W, T)]
    mid = len(tiles) // 2
    nt = min(a.tiles, len(tiles))
    order = [(mid + i) % len(tiles) for i in range(nt)]  # the bench's sample first, then outwards
    osc = O.OracleScene(pg.capi, scene)
    tree = O.OracleSDTree(osc)
    tree.deserialize(blob)
    off = 2 ** 5 - 1
    gt = bench.load_gt()[0].reshape(-1, 3).astype(np.float64)
    g = bench.image(final).reshape(-1, 3).astype(np.float64)
    cpu_gt = None
    if os.path.exists(bench.GT_C3_CPU):
        z = np.load(bench.GT_C3_CPU)
        cpu_gt = {int(p): z["mean"][i].astype(np.float64) for i, p in enumerate(z["pixels"])}
    se_g, se_c, se_g2, se_c2, rel, t_cpu = [], [], [], [], [], 0.0
    report = []
    batch = max(a.threads, 16)
    for b0 in range(0, nt, batch):
        ids = order[b0:b0 + batch]
        pix = np.array([p for i in ids for p in tiles[i]], np.uint32)
        t = time.perf_counter()
        c_rgbw = O.render(osc, cfg, a.spp, off, sdtree=tree, pixels=pix, nthreads=a.threads)[0]
        t_cpu += time.perf_counter() - t
        c = bench.image(c_rgbw).reshape(-1, 3).astype(np.float64)
        for i in ids:
            p = np.array(tiles[i])
            se_g.append(((g[p] - gt[p]) ** 2).sum())
            se_c.append(((c[p] - gt[p]) ** 2).sum())
            rel.append(float((np.abs(g[p] - c[p]).max(-1) / np.maximum(c[p].max(-1), 1e-3) > 1e-3).mean()))
            if cpu_gt is not None and all(int(q) in cpu_gt for q in p):
                gc = np.array([cpu_gt[int(q)] for q in p])
                se_g2.append(((g[p] - gc) ** 2).sum())
                se_c2.append(((c[p] - gc) ** 2).sum())
        r, e = ratio_se(np.array(se_g), np.array(se_c))
        row = {"tiles": len(se_g), "pixels": int(len(se_g) * T * T), "rmse_ratio_gpu_over_cpu": round(r, 5),
               "jackknife_se": round(e, 5), "pixels_diverged_frac": round(float(np.mean(rel)), 5),
               "cpu_seconds": round(t_cpu, 1)}
        if len(se_g2) >= 2:
            r2, e2 = ratio_se(np.array(se_g2), np.array(se_c2))
            row["vs_cpu_ground_truth"] = {"tiles": len(se_g2), "ratio": round(r2, 5), "jackknife_se": round(e2, 5)}
        report.append(row)
        print(json.dumps(row), flush=True)
    out = {"workload": "C3 1280x720 guided job (5 training iterations) + the 1024-spp final render; the CPU "
                       "oracle renders the same final pass with the GPU's SD-tree and random streams (paired)",
           "ground_truth": "tests/golden/c3_gt.npz (GPU, 65,536 spp); vs_cpu_ground_truth: "
                           "tests/golden/c3_cpu_gt_tiles.npz (CPU oracle, unguided, 8192 spp)",
           "criterion": "ratio <= 1.01 with jackknife SE < 0.01 (SURVEY.md §8c(3))", "by_sample_size": report}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
