"""Which paths make C3's guided image worse than the unguided one in the dark class?  

Trains the bench's guided job, renders its 1024-spp final pass and an unguided 1024-spp pass, and
splits the dark-class relMSE (bench.errors' normalisation) into per-pixel variance (the films' sum of
squares) and the pixels that dominate it.  For the worst dark pixels of the guided image the CPU oracle
replays all 1024 final-pass samples with the GPU's SD-tree and the same random streams (paired, the
checker role of oracle/) and logs the vertices of the largest-contribution path: depth, material,
guided or not, the mixture weight and the throughput.  GPU box only.

  python tools/outlier_paths_c3.py OUT.json [--pixels 24]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

MODES = {0: "bsdf", 1: "mix:bsdf", 2: "mix:guide", 11: "mix:bsdf, zero weight (end)", 12: "mix:guide, zero weight (end)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--pixels", type=int, default=24)
    ap.add_argument("--spp", type=int, default=1024)
    a = ap.parse_args()
    import pgload
    pg = pgload.load()
    import bench
    import oracle_py as O  # checker
    from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer
    scene = pg.scenes.ajar_door(1280, 720)
    W = scene.width
    gt = bench.load_gt()[0].astype(np.float64)
    norm = (gt ** 2 + 1e-2 * float(gt.mean()) ** 2).mean(-1).ravel()  # per-pixel relMSE denominator (channel mean)
    integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": a.spp, **bench.BENCH_GUIDING}, device=0)
    integ.preprocess(scene)
    integ.reset()
    g_rgbw, g_sq = integ.render(a.spp)
    blob = integ.dev.get_sdtree()
    cfg = integ.cfg
    integ.postprocess()
    dev = Device(pg.capi.default_config())
    dev.upload(scene)
    dev.render_pass(a.spp, 0)
    u_rgbw, u_sq = dev.read_film()[:2]
    dev.close()

    def stats(rgbw, sq):
        n = np.maximum(rgbw[..., 3:4].astype(np.float64), 1)
        m = rgbw[..., :3] / n
        var = np.maximum(sq[..., :3] / n - m ** 2, 0) / n  # variance of the pixel mean
        rel = (((m - gt) ** 2).mean(-1)).ravel() / norm
        return m, (var.mean(-1)).ravel() / norm, rel

    gm, gvar, grel = stats(g_rgbw, g_sq)
    um, uvar, urel = stats(u_rgbw, u_sq)
    dark = (gt.mean(-1) < gt.mean()).ravel()
    n = len(dark)
    res = {"workload": "C3 1280x720, bench guided job (5 training iterations, albedo bound + glossy prior) vs the "
                       "unguided tracer, both 1024 spp final",
           "classes": {}}
    for name, m in (("dark", dark), ("bright", ~dark)):
        r = {"pixels": int(m.sum()),
             "relmse_sum_guided": float(grel[m].sum() / n), "relmse_sum_unguided": float(urel[m].sum() / n),
             "variance_sum_guided": float(gvar[m].sum() / n), "variance_sum_unguided": float(uvar[m].sum() / n),
             "pixels_guided_variance_higher": float((gvar[m] > uvar[m]).mean()),
             "median_variance_ratio": float(np.median(gvar[m] / np.maximum(uvar[m], 1e-30)))}
        gs = np.sort(gvar[m])[::-1]
        us = np.sort(uvar[m])[::-1]
        for k in (10, 100, 1000, 10000):
            r[f"variance_share_top{k}_guided"] = float(gs[:k].sum() / max(gs.sum(), 1e-30))
            r[f"variance_share_top{k}_unguided"] = float(us[:k].sum() / max(us.sum(), 1e-30))
        res["classes"][name] = r
        print(json.dumps({name: r}), flush=True)

    # material of each original triangle
    tri_mat = np.zeros(sum(s.tri_count for s in scene.shapes), np.int32)
    for s in scene.shapes:
        tri_mat[s.tri_begin:s.tri_begin + s.tri_count] = s.material
    names = {v: k[7:].lower() for k, v in vars(pg.capi).items() if k.startswith("PG_BSDF_") and isinstance(v, int)}
    mat_names = [f"{i}:{names.get(int(m.type), m.type)}" for i, m in enumerate(scene.materials)]

    live_mat = np.array([not (m.type == pg.capi.PG_BSDF_DIFFUSE and max(m.diffuse_reflectance[:3]) == 0)
                         for m in scene.materials])
    osc = O.OracleScene(pg.capi, scene)
    tree = O.OracleSDTree(osc)
    tree.deserialize(blob)
    off = 2 ** 5 - 1

    def replay(p):
        """per-sample radiance of pixel p in the guided final pass (the GPU's tree) and unguided (no
        tree), same sample indices, and whether the guided path took a direction at a D-tree vertex
        (an unguided-prefix path, flag 0, is the same path bit for bit in both renders)"""
        Lg, Lu, fl = np.zeros(a.spp), np.zeros(a.spp), np.zeros(a.spp, bool)
        for s in range(a.spp):
            _, L, vtx = osc.path_rays(cfg, tree, p, off + s, max_rays=64)
            Lg[s] = float(np.mean(L))
            if len(vtx):
                # a D-tree vertex changes the path if it continued, added NEE (mixture MIS weight) or
                # ended on a guided direction of a non-black BSDF (the unguided path samples the BSDF there)
                tri = vtx[:, 1].astype(np.int64)
                nb = live_mat[tri_mat[np.clip(tri, 0, len(tri_mat) - 1)]]
                nee = (vtx[:, 21] > 0) | (vtx[:, 22] > 0) | (vtx[:, 23] > 0)
                fl[s] = bool(np.any((vtx[:, 9] == 1) & ((vtx[:, 28] == 1) | nee | ((vtx[:, 10] == 12) & nb))))
            _, L, _ = osc.path_rays(cfg, None, p, off + s, max_rays=64)
            Lu[s] = float(np.mean(L))
        return Lg, Lu, fl

    def var_mean(x, p):  # variance of the pixel mean, relMSE-normalised
        return float(x.var() / len(x) / norm[p])

    rng = np.random.default_rng(5)
    groups = {"worst_200_dark_by_guided_variance": [int(p) for p in np.argsort(np.where(dark, gvar, -1))[::-1][:200]],
              "random_200_dark": [int(p) for p in rng.choice(np.flatnonzero(dark), 200, replace=False)]}
    res["decomposition"] = {}
    rows = []
    for gname, pix in groups.items():
        acc = dict.fromkeys(("guided", "unguided", "unguided_prefix_part", "guided_part_guided", "guided_part_unguided"), 0.0)
        frac = []
        for p in pix:
            Lg, Lu, fl = replay(p)
            U = np.where(fl, 0.0, Lg)
            acc["guided"] += var_mean(Lg, p)
            acc["unguided"] += var_mean(Lu, p)
            acc["unguided_prefix_part"] += var_mean(U, p)
            acc["guided_part_guided"] += var_mean(np.where(fl, Lg, 0.0), p)
            acc["guided_part_unguided"] += var_mean(np.where(fl, Lu, 0.0), p)
            frac.append(fl.mean())
            if gname.startswith("worst") and len(rows) < 6:
                s = int(np.argmax(Lg))
                _, L, vtx = osc.path_rays(cfg, tree, p, off + s)
                verts = [{"depth": int(v[0]), "mat": mat_names[tri_mat[int(v[1])]] if 0 <= int(v[1]) < len(tri_mat) else "-",
                          "mode": MODES.get(int(v[10]), str(int(v[10]))), "weight": round(float(np.mean(v[12:15])), 4),
                          "T": round(float(np.mean(v[5:8])), 4)} for v in vtx]
                rows.append({"pixel": [p % W, p // W], "gt": float(gt.reshape(-1, 3)[p].mean()),
                             "gpu_mean": float(gm.reshape(-1, 3)[p].mean()), "cpu_mean": float(Lg.mean()),
                             "unguided_gpu_mean": float(um.reshape(-1, 3)[p].mean()), "unguided_cpu_mean": float(Lu.mean()),
                             "top_sample_share": float(Lg.max() / max(Lg.sum(), 1e-30)),
                             "top_sample_guided_prefix": bool(fl[s]), "top_path": verts})
                print(json.dumps({k: rows[-1][k] for k in ("pixel", "gpu_mean", "cpu_mean", "unguided_cpu_mean",
                                                          "top_sample_share", "top_sample_guided_prefix")}), flush=True)
        d = {k: round(v / n, 6) for k, v in acc.items()}
        d["pixels"] = len(pix)
        d["samples_with_guided_prefix"] = round(float(np.mean(frac)), 4)
        d["unguided_prefix_share_of_guided_variance"] = round(acc["unguided_prefix_part"] / max(acc["guided"], 1e-30), 4)
        d["guided_part_variance_ratio"] = round(acc["guided_part_guided"] / max(acc["guided_part_unguided"], 1e-30), 4)
        res["decomposition"][gname] = d
        print(json.dumps({gname: d}), flush=True)
    res["worst_dark_pixels"] = rows
    res["note"] = ("variance sums are over the listed pixels, relMSE-normalised and divided by the image's pixel count "
                   "like bench.errors; unguided_prefix_part = the samples whose guided path never sampled at a "
                   "D-tree vertex (bit-identical in both renders), guided_part_* = the other samples' radiance in the "
                   "guided and in the unguided render")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
