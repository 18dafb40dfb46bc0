"""Where do the GPU and the CPU oracle part ways on C3 with one SD-tree and the same random numbers?

The bench's `rmse_vs_cpu.same_tree` compares the GPU final render with the oracle's render of the same
32 centre tiles using the GPU-trained tree.  This tool finds the pixels that dominate that relative
RMSE, the samples of those pixels whose radiance differs, and for each such path the first ray on which
the GPU's traversal (pg_trace_rays) and the oracle's (Scene::traverse) disagree, with a brute-force
verdict over every triangle (OracleScene.trace_brute).  GPU box only; writes JSON to argv[1].

  python tools/diverge_c3.py gpurun_out/r04b/diverge.json [--top 12]

With the debug build (make -C mitsuba-path-guiding_amd watch: PG_WATCH, loaded through PG_LIB) each
diverged path is also replayed with its vertex log on the GPU and compared with the oracle's Li log
field by field (FIELDS below): the first vertex and quantity where the two part ways.
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


FIELDS = ["depth", "tri", "px", "py", "pz", "Tr", "Tg", "Tb", "alpha", "guided", "mode", "woPdf", "wr", "wg", "wb",
          "wox", "woy", "woz", "Lr", "Lg", "Lb", "neeR", "neeG", "neeB", "neeEmPdf", "neeBsdfPdf", "rrQ", "rrSurvived",
          "alive", "shadow", "b0", "b1"]
WATCH_LIB = os.path.join(ROOT, "mitsuba-path-guiding_amd", "build", "libpgamd_watch.so")


def first_difference(gv, cv):
    """first (vertex, field) where the GPU and oracle vertex logs differ beyond fp32 noise"""
    for i in range(max(len(gv), len(cv))):
        if i >= len(gv) or i >= len(cv):
            return {"vertex": i, "field": "count", "gpu_vertices": len(gv), "cpu_vertices": len(cv)}
        for k, name in enumerate(FIELDS):
            if name in ("shadow", "neeR", "neeG", "neeB"):
                continue  # the kernels log every queued shadow ray, the oracle visible ones only
            a, b = float(gv[i][k]), float(cv[i][k])
            if name == "tri":
                if int(a) != int(b):
                    return {"vertex": i, "field": name, "gpu": a, "cpu": b}
                continue
            if not (abs(a - b) <= 2e-4 * max(1.0, abs(a), abs(b))):
                return {"vertex": i, "field": name, "gpu": a, "cpu": b,
                        "gpu_vertex": [float(x) for x in gv[i]], "cpu_vertex": [float(x) for x in cv[i]]}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--tiles", type=int, default=32)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    watch = os.path.exists(WATCH_LIB)
    if watch:
        os.environ["PG_LIB"] = WATCH_LIB
    import ctypes as C
    import pgload
    pg = pgload.load()
    import bench
    import oracle_py as O  # checker
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    scene = pg.scenes.ajar_door(1280, 720)
    integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": a.spp, **bench.BENCH_GUIDING},
                             device=0)
    integ.preprocess(scene)
    integ.reset()
    final, _ = integ.render(a.spp)
    dev = integ.dev
    if watch:
        from mitsuba_path_guiding_amd import integrator as I
        wl = I.library()
        wl.pg_debug_watch.argtypes = [C.c_uint32, C.c_uint32]
        wl.pg_debug_watch_read.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    off = 2 ** 5 - 1
    W, T = scene.width, 32
    tiles = [[y * W + x for y in range(ty, min(ty + T, scene.height)) for x in range(tx, min(tx + T, W))]
             for ty in range(0, scene.height, T) for tx in range(0, W, T)]
    mid = len(tiles) // 2
    pix = np.array([p for i in range(a.tiles) for p in tiles[(mid + i) % len(tiles)]], np.uint32)
    osc = O.OracleScene(pg.capi, scene)
    tree = O.OracleSDTree(osc)
    tree.deserialize(dev.get_sdtree())
    cfg = integ.cfg
    t0 = time.perf_counter()
    s_rgbw = O.render(osc, cfg, a.spp, off, sdtree=tree, pixels=pix, nthreads=a.threads)[0]
    t_cpu = time.perf_counter() - t0
    g = bench.image(final).reshape(-1, 3)[pix].astype(np.float64)
    s = bench.image(s_rgbw).reshape(-1, 3)[pix].astype(np.float64)
    se = ((g - s) ** 2).sum(1)
    rel_rmse = float(np.sqrt(se.mean() / 3) / np.sqrt((s ** 2).mean()))
    rel = np.abs(g - s).max(-1) / np.maximum(s.max(-1), 1e-3)
    order = np.argsort(-se)
    top = order[: a.top]
    out = {"same_tree_relative_rmse": rel_rmse, "pixels": int(len(pix)),
           "pixels_diverged_frac": float((rel > 1e-3).mean()), "cpu_render_s": round(t_cpu, 1),
           "top_share_of_squared_error": [float(se[top[: k + 1]].sum() / se.sum()) for k in range(len(top))],
           "relative_rmse_without_top": [float(np.sqrt(np.delete(se, top[: k + 1]).mean() / 3) /
                                               np.sqrt((s ** 2).mean())) for k in range(len(top))],
           "top": []}
    print(json.dumps({k: v for k, v in out.items() if k != "top"}), flush=True)
    # per-sample radiance of the top pixels on the GPU: one 1-spp pass per sample index
    tp = pix[top]
    gs = np.zeros((len(tp), a.spp, 3), np.float32)
    for k in range(a.spp):
        dev.reset_film()
        dev.render_pass(1, off + k)
        f = dev.read_film()[0].reshape(-1, 4)
        gs[:, k] = f[tp, :3] / np.maximum(f[tp, 3:4], 1)
        if k % 256 == 0:
            print(f"gpu per-sample pass {k}", flush=True)
    for j, p in enumerate(tp):
        ent = {"pixel": int(p), "xy": [int(p % W), int(p // W)], "gpu": g[top[j]].tolist(), "cpu": s[top[j]].tolist(),
               "share": float(se[top[j]] / se.sum()), "samples": []}
        for k in range(a.spp):
            rays, L, cv = osc.path_rays(cfg, tree, int(p), off + k)
            d = np.abs(gs[j, k] - L).max()
            if d <= 1e-3 * max(float(np.abs(L).max()), float(np.abs(gs[j, k]).max()), 1e-6):
                continue
            smp = {"sample": off + k, "gpu_L": gs[j, k].tolist(), "cpu_L": L.tolist(), "rays": int(len(rays))}
            if watch:  # replay the path with the kernels' vertex log
                assert wl.pg_debug_watch(int(p), off + k) == 0
                dev.reset_film()
                dev.render_pass(1, off + k)
                gv = np.zeros((256, 32), np.float32)
                nv = C.c_uint32()
                assert wl.pg_debug_watch_read(gv.ctypes.data, 256, C.byref(nv)) == 0
                gv = gv[: nv.value]
                gv = gv[np.argsort(gv[:, 0], kind="stable")]
                smp["first_vertex_difference"] = first_difference(gv, cv)
                smp["gpu_vertices"] = gv.tolist()
                smp["cpu_vertices"] = cv.tolist()
            # re-trace the oracle path's rays on the GPU: first disagreement
            for i, r in enumerate(rays):
                kind = int(r[0])
                q = r[1:9][None].copy()
                h = dev.trace_rays(q, any_hit=kind == 1)[0]
                if kind == 1:
                    if bool(h[0] > 0.5) != bool(r[9] > 0.5):
                        smp["first_ray_mismatch"] = {"index": i, "kind": "shadow", "ray": q[0].tolist(),
                                                     "gpu_occluded": float(h[0]), "cpu_occluded": float(r[9])}
                        break
                    continue
                gp, cp = int(h[1:2].view(np.uint32)[0]), int(r[10:11].view(np.uint32)[0])
                if gp != cp or (gp != 0xFFFFFFFF and abs(h[0] - r[9]) > 1e-4 * max(1.0, abs(r[9]))):
                    b = osc.trace_brute(q)[0]
                    smp["first_ray_mismatch"] = {"index": i, "kind": "closest", "ray": q[0].tolist(),
                                                 "gpu": [float(h[0]), gp, float(h[2]), float(h[3])],
                                                 "cpu": [float(r[9]), cp],
                                                 "brute": [float(b[0]), int(b[1:2].view(np.uint32)[0])]}
                    break
            else:
                smp["first_ray_mismatch"] = None  # every ray of the oracle path traces alike: shading arithmetic
            ent["samples"].append(smp)
        out["top"].append(ent)
        print(json.dumps({k: v for k, v in ent.items() if k != "samples"}), len(ent["samples"]), "diverged samples",
              flush=True)
        for smp in ent["samples"][:4]:
            print("   ", json.dumps({k: v for k, v in smp.items() if not k.endswith("_vertices")}), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    integ.postprocess()


if __name__ == "__main__":
    main()
