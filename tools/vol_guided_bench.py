"""C5 guided volpath probe (one GPU): the guided job (5 training iterations of 1..16 spp + a final
render) on the smoke scene, its throughput, and equal-spp relative RMSE of guided (distance guiding
off / on) vs unguided renders against a high-spp unguided ground truth.
  python tools/vol_guided_bench.py [--size 256] [--res 256] [--spp 64] [--gt-spp 8192]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--gt-spp", type=int, default=8192)
    ap.add_argument("--betas", default="0,0.5")
    a = ap.parse_args()
    import pgload
    pg = pgload.load()
    from mitsuba_path_guiding_amd.integrator import Device, GuidedVolumetricPathTracer
    sc = pg.scenes.smoke(a.size, a.size, res=a.res)
    vcfg = dict(integrator=pg.capi.PG_INTEGRATOR_VOLPATH)

    def img(film):
        rgbw, _ = film
        return rgbw[..., :3] / np.maximum(rgbw[..., 3:], 1)

    dev = Device(pg.capi.default_config(seed=4242, **vcfg))
    dev.upload(sc)
    t = time.perf_counter()
    chunk = 512
    for k in range(0, a.gt_spp, chunk):
        dev.render_pass(chunk, k)
    gt = img(dev.read_film())
    print(f"ground truth {a.gt_spp} spp: {time.perf_counter() - t:.1f} s", flush=True)
    dev.close()
    denom = np.mean(gt) ** 2

    def rel_rmse(x):
        return float(np.sqrt(np.mean((x - gt) ** 2) / denom))

    out = {"scene": f"smoke {a.size}^2, grid {a.res}^3", "spp": a.spp}
    dev = Device(pg.capi.default_config(**vcfg))
    dev.upload(sc)
    dev.render_pass(1, 1 << 20)
    dev.reset_film()
    s0 = dev.stats()
    t = time.perf_counter()
    dev.render_pass(a.spp, 1 << 21)
    film = dev.read_film()
    el = time.perf_counter() - t
    s1 = dev.stats()
    out["unguided"] = {"rel_rmse": rel_rmse(img(film)), "mpaths_s": round((s1["paths"] - s0["paths"]) / el / 1e6, 2)}
    dev.close()
    for beta in [float(b) for b in a.betas.split(",")]:
        integ = GuidedVolumetricPathTracer({"trainingIterations": 5, "distanceGuiding": beta})
        integ.preprocess(sc)
        integ.render(1)  # warm-up job
        integ.reset()
        t = time.perf_counter()
        integ.train()
        tt = time.perf_counter() - t
        integ.dev.reset_film()
        t2 = time.perf_counter()
        integ.dev.render_pass(a.spp, integ.sample_offset)
        film = integ.dev.read_film()
        tr = time.perf_counter() - t2
        st = integ.postprocess()
        train_paths = a.size * a.size * 31
        out[f"guided_beta{beta}"] = {
            "rel_rmse": rel_rmse(img(film)), "train_s": round(tt, 3), "render_s": round(tr, 3),
            "render_mpaths_s": round(a.size * a.size * a.spp / tr / 1e6, 2),
            "job_mpaths_s": round((train_paths + a.size * a.size * a.spp) / (tt + tr) / 1e6, 2),
            "stree_nodes": st["stree_nodes"], "dtree_nodes": st["dtree_nodes"]}
        print(json.dumps(out[f"guided_beta{beta}"]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
