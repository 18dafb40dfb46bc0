"""Quality half of the headline metric on C3: relative error of the guided
job against a high-spp unguided ground truth, next to the unguided path tracer at equal spp and at
equal time.  One GPU.

  python tools/quality_c3.py [--gt-spp 65536] [--spp 1024] [--save-gt gpurun_out/c3_gt.npz]
                             [--gt gpurun_out/c3_gt.npz]   # reuse a ground truth

Error metrics (per pixel, per channel, over the whole image; gt = ground-truth mean):
  rel_rmse = sqrt(mean((x - gt)^2)) / mean(gt)
  relmse   = mean((x - gt)^2 / (gt^2 + 1e-2))      (Mueller et al. 2017's relMSE convention)
  relmse_exposed = the same with epsilon 1e-2 * mean(gt)^2, i.e. on the image exposed to mean 1
    (C3 is dark: mean 0.0018, so the absolute 1e-2 turns relmse into a plain MSE of the bright
    door-gap pixels); _trim999 drops the worst 0.1 % of pixels (single-sample fireflies);
    _dark is the median over pixels darker than the image mean (the camera room lit through the gap)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def img(film):
    rgbw = film[0]
    return rgbw[..., :3] / np.maximum(rgbw[..., 3:], 1)


def load_gt(path):
    z = np.load(path)
    if "mean" in z:
        return z["mean"].astype(np.float32)
    return z["mean_x256"].astype(np.float32) / np.float32(z["scale"])  # tests/golden/c3_gt.npz


def errors(x, gt):
    d2 = (x.astype(np.float64) - gt) ** 2
    g2 = gt.astype(np.float64) ** 2
    rel = (d2 / (g2 + 1e-2 * float(gt.mean()) ** 2)).mean(-1).ravel()
    trim = np.sort(rel)[: int(len(rel) * 0.999)]
    dark = (gt.mean(-1) < gt.mean()).ravel()
    return {"rel_rmse": round(float(np.sqrt(d2.mean()) / gt.mean()), 6),
            "relmse": round(float((d2 / (g2 + 1e-2)).mean()), 7),
            "relmse_exposed": round(float(rel.mean()), 5),
            "relmse_exposed_trim999": round(float(trim.mean()), 5),
            "relmse_exposed_dark": round(float(np.median(rel[dark])), 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="ajar_door")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--gt-spp", type=int, default=65536)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--train", type=int, default=5)
    ap.add_argument("--gt", default=None, help="existing ground truth (.npz with 'mean')")
    ap.add_argument("--save-gt", default=None)
    ap.add_argument("--props", default="{}", help="extra guided-integrator properties (JSON)")
    ap.add_argument("--dump", default=None, help="save the compared images (.npz, f16)")
    ap.add_argument("--reps", type=int, default=3, help="timed runs per render (best wall clock)")
    a = ap.parse_args()
    import pgload
    pg = pgload.load()
    from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer
    sc = pg.scenes.SCENES[a.scene](a.width, a.height)
    npx = a.width * a.height
    out = {"scene": f"{a.scene} {a.width}x{a.height}", "spp": a.spp, "train": a.train}

    if a.gt:
        gt = load_gt(a.gt)
        out["gt"] = {"file": a.gt}
    else:
        dev = Device(pg.capi.default_config(seed=4242))  # independent streams from every render below
        dev.upload(sc)
        t = time.perf_counter()
        for k in range(0, a.gt_spp, 1024):
            dev.render_pass(min(1024, a.gt_spp - k), k)
            if k % 8192 == 0:
                print(f"gt {k} spp {time.perf_counter() - t:.1f} s", flush=True)
        gt = img(dev.read_film())
        el = time.perf_counter() - t
        dev.close()
        out["gt"] = {"spp": a.gt_spp, "seconds": round(el, 1), "mpaths_s": round(a.gt_spp * npx / el / 1e6, 1),
                     "seed": 4242, "integrator": "unguided progressive path tracer (GPU, oracle-parity-tested)"}
        if a.save_gt:
            np.savez_compressed(a.save_gt, mean=gt, spp=a.gt_spp)
    print(json.dumps(out["gt"]), flush=True)
    out["gt_mean"] = round(float(gt.mean()), 6)

    # ---- unguided at equal spp
    dev = Device(pg.capi.default_config())
    dev.upload(sc)
    dev.render_pass(16, 1 << 24)  # warm-up
    dev.reset_film()
    dev.render_pass(a.spp, 0)
    dev.read_film()
    # wall clocks: the best of a.reps runs (the renders are deterministic, so every run gives the same
    # image); one cold measurement on a fresh box can be 10-15 % off
    tu = float("inf")
    for _ in range(a.reps):
        dev.reset_film()
        s0 = dev.stats()
        t = time.perf_counter()
        dev.render_pass(a.spp, 0)
        ug = img(dev.read_film())
        tu = min(tu, time.perf_counter() - t)
        s1 = dev.stats()
    rate = a.spp * npx / tu
    dumps = {"unguided": ug}
    seg_u = (s1["segments"] - s0["segments"]) / max(1, s1["paths"] - s0["paths"])
    out["unguided_equal_spp"] = dict(errors(ug, gt), seconds=round(tu, 3), mpaths_s=round(rate / 1e6, 1),
                                     segments_per_path=round(seg_u, 4), gsegments_s=round(rate * seg_u / 1e9, 3))
    print("unguided", json.dumps(out["unguided_equal_spp"]), flush=True)

    # ---- guided job (training + final render), discard and inverse-variance combination
    props = json.loads(a.props)
    tg = None
    for comb in ("discard", "inversevar"):
        integ = GuidedPathTracer(dict({"trainingIterations": a.train, "samplesPerProgression": a.spp,
                                       "sampleCombination": comb}, **props))
        integ.preprocess(sc)
        integ.render(a.spp)  # warm-up job
        el = float("inf")
        for _ in range(a.reps):
            integ.reset()
            s0 = integ.dev.stats()
            t = time.perf_counter()
            rgbw, sq = integ.render(a.spp)
            el = min(el, time.perf_counter() - t)
            st = integ.dev.stats()
        seg_g = (st["segments"] - s0["segments"]) / max(1, st["paths"] - s0["paths"])
        x = rgbw[..., :3] / np.maximum(rgbw[..., 3:], 1)
        dumps[comb] = x
        r = dict(errors(x, gt), seconds=round(el, 3),
                 mpaths_s=round((2 ** a.train - 1 + a.spp) * npx / el / 1e6, 1),
                 stree_nodes=int(st["stree_nodes"]), dtree_nodes=int(st["dtree_nodes"]),
                 segments_per_path=round(seg_g, 4),
                 gsegments_s=round((st["segments"] - s0["segments"]) / el / 1e9, 3))
        if comb == "inversevar":
            r["weights"] = [round(w, 4) for w in integ.combination_weights]
        else:
            tg = el
        out[f"guided_{comb}"] = r
        print(comb, json.dumps(r), flush=True)
        integ.postprocess()

    # ---- unguided at equal time (the whole guided job's wall clock, training included)
    spp_eq = max(1, int(tg * rate / npx))
    dev.reset_film()
    t = time.perf_counter()
    done = 0
    while done < spp_eq:
        k = min(1024, spp_eq - done)
        dev.render_pass(k, done)
        done += k
    ue = img(dev.read_film())
    out["unguided_equal_time"] = dict(errors(ue, gt), spp=spp_eq, seconds=round(time.perf_counter() - t, 3))
    dev.close()
    g = out["guided_discard"]
    out["guided_vs_unguided"] = {
        "relmse_ratio_equal_spp": round(g["relmse"] / out["unguided_equal_spp"]["relmse"], 4),
        "relmse_ratio_equal_time": round(g["relmse"] / out["unguided_equal_time"]["relmse"], 4),
        "rel_rmse_ratio_equal_spp": round(g["rel_rmse"] / out["unguided_equal_spp"]["rel_rmse"], 4),
        "rel_rmse_ratio_equal_time": round(g["rel_rmse"] / out["unguided_equal_time"]["rel_rmse"], 4),
        "exposed_ratio_equal_spp": round(g["relmse_exposed"] / out["unguided_equal_spp"]["relmse_exposed"], 4),
        "exposed_ratio_equal_time": round(g["relmse_exposed"] / out["unguided_equal_time"]["relmse_exposed"], 4)}
    iv = out["guided_inversevar"]  # every iteration's film, inverse-variance weighted (same wall clock + combine)
    out["inversevar_vs_unguided"] = {
        "relmse_ratio_equal_time": round(iv["relmse"] / out["unguided_equal_time"]["relmse"], 4),
        "exposed_ratio_equal_time": round(iv["relmse_exposed"] / out["unguided_equal_time"]["relmse_exposed"], 4)}
    print(json.dumps(out), flush=True)
    if a.dump:
        np.savez_compressed(a.dump, **{k: v.astype(np.float16) for k, v in dumps.items()})


if __name__ == "__main__":
    main()
