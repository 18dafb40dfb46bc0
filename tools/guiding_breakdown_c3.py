"""Does guiding pay at equal time on C3, and where does it lose?  

Times the guided C3 job in several configurations (each the best of two warm runs, the whole job:
training, exchange-free splat + refit, final render) and the unguided path tracer, renders the unguided
tracer at the spp each guided job's wall clock buys, and compares relMSE (bench.py errors: the image
exposed to mean 1; trim999; dark median) against the 65,536-spp ground truth.  The per-pixel breakdown
splits the summed relMSE of each image into pixel classes -- the ground truth's dark pixels (the camera
room lit through the door gap) and bright pixels, and the glint pixels (the 0.1 % of pixels with the
largest unguided equal-spp error) -- so the classes where guiding wins and loses are visible.  The glint class is chosen on the unguided
image, so the class ratios are selection-biased; tools/outlier_paths_c3.py has the
unbiased per-sample decomposition.

  python tools/guiding_breakdown_c3.py OUT.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "albedo_prior (bench)": {"bsdfSamplingFractionBound": "albedo", "glossyPrior": True},
    "albedo_prior + inversevar": {"bsdfSamplingFractionBound": "albedo", "glossyPrior": True,
                                  "sampleCombination": "inversevar"},
    "learned_prior + inversevar": {"bsdfSamplingFractionBound": "learned", "glossyPrior": True,
                                   "sampleCombination": "inversevar"},
    "albedo_prior, 4 iterations": {"bsdfSamplingFractionBound": "albedo", "glossyPrior": True, "trainingIterations": 4},
}


def rel_map(x, gt):
    d2 = (x.astype(np.float64) - gt) ** 2
    return (d2 / (gt.astype(np.float64) ** 2 + 1e-2 * float(gt.mean()) ** 2)).mean(-1).ravel()


def main():
    out_path = sys.argv[1]
    import pgload
    pg = pgload.load()
    import bench
    from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer
    scene = pg.scenes.ajar_door(1280, 720)
    gt, _ = bench.load_gt()
    spp = 1024
    dev = Device(pg.capi.default_config())
    dev.upload(scene)
    dev.render_pass(spp, 0)
    ug = bench.image(dev.read_film()[0])
    best = float("inf")
    for _ in range(2):
        dev.reset_film()
        t = time.perf_counter()
        dev.render_pass(spp, 0)
        dev.read_film()
        best = min(best, time.perf_counter() - t)
    rate = spp / best
    rel_u = rel_map(ug, gt)
    n = len(rel_u)
    dark = (gt.mean(-1) < gt.mean()).ravel()
    glint = np.zeros(n, bool)
    glint[np.argsort(rel_u)[::-1][: n // 1000]] = True
    classes = {"dark (gt < mean)": dark & ~glint, "bright": ~dark & ~glint, "glint (worst 0.1 % unguided)": glint}

    def breakdown(rel):
        return {k: {"pixels": int(m.sum()), "relmse_sum_share": round(float(rel[m].sum() / n / max(rel.mean(), 1e-30)), 4),
                    "relmse_mean": round(float(rel[m].mean()), 5)} for k, m in classes.items()}

    res = {"unguided_1024": dict(bench.errors(ug, gt), seconds=round(best, 4), breakdown=breakdown(rel_u)),
           "configs": {}}
    print(json.dumps({"unguided_seconds": best}), flush=True)
    for name, props in CONFIGS.items():
        p = {"trainingIterations": 5, "samplesPerProgression": spp, **props}
        integ = GuidedPathTracer(p, device=0)
        integ.preprocess(scene)
        tbest, img = float("inf"), None
        for run in range(3):  # the first run warms up
            integ.reset()
            t = time.perf_counter()
            rgbw, _sq = integ.render(spp)
            el = time.perf_counter() - t
            if run > 0:
                tbest = min(tbest, el)
            img = bench.image(rgbw)
        integ.postprocess()
        spp_eq = max(1, int(round(tbest * rate)))
        dev.reset_film()
        done = 0
        while done < spp_eq:
            k = min(1024, spp_eq - done)
            dev.render_pass(k, done)
            done += k
        ue = bench.image(dev.read_film()[0])
        g, u, u1 = bench.errors(img, gt), bench.errors(ue, gt), res["unguided_1024"]
        rel_g, rel_ue = rel_map(img, gt), rel_map(ue, gt)
        bg, bu = breakdown(rel_g), breakdown(rel_ue)
        entry = {"props": props, "job_seconds": round(tbest, 4), "unguided_equal_time_spp": spp_eq,
                 "guided": g, "unguided_equal_time": u,
                 "ratio_equal_spp": {m: round(g[m] / u1[m], 4) for m in ("relmse", "relmse_trim999", "relmse_dark_median")},
                 "ratio_equal_time": {m: round(g[m] / u[m], 4) for m in ("relmse", "relmse_trim999", "relmse_dark_median")},
                 "breakdown_guided": bg, "breakdown_unguided_equal_time": bu,
                 "class_ratio_equal_time": {k: round(bg[k]["relmse_mean"] / max(bu[k]["relmse_mean"], 1e-30), 4) for k in classes}}
        res["configs"][name] = entry
        print(json.dumps({"config": name, "job_seconds": entry["job_seconds"], "equal_spp": entry["ratio_equal_spp"],
                          "equal_time": entry["ratio_equal_time"], "class_ratio_equal_time": entry["class_ratio_equal_time"]}),
              flush=True)
    dev.close()
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
