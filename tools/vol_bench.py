"""C5 volumetric throughput probe: smoke scene (256^3 fBm grid) at 1024^2, unguided volpath.
  python tools/vol_bench.py [--spp 8] [--res 256] [--size 1024] [--steps 2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--scale", type=float, default=40.0)
    ap.add_argument("--global-majorant", action="store_true")
    a = ap.parse_args()
    import pgload
    pg = pgload.load()
    from mitsuba_path_guiding_amd.integrator import Device
    t = time.time()
    sc = pg.scenes.smoke(a.size, a.size, res=a.res, scale=a.scale)
    print("scene", round(time.time() - t, 2), "s", flush=True)
    dev = Device(pg.capi.default_config(integrator=pg.capi.PG_INTEGRATOR_VOLPATH,
                                        volume_majorant=int(a.global_majorant)))
    dev.upload(sc)
    dev.render_pass(1, 0)  # warm-up
    s0 = dev.stats()
    t = time.perf_counter()
    for k in range(a.steps):
        dev.render_pass(a.spp, 1 + k * a.spp)
    el = time.perf_counter() - t
    s1 = dev.stats()
    d = {k: s1[k] - s0[k] for k in s1}
    out = {"mpaths_s": round(d["paths"] / el / 1e6, 3), "wall_s": round(el, 3), "paths": d["paths"],
           "segments_per_path": round(d["segments"] / d["paths"], 3),
           "nee_per_path": round(d["shadow_rays"] / d["paths"], 3),
           "volume_ms": round(d["volume_ms"], 2), "launches": d["volume_launches"]}
    print(json.dumps(out), flush=True)
    rgbw, _ = dev.read_film()
    import numpy as np
    np.save(os.path.join(ROOT, "gpurun_out", "smoke_img.npy"), (rgbw[..., :3] / np.maximum(rgbw[..., 3:], 1)).astype(np.float16))
    dev.close()


if __name__ == "__main__":
    main()
