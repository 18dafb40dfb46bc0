"""One-lane calibration pass of C3 (the bench's trained tree, 32 spp) with the bounce's shadow rays and closest hits
in separate launches (PG_NO_RAYS_FUSION=1): how k_rays' time splits between its any-hit and closest-hit halves."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer  # noqa: E402

sc = pg.scenes.ajar_door(1280, 720)
integ = GuidedPathTracer({"trainingIterations": 5, "bsdfSamplingFractionBound": "albedo", "glossyPrior": True})
integ.preprocess(sc)
integ.train()
blob = integ.dev.get_sdtree()
out = {}
for fuse in ("1", "0"):
    if fuse == "0":
        os.environ["PG_NO_RAYS_FUSION"] = "1"
    cfg = pg.capi.default_config(guiding=1, path_lanes=1, kernel_timing=1, bsdf_fraction_bound=integ.cfg.bsdf_fraction_bound,
                                 glossy_prior=integ.cfg.glossy_prior)
    d = Device(cfg)
    d.upload(sc)
    d.put_sdtree(blob)
    for rep in range(2):
        s0 = d.stats()
        d.render_pass(32, 31)
        s1 = d.stats()
        st = {k: s1[k] - s0[k] for k in ("trace_ms", "shade_ms", "shadow_ms", "rays_ms", "trace_launches", "shadow_launches",
                                         "rays_launches", "segments", "shadow_rays", "paths")}
        out[f"fused{fuse}_rep{rep}"] = st
        print(f"fused={fuse} rep={rep}", json.dumps(st), flush=True)
    d.close()
integ.postprocess()
