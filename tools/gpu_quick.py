"""Quick GPU sanity/timing run (development helper)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import pgload
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer

for name, sc, spp in [("cornell", pg.scenes.cornell(512, 512), 64), ("ajar", pg.scenes.ajar_door(1280, 720), 16)]:
    d = Device(pg.capi.default_config(kernel_timing=1))
    t = time.time(); d.upload(sc); print(name, "upload", time.time() - t, "tris", sc.num_triangles, flush=True)
    d.render_pass(1, 0)
    t = time.time(); d.render_pass(spp, 1); dt = time.time() - t
    st = d.stats()
    n = sc.width * sc.height * spp
    print(name, f"unguided {n/dt/1e6:.1f} Mpaths/s, seg/path {st['segments']/st['paths']:.2f}, "
          f"trace {st['trace_ms']:.1f} shade {st['shade_ms']:.1f} shadow {st['shadow_ms']:.1f} ms", flush=True)
    f = d.read_film()[0]
    print(name, "mean", (f[..., :3].sum((0, 1)) / f[..., 3].sum()), flush=True)
    d.close()
    integ = GuidedPathTracer({"trainingIterations": 5})
    integ.preprocess(sc)
    t = time.time(); integ.render(spp); dt = time.time() - t
    st = integ.postprocess()
    print(name, f"guided job {st['paths']/dt/1e6:.1f} Mpaths/s records {st['records']} snodes {st['stree_nodes']} "
          f"dnodes {st['dtree_nodes']}", flush=True)
