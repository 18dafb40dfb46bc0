"""How much of k_shade is the SD-tree (guided vs unguided shading on the same C3 scene, one lane).

Prints per-segment shading time for: unguided, guided with the trained tree.  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer  # noqa: E402

sc = pg.scenes.ajar_door(1280, 720)
g = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": 4})
g.preprocess(sc)
g.render(4)
tree = g.dev.get_sdtree()
g.postprocess()
for guided in (0, 1):
    d = Device(pg.capi.default_config(guiding=guided, path_lanes=1, kernel_timing=1))
    d.upload(sc)
    if guided:
        d.put_sdtree(tree)
    d.render_pass(2, 31)
    s0 = d.stats()
    d.render_pass(32, 33)
    s1 = d.stats()
    x = {k: s1[k] - s0[k] for k in s1}
    seg = max(x["segments"], 1)
    print(f"guided={guided}: shade {x['shade_ms']:.1f} ms, trace {x['trace_ms']:.1f} ms, shadow {x['shadow_ms']:.1f} ms, "
          f"segments {seg}, shade ns/segment {x['shade_ms'] * 1e6 / seg:.2f}, trace ns/seg {x['trace_ms'] * 1e6 / seg:.2f}",
          flush=True)
    d.close()
