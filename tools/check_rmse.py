"""GPU vs oracle agreement at equal RNG streams, and 1-lane vs 3-lane bit-identity (development helper)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import pgload
pg = pgload.load()
import oracle_py as O
from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer

def rel_rmse(g, c):
    gm = g[..., :3] / np.maximum(g[..., 3:4], 1)
    cm = c[..., :3] / np.maximum(c[..., 3:4], 1)
    d = np.abs(gm - cm).max(-1) / np.maximum(cm.max(-1), 1e-3)
    return float(np.sqrt(np.mean((gm - cm) ** 2)) / np.sqrt(np.mean(cm ** 2))), float((d > 1e-3).mean())

for name, sc in [("cornell", pg.scenes.cornell(128, 128)), ("ajar", pg.scenes.ajar_door(320, 180))]:
    osc = O.OracleScene(pg.capi, sc)
    spp = 16
    films = {}
    for lanes in (1, 3):
        d = Device(pg.capi.default_config(path_lanes=lanes))
        d.upload(sc)
        d.render_pass(spp, 0)
        films[lanes] = d.read_film()[0]
        d.close()
    c = O.render(osc, pg.capi.default_config(), spp, nthreads=16)[0]
    print(name, "unguided lanes1==lanes3:", np.array_equal(films[1], films[3]), "rmse/diverged vs oracle:", rel_rmse(films[3], c), flush=True)
    integ = GuidedPathTracer({"trainingIterations": 4, "samplesPerProgression": spp})
    integ.preprocess(sc)
    integ.render(spp)
    tree = O.OracleSDTree(osc)
    tree.deserialize(integ.dev.get_sdtree())
    off = 2 ** 4 - 1
    integ.dev.reset_film()
    integ.dev.render_pass(spp, off, False)
    g = integ.dev.read_film()[0]
    c = O.render(osc, pg.capi.default_config(guiding=1), spp, off, sdtree=tree, nthreads=16)[0]
    print(name, "guided rmse/diverged vs oracle:", rel_rmse(g, c), flush=True)
