"""Traversal statistics of the C3 calibration pass (the travstats build, PG_LIB=.../build_travstats/libpgamd.so):
closest-hit walks, node visits and triangle tests per walk; any-hit walks, node visits, triangle tests per walk."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer, library  # noqa: E402

lib = library()
lib.pg_debug_trav_stats.argtypes = [C.c_void_p, C.c_int]
sc = pg.scenes.ajar_door(1280, 720)
integ = GuidedPathTracer({"trainingIterations": 5, "bsdfSamplingFractionBound": "albedo", "glossyPrior": True})
integ.preprocess(sc)
integ.train()
blob = integ.dev.get_sdtree()
out = np.zeros(8, np.uint64)
assert lib.pg_debug_trav_stats(out.ctypes.data, 1) == 0
cfg = pg.capi.default_config(guiding=1, path_lanes=1, bsdf_fraction_bound=integ.cfg.bsdf_fraction_bound,
                             glossy_prior=integ.cfg.glossy_prior)
d = Device(cfg)
d.upload(sc)
d.put_sdtree(blob)
d.render_pass(32, 31)
assert lib.pg_debug_trav_stats(out.ctypes.data, 1) == 0
cw, cv, ct, _, aw, av, at, _ = (int(x) for x in out)
print(f"closest-hit walks {cw}, node visits/walk {cv / cw:.2f}, triangle tests/walk {ct / cw:.2f}")
print(f"any-hit walks {aw}, node visits/walk {av / aw:.2f}, triangle tests/walk {at / aw:.2f}")
d.close()
integ.postprocess()
