import sys, numpy as np
sys.path.insert(0, '/root/repo')
import pgload
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device
for name, sc in [("cornell", pg.scenes.cornell(64, 64)), ("ajar", pg.scenes.ajar_door(320, 180))]:
    d = Device(pg.capi.default_config()); d.upload(sc)
    lo, hi = sc.bounds(); rng = np.random.default_rng(1); n = 20000
    o = lo + (hi - lo) * rng.random((n, 3)); dd = rng.normal(size=(n, 3)); dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32); r[:, 0:3] = o; r[:, 3] = 1e-4; r[:, 4:7] = dd; r[:, 7] = np.inf
    h = d.trace_rays(r)
    print(name, "nodes/ray", h[:, 2].mean(), "tris/ray", h[:, 3].mean(), "max nodes", h[:, 2].max(), flush=True)
