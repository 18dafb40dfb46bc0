"""C4 kitchen sanity: upload (BVH build), unguided pass timing, small-image parity vs oracle (dev helper)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import pgload
pg = pgload.load()
import oracle_py as O
from mitsuba_path_guiding_amd.integrator import Device, GuidedPathTracer
t = time.time(); sc = pg.scenes.kitchen(1920, 1080); print("scene", sc.num_triangles, "tris", f"{time.time()-t:.1f}s", flush=True)
d = Device(pg.capi.default_config())
t = time.time(); d.upload(sc); print("upload", f"{time.time()-t:.2f}s", flush=True)
d.render_pass(1, 0)
t = time.time(); d.render_pass(16, 1); dt = time.time() - t
st = d.stats(); n = 1920 * 1080 * 16
print(f"unguided {n/dt/1e6:.1f} Mpaths/s seg/path {st['segments']/st['paths']:.2f}", flush=True)
d.close()
integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": 64})
integ.preprocess(sc)
t = time.time(); integ.render(64); dt = time.time() - t
st = integ.postprocess()
print(f"guided job 31+64 spp: {(31+64)*1920*1080/dt/1e6:.1f} Mpaths/s, records {st['records']}, snodes {st['stree_nodes']}", flush=True)
small = pg.scenes.kitchen(96, 54)
d = Device(pg.capi.default_config()); d.upload(small); d.render_pass(64, 0); g = d.read_film(); d.close()
c = O.render(O.OracleScene(pg.capi, small), pg.capi.default_config(), 64, nthreads=16)[:2]
n1 = np.maximum(g[0][..., 3:4], 1); n2 = np.maximum(c[0][..., 3:4], 1)
m1, m2 = g[0][..., :3] / n1, c[0][..., :3] / n2
v1 = np.maximum(g[1][..., :3] / n1 - m1 ** 2, 0) / n1; v2 = np.maximum(c[1][..., :3] / n2 - m2 ** 2, 0) / n2
z = (m1 - m2) / np.sqrt(v1 + v2 + 1e-12)
print("kitchen 96x54 parity: |z|<5 frac", (np.abs(z) < 5).mean(), "mean rel", abs(m1.mean() - m2.mean()) / m2.mean(), flush=True)
