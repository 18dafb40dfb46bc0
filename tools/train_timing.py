"""Host-side timing of the guided training loop phases on C3 (development helper)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import GuidedPathTracer

sc = pg.scenes.ajar_door(1280, 720)
world = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # emulate rank 0 of `world` (its tile shard)
integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": 1024}, rank=0, world_size=world)
integ.preprocess(sc)
d = integ.dev
for rep in range(int(os.environ.get("PG_TRAIN_REPS", 2))):
    T = {}
    def tm(k, f, *a, **kw):
        t = time.perf_counter(); r = f(*a, **kw); T[k] = T.get(k, 0) + time.perf_counter() - t; return r
    t0 = time.perf_counter()
    tm("reset", integ.reset)
    off = 0
    for it in range(5):
        tm(f"pass{it}", d.render_pass, 2 ** it, off, True)
        off += 2 ** it
        tm(f"splat{it}", d.splat_local)
        tm(f"refit{it}", d.refit, it)
    tm("reset_film", d.reset_film)
    if not os.environ.get("PG_TRAIN_ONLY"):
        tm("final", d.render_pass, 1024, off, False)
    print(f"world {world} rep {rep}: total {time.perf_counter()-t0:.3f} s  " + "  ".join(f"{k} {v*1e3:.1f}" for k, v in T.items()), flush=True)
    st = d.stats()
    print("  stree", st["stree_nodes"], "dtree", st["dtree_nodes"], flush=True)
