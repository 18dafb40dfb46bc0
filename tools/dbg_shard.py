"""Debug helper: full context vs 4 tile-shard contexts, per training iteration (record counts, building stats)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import pgload
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device
name = sys.argv[1] if len(sys.argv) > 1 else "kitchen"
sc = pg.scenes.SCENES[name](192, 108)
cfg = dict(guiding=1, s_tree_threshold=2000.0)
def mk(**k):
    d = Device(pg.capi.default_config(**cfg, **k)); d.upload(sc); return d
full = mk(); shards = [mk(rank=r, world_size=4) for r in range(4)]
full2 = mk()
print("bvh/tree equal at start:", all(np.array_equal(d.get_sdtree(), full.get_sdtree()) for d in shards))
rays = np.random.default_rng(1).random((200000, 8)).astype(np.float32)
lo, hi = sc.bounds(); rays[:, :3] = lo + (hi - lo) * rays[:, :3]; rays[:, 3] = 1e-4
d = np.random.default_rng(2).normal(size=(200000, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
rays[:, 4:7] = d; rays[:, 7] = np.inf
h0 = full.trace_rays(rays); print("trace equal full vs shard0:", np.array_equal(h0.view(np.uint32), shards[0].trace_rays(rays).view(np.uint32)), "full vs full2:", np.array_equal(h0.view(np.uint32), full2.trace_rays(rays).view(np.uint32)))
off = 0
for it in range(4):
    full.render_pass(2 ** it, off, True)
    full2.render_pass(2 ** it, off, True)
    for s in shards: s.render_pass(2 ** it, off, True)
    ff = full.read_film()[0]; fs = sum(s.read_film()[0] for s in shards)
    bad = np.argwhere((ff != fs).any(-1))
    print("   film pixels differing:", len(bad), bad[:8].tolist(), [ (ff[y,x].tolist(), fs[y,x].tolist()) for y, x in bad[:3]])
    full.reset_film(); full2.reset_film()
    for s in shards: s.reset_film()
    rc = [s.record_count() for s in shards]
    print(it, "records full", full.record_count(), "full2", full2.record_count(), "shards", rc, sum(rc))
    ra = np.frombuffer(full.get_records().tobytes(), np.float32).reshape(-1, 8)
    rb = np.concatenate([np.frombuffer(s.get_records().tobytes(), np.float32).reshape(-1, 8) for s in shards])
    ka = np.sort(ra.view(np.uint32)[:, :6].copy().view("V24").ravel()); kb = np.sort(rb.view(np.uint32)[:, :6].copy().view("V24").ravel())
    print("   records equal as multisets:", len(ka) == len(kb) and bool(np.all(ka == kb)))
    full.splat_local(); full2.splat_local()
    for s in shards: s.splat_local()
    tf = full.get_tree_stats(); tot = sum(s.get_tree_stats() for s in shards)
    diff = np.nonzero(tf != tot)[0]
    print("   stats words", len(tf), "differ", len(diff), diff[:10], "full==full2", np.array_equal(tf, full2.get_tree_stats()))
    for s in shards: s.put_tree_stats(tot)
    full.refit(it); full2.refit(it)
    for s in shards: s.refit(it)
    print("   trees equal:", [np.array_equal(s.get_sdtree(), full.get_sdtree()) for s in shards], np.array_equal(full.get_sdtree(), full2.get_sdtree()))
    off += 2 ** it
