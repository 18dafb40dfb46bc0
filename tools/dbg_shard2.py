"""Debug helper: which configuration factor makes a tile-shard context's paths differ from the full context's."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import pgload
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device
sc = pg.scenes.kitchen(192, 108)
def run(extra_full, extra_shard, label, spp_final=8):
    cfg = dict(guiding=1, s_tree_threshold=2000.0)
    def mk(**k):
        d = Device(pg.capi.default_config(**cfg, **k)); d.upload(sc); return d
    full = mk(**extra_full); shards = [mk(rank=r, world_size=4, **extra_shard) for r in range(4)]
    off = 0
    for it in range(3):
        full.render_pass(2 ** it, off, True); full.splat_local(); full.refit(it)
        for s in shards: s.render_pass(2 ** it, off, True); s.splat_local()
        tot = sum(s.get_tree_stats() for s in shards)
        for s in shards: s.put_tree_stats(tot); s.refit(it)
        off += 2 ** it
    assert all(np.array_equal(s.get_sdtree(), full.get_sdtree()) for s in shards)
    full.reset_film()
    for s in shards: s.reset_film()
    full.render_pass(spp_final, off, False)
    for s in shards: s.render_pass(spp_final, off, False)
    ff = full.read_film()[0]; fs = sum(s.read_film()[0] for s in shards)
    bad = np.argwhere((ff != fs).any(-1))
    print(label, "differing pixels:", len(bad), bad[:6].tolist(), flush=True)
    per = []
    for y, x in bad[:2]:
        for k in range(spp_final):
            full.reset_film(); [s.reset_film() for s in shards]
            full.render_pass(1, off + k, False); [s.render_pass(1, off + k, False) for s in shards]
            a = full.read_film()[0][y, x]; b = sum(s.read_film()[0] for s in shards)[y, x]
            if not np.array_equal(a, b): per.append((int(y), int(x), k, a.tolist(), b.tolist()))
    print("   per-sample:", per, flush=True)
    for d in shards + [full]: d.close()
run({}, {}, "default")
run(dict(path_lanes=1), dict(path_lanes=1), "lanes=1")
run(dict(max_paths_in_flight=5184 * 8), dict(max_paths_in_flight=5184 * 8), "cap=41472")
run(dict(bsdf_fraction_bound=0), dict(bsdf_fraction_bound=0), "fraction fixed")
