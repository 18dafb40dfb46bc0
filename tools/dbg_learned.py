"""Debug helper: where do the GPU and oracle learned-mode trees differ after a refit?"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import pgload
import oracle_py as O
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device
from test_learned_fraction import tree_alphas
sc = pg.scenes.cornell(48, 48)
cfg = pg.capi.default_config(guiding=1, s_tree_threshold=400.0, bsdf_fraction_bound=pg.capi.PG_FRACTION_LEARNED)
osc = O.OracleScene(pg.capi, sc)
ot = O.OracleSDTree(osc)
d = Device(cfg); d.upload(sc)
off = 0
for it in range(3):
    O.render(osc, cfg, 2 ** it, off, record=True, sdtree=ot)
    off += 2 ** it
    recs = ot.take_records(pg.capi)
    d.splat_records(recs); ot.splat_bytes(recs)
    gs = d.get_tree_stats()
    d.refit(it); ot.refit(it, cfg)
    g, c = d.get_sdtree(), ot.serialize()
    print("it", it, "len", len(g), len(c), "equal", np.array_equal(g, c))
    if not np.array_equal(g, c) and len(g) == len(c):
        diff = np.flatnonzero(g != c)
        print("  first diffs", diff[:10], "n", len(diff))
        ag, ac = tree_alphas(g), tree_alphas(c)
        print("  alphas differ at", np.flatnonzero(ag != ac)[:10], ag[ag != ac][:10], ac[ag != ac][:10])
        ns, nd, nsamp, nb = (int(x) for x in np.frombuffer(g[48:64].tobytes(), np.uint32))
        print("  layout snodes end", 64 + 8 * ns, "meta end", 64 + 8 * ns + 32 * nd, "samp end", 64 + 8 * ns + 32 * nd + 32 * nsamp)
        frac = gs[-11 * nd:].reshape(nd, 11)
        bad = np.flatnonzero(ag != ac)
        for b in bad[:3]:
            print("  leaf", b, "stats", frac[b].view(np.int64))
