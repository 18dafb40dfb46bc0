"""Repeated guided kitchen training on fresh contexts (iterations 0..3), per-pass record/film hashes and
statistics; --lanes N sets pg_config.path_lanes (1 serialises the chunks)."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device  # noqa: E402

lanes = int(sys.argv[sys.argv.index("--lanes") + 1]) if "--lanes" in sys.argv else 0
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 6
md5 = lambda a: hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()[:8]
sc = pg.scenes.kitchen(192, 108)
seen = {}
for r in range(reps):
    d = Device(pg.capi.default_config(guiding=1, s_tree_threshold=2000.0, path_lanes=lanes))
    d.upload(sc)
    off = 0
    out = []
    for it in range(4):
        s0 = d.stats()
        d.render_pass(2 ** it, off, True)
        s1 = d.stats()
        rec = d.get_records().reshape(-1, 32)
        if "--dump" in sys.argv and it == 1:
            np.save(os.path.join(ROOT, "gpurun_out", f"kit_rec_it1_{lanes}_{r}.npy"), rec[np.lexsort(rec.T[::-1])])
        out.append(f"{it}:{len(rec)}:{md5(rec[np.lexsort(rec.T[::-1])])}:{md5(d.read_film()[0])}:"
                   f"seg{s1['segments'] - s0['segments']}:sh{s1['shadow_rays'] - s0['shadow_rays']}")
        d.splat_local()
        d.refit(it)
        off += 2 ** it
    d.close()
    line = " ".join(out)
    seen[line] = seen.get(line, 0) + 1
    print(f"lanes {lanes} rep {r}: {line}", flush=True)
print(f"lanes {lanes}: {len(seen)} distinct outcome(s) in {reps} runs")
