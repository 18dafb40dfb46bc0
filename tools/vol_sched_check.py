"""Which k_volpath scheduling variants change films / trees?  (development check, one GPU)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer, ProgressiveVolumetricPathTracer  # noqa: E402

sc = pg.scenes.smoke(96, 96, res=48)
for guided in (False, True):
    out = {}
    for r, w in (("1", "0"), ("1", "0"), ("24", "0"), ("64", "0"), ("40", "2"), ("40", "8"), ("1", "1")):
        os.environ["PG_VOL_REFILL"], os.environ["PG_VOL_SURF_WAIT"] = r, w
        if guided:
            t = GuidedVolumetricPathTracer({"trainingIterations": 3, "samplesPerProgression": 8})
        else:
            t = ProgressiveVolumetricPathTracer({"samplesPerProgression": 8})
        t.preprocess(sc)
        rgbw, sq = t.render(8)
        tree = t.dev.get_sdtree() if guided else None
        t.postprocess()
        key = (r, w)
        if out:
            r0 = next(iter(out.values()))
            d = np.abs(rgbw - r0[0])
            print("guided" if guided else "plain", key, "film identical" if np.array_equal(rgbw, r0[0]) else
                  f"film DIFF {int((d > 0).any(-1).sum())} px max {d.max():.3g}",
                  "" if tree is None else ("tree identical" if np.array_equal(tree, r0[2]) else "tree DIFF"), flush=True)
        out.setdefault(key, (rgbw, sq, tree))
