"""k_volpath refill threshold (PG_VOL_REFILL): films and trees must not depend on it (every work item
draws from its own stream and writes its own slot).  Development check, one GPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import GuidedVolumetricPathTracer  # noqa: E402

sc = pg.scenes.smoke(128, 128, res=64)
ref = None
for r in ("1", "16", "48"):
    os.environ["PG_VOL_REFILL"] = r
    t = GuidedVolumetricPathTracer({"trainingIterations": 3, "samplesPerProgression": 16})
    t.preprocess(sc)
    rgbw, sq = t.render(16)
    tree = t.dev.get_sdtree()
    t.postprocess()
    if ref is None:
        ref = (rgbw, sq, tree)
    else:
        same = np.array_equal(rgbw, ref[0]) and np.array_equal(sq, ref[1]) and np.array_equal(tree, ref[2])
        print("refill", r, "identical" if same else "DIFFERENT", flush=True)
        assert same
print("ok")
