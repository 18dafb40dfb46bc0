"""Train the bench's guided C3 job's SD-tree on the GPU and save its serialized blob (tools/dtree_depths.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import GuidedPathTracer  # noqa: E402

integ = GuidedPathTracer({"trainingIterations": 5, "bsdfSamplingFractionBound": "albedo", "glossyPrior": True})
integ.preprocess(pg.scenes.ajar_door(1280, 720))
integ.train()
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "c3_tree.npy")
os.makedirs(os.path.dirname(out), exist_ok=True)
np.save(out, integ.dev.get_sdtree())
print("saved", out, integ.dev.stats()["stree_nodes"], integ.dev.stats()["dtree_nodes"])
