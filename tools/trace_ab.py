"""Dump closest hits of a fixed ray set (C3 scene) for A/B comparison of traversal builds.
  PG_LIB=... python tools/trace_ab.py OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pgload  # noqa: E402
from test_gpu_parity import random_rays  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device  # noqa: E402

sc = pg.scenes.ajar_door(1280, 720)
d = Device(pg.capi.default_config())
d.upload(sc)
rays = random_rays(sc, 1_500_000, 3)
h = d.trace_rays(rays)
a = d.trace_rays(rays, any_hit=True)
np.savez_compressed(sys.argv[1], h=h, a=a[:, 0])
print("hits", (h[:, 1].view(np.uint32) != 0xFFFFFFFF).mean())
