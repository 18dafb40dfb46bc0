"""Determinism of the 4-shard kitchen training (tests/test_gpu_configs.py::test_c4_guided_four_rank_shard):
per iteration, md5 of every context's sorted records and film, and of the trees after the exchange."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device  # noqa: E402


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()[:8]


def dev(sc, **cfg):
    d = Device(pg.capi.default_config(**cfg))
    d.upload(sc)
    return d


PROBE = "--probe" in sys.argv
sc = pg.scenes.kitchen(192, 108)
cfg = dict(guiding=1, s_tree_threshold=2000.0)
full = dev(sc, **cfg)
shards = [dev(sc, rank=r, world_size=4, **cfg) for r in range(4)]
off = 0
for it in range(4):
    line = []
    for name, d in [("F", full)] + [(f"S{r}", s) for r, s in enumerate(shards)]:
        d.render_pass(2 ** it, off, True)
        if PROBE:
            rec = d.get_records().reshape(-1, 32)
            rec = rec[np.lexsort(rec.T[::-1])]
            line.append(f"{name}:{len(rec)}:{md5(rec)}:{md5(d.read_film()[0])}")
    if "--probe2" in sys.argv:
        rec = full.get_records().reshape(-1, 32)
        line.append(f"Frec:{len(rec)}:{md5(rec[np.lexsort(rec.T[::-1])])}:{md5(full.read_film()[0])}")
    full.splat_local()
    full.refit(it)
    for d in shards:
        d.splat_local()
    total = sum(d.get_tree_stats() for d in shards)
    for d in shards:
        d.put_tree_stats(total)
        d.refit(it)
    off += 2 ** it
    print(f"it {it} " + " ".join(line) + f" treeF {md5(full.get_sdtree())} treeS {md5(shards[0].get_sdtree())}", flush=True)
