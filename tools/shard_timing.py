"""Strong-scaling rehearsal on ONE GPU (development helper): time rank 0's shard of the C3 job for
world sizes 1, 2, 4, 8 (tile shard = 1/W of the image, local splat only, no collective), with the
training / final-render split.  Rank 0's time at W approximates the N=W job time minus the
all-reduce of the tree statistics (a few MB per iteration over xGMI)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import GuidedPathTracer  # noqa: E402

sc = pg.scenes.ajar_door(1280, 720)
worlds = [int(w) for w in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "2", "4", "8"])]
base = None
for W in worlds:
    # the bench's guided configuration (bench.py BENCH_GUIDING)
    integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": 1024,
                              "bsdfSamplingFractionBound": "albedo", "glossyPrior": True}, rank=0, world_size=W)
    integ.preprocess(sc)
    d = integ.dev
    best = None
    for rep in range(3):
        integ.reset()
        t0 = time.perf_counter()
        ph = {}
        off = 0
        for it in range(5):
            t = time.perf_counter()
            d.render_pass(2 ** it, off, True)
            off += 2 ** it
            t1 = time.perf_counter()
            d.splat_local()
            t2 = time.perf_counter()
            d.refit(it)
            t3 = time.perf_counter()
            ph[f"p{it}"] = (t1 - t) * 1e3
            ph[f"s{it}"] = (t2 - t1) * 1e3
            ph[f"r{it}"] = (t3 - t2) * 1e3
        t_train = time.perf_counter() - t0
        d.reset_film()
        d.render_pass(1024, off, False)
        d.read_film()
        tot = time.perf_counter() - t0
        if best is None or tot < best[0]:
            best = (tot, t_train, ph)
    tot, t_train, ph = best
    if base is None:
        base = tot
    print(f"W={W}: job {tot*1e3:.1f} ms  train {t_train*1e3:.1f} ms  final {(tot-t_train)*1e3:.1f} ms  "
          f"est. speedup {base/tot:.2f}x", flush=True)
    print("   " + " ".join(f"{k}={v:.1f}" for k, v in ph.items()), flush=True)
    integ.postprocess()
