"""Wall-clock split of one C3 guided job (bench configuration): each training iteration's recording pass,
splat and refit, then the final render; two jobs, the second reported."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import GuidedPathTracer  # noqa: E402

sc = pg.scenes.ajar_door(1280, 720)
integ = GuidedPathTracer({"trainingIterations": 5, "samplesPerProgression": 1024, "bsdfSamplingFractionBound": "albedo",
                          "glossyPrior": True})
integ.preprocess(sc)
dev = integ.dev
for job in range(2):
    integ.reset()
    ph = []
    t0 = time.perf_counter()
    for it in range(5):
        a = time.perf_counter()
        dev.render_pass(2 ** it, integ.sample_offset, record=True)
        integ.sample_offset += 2 ** it
        b = time.perf_counter()
        dev.splat_local()
        c = time.perf_counter()
        dev.refit(it)
        d = time.perf_counter()
        ph.append({"it": it, "pass_ms": 1e3 * (b - a), "splat_ms": 1e3 * (c - b), "refit_ms": 1e3 * (d - c)})
    t1 = time.perf_counter()
    dev.reset_film()
    dev.render_pass(1024, integ.sample_offset)
    dev.read_film()
    t2 = time.perf_counter()
    print(json.dumps({"job": job, "train_ms": 1e3 * (t1 - t0), "final_ms": 1e3 * (t2 - t1), "iterations": ph}), flush=True)
integ.postprocess()
