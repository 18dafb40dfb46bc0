"""Benchmark: Mpaths/s of the SD-tree guided integrator on the Veach ajar-door-class scene (C3).

A step is one complete guided render job of C3 (BASELINE.json configs[2]): 1280x720, five training
progressions of 1, 2, 4, 8, 16 spp (training-record write, RCCL all-gather of records across ranks,
fixed-point splat, SD-tree refit) followed by the 1024-spp final render with the trained tree —
(31 + 1024) x 921,600 = 972.3 M camera paths per step.  Inputs (scene, BVH, path buffers) are
resident in HBM before timing starts.  With N ranks the image tiles are sharded (total work fixed:
"strong" scaling); value = all paths of the job / max-over-ranks wall time.

Also reported: the dominant kernel's roofline (algorithmic bytes per launch, SURVEY.md §8d /
DESIGN.md §"Measurement", over its HIP-event-measured average duration on a one-lane context, since
the timed job overlaps three lanes), the timed-region pipeline figure, and on rank 0 at N=1 the
CPU oracle timed on a bounded sample of the same job (kind "port"), plus the equal-spp relative RMSE
between GPU and CPU on that sample.

  python bench.py [--gpus N --steps K --warmup W] [--spp 1024] [--no-cpu] [--quick]
  python bench.py --scene smoke      # C5: the guided volumetric job on the 256^3 smoke cloud at 1024^2
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# algorithmic bytes per unit (DESIGN.md §"Measurement"; SURVEY.md §8d decomposition of B_seg)
BYTES_TRACE_PER_RAY = 52      # queue id 4 + ray o/tmin 16 + ray d/tmax 16 + hit write 16
BYTES_SHADOW_PER_RAY = 84     # queue id 4 + shadow ray 32 + contribution 16 + radiance RMW 32
BYTES_SHADE_PER_VERTEX = 488  # path state read 96 + write 96 + tri gather 80 + material 32 + shadow write 48
#                               + emitter-tri gather 80 + training vertex 48 + queue writes 8
BYTES_DENSITY_LOOKUP = 32     # k_volpath (C5): one trilinear lookup gathers 8 f32 voxels


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="ajar_door")
    ap.add_argument("--width", type=int, default=None, help="default 1280 (C3), 1024 (C5 smoke)")
    ap.add_argument("--height", type=int, default=None, help="default 720 (C3), 1024 (C5 smoke)")
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--train", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--lanes", type=int, default=0, help="path chunks in flight (pg_config.path_lanes, 0 = 3)")
    ap.add_argument("--paths-in-flight", type=int, default=0, help="paths per chunk (0 = 2^22)")
    ap.add_argument("--exchange", default="allreduce", choices=["allreduce", "allgather"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--quick", action="store_true", help="small smoke configuration (not a bench line)")
    return ap.parse_args()


def main():
    a = parse()
    vol = a.scene == "smoke"  # C5: guided volumetric path tracer on the smoke cloud
    if a.width is None:
        a.width = 1024 if vol else 1280
    if a.height is None:
        a.height = 1024 if vol else 720
    if a.quick:
        a.width, a.height, a.spp, a.steps, a.warmup = 320, 180, 64, 1, 1
    import pgload
    pg = pgload.load()
    from mitsuba_path_guiding_amd import distributed as D
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer, GuidedVolumetricPathTracer

    rank, world, local = D.env_rank()
    world = max(world, 1)
    # RCCL ("nccl") over xGMI; PG_DIST_BACKEND=gloo rehearses the multi-rank path with ranks
    # sharing the visible GPUs (collectives through host memory)
    backend = os.environ.get("PG_DIST_BACKEND", "nccl")
    if world > 1:
        D.init(backend)
    import torch

    on_dev = torch.cuda.is_available() and backend == "nccl"
    device = local % max(1, torch.cuda.device_count())
    scene = pg.scenes.SCENES[a.scene](a.width, a.height)
    # postprogression exchange: all-reduce of the SD-tree building statistics
    exchange = D.make_exchange(on_dev, mode=a.exchange) if world > 1 else None
    # one progression for the final render (the device chunks it into waves of <= 4M paths)
    Tracer = GuidedVolumetricPathTracer if vol else GuidedPathTracer
    integ = Tracer({"trainingIterations": a.train, "samplesPerProgression": a.spp, "pathLanes": a.lanes,
                    "maxPathsInFlight": a.paths_in_flight}, device=device,
                   rank=rank, world_size=world, exchange=exchange)
    integ.preprocess(scene)
    dev = integ.dev

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def job():
        integ.reset()
        integ.render(a.spp)

    for _ in range(a.warmup):
        job()
    barrier()
    s0 = dev.stats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        job()
    barrier()
    elapsed = time.perf_counter() - t0
    s1 = dev.stats()
    if world > 1:
        elapsed = D.max_over_ranks(elapsed, on_dev)
    paths_per_job = (2 ** a.train - 1 + a.spp) * a.width * a.height
    total_paths = paths_per_job * a.steps
    value = total_paths / elapsed / 1e6

    # ---- timed-region pipeline figure: algorithmic bytes of trace + shade + shadow per wall second
    d = {k: s1[k] - s0[k] for k in s1}
    if vol:
        pipe_bytes = d["density_lookups"] * BYTES_DENSITY_LOOKUP
        pipeline = {"achieved": round(pipe_bytes / elapsed / 1e9, 2), "unit": "GB/s",
                    "frac": round(pipe_bytes / elapsed / 1e9 / HBM_PEAK_GBS, 5),
                    "algorithmic_bytes_per_step": int(pipe_bytes / a.steps),
                    "note": "density-grid gathers of k_volpath over the timed wall clock"}
        roofline = volume_roofline(d)
    else:
        pipe_bytes = d["segments"] * (BYTES_TRACE_PER_RAY + BYTES_SHADE_PER_VERTEX) + d["shadow_rays"] * BYTES_SHADOW_PER_RAY
        pipeline = {"achieved": round(pipe_bytes / elapsed / 1e9, 2), "unit": "GB/s",
                    "frac": round(pipe_bytes / elapsed / 1e9 / HBM_PEAK_GBS, 5),
                    "algorithmic_bytes_per_step": int(pipe_bytes / a.steps),
                    "note": "all path kernels over the timed wall clock (3 path lanes run concurrently)"}
        roofline = kernel_roofline(pg, scene, integ, device, a)

    # ---- CPU baseline (oracle, rank 0, N = 1, bounded sample) + equal-spp RMSE on the sample
    cpu = None
    rmse = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu, rmse = cpu_baseline(pg, scene, integ, a)

    if rank == 0:
        line = {
            "metric": "Mpaths/sec + equal-spp RMSE vs CPU ref, ajar-door scene at 1/2/4/8 GPUs",
            "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{'C5' if vol else 'C3'} {a.scene} {a.width}x{a.height}, guided SD-tree"
                                   f"{' volpath (phase MIS + guided free flight)' if vol else ''}, {a.train} training "
                                   f"iterations (1..{2 ** (a.train - 1)} spp) + {a.spp} spp render",
                       "scene": a.scene, "triangles": scene.num_triangles, "width": a.width, "height": a.height,
                       "spp": a.spp, "training_iterations": a.train, "paths_per_step": paths_per_job,
                       "parallelism": f"tile-shard x{world}, RCCL {a.exchange} per training iteration"},
            "roofline": roofline,
            "pipeline": pipeline,
            "cpu_baseline": cpu,
            "rmse_vs_cpu": rmse,
            "segments_per_path": round(d["segments"] / max(d["paths"], 1), 3),
            "kernel_event_ms_per_step": {k: round(d[k] / a.steps, 2)
                                         for k in (("volume_ms",) if vol else ("trace_ms", "shade_ms", "shadow_ms"))},
        }
        print(json.dumps(line), flush=True)
    integ.postprocess()
    if world > 1:
        torch.distributed.destroy_process_group()


def kernel_roofline(pg, scene, integ, local, a, spp=32):
    """Roofline of the dominant kernel.  The timed job runs three path lanes concurrently, so a HIP
    event pair around one launch also covers the other lanes' kernels; per-kernel durations are
    therefore measured on a one-lane context (same scene, same trained SD-tree, guided final-render
    passes, launches serialized on one stream) right after the timed region."""
    from mitsuba_path_guiding_amd.integrator import Device
    cfg = pg.capi.default_config(guiding=1, device=local, path_lanes=1, rank=integ.dev.cfg.rank,
                                 world_size=integ.dev.cfg.world_size)
    dev = Device(cfg)
    dev.upload(scene)
    dev.put_sdtree(integ.dev.get_sdtree())
    off = 2 ** a.train - 1
    # no warm-up pass: the kernels are loaded by the timed job, and the rocprofv3 summary of this
    # context's stream (tools/pmc_summary.py "calibration") must cover exactly these launches
    s0 = dev.stats()
    dev.render_pass(spp, off)
    s1 = dev.stats()
    d = {k: s1[k] - s0[k] for k in s1}
    kernels = {  # name: (total ms, algorithmic bytes, launches)
        "k_trace": (d["trace_ms"], d["segments"] * BYTES_TRACE_PER_RAY, d["trace_launches"]),
        "k_shade": (d["shade_ms"], d["segments"] * BYTES_SHADE_PER_VERTEX, d["shade_launches"]),
        "k_shadow": (d["shadow_ms"], d["shadow_rays"] * BYTES_SHADOW_PER_RAY, d["trace_launches"]),
    }
    dev.close()
    dom = max(kernels, key=lambda k: kernels[k][0])
    ms, nbytes, launches = kernels[dom]
    achieved = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            traffic = pj.get("kernels", {}).get(dom, {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": dom,
            "algorithmic_bytes_per_launch": int(nbytes / max(launches, 1)),
            "avg_launch_ms": round(ms / max(launches, 1), 4),
            "measured": f"1-lane context, guided {scene.width}x{scene.height} x {spp} spp with the trained tree",
            "kernels": {k: {"ms": round(v[0], 2), "launches": int(v[2]),
                            "achieved_gbs": round(v[1] / (v[0] / 1e3) / 1e9, 2) if v[0] > 0 else 0.0}
                        for k, v in kernels.items()}}


def volume_roofline(d):
    """k_volpath (C5) roofline from the timed job itself: the volumetric path runs one launch at a time
    on the context stream, so its HIP-event durations are exact.  Algorithmic bytes = density-grid
    gathers (8 voxels x 4 B per lookup); the 64 MiB grid stays in the 256 MiB Infinity Cache, so
    this is an on-die gather rate measured against the HBM peak."""
    ms, launches = d["volume_ms"], max(d["volume_launches"], 1)
    nbytes = d["density_lookups"] * BYTES_DENSITY_LOOKUP
    achieved = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_volpath_latest.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("kernels", {}).get("k_volpath", {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": "k_volpath",
            "algorithmic_bytes_per_launch": int(nbytes / launches), "avg_launch_ms": round(ms / launches, 4),
            "density_lookups_per_launch": int(d["density_lookups"] / launches),
            "measured": "timed job, HIP events around every k_volpath launch (one stream)"}


def cpu_baseline(pg, scene, integ, a):
    """Time the oracle (CPU restatement, all host cores) on a bounded sample of the same job: the
    guided final render of the first tiles with the GPU-trained SD-tree, then compare GPU vs CPU at
    equal spp on those pixels."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O  # checker / CPU baseline only
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = max(1, min(cores, 16))  # the GPU box's CPU share is 16 threads
    osc = O.OracleScene(pg.capi, scene)
    tree = O.OracleSDTree(osc)
    tree.deserialize(integ.dev.get_sdtree())
    cfg = pg.capi.default_config(guiding=1)
    vol = a.scene == "smoke"
    if vol:
        cfg = integ.cfg  # guided volpath, same parameters as the GPU job
    W = scene.width
    T = 32
    tiles = []
    for ty in range(0, scene.height, T):
        for tx in range(0, W, T):
            tiles.append([(y * W + x) for y in range(ty, min(ty + T, scene.height)) for x in range(tx, min(tx + T, W))])
    spp = 64
    off = 2 ** a.train - 1
    # warm up on one tile, calibrate on 16 tiles from the image centre, then size the sample to
    # ~cpu_seconds of work
    mid = len(tiles) // 2
    O.render(osc, cfg, 4, off, sdtree=tree, pixels=np.array(tiles[mid], np.uint32), nthreads=cores)
    cal = np.array([p for i in range(16) for p in tiles[(mid + i) % len(tiles)]], np.uint32)
    t = time.perf_counter()
    O.render(osc, cfg, spp, off, sdtree=tree, pixels=cal, nthreads=cores)
    per_tile = (time.perf_counter() - t) / 16
    ntiles = int(max(1, min(len(tiles), a.cpu_seconds / max(per_tile, 1e-4))))
    sel = [tiles[(mid + i) % len(tiles)] for i in range(ntiles)]
    pix = np.array([p for tl in sel for p in tl], np.uint32)
    t = time.perf_counter()
    c_rgbw, _, st = O.render(osc, cfg, spp, off, sdtree=tree, pixels=pix, nthreads=cores)
    dt = time.perf_counter() - t
    cpu = {"value": round(float(st[0]) / dt / 1e6, 4), "unit": "Mpaths/s", "cores": cores, "kind": "port",
           "sample": f"{ntiles} tiles of 32x32 ({len(pix)} px) x {spp} spp of the guided {'C5' if vol else 'C3'} final render "
                     f"with the GPU-trained SD-tree ({int(st[0])} paths, {dt:.1f} s)"}
    # equal-spp GPU render of the same sample indices (fresh film; timed region is over)
    integ.dev.reset_film()
    integ.dev.render_pass(spp, off, False)
    g_rgbw, _ = integ.dev.read_film()
    g = g_rgbw.reshape(-1, 4)[pix]
    c = c_rgbw.reshape(-1, 4)[pix]
    gm = g[:, :3] / np.maximum(g[:, 3:4], 1)
    cm = c[:, :3] / np.maximum(c[:, 3:4], 1)
    rmse = float(np.sqrt(np.mean((gm - cm) ** 2)) / max(float(np.sqrt(np.mean(cm ** 2))), 1e-12))
    rel = np.abs(gm - cm).max(-1) / np.maximum(cm.max(-1), 1e-3)
    return cpu, {"relative_rmse": round(rmse, 6), "pixels_diverged_frac": round(float((rel > 1e-3).mean()), 6),
                 "spp": spp, "pixels": int(len(pix)),
                 "note": "same RNG streams on both sides; a path whose fp32 libm/FMA rounding flips one "
                         "branch diverges, so the RMSE is dominated by the few diverged firefly pixels"}


if __name__ == "__main__":
    main()
