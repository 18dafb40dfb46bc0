"""Benchmark: Mpaths/s + equal-spp RMSE of the SD-tree guided integrator on the Veach ajar-door-class
scene (C3).

A step is one complete guided render job of C3 (BASELINE.json configs[2]): 1280x720, five training
progressions of 1, 2, 4, 8, 16 spp (training-record write, fixed-point splat, all-reduce of the
SD-tree building statistics across ranks, refit) followed by the 1024-spp final render with the
trained tree -- (31 + 1024) x 921,600 = 972.3 M camera paths per step.  Inputs (scene, BVH, path
buffers) are resident in HBM before timing starts.  With N ranks the image tiles are sharded (total
work fixed: "strong" scaling) and the film tiles are reduced to rank 0 inside the timed job;
value = all paths of the job / max-over-ranks wall time.

Also reported:
  roofline   the dominant kernel's algorithmic bytes per launch (SURVEY.md §8d's 420 B per segment,
             split per kernel) over its average launch on a one-lane calibration context
             (the timed job overlaps three lanes): the headline `frac` with the duration from the
             committed rocprofv3 kernel trace of those launches (profiles/pmc_latest.json), this run's
             HIP-event figure as `frac_hip_events`; `traffic` from the committed rocprofv3 PMC summary
             named in `traffic_source` (with its code revision);
  pipeline   §8d's pipeline figure: segments/s x 420 B over the timed wall clock;
  quality    (N = 1, C3 at 1280x720) relative errors of the timed job's guided image against the
             65,536-spp unguided ground truth tests/golden/c3_gt.npz, next to the unguided path
             tracer at equal spp and at equal time (tools/quality_c3.py has the definitions);
  cpu_baseline  (rank 0, N = 1) the CPU oracle running the same guided job on a bounded sample: the
             full 31-spp training (its own records, splat and refit) and the 1024-spp final render
             of a block of tiles; with the GPU/CPU relative-RMSE ratio on those tiles.

  python bench.py [--gpus N --steps K --warmup W] [--spp 1024] [--no-cpu] [--no-quality] [--quick]
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
# B_seg = 420 B per path segment (state read 72 + write 68, hit record write + read
# 32, hit-triangle gather 76, material 32, shadow-queue write + read 64, emitter-triangle gather 36,
# training record 40), split over the three path kernels:
BYTES_SEGMENT = 420
BYTES_TRACE_PER_RAY = 48       # ray o/d read 32 + hit write 16
BYTES_SHADE_PER_VERTEX = 300   # state read 40 + write 68 + hit read 16 + triangle 76 + material 32
#                                + shadow-queue write 32 + emitter triangle 36
BYTES_SHADE_RECORD = 40        # + training record (recording passes only)
BYTES_SHADOW_PER_RAY = 32      # shadow-queue read 32
assert BYTES_TRACE_PER_RAY + BYTES_SHADE_PER_VERTEX + BYTES_SHADE_RECORD + BYTES_SHADOW_PER_RAY == BYTES_SEGMENT
BYTES_DENSITY_LOOKUP = 32      # k_volpath (C5): one trilinear lookup gathers 8 f32 voxels
# the volumetric wavefront's SoA path state (pg_kernels.h VolWave) moved per item: a free flight reads
# origin, direction, its / medium record and random stream (64 B), writes the stream and the interaction
# point (32 B) and moves its two queue entries (8 B); an interaction reads the whole state and the
# interaction point (112 B), writes it back (96 B) and moves its queue entries (8 B)
BYTES_VOL_FLIGHT = 104
BYTES_VOL_VERTEX = 216
# round 5: the interactions' transmittance walks as a stage of their own (k_vnee): per walked slot the flags
# word (16 B), the NEE record (48 B), the random stream (16 B), L read + write (32 B) and the queue entry
# (4 B); an emitter walk through media adds its 48-B record (rare: not in the floor)
BYTES_VOL_NEE = 116
GT_C3 = os.path.join(ROOT, "tests", "golden", "c3_gt.npz")
GT_C3_CPU = os.path.join(ROOT, "tests", "golden", "c3_cpu_gt_tiles.npz")  # make_c3_cpu_gt.py


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Without a torchrun environment and N > 1, bench.py launches N "
                         "ranks itself (torch.distributed.run, 127.0.0.1); under torchrun N must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="ajar_door")
    ap.add_argument("--width", type=int, default=None, help="default 1280 (C3), 1024 (C5 smoke)")
    ap.add_argument("--height", type=int, default=None, help="default 720 (C3), 1024 (C5 smoke)")
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--train", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-quality", action="store_true")
    ap.add_argument("--lanes", type=int, default=0, help="path chunks in flight (pg_config.path_lanes, 0 = 3)")
    ap.add_argument("--paths-in-flight", type=int, default=0, help="paths per chunk (0 = auto: C3's final render on one GPU in 12 chunks, else 2^25)")
    ap.add_argument("--exchange", default=None, choices=["allreduce", "allgather", "capi", "capi-allgather"],
                    help="postprogression exchange (N > 1): the library's own RCCL communicator (pg_comm_*, the C++ "
                         "adapter's path): all-reduce of the tree statistics ('capi', default with RCCL) or all-gather "
                         "of the records ('capi-allgather'); or torch.distributed: 'allreduce' (default with "
                         "PG_DIST_BACKEND=gloo, whose ranks may share a GPU, which RCCL refuses) or 'allgather'")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="launcher self-test: every rank joins the process group and reports (rank, world); no GPU")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU budget of the final-render sample")
    ap.add_argument("--quick", action="store_true", help="small smoke configuration (not a bench line)")
    ap.add_argument("--props", default=None,
                    help="integrator properties (JSON); default: the guided configuration DESIGN.md §8a measured best "
                         "on C3 (albedo-bounded BSDF fraction + glossy prior)")
    return ap.parse_args()


def launch_ranks(n, argv):
    """Start n ranks of this script through torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) and return their exit status.  Runs in a parent that has not touched the GPU (no torch
    or library import yet): the ranks are child processes, never an exec of this one."""
    import socket
    import subprocess
    with socket.socket() as s:  # a free port for the rendezvous
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    return subprocess.call(cmd, env=env)


def deadline_seconds():
    """PG_BENCH_DEADLINE: seconds a multi-rank start-up stage may take before the rank exits naming the stuck
    rank (distributed.Watchdog); the first job (kernel loading, the first pg_comm collectives) gets 3x."""
    return float(os.environ.get("PG_BENCH_DEADLINE", "300"))


def first_collective(wd, world, on_dev):
    """One small all-reduce of the rank ids, timed and reported per rank (the first traffic of the group)."""
    import torch
    import torch.distributed as dist
    stall = os.environ.get("PG_BENCH_STALL_RANK")  # test hook: this rank stalls before its first collective
    if stall is not None and int(stall) == dist.get_rank():
        wd.stage("stall (test hook)")
        time.sleep(3600)
    wd.stage("first collective", collective=True)
    t0 = time.perf_counter()
    tdev = torch.device("cuda", torch.cuda.current_device()) if on_dev else torch.device("cpu")
    t = torch.tensor([float(dist.get_rank())], dtype=torch.float64, device=tdev)
    dist.all_reduce(t)
    total = float(t.item())
    wd._say(f"first collective complete in {time.perf_counter() - t0:.3f} s (rank sum {total:.0f}, "
            f"expected {world * (world - 1) / 2:.0f})")
    assert total == world * (world - 1) / 2, total
    return total


def plumbing_check(a, rank, world):
    """--plumbing-check: the launcher's rank / world wiring without a GPU (gloo process group)."""
    from mitsuba_path_guiding_amd import distributed as D
    import torch
    import torch.distributed as dist
    wd = D.Watchdog(rank, world, device="cpu", seconds=deadline_seconds())
    wd.stage("process group init", collective=True)
    D.init("gloo")
    wd.attach_store()
    assert dist.get_world_size() == world == a.gpus, (dist.get_world_size(), world, a.gpus)
    first_collective(wd, world, False)
    wd.done()
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", -1)),
                                 "world": dist.get_world_size(), "pid": os.getpid()})
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"plumbing_check": True, "n_gpus": world, "ranks": got,
                          "rank_sum": float(t.item())}), flush=True)
    dist.destroy_process_group()


def main():
    a = parse()
    rank, world, _ = (int(os.environ.get(k, d)) for k, d in (("RANK", 0), ("WORLD_SIZE", 1), ("LOCAL_RANK", 0)))
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        # the driver's `bench.py --gpus N` without torchrun: launch the N ranks here (before any GPU use)
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    if a.gpus is None:
        a.gpus = world
    if a.gpus != world:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)")
    if a.plumbing_check:
        import pgload
        pgload.load()
        return plumbing_check(a, rank, world)
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
    import torch
    if world > 1 and backend == "nccl" and torch.cuda.device_count() < world:
        sys.exit(f"bench.py: {world} ranks need {world} visible GPUs, found {torch.cuda.device_count()} "
                 "(PG_DIST_BACKEND=gloo rehearses ranks that share a GPU)")
    device = local % max(1, torch.cuda.device_count())
    # per-rank start-up report and deadlines (stderr; rank 0's stdout keeps the one JSON line)
    wd = D.Watchdog(rank, world, device=device, seconds=deadline_seconds()) if world > 1 else None
    if world > 1:
        wd.stage(f"process group init ({backend})", collective=True)
        D.init(backend)
        wd.attach_store()
        assert torch.distributed.get_world_size() == world == a.gpus

    on_dev = torch.cuda.is_available() and backend == "nccl"
    if world > 1:
        wd._say(f"world {world}, local rank {local}, device {device}"
                + (f" ({torch.cuda.get_device_name(device)})" if torch.cuda.is_available() else ""))
        first_collective(wd, world, on_dev)
        wd.stage("scene flatten + upload (pg_create, pg_upload_scene)")
    scene = pg.scenes.SCENES[a.scene](a.width, a.height)
    # postprogression exchange (N > 1): by default the library's own RCCL communicator (pg_comm_*, what
    # the C++ adapter runs): all-reduce of the SD-tree building statistics.  RCCL
    # refuses two ranks on one device, so gloo rehearsals use the torch.distributed exchange.
    if a.exchange is None:
        a.exchange = "capi" if backend == "nccl" else "allreduce"
    capi_comm = world > 1 and a.exchange.startswith("capi")
    if world > 1:
        exchange = (D.make_capi_exchange(mode="allgather" if a.exchange == "capi-allgather" else "allreduce")
                    if capi_comm else D.make_exchange(on_dev, mode=a.exchange))
    else:
        exchange = None
    # one progression for the final render (the device cuts it into 12 chunks on one GPU, 3 in flight)
    Tracer = GuidedVolumetricPathTracer if vol else GuidedPathTracer
    if a.props is None:
        a.props = "{}" if vol else json.dumps(BENCH_GUIDING)
    integ = Tracer({"trainingIterations": a.train, "samplesPerProgression": a.spp, "pathLanes": a.lanes,
                    "maxPathsInFlight": a.paths_in_flight, **json.loads(a.props)}, device=device,
                   rank=rank, world_size=world, exchange=exchange,
                   reduce_sum=D.make_reduce_sum(on_dev) if world > 1 else None)
    integ.preprocess(scene)
    dev = integ.dev
    if capi_comm:
        wd.stage("pg_comm_init (the library's RCCL communicator)", collective=True)
        D.init_capi_comm(dev)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def job():
        integ.reset()
        rgbw, sq = integ.render(a.spp)
        if capi_comm:  # RCCL reduce of the device films inside the library, then rank 0 reads it
            dev.comm_reduce_film(0)
            rgbw = dev.read_film()[0]
        elif world > 1:  # gather the disjoint film tiles on rank 0
            rgbw, sq = D.reduce_film(rgbw, sq, on_dev)
        return rgbw

    for w in range(a.warmup):
        if wd is not None and w == 0:  # kernel loading and the first pg_comm collectives
            wd.stage("first job (warm-up)", seconds=3 * deadline_seconds())
        job()
    if wd is not None:
        wd.stage("barrier before the timed region", collective=True)
    barrier()
    if wd is not None:
        wd.done()
    s0 = dev.stats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        final = job()
    barrier()
    elapsed = time.perf_counter() - t0
    s1 = dev.stats()
    if world > 1:
        elapsed = D.max_over_ranks(elapsed, on_dev)
    paths_per_job = (2 ** a.train - 1 + a.spp) * a.width * a.height
    total_paths = paths_per_job * a.steps
    value = total_paths / elapsed / 1e6

    # ---- §8d pipeline figure over the timed wall clock
    d = {k: s1[k] - s0[k] for k in s1}
    if world > 1:
        for k in ("segments", "escaped", "records", "shadow_rays", "density_lookups", "vol_flights", "vol_vertices"):
            d[k] = int(D.sum_over_ranks(d[k], on_dev))
    if vol:
        # density gathers (every lookup: k_vcam / k_vflight / k_vvertex / k_vtail, or k_volpath) plus the
        # wavefront's state traffic per flight and interaction (0 with the megakernel, PG_VOL_WAVEFRONT=0)
        pipe_bytes = (d["density_lookups"] * BYTES_DENSITY_LOOKUP + d.get("vol_flights", 0) * BYTES_VOL_FLIGHT +
                      d.get("vol_vertices", 0) * BYTES_VOL_VERTEX + d.get("vol_nee_walks", 0) * BYTES_VOL_NEE)
        pipeline = {"achieved": round(pipe_bytes / elapsed / 1e9, 2), "unit": "GB/s",
                    "frac": round(pipe_bytes / elapsed / 1e9 / HBM_PEAK_GBS, 5),
                    "algorithmic_bytes_per_step": int(pipe_bytes / a.steps),
                    "note": "density-grid gathers plus the wavefront stages' path-state bytes (bytes_model) over "
                            "the timed wall clock, all ranks"}
        roofline = volume_roofline(d, pg, scene, integ, device, a)
    else:
        # §8d's 420 B per segment, split by what each segment does: every segment is traced, escaped
        # ones are not shaded, only recording passes write training records, and only NEE vertices
        # send a shadow ray
        pipe_bytes = (d["segments"] * BYTES_TRACE_PER_RAY + (d["segments"] - d["escaped"]) * BYTES_SHADE_PER_VERTEX
                      + d["records"] * BYTES_SHADE_RECORD + d["shadow_rays"] * BYTES_SHADOW_PER_RAY)
        pipeline = {"achieved": round(pipe_bytes / elapsed / 1e9, 2), "unit": "GB/s",
                    "frac": round(pipe_bytes / elapsed / 1e9 / HBM_PEAK_GBS, 5),
                    "bytes_per_segment_nominal": BYTES_SEGMENT, "segments_per_step": int(d["segments"] / a.steps),
                    "algorithmic_bytes_per_step": int(pipe_bytes / a.steps),
                    "note": "SURVEY.md §8d over the timed wall clock, all ranks: segments x 48 B (trace) + shaded "
                            "segments x 300 B + training records x 40 B + shadow rays x 32 B"}
        roofline = kernel_roofline(pg, scene, integ, device, a)

    quality = None
    if rank == 0 and world == 1 and not vol and not a.no_quality:
        quality = quality_block(pg, scene, final, elapsed / a.steps, a)
    # ---- CPU baseline (oracle, rank 0, N = 1, bounded sample of the same guided job)
    cpu = None
    rmse = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu, rmse = cpu_baseline(pg, scene, integ, final, a)

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
                       "integrator_props": json.loads(a.props),
                       "parallelism": f"tile-shard x{world}, "
                                      + (f"{'RCCL' if backend == 'nccl' else backend} {a.exchange} per training iteration"
                                         if world > 1 else "no exchange (one rank)")
                                      + (", film reduce to rank 0" if world > 1 else "")},
            "roofline": roofline,
            "pipeline": pipeline,
            "quality": quality,
            "cpu_baseline": cpu,
            "rmse_vs_cpu": rmse,
            "segments_per_path": round(d["segments"] / max(total_paths, 1), 3),
        }
        print(json.dumps(line), flush=True)
    integ.postprocess()
    if world > 1:
        torch.distributed.destroy_process_group()


# C3's guided configuration: the BSDF-sampling fraction bounded below by the BSDF's
# albedo, and the glossy prior (BSDF::getGlossySamplingRate) -- rough metals and glass are not guided
BENCH_GUIDING = {"bsdfSamplingFractionBound": "albedo", "glossyPrior": True}


def kernel_roofline(pg, scene, integ, local, a, spp=32):
    """Roofline of the dominant kernel of the kernels the render ships: k_shade_all (every material
    class of a bounce in one launch), k_rays (a bounce's shadow rays + the next bounce's closest hits
    in one launch) and k_trace (the camera rays' closest hits).  The timed job runs three path lanes
    concurrently, so a HIP event pair around one launch would also cover the other lanes' kernels;
    the durations therefore come from a one-lane context (same scene, same trained SD-tree, a guided
    final-render pass without records, the same fused launches serialized on its one stream, each
    bracketed by a HIP event pair on that stream) right after the timed region.  rocprofv3 sees the
    same launches on that stream (tools/pmc_summary.py "calibration")."""
    from mitsuba_path_guiding_amd.integrator import Device
    cfg = pg.capi.default_config(guiding=1, device=local, path_lanes=1, kernel_timing=1, rank=integ.dev.cfg.rank,
                                 world_size=integ.dev.cfg.world_size,
                                 bsdf_fraction_bound=integ.cfg.bsdf_fraction_bound,
                                 glossy_prior=integ.cfg.glossy_prior)
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
    shaded = d["segments"] - d["escaped"]
    shade_name = "k_shade" if scene.envmap is not None else "k_shade_all"  # env scenes shade per class
    kernels = {  # name: (total ms, algorithmic bytes, launches); no records: no training-record bytes
        "k_trace": (d["trace_ms"], d["paths"] * BYTES_TRACE_PER_RAY, d["trace_launches"]),
        shade_name: (d["shade_ms"], shaded * BYTES_SHADE_PER_VERTEX, d["shade_launches"]),
        "k_rays": (d["rays_ms"], (d["segments"] - d["paths"]) * BYTES_TRACE_PER_RAY
                   + d["shadow_rays"] * BYTES_SHADOW_PER_RAY, d["rays_launches"]),
    }
    dev.close()
    # the HBM roofline is reported for the shipped kernel that carries the most algorithmic bytes
    # (the shading launch: ~70 % of SURVEY §8d's 420 B per segment); the traversal launches (k_rays,
    # k_trace) are latency-bound gathers of cache-resident BVH nodes, excluded from the byte model by
    # §8d, and are listed under "kernels" with their own time share and fraction
    dom = max(kernels, key=lambda k: kernels[k][1])
    total_ms = sum(v[0] for v in kernels.values()) or 1.0
    ms, nbytes, launches = kernels[dom]
    achieved = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    per_launch = nbytes / max(launches, 1)
    traffic, source, measured = None, None, {}
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            measured = pj.get("kernels", {})
            traffic = measured.get(dom, {}).get("hbm_bytes_per_launch")
            source = {"file": "profiles/pmc_latest.json", "profiled": pj.get("source"),
                      "revision": pj.get("revision")}
        except (OSError, ValueError):
            traffic = None
    out = {}
    for k, v in kernels.items():
        e = {"ms": round(v[0], 2), "launches": int(v[2]),
             "algorithmic_bytes_per_launch": int(v[1] / max(v[2], 1)),
             "avg_launch_ms": round(v[0] / max(v[2], 1), 4),
             "time_share": round(v[0] / total_ms, 3),
             "achieved_gbs": round(v[1] / (v[0] / 1e3) / 1e9, 2) if v[0] > 0 else 0.0,
             "frac": round(v[1] / (v[0] / 1e3) / 1e9 / HBM_PEAK_GBS, 5) if v[0] > 0 else 0.0}
        t = measured.get(k, {}).get("hbm_bytes_per_launch")
        if t and v[2]:
            e["traffic_bytes_per_launch"] = t
            e["traffic_over_algorithmic"] = round(t / (v[1] / v[2]), 3)
        cal = measured.get(k, {}).get("calibration_avg_ns")
        if cal and v[2]:  # the same launches' duration in the committed rocprofv3 summary
            e["avg_launch_ms_rocprof"] = round(cal / 1e6, 4)
            e["frac_rocprof"] = round(v[1] / v[2] / (cal / 1e9) / 1e9 / HBM_PEAK_GBS, 5)
        out[k] = e
    return {"bound": "hbm", **headline_frac(achieved, per_launch, ms / max(launches, 1), out[dom],
                                            profiled_workload(a, integ.dev.cfg.world_size)),
            "traffic": traffic, "traffic_source": source,
            "traffic_over_algorithmic": round(traffic / per_launch, 3) if traffic else None,
            "kernel": dom, "dominant_by": "algorithmic bytes per pass (time shares under kernels)",
            "algorithmic_bytes_per_launch": int(per_launch),
            "bytes_model": {"k_trace": f"{BYTES_TRACE_PER_RAY} B/camera ray",
                            shade_name: f"{BYTES_SHADE_PER_VERTEX} B/shaded vertex (+{BYTES_SHADE_RECORD} B when "
                                        "recording)",
                            "k_rays": f"{BYTES_TRACE_PER_RAY} B/bounce ray + {BYTES_SHADOW_PER_RAY} B/shadow ray",
                            "sum": f"{BYTES_SEGMENT} B/segment (SURVEY.md §8d)"},
            "measured": f"1-lane context, guided {scene.width}x{scene.height} x {spp} spp with the trained tree, "
                        f"no records; the fused launches the timed job runs, HIP events on the lane's stream",
            "kernels": out}


def profiled_workload(a, world):
    """Whether this run's calibration launches are the ones tools/profile.sh profiled: the default bench
    workload of its scene on one rank (a shard of N ranks, --quick or another size launches smaller passes)."""
    dflt = (1024, 1024) if a.scene == "smoke" else (1280, 720)
    return (world == 1 and a.scene in ("ajar_door", "smoke") and not a.quick and (a.width, a.height) == dflt
            and a.spp == 1024 and a.train == 5)


def headline_frac(achieved_hip, per_launch, avg_ms_hip, dom, profiled=True):
    """The roofline's headline figures.  `achieved` / `frac` / `avg_launch_ms` take the dominant kernel's
    average launch duration from the committed rocprofv3 kernel trace of the same calibration launches
    (profiles/pmc_*_latest.json "calibration_avg_ns"), so they reproduce from profiles/ alone; this run's
    HIP-event duration on the driver's box is reported beside them (`frac_hip_events`), with the ratio of
    the two boxes' durations named when they differ by more than 2 %.  Without a committed summary, or when
    this run's calibration is not the profiled workload (`profiled`: a rank of an N-GPU shard, --quick, another
    size), the HIP events are the headline."""
    cal_ms = dom.get("avg_launch_ms_rocprof")
    hip = {"frac_hip_events": round(achieved_hip / HBM_PEAK_GBS, 5), "avg_launch_ms_hip_events": round(avg_ms_hip, 4)}
    if not cal_ms or not profiled:
        why = "HIP events, this run" + ("" if not cal_ms else
                                        " (the committed profile is of the one-rank default workload, not this one)")
        return {"achieved": round(achieved_hip, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved_hip / HBM_PEAK_GBS, 5), "frac_source": why,
                "avg_launch_ms": round(avg_ms_hip, 4), **hip}
    achieved = per_launch / (cal_ms / 1e3) / 1e9
    out = {"achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
           "frac_source": "rocprofv3 kernel trace of the calibration launches (traffic_source file)",
           "avg_launch_ms": round(cal_ms, 4), **hip}
    ratio = avg_ms_hip / cal_ms
    if abs(ratio - 1) > 0.02:
        out["box_difference"] = (f"this run's HIP-event launch average is {ratio:.3f}x the profiled one: a different "
                                 "box (clocks, memory, other tenants) or a kernel revision newer than the profile")
    return out


def volume_roofline(d, pg=None, scene=None, integ=None, local=0, a=None, spp=64):
    """C5 roofline.  The volumetric wavefront (default): a calibration context after the timed region
    (same scene, the job's trained tree, a 64-spp final-render pass, pg_config.kernel_timing) times
    every free-flight (k_vflight) and interaction (k_vvertex) launch with a HIP event pair on its one
    stream; algorithmic bytes = density gathers (32 B per trilinear lookup) + the SoA path state each
    launch moves (BYTES_VOL_FLIGHT / BYTES_VOL_VERTEX per item); the kernel with the most bytes is
    reported.  With PG_VOL_WAVEFRONT=0: k_volpath from the timed job itself (one launch at a time on
    the context stream), density gathers only."""
    if os.environ.get("PG_VOL_WAVEFRONT", "1") != "0" and integ is not None:
        return wavefront_roofline(pg, scene, integ, local, a, spp)
    ms, launches = d["volume_ms"], max(d["volume_launches"], 1)
    nbytes = d["density_lookups"] * BYTES_DENSITY_LOOKUP
    achieved = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    traffic, source, cal = None, None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_volpath_latest.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            traffic = pj.get("kernels", {}).get("k_volpath", {}).get("hbm_bytes_per_launch")
            cal = pj.get("kernels", {}).get("k_volpath", {}).get("avg_ns")
            source = {"file": "profiles/pmc_volpath_latest.json", "profiled": pj.get("source"),
                      "revision": pj.get("revision")}
        except (OSError, ValueError):
            traffic = None
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_source": source,
            "frac_rocprof": round(nbytes / launches / (cal / 1e9) / 1e9 / HBM_PEAK_GBS, 5) if cal else None,
            "avg_launch_ms_rocprof": round(cal / 1e6, 4) if cal else None,
            "kernel": "k_volpath", "algorithmic_bytes_per_launch": int(nbytes / launches),
            "avg_launch_ms": round(ms / launches, 4),
            "density_lookups_per_launch": int(d["density_lookups"] / launches),
            "measured": "timed job, HIP events around every k_volpath launch (one stream)"}


def wavefront_roofline(pg, scene, integ, local, a, spp):
    from mitsuba_path_guiding_amd.integrator import Device
    cfg = type(integ.dev.cfg).from_buffer_copy(integ.dev.cfg)  # the job's configuration, stage timing on
    cfg.kernel_timing = 1
    dev = Device(cfg)
    dev.upload(scene)
    dev.put_sdtree(integ.dev.get_sdtree())
    s0 = dev.stats()
    dev.render_pass(spp, 2 ** a.train - 1)
    s1 = dev.stats()
    dev.close()
    d = {k: s1[k] - s0[k] for k in s1}
    kernels = {
        "k_vflight": (d["vol_flight_ms"], d["vol_flights"] * BYTES_VOL_FLIGHT + d["vol_flight_lookups"] * BYTES_DENSITY_LOOKUP,
                      d["vol_flight_launches"], d["vol_flight_lookups"]),
        "k_vvertex": (d["vol_vertex_ms"], d["vol_vertices"] * BYTES_VOL_VERTEX + d["vol_vertex_lookups"] * BYTES_DENSITY_LOOKUP,
                      d["vol_vertex_launches"], d["vol_vertex_lookups"]),
    }
    if d.get("vol_nee_launches"):
        kernels["k_vnee"] = (d["vol_nee_ms"], d["vol_nee_walks"] * BYTES_VOL_NEE + d["vol_nee_lookups"] * BYTES_DENSITY_LOOKUP,
                             d["vol_nee_launches"], d["vol_nee_lookups"])
    measured, source = {}, None
    pmc = os.path.join(ROOT, "profiles", "pmc_volpath_latest.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            measured = pj.get("kernels", {})
            source = {"file": "profiles/pmc_volpath_latest.json", "profiled": pj.get("source"), "revision": pj.get("revision")}
        except (OSError, ValueError):
            measured = {}
    out = {}
    total_ms = sum(v[0] for v in kernels.values()) or 1.0
    for k, (ms, nbytes, launches, lookups) in kernels.items():
        e = {"ms": round(ms, 2), "launches": int(launches), "algorithmic_bytes_per_launch": int(nbytes / max(launches, 1)),
             "density_lookups_per_launch": int(lookups / max(launches, 1)),
             "avg_launch_ms": round(ms / max(launches, 1), 4), "time_share": round(ms / total_ms, 3),
             "achieved_gbs": round(nbytes / (ms / 1e3) / 1e9, 2) if ms > 0 else 0.0,
             "frac": round(nbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5) if ms > 0 else 0.0}
        m = measured.get(k, {})
        if m.get("hbm_bytes_per_launch") and launches:
            e["traffic_bytes_per_launch"] = m["hbm_bytes_per_launch"]
            e["traffic_over_algorithmic"] = round(m["hbm_bytes_per_launch"] / (nbytes / launches), 3)
        cal = m.get("calibration_avg_ns")
        if cal and launches:  # the profiled calibration context's average duration (rocprofv3 kernel trace)
            e["avg_launch_ms_rocprof"] = round(cal / 1e6, 4)
            e["frac_rocprof"] = round(nbytes / launches / (cal / 1e9) / 1e9 / HBM_PEAK_GBS, 5)
        out[k] = e
    dom = max(kernels, key=lambda k: kernels[k][1])
    ms, nbytes, launches, _ = kernels[dom]
    achieved = nbytes / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    return {"bound": "hbm", **headline_frac(achieved, nbytes / max(launches, 1), ms / max(launches, 1), out[dom],
                                            profiled_workload(a, integ.dev.cfg.world_size)),
            "kernel": dom,
            "traffic": out[dom].get("traffic_bytes_per_launch"), "traffic_source": source,
            "traffic_over_algorithmic": out[dom].get("traffic_over_algorithmic"),
            "algorithmic_bytes_per_launch": int(nbytes / max(launches, 1)),
            "bytes_model": {"k_vflight": f"{BYTES_VOL_FLIGHT} B state per flight + {BYTES_DENSITY_LOOKUP} B per density lookup",
                            "k_vvertex": f"{BYTES_VOL_VERTEX} B state per interaction + {BYTES_DENSITY_LOOKUP} B per density lookup",
                            "k_vnee": f"{BYTES_VOL_NEE} B per deferred walk slot + {BYTES_DENSITY_LOOKUP} B per density lookup"},
            "measured": f"calibration context after the timed region: {scene.width}x{scene.height} x {spp} spp final-render "
                        "pass with the job's tree, HIP events around every stage launch (one stream)",
            "kernels": out}


def load_gt(path=GT_C3):
    z = np.load(path)
    return z["mean_x256"].astype(np.float32) / np.float32(z["scale"]), int(z["spp"])


def errors(x, gt):
    """rel_rmse = sqrt(mean((x - gt)^2)) / mean(gt); relmse = mean((x - gt)^2 / (gt^2 + 1e-2 mean(gt)^2))
    (relMSE on the image exposed to mean 1; C3's mean is 0.0018); _trim999 without the worst 0.1 %
    of pixels; _dark = median over pixels darker than the mean (the room lit through the door, 96 % of
    the image); _top100_share = the 100 worst pixels' share of relmse (single-sample glints)."""
    d2 = (x.astype(np.float64) - gt) ** 2
    rel = (d2 / (gt.astype(np.float64) ** 2 + 1e-2 * float(gt.mean()) ** 2)).mean(-1).ravel()
    trim = np.sort(rel)[: max(1, int(len(rel) * 0.999))]
    dark = (gt.mean(-1) < gt.mean()).ravel()
    top = np.sort(rel)[::-1][:100]
    return {"rel_rmse": round(float(np.sqrt(d2.mean()) / gt.mean()), 5), "relmse": round(float(rel.mean()), 5),
            "relmse_trim999": round(float(trim.mean()), 5),
            "relmse_top100_share": round(float(top.sum() / max(rel.sum(), 1e-30)), 4),
            "relmse_dark_median": round(float(np.median(rel[dark])), 5) if dark.any() else None}


def image(rgbw):
    return rgbw[..., :3] / np.maximum(rgbw[..., 3:4], 1)


def quality_block(pg, scene, final, job_s, a):
    """Equal-spp / equal-time relative errors against the committed 65,536-spp ground truth."""
    if a.scene != "ajar_door" or (a.width, a.height) != (1280, 720) or not os.path.exists(GT_C3):
        return None
    from mitsuba_path_guiding_amd.integrator import Device
    gt, gt_spp = load_gt()
    out = {"ground_truth": f"tests/golden/c3_gt.npz: unguided GPU path tracer, {gt_spp} spp, seed 4242",
           "guided": errors(image(final), gt)}
    dev = Device(pg.capi.default_config())
    dev.upload(scene)
    dev.render_pass(a.spp, 0)  # warm-up + equal-spp image (sample indices 0.., the guided final pass 31..: paired)
    ug = image(dev.read_film()[0])
    best = float("inf")  # best of two warm runs, like the timed job's steady state
    for _ in range(2):
        dev.reset_film()
        t = time.perf_counter()
        dev.render_pass(a.spp, 0)
        dev.read_film()
        best = min(best, time.perf_counter() - t)
    rate = a.spp / best
    out["unguided_equal_spp"] = dict(errors(ug, gt), spp=a.spp)
    spp_eq = max(1, int(round(job_s * rate)))
    dev.reset_film()
    done = 0
    while done < spp_eq:
        k = min(1024, spp_eq - done)
        dev.render_pass(k, done)
        done += k
    out["unguided_equal_time"] = dict(errors(image(dev.read_film()[0]), gt), spp=spp_eq)
    dev.close()
    g = out["guided"]
    out["guided_over_unguided"] = {
        f"{m}_{w}": round(g[m] / out[f"unguided_{w}"][m], 4)
        for m in ("relmse", "relmse_trim999", "relmse_dark_median") for w in ("equal_spp", "equal_time")}
    return out


def cpu_share():
    """Host threads the CPU baseline may use, and where that number comes from: the smallest of the
    scheduler affinity, the cgroup CPU quota (cgroup v2 cpu.max, v1 cfs_quota/period) and the job's
    declared thread budget (OMP_NUM_THREADS, which gpurun sets to the box's CPU share)."""
    import math
    limits = {}
    if hasattr(os, "sched_getaffinity"):
        limits["affinity"] = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else (float(q), float(p))
        limits["cgroup_cpu.max"] = "max" if quota is None else math.ceil(quota[0] / quota[1])
    except (OSError, ValueError):
        try:
            q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            limits["cgroup_cfs_quota"] = "max" if q <= 0 else math.ceil(q / p)
        except (OSError, ValueError):
            pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        limits["OMP_NUM_THREADS"] = int(os.environ["OMP_NUM_THREADS"])
    nums = {k: v for k, v in limits.items() if isinstance(v, int) and v > 0}
    src = min(nums, key=nums.get) if nums else "os.cpu_count"
    cores = max(1, nums[src] if nums else (os.cpu_count() or 1))
    return cores, {"used": src, **{k: v for k, v in limits.items()}}


def cpu_baseline(pg, scene, integ, final, a):
    """The oracle (CPU restatement, up to 16 host threads = the GPU box's CPU share) runs the same
    guided job on a bounded sample: the full training (every pixel, 1..16 spp, its own records,
    splat and refit) and the final render of a block of tiles from the image centre.  Returns the
    CPU throughput over both, and the equal-spp RMSE of the GPU and the CPU images on those tiles
    against the ground truth (RMSE_gpu / RMSE_cpu <= 1.01)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O  # checker / CPU baseline only
    host_cpus = os.cpu_count()
    cores, cores_source = cpu_share()
    vol = a.scene == "smoke"
    osc = O.OracleScene(pg.capi, scene)
    cfg = integ.cfg  # same integrator parameters as the GPU job
    tree = O.OracleSDTree(osc)
    t0 = time.perf_counter()
    paths = 0
    for it in range(a.train):
        st = O.render(osc, cfg, 2 ** it, 2 ** it - 1, record=True, sdtree=tree, nthreads=cores)[2]
        paths += int(st[0])
        tree.splat_pending()
        tree.refit(it, cfg)
    t_train = time.perf_counter() - t0
    same_tree = bool(np.array_equal(tree.serialize(), integ.dev.get_sdtree()))
    W, T = scene.width, 32
    tiles = [[y * W + x for y in range(ty, min(ty + T, scene.height)) for x in range(tx, min(tx + T, W))]
             for ty in range(0, scene.height, T) for tx in range(0, W, T)]
    off = 2 ** a.train - 1
    mid = len(tiles) // 2
    # calibrate on `cores` tiles (the oracle's threads take whole tiles) at 1/16 of the spp, then size
    # the sample to ~cpu_seconds
    cal = np.array([p for i in range(cores) for p in tiles[(mid + i) % len(tiles)]], np.uint32)
    t = time.perf_counter()
    O.render(osc, cfg, max(1, a.spp // 16), off, sdtree=tree, pixels=cal, nthreads=cores)
    per_tile = (time.perf_counter() - t) / cores * a.spp / max(1, a.spp // 16)
    ntiles = int(max(cores, min(len(tiles), a.cpu_seconds / max(per_tile, 1e-4))))
    ntiles = ntiles // cores * cores  # whole rounds of the oracle's tile workers
    pix = np.array([p for i in range(ntiles) for p in tiles[(mid + i) % len(tiles)]], np.uint32)
    t = time.perf_counter()
    c_rgbw, _, st = O.render(osc, cfg, a.spp, off, sdtree=tree, pixels=pix, nthreads=cores)
    t_render = time.perf_counter() - t
    paths += int(st[0])
    cpu = {"value": round(paths / (t_train + t_render) / 1e6, 4), "unit": "Mpaths/s", "cores": cores,
           "cores_source": cores_source, "host_cpus": host_cpus, "kind": "port",
           "sample": f"the guided {'C5' if vol else 'C3'} job on the CPU oracle: full training "
                     f"({a.train} iterations, every pixel, {t_train:.1f} s) + the {a.spp}-spp final render of "
                     f"{ntiles} tiles of 32x32 ({len(pix)} px, {t_render:.1f} s); {paths} paths"}
    g = image(final).reshape(-1, 3)[pix]
    c = image(c_rgbw).reshape(-1, 3)[pix]
    rmse = {"spp": a.spp, "pixels": int(len(pix)), "same_sdtree": same_tree}
    gt, se_g = None, None
    if not vol and os.path.exists(GT_C3) and (a.width, a.height) == (1280, 720):
        # independent guided jobs (each trained its own tree; any differing record changes the trees, so
        # the final renders decorrelate): RMSE ratio against the ground truth, with a jackknife error
        # over the tiles because single-sample fireflies dominate C3's squared errors
        gt = load_gt()[0].reshape(-1, 3)[pix]
        se_g = ((g - gt) ** 2).reshape(ntiles, -1).sum(1)
        se_c = ((c - gt) ** 2).reshape(ntiles, -1).sum(1)
        ratio = float(np.sqrt(se_g.sum() / se_c.sum()))
        jk = np.sqrt((se_g.sum() - se_g) / (se_c.sum() - se_c))
        err = float(np.sqrt((ntiles - 1) / ntiles * ((jk - jk.mean()) ** 2).sum()))
        rmse.update({"rmse_gpu_vs_gt": float(np.sqrt(se_g.sum() / g.size)),
                     "rmse_cpu_vs_gt": float(np.sqrt(se_c.sum() / c.size)),
                     "rmse_ratio_gpu_over_cpu": round(ratio, 5), "rmse_ratio_jackknife_se": round(err, 5),
                     "target": "<= 1.01 (SURVEY.md §8c(3))"})
        # the same ratio against a ground truth the system under test did not render: the unguided
        # CPU oracle at 8192 spp on the first tiles of the same run (tests/golden/make_c3_cpu_gt.py)
        if os.path.exists(GT_C3_CPU):
            z = np.load(GT_C3_CPU)
            at = {int(p): i for i, p in enumerate(z["pixels"])}
            if all(int(p) in at for p in pix):
                gtc = z["mean"][[at[int(p)] for p in pix]].astype(np.float64)
                se_g2 = ((g - gtc) ** 2).reshape(ntiles, -1).sum(1)
                se_c2 = ((c - gtc) ** 2).reshape(ntiles, -1).sum(1)
                jk2 = np.sqrt((se_g2.sum() - se_g2) / (se_c2.sum() - se_c2))
                rmse["vs_cpu_ground_truth"] = {
                    "ground_truth": f"tests/golden/c3_cpu_gt_tiles.npz: CPU oracle, unguided, {int(z['spp'])} spp",
                    "rmse_ratio_gpu_over_cpu": round(float(np.sqrt(se_g2.sum() / se_c2.sum())), 5),
                    "rmse_ratio_jackknife_se": round(float(np.sqrt((ntiles - 1) / ntiles *
                                                                   ((jk2 - jk2.mean()) ** 2).sum())), 5)}
    # same-stream parity: the CPU final render of the same tiles with the GPU-trained tree
    tree.deserialize(integ.dev.get_sdtree())
    s_rgbw = O.render(osc, cfg, a.spp, off, sdtree=tree, pixels=pix, nthreads=cores)[0]
    s = image(s_rgbw).reshape(-1, 3)[pix]
    rel = np.abs(g - s).max(-1) / np.maximum(s.max(-1), 1e-3)
    rmse["same_tree"] = {"gpu_vs_cpu_relative_rmse": round(float(np.sqrt(np.mean((g - s) ** 2)) /
                                                                 max(float(np.sqrt(np.mean(s ** 2))), 1e-12)), 6),
                         "pixels_diverged_frac": round(float((rel > 1e-3).mean()), 6),
                         "note": "GPU and CPU final renders with one tree and the same RNG streams; a path whose "
                                 "fp32 libm/FMA rounding flips one branch diverges"}
    # single-sample glints set the figure: the worst pixel's share and the figure without
    # the worst 3 pixels
    d2 = ((g - s) ** 2).sum(-1)
    keep = np.ones(len(d2), bool)
    keep[np.argsort(d2)[::-1][:3]] = False
    rmse["same_tree"].update({
        "worst_pixel_share_of_squared_difference": round(float(d2.max() / max(d2.sum(), 1e-30)), 4),
        "gpu_vs_cpu_relative_rmse_without_worst_3_pixels": round(float(
            np.sqrt(np.mean((g[keep] - s[keep]) ** 2)) / max(float(np.sqrt(np.mean(s[keep] ** 2))), 1e-12)), 6)})
    if gt is not None:
        # the paired form of the RMSE ratio: both renders draw the same paths, so only the diverged
        # pixels separate them and the jackknife error over the tiles is small
        se_s = ((s - gt) ** 2).reshape(ntiles, -1).sum(1)
        jk3 = np.sqrt((se_g.sum() - se_g) / (se_s.sum() - se_s))
        rmse["same_tree"].update({
            "rmse_ratio_gpu_over_cpu": round(float(np.sqrt(se_g.sum() / se_s.sum())), 5),
            "rmse_ratio_jackknife_se": round(float(np.sqrt((ntiles - 1) / ntiles * ((jk3 - jk3.mean()) ** 2).sum())), 5)})
    return cpu, rmse


if __name__ == "__main__":
    main()
