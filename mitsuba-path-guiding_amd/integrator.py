"""Host-side mirror of the reference's progressive integrator plugin surface, over the C-ABI.

    reference                                              here
    -----------------------------------------------------  ---------------------------------------
    ProgressiveMIPathTracer (progressive_path.cpp:89-124)   ProgressivePathTracer
    ProgressiveVolumetricPathTracer (progressive_volpath.   ProgressiveVolumetricPathTracer
      cpp:71-96)
    <guided progressive path tracer> (absent)     GuidedPathTracer
    <guided volumetric path tracer> (absent; config C5)     GuidedVolumetricPathTracer
    Integrator::preprocess (integrator.h:61)                .preprocess(scene)
    ProgressiveMonteCarloIntegrator::render (progressive-   .render()
      integrator.cpp:170-220) / renderSamples (:65-114)
    preprogression / postprogression (:308-317)             .preprogression() / .postprogression()
    Integrator::cancel (integrator.h:84)                    .cancel()  (thread-safe)
    Integrator::postprocess (integrator.h:96)               .postprocess()

Properties use the reference's XML names (maxDepth, rrDepth, strictNormals, hideEmitters, useNee,
samplesPerProgression, maxComponentValue; guiding: trainingIterations, sTreeThreshold,
dTreeThreshold, bsdfSamplingFraction, distanceGuiding).  Errors raise RuntimeError with pg_last_error(), like
Log(EError, ...) throws in Mitsuba.  There is no CPU fallback: without libpgamd.so or a gfx950
device every entry point raises.
"""
import ctypes as C
import threading

import numpy as np

from . import capi

_lib = None
_lib_lock = threading.Lock()


def library():
    global _lib
    with _lib_lock:
        if _lib is None:
            _lib = capi.load_library()
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


_FRACTION_BOUNDS = {"fixed": capi.PG_FRACTION_FIXED, "albedo": capi.PG_FRACTION_ALBEDO,
                    "throughput": capi.PG_FRACTION_THROUGHPUT, "learned": capi.PG_FRACTION_LEARNED}


class PGError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"pg status {status}: {msg}")
        self.status = status


def rough_transmittance(distribution, alpha, eta):
    """roughplastic's rough-transmittance slice (pg_rough_transmittance): the 100-entry table over
    cos^(1/4) and the internal diffuse Fresnel reflectance.  Host-only, no device needed."""
    lib = library()
    table = np.zeros(100, np.float32)
    fdr = C.c_float()
    st = lib.pg_rough_transmittance(int(distribution), float(alpha), float(eta), _p(table), C.byref(fdr))
    if st != capi.PG_OK:
        raise PGError(st, lib.pg_last_error(None).decode())
    return table, fdr.value


class Device:
    """One pg_ctx: a render context bound to one HIP device and one image-tile shard."""

    def __init__(self, config=None, **overrides):
        self.lib = library()
        self.cfg = config if config is not None else capi.default_config(**overrides)
        h = C.c_void_p()
        st = self.lib.pg_create(C.byref(self.cfg), C.byref(h))
        if st != capi.PG_OK:
            raise PGError(st, self.lib.pg_last_error(None).decode())
        self.h = h
        self.scene = None

    def _chk(self, st):
        if st != capi.PG_OK:
            raise PGError(st, self.lib.pg_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.pg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- scene / passes
    def upload(self, scene):
        self.scene = scene
        self._chk(self.lib.pg_upload_scene(self.h, C.byref(scene.desc())))

    def render_pass(self, spp, sample_offset=0, record=False):
        self._chk(self.lib.pg_render_pass(self.h, spp, sample_offset, int(bool(record))))

    def render_time(self, seconds, spp_per_progression=1, sample_offset=0, max_spp=0):
        """pg_render_time: whole progressions until `seconds` of wall clock; returns the spp rendered."""
        n = C.c_uint32()
        self._chk(self.lib.pg_render_time(self.h, float(seconds), int(spp_per_progression), int(sample_offset),
                                          int(max_spp), C.byref(n)))
        return n.value

    def cancel(self):
        self._chk(self.lib.pg_cancel(self.h))

    # -- records / SD-tree
    def record_count(self):
        n = C.c_uint64()
        self._chk(self.lib.pg_get_record_count(self.h, C.byref(n)))
        return n.value

    def get_records(self, dst_ptr=None, max_records=None):
        """Host copy (np.uint8 view, 32 B per record), or copy into a device pointer."""
        n = self.record_count() if max_records is None else max_records
        w = C.c_uint64()
        if dst_ptr is not None:
            self._chk(self.lib.pg_get_records(self.h, C.c_void_p(dst_ptr), n, 1, C.byref(w)))
            return w.value
        buf = np.zeros(n * 32, np.uint8)
        self._chk(self.lib.pg_get_records(self.h, _p(buf), n, 0, C.byref(w)))
        return buf[: w.value * 32]

    def splat_records(self, recs=None, device_ptr=None, count=None):
        if device_ptr is not None:
            self._chk(self.lib.pg_splat_records(self.h, C.c_void_p(device_ptr), count, 1))
        else:
            recs = np.ascontiguousarray(recs, np.uint8)
            self._chk(self.lib.pg_splat_records(self.h, _p(recs), len(recs) // 32, 0))

    def splat_local(self):
        self._chk(self.lib.pg_splat_local_records(self.h))

    def tree_stats_words(self):
        n = C.c_uint64()
        self._chk(self.lib.pg_get_tree_stats(self.h, None, 0, 0, C.byref(n)))
        return n.value

    def get_tree_stats(self, dst_ptr=None, words=None):
        """Building-tree statistics (pg_get_tree_stats): numpy uint64 array, or into device memory."""
        n = C.c_uint64()
        if dst_ptr is not None:
            self._chk(self.lib.pg_get_tree_stats(self.h, C.c_void_p(dst_ptr), int(words), 1, C.byref(n)))
            return n.value
        out = np.zeros(self.tree_stats_words(), np.uint64)
        self._chk(self.lib.pg_get_tree_stats(self.h, _p(out), len(out), 0, C.byref(n)))
        return out

    def put_tree_stats(self, stats=None, device_ptr=None, words=None):
        if device_ptr is not None:
            self._chk(self.lib.pg_put_tree_stats(self.h, C.c_void_p(device_ptr), int(words), 1))
        else:
            stats = np.ascontiguousarray(stats, np.uint64)
            self._chk(self.lib.pg_put_tree_stats(self.h, _p(stats), len(stats), 0))

    def refit(self, iteration):
        self._chk(self.lib.pg_refit(self.h, iteration))

    # -- multi-GPU inside the library (RCCL): the C++ adapter's exchange path
    def comm_unique_id(self):
        buf = np.zeros(capi.PG_COMM_ID_BYTES, np.uint8)
        self._chk(self.lib.pg_comm_unique_id(_p(buf)))
        return buf

    def comm_init(self, uid):
        uid = np.ascontiguousarray(uid, np.uint8)
        self._chk(self.lib.pg_comm_init(self.h, _p(uid)))

    def comm_allreduce_tree_stats(self):
        self._chk(self.lib.pg_comm_allreduce_tree_stats(self.h))

    def comm_reduce_film(self, root=0):
        self._chk(self.lib.pg_comm_reduce_film(self.h, int(root)))

    def comm_allgather_records(self):
        """pg_comm_allgather_records: every rank's records splatted into every rank's building tree;
        returns the per-rank record counts."""
        out = np.zeros(self.cfg.world_size, np.uint64)
        self._chk(self.lib.pg_comm_allgather_records(self.h, _p(out)))
        return [int(x) for x in out]

    def comm_allreduce_f64(self, values):
        v = np.ascontiguousarray(values, np.float64).copy()
        self._chk(self.lib.pg_comm_allreduce_f64(self.h, _p(v), len(v)))
        return v

    def get_sdtree(self):
        n = C.c_uint64()
        self._chk(self.lib.pg_get_sdtree(self.h, None, 0, C.byref(n)))
        buf = np.zeros(n.value, np.uint8)
        self._chk(self.lib.pg_get_sdtree(self.h, _p(buf), n.value, C.byref(n)))
        return buf

    def put_sdtree(self, blob):
        blob = np.ascontiguousarray(blob, np.uint8)
        self._chk(self.lib.pg_put_sdtree(self.h, _p(blob), len(blob)))

    def sdtree_pdf(self, pos, d):
        pos = np.ascontiguousarray(pos, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        out = np.zeros(len(pos), np.float32)
        self._chk(self.lib.pg_sdtree_pdf(self.h, _p(pos), _p(d), len(pos), _p(out)))
        return out

    def sdtree_sample(self, pos, u):
        pos = np.ascontiguousarray(pos, np.float32)
        u = np.ascontiguousarray(u, np.float32)
        d = np.zeros((len(pos), 3), np.float32)
        pdf = np.zeros(len(pos), np.float32)
        self._chk(self.lib.pg_sdtree_sample(self.h, _p(pos), _p(u), len(pos), _p(d), _p(pdf)))
        return d, pdf

    # -- film / stats
    def read_film(self):
        W, H = self.scene.width, self.scene.height
        rgbw = np.zeros((H, W, 4), np.float32)
        sq = np.zeros((H, W, 4), np.float32)
        self._chk(self.lib.pg_read_film(self.h, _p(rgbw), _p(sq)))
        return rgbw, sq

    def reset_film(self):
        self._chk(self.lib.pg_reset_film(self.h))

    def read_aovs(self):
        """Denoiser feature sums (pg_config.aovs = 1): (albedo rgb + count, normal xyz + 0), (H, W, 4) each."""
        W, H = self.scene.width, self.scene.height
        alb = np.zeros((H, W, 4), np.float32)
        nrm = np.zeros((H, W, 4), np.float32)
        self._chk(self.lib.pg_read_aovs(self.h, _p(alb), _p(nrm)))
        return alb, nrm

    def stats(self):
        s = capi.pg_stats()
        self._chk(self.lib.pg_get_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in capi.pg_stats._fields_}

    def local_pixel_count(self):
        n = C.c_uint64()
        self._chk(self.lib.pg_local_pixel_count(self.h, C.byref(n)))
        return n.value

    # -- unit-level queries
    def trace_rays(self, rays, any_hit=False):
        rays = np.ascontiguousarray(rays, np.float32)
        hits = np.zeros((len(rays), 4), np.float32)
        self._chk(self.lib.pg_trace_rays(self.h, _p(rays), len(rays), int(any_hit), _p(hits)))
        return hits

    def hit_records(self, rays):
        """pg_hit_records: n x 16 (p, t, geoN, shN, shading frame s, wi local) of each ray's closest hit."""
        rays = np.ascontiguousarray(rays, np.float32)
        out = np.zeros((len(rays), 16), np.float32)
        self._chk(self.lib.pg_hit_records(self.h, _p(rays), len(rays), _p(out)))
        return out

    def bsdf_query(self, material, wi, u, wo_given=None):
        wi = np.ascontiguousarray(wi, np.float32)
        u = np.ascontiguousarray(u, np.float32)
        wg = None if wo_given is None else np.ascontiguousarray(wo_given, np.float32)
        out = np.zeros((len(wi), 12), np.float32)
        self._chk(self.lib.pg_bsdf_query(self.h, material, _p(wi), _p(u), _p(wg), len(wi), _p(out)))
        return out

    def phase_query(self, medium, wi, u, wo_given=None):
        """(wo.xyz, pdf, eval(wi, wo_given)) per query, HG of `medium` on the device."""
        a = np.ascontiguousarray(np.concatenate([np.asarray(wi, np.float32), np.asarray(u, np.float32)], 1))
        wg = None if wo_given is None else np.ascontiguousarray(wo_given, np.float32)
        out = np.zeros((len(a), 5), np.float32)
        self._chk(self.lib.pg_phase_query(self.h, medium, _p(a), _p(wg), len(a), _p(out)))
        return out

    def envmap_query(self, op, x):
        """Environment emitter on the device: op 0 sampleDirect (x: n x 2 samples -> n x 8: d, pdf,
        value/pdf, dist), op 1 pdfDirect (x: n x 3 directions -> n), op 2 evalEnvironment (-> n x 3)."""
        x = np.ascontiguousarray(x, np.float32)
        n = len(x)
        out = np.zeros((n, 8) if op == 0 else (n,) if op == 1 else (n, 3), np.float32)
        self._chk(self.lib.pg_envmap_query(self.h, int(op), _p(x), n, _p(out)))
        return out

    def medium_lookup(self, medium, pts):
        pts = np.ascontiguousarray(pts, np.float32)
        out = np.zeros(len(pts), np.float32)
        self._chk(self.lib.pg_medium_query(self.h, medium, 0, _p(pts), None, len(pts), _p(out)))
        return out

    def medium_sample(self, medium, rays, keys, transmittance=False, grid=False):
        """rays n x 8 (o, mint, d, maxt); keys n x 2 u32 (rng key, sample); returns n x 4."""
        rays = np.ascontiguousarray(rays, np.float32)
        keys = np.ascontiguousarray(keys, np.uint32)
        out = np.zeros((len(rays), 4), np.float32)
        op = (2 if transmittance else 1) + (2 if grid else 0)
        self._chk(self.lib.pg_medium_query(self.h, medium, op, _p(rays), _p(keys), len(rays), _p(out)))
        return out


class ProgressivePathTracer:
    """Mirror of ProgressiveMIPathTracer: plain (unguided) progressive path tracing on the GPU."""

    guided = False
    integrator = capi.PG_INTEGRATOR_PATH

    def __init__(self, props=None, device=0, rank=0, world_size=1, reduce_sum=None):
        props = dict(props or {})
        self.props = props
        # callable(np.float64 array) -> its element-wise sum over ranks (world_size > 1): maxRenderTime's
        # progression agreement, inverse-variance weights over the whole image
        self.reduce_sum = reduce_sum
        self.cfg = capi.default_config(
            device=device, rank=rank, world_size=world_size,
            max_depth=int(props.get("maxDepth", -1)), rr_depth=int(props.get("rrDepth", 5)),
            strict_normals=int(bool(props.get("strictNormals", False))),
            hide_emitters=int(bool(props.get("hideEmitters", False))),
            use_nee=int(bool(props.get("useNee", True))),
            max_component_value=float(props.get("maxComponentValue", float("inf"))),
            seed=int(props.get("seed", 1337)), guiding=int(self.guided),
            bsdf_sampling_fraction=float(props.get("bsdfSamplingFraction", 0.5)),
            s_tree_threshold=float(props.get("sTreeThreshold", 12000.0)),
            d_tree_threshold=float(props.get("dTreeThreshold", 0.01)),
            max_paths_in_flight=int(props.get("maxPathsInFlight", 0)), integrator=self.integrator,
            path_lanes=int(props.get("pathLanes", 0)),
            distance_guiding=float(props.get("distanceGuiding", 0.25)),
            aovs=int(bool(props.get("aovs", False))),
            volpath_exact_mis=int(bool(props.get("exactMis", False))),
            tail_paths=int(props.get("tailPaths", 0)),
            glossy_prior=int(bool(props.get("glossyPrior", False))),
            bsdf_fraction_bound=_FRACTION_BOUNDS[str(props.get("bsdfSamplingFractionBound", "fixed")).lower()])
        self.spp_per_progression = int(props.get("samplesPerProgression", 1))
        # maxRenderTime (progressiveintegrator.cpp:296-300): > 0 renders whole progressions until this
        # many seconds have passed (renderTime, :117-168); rendered_spp / render_seconds report the
        # outcome (the reference's m_spp and m_renderTime, :207-208)
        self.max_render_time = float(props.get("maxRenderTime", -1.0))
        self.rendered_spp = 0
        self.render_seconds = 0.0
        self.dev = None
        self.progression = 0
        self.sample_offset = 0
        self._cancel = threading.Event()

    def preprocess(self, scene):
        self.dev = Device(self.cfg)
        self.dev.upload(scene)
        self.progression = 0
        self.sample_offset = 0
        return True

    def preprogression(self):
        self.progression += 1

    def postprogression(self):
        pass

    def render_progression(self, spp, record=False):
        self.preprogression()
        self.dev.render_pass(spp, self.sample_offset, record)
        self.sample_offset += spp
        self.postprogression()

    def render(self, spp, budget_start=None):
        """renderSamples: spp / samplesPerProgression progressions, or with maxRenderTime > 0 renderTime
        (whole progressions until the budget, counted from budget_start, is spent); returns (rgbw, sumsq)."""
        import time
        t0 = time.perf_counter() if budget_start is None else budget_start
        if self.max_render_time > 0 and self.cfg.world_size > 1:
            self.rendered_spp = self._render_time_sharded(t0)
        elif self.max_render_time > 0:
            left = self.max_render_time - (time.perf_counter() - t0)
            done = 0
            if left > 0 and not self._cancel.is_set():
                self.preprogression()
                done = self.dev.render_time(left, self.spp_per_progression, self.sample_offset)
                self.sample_offset += done
                self.postprogression()
            self.rendered_spp = done
        else:
            passes = max(1, spp // self.spp_per_progression)
            for _ in range(passes):
                if self._cancel.is_set():
                    return None
                self.render_progression(self.spp_per_progression)
            self.rendered_spp = passes * self.spp_per_progression
        self.render_seconds = time.perf_counter() - t0
        rgbw, sq = self.dev.read_film()
        if getattr(self.dev.scene, "mirror_x", False):  # a mirrored sensor (e.g. <scale x="-1"/> in toWorld)
            rgbw, sq = rgbw[:, ::-1].copy(), sq[:, ::-1].copy()
        return rgbw, sq

    def _render_time_sharded(self, t0):
        """maxRenderTime with a tile shard (world_size > 1): the ranks must render the same number of
        whole progressions, or the reduced image would mix tile-dependent sample counts (the
        reference's renderTime keeps progressions image-wide, progressiveintegrator.cpp:117-168).
        Every decision is taken from all-reduced clocks, so it is identical on every rank: before
        each batch the ranks sum a vector holding each rank's elapsed time and seconds per progression
        in its own slot; the slowest rank's figures size the next batch (at most half the remaining
        budget, as pg_render_time does) or stop the render.  Needs reduce_sum (a sum over ranks)."""
        import time
        reduce_sum = self.reduce_sum
        if reduce_sum is None:
            raise ValueError("maxRenderTime with world_size > 1 needs reduce_sum (a sum over ranks) to keep the "
                             "ranks' progression counts equal")
        W, r = self.cfg.world_size, self.cfg.rank
        done, per_prog = 0, 0.0
        while not self._cancel.is_set():
            v = np.zeros(2 * W, np.float64)
            v[r], v[W + r] = time.perf_counter() - t0, per_prog
            v = np.asarray(reduce_sum(v), np.float64)
            elapsed, pp = float(v[:W].max()), float(v[W:].max())
            if elapsed >= self.max_render_time:
                break
            progs = 1 if done == 0 else int(max(1.0, min(np.floor(0.5 * (self.max_render_time - elapsed) /
                                                                   max(pp, 1e-9)), 1e6)))
            t = time.perf_counter()
            self.render_progression(progs * self.spp_per_progression)
            done += progs * self.spp_per_progression
            per_prog = (time.perf_counter() - t) / progs
        return done

    def denoiser_features(self):
        """Per-pixel means of the first-hit albedo and normal (what Denoiser::add averages,
        denoiser.cpp:138-144), shape (H, W, 3) each; needs props {"aovs": True}."""
        alb, nrm = self.dev.read_aovs()
        if getattr(self.dev.scene, "mirror_x", False):  # same read-out flip as render()
            alb, nrm = alb[:, ::-1], nrm[:, ::-1]
        n = np.maximum(alb[..., 3:4], 1)
        return alb[..., :3] / n, nrm[..., :3] / n

    def cancel(self):
        self._cancel.set()
        if self.dev is not None:
            self.dev.cancel()

    def postprocess(self):
        st = self.dev.stats() if self.dev else {}
        if self.dev:
            self.dev.close()
        return st


class ProgressiveVolumetricPathTracer(ProgressivePathTracer):
    """Mirror of ProgressiveVolumetricPathTracer: unguided progressive volumetric path tracing
    (heterogeneous media with Woodcock tracking, HG phase functions, null-BSDF medium boundaries)
    on the GPU.  Same properties as ProgressivePathTracer."""

    integrator = capi.PG_INTEGRATOR_VOLPATH


class GuidedPathTracer(ProgressivePathTracer):
    """SD-tree guided progressive path tracer (Mueller et al. 2017 on the fork's scaffolding).

    Training: iteration k renders 2^k progressions' worth of spp with training records, then the
    postprogression hook splats them into the building SD-tree (one GPU), or runs `exchange` (several
    ranks: by default distributed.make_exchange's all-reduce of the building statistics over RCCL;
    distributed.make_capi_exchange uses the library's own communicator), and refits.  The film is reset before the
    final render, which samples with the last trained tree.

    sampleCombination (after Mueller's practical-path-guiding course notes):
    "discard" (default) keeps only the final render's samples; "inversevar" keeps every training
    iteration's image too and returns the inverse-variance weighted combination of all of them,
    each image weighted by 1 / (its mean per-pixel variance of the mean), since the early, poorly
    guided iterations are noisier.  All images are unbiased, so the combination is too.
    """

    guided = True

    def __init__(self, props=None, device=0, rank=0, world_size=1, exchange=None, reduce_sum=None):
        super().__init__(props, device, rank, world_size, reduce_sum)
        self.training_iterations = int(self.props.get("trainingIterations", 5))
        self.exchange = exchange  # callable(dev): the postprogression statistics exchange (N > 1)
        self.initial_tree = None
        self.sample_combination = str(self.props.get("sampleCombination", "discard")).lower()
        if self.sample_combination not in ("discard", "inversevar"):
            raise ValueError(f"sampleCombination must be discard or inversevar, not {self.sample_combination!r}")
        self.iteration_films = []
        self.combination_weights = None

    def preprocess(self, scene):
        super().preprocess(scene)
        self.initial_tree = self.dev.get_sdtree()
        return True

    def reset(self):
        """Start a new job on the uploaded scene: untrained SD-tree, empty film, sample index 0."""
        self.dev.put_sdtree(self.initial_tree)
        self.dev.reset_film()
        self.sample_offset = 0
        self.progression = 0

    def train(self):
        for it in range(self.training_iterations):
            if self._cancel.is_set():
                return
            self.preprogression()
            self.dev.render_pass(2 ** it, self.sample_offset, record=True)
            self.sample_offset += 2 ** it
            if self.sample_combination == "inversevar":
                self.iteration_films.append(self.dev.read_film())
                self.dev.reset_film()
            self.postprogression_train(it)

    def postprogression_train(self, it):
        if self.exchange is None:
            self.dev.splat_local()
        else:
            self.exchange(self.dev)
        self.dev.refit(it)

    def render(self, spp):
        """Training iterations, then the final render (spp, or with maxRenderTime > 0 whole
        progressions until the budget, which includes the training time, is spent)."""
        import time
        t0 = time.perf_counter()
        self.iteration_films = []
        self.train()
        self.dev.reset_film()
        out = super().render(spp, budget_start=t0)
        if out is None or self.sample_combination == "discard":
            return out
        films = [(f[0][:, ::-1], f[1][:, ::-1]) if getattr(self.dev.scene, "mirror_x", False) else f
                 for f in self.iteration_films] + [out]
        return combine_inverse_variance(films, self, self.reduce_sum)


def combine_inverse_variance(films, owner=None, reduce_sum=None):
    """Inverse-variance weighted combination of unbiased images given as film sums (rgbw, sumsq):
    image i has per-pixel means m_i and variance estimate v_i = mean over the rendered pixels and
    channels of (E[x^2] - m^2) / n.  With a tile shard, each rank holds only its tiles: reduce_sum
    (a sum over ranks) turns the local sums and pixel counts into the whole image's, so every rank
    uses the same weights and the result does not depend on the rank count.  Returns film-like sums
    (combined mean x total count, combined second moment x total count) so that callers can keep
    dividing by the count channel."""
    means, seconds, counts = [], [], []
    stats = np.zeros(2 * len(films), np.float64)  # per image: variance sum, channel count
    for i, (rgbw, sq) in enumerate(films):
        cnt = rgbw[..., 3:4]
        n = np.maximum(cnt, 1)
        m = rgbw[..., :3] / n
        m2 = sq[..., :3] / n
        mask = np.broadcast_to(cnt > 0, m.shape)
        stats[2 * i] = float(np.sum((np.maximum(m2 - m * m, 0) / n)[mask], dtype=np.float64))
        stats[2 * i + 1] = float(mask.sum())
        means.append(m)
        seconds.append(m2)
        counts.append(cnt)
    if reduce_sum is not None:
        stats = np.asarray(reduce_sum(stats), np.float64)
    weights = []
    for i in range(len(films)):
        v = stats[2 * i] / stats[2 * i + 1] if stats[2 * i + 1] > 0 else 0.0
        weights.append(1.0 / v if v > 0 and np.isfinite(v) else 0.0)
    W = np.asarray(weights, np.float64)
    if W.sum() <= 0:
        W = np.zeros_like(W)
        W[-1] = 1.0
    W = W / W.sum()
    if owner is not None:
        owner.combination_weights = W.tolist()
    total = np.sum(counts, 0)
    mean = sum(w * m for w, m in zip(W, means))
    second = sum(w * m2 for w, m2 in zip(W, seconds))
    rgbw = np.concatenate([mean * total, total], -1).astype(np.float32)
    sq = np.concatenate([second * total, np.zeros_like(total)], -1).astype(np.float32)
    return rgbw, sq


class GuidedVolumetricPathTracer(GuidedPathTracer):
    """SD-tree guided progressive volumetric path tracer (config C5).  Training records come from
    medium vertices and smooth surface vertices; directions at both are one-sample MIS between the
    phase function / BSDF and the D-tree (`bsdfSamplingFraction`), and free flights use guided
    weighted delta tracking with mixing weight `distanceGuiding` (0 = the reference's free flight;
    oracle/orc_volpath.h GuidedAccept).  Same training schedule and exchange as GuidedPathTracer."""

    integrator = capi.PG_INTEGRATOR_VOLPATH
