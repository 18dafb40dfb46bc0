"""ORACLE — test infrastructure only.

ctypes bindings of oracle/_build/liboracle.so (the CPU restatement).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as the
checker / the timed CPU baseline.  The product never imports it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")  # ORACLE_LIB: sanitizer builds
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib(capi):
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        VP = C.c_void_p
        sig = {
            "oracle_scene_create": (VP, [C.POINTER(capi.pg_scene_desc)]),
            "oracle_scene_destroy": (None, [VP]),
            "oracle_scene_bounds": (None, [VP, VP, VP]),
            "oracle_hardware_threads": (C.c_int, []),
            "oracle_sdtree_create": (VP, [VP]),
            "oracle_sdtree_destroy": (None, [VP]),
            "oracle_render": (C.c_int, [VP, C.POINTER(capi.pg_config), VP, C.c_uint32, C.c_uint32, C.c_int32, VP,
                                        C.c_uint64, C.c_int32, VP, VP, VP]),
            "oracle_sdtree_pending_count": (C.c_uint64, [VP]),
            "oracle_sdtree_take_pending": (C.c_uint64, [VP, VP, C.c_uint64]),
            "oracle_sdtree_splat": (None, [VP, VP, C.c_uint64]),
            "oracle_sdtree_splat_pending": (None, [VP]),
            "oracle_sdtree_refit": (None, [VP, C.c_uint32, C.c_float, C.c_float, C.c_int32]),
            "oracle_sdtree_configure": (None, [VP, C.c_int32, C.c_float]),
            "oracle_sdtree_serialize": (C.c_uint64, [VP, VP, C.c_uint64]),
            "oracle_sdtree_deserialize": (C.c_int, [VP, VP, C.c_uint64]),
            "oracle_sdtree_pdf": (None, [VP, VP, VP, C.c_uint64, VP]),
            "oracle_sdtree_sample": (None, [VP, VP, VP, C.c_uint64, VP, VP]),
            "oracle_trace_rays": (None, [VP, VP, C.c_uint64, C.c_int32, VP]),
            "oracle_trace_rays_brute": (None, [VP, VP, C.c_uint64, VP]),
            "oracle_path_rays": (C.c_uint64, [VP, C.POINTER(capi.pg_config), VP, C.c_uint32, C.c_uint32, VP,
                                              C.c_uint64, VP, VP, C.c_uint64, VP]),
            "oracle_bsdf_query": (None, [C.POINTER(capi.pg_material), VP, VP, VP, C.c_uint64, VP]),
            "oracle_material_type": (C.c_uint32, [C.POINTER(capi.pg_material)]),
            "oracle_rough_transmittance": (None, [C.c_uint32, C.c_float, C.c_float, VP, VP]),
            "oracle_intersect": (None, [VP, VP, C.c_uint64, VP]),
            "oracle_hit_records": (None, [VP, VP, C.c_uint64, VP]),
            "oracle_set_volpath_eager": (None, [C.c_int32]),
            "oracle_medium_query": (None, [VP, C.c_int32, C.c_int32, VP, VP, C.c_uint64, VP]),
            "oracle_hg_query": (None, [C.c_float, VP, VP, C.c_uint64, VP]),
            "oracle_microfacet_query": (None, [C.c_int32, C.c_float, C.c_float, VP, VP, VP, C.c_uint64, VP]),
            "oracle_render_aovs": (None, [VP, C.c_uint32, C.c_uint32, C.c_uint32, VP, VP]),
            "oracle_envmap_query": (C.c_int, [VP, C.c_int32, VP, C.c_uint64, VP]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleScene:
    def __init__(self, capi, scene):
        self.capi = capi
        self.scene = scene
        self.L = lib(capi)
        self.h = self.L.oracle_scene_create(C.byref(scene.desc()))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_scene_destroy(self.h)
            self.h = None

    def bounds(self):
        lo = np.zeros(3, np.float32)
        hi = np.zeros(3, np.float32)
        self.L.oracle_scene_bounds(self.h, _p(lo), _p(hi))
        return lo, hi

    def intersect(self, rays):
        rays = np.ascontiguousarray(rays, np.float32)
        out = np.zeros((len(rays), 16), np.float32)
        self.L.oracle_intersect(self.h, _p(rays), len(rays), _p(out))
        return out

    def hit_records(self, rays):
        """n x 16 (p, t, geoN, shN, shading frame s, wi local): the layout of the library's pg_hit_records."""
        rays = np.ascontiguousarray(rays, np.float32)
        out = np.zeros((len(rays), 16), np.float32)
        self.L.oracle_hit_records(self.h, _p(rays), len(rays), _p(out))
        return out

    def medium_lookup(self, m, pts):
        pts = np.ascontiguousarray(pts, np.float32)
        out = np.zeros(len(pts), np.float32)
        self.L.oracle_medium_query(self.h, m, 0, _p(pts), None, len(pts), _p(out))
        return out

    def medium_sample(self, m, rays, keys, transmittance=False, grid=False):
        """rays: n x 8 (o, mint, d, maxt); keys: n x 2 u32 (rng key, sample).  Returns n x 4."""
        rays = np.ascontiguousarray(rays, np.float32)
        keys = np.ascontiguousarray(keys, np.uint32)
        out = np.zeros((len(rays), 4), np.float32)
        op = (2 if transmittance else 1) + (2 if grid else 0)
        self.L.oracle_medium_query(self.h, m, op, _p(rays), _p(keys), len(rays), _p(out))
        return out

    def envmap_query(self, op, x):
        """Same layout as integrator.Device.envmap_query."""
        x = np.ascontiguousarray(x, np.float32)
        n = len(x)
        out = np.zeros((n, 8) if op == 0 else (n,) if op == 1 else (n, 3), np.float32)
        if self.L.oracle_envmap_query(self.h, int(op), _p(x), n, _p(out)) != 0:
            raise ValueError("the scene has no environment emitter")
        return out

    def render_aovs(self, spp, sample_offset=0, seed=1337):
        """First-hit denoiser feature sums: (albedo rgb + count, normal xyz + 0), (H, W, 4) each."""
        W, H = self.scene.width, self.scene.height
        alb = np.zeros((H, W, 4), np.float32)
        nrm = np.zeros((H, W, 4), np.float32)
        self.L.oracle_render_aovs(self.h, seed, spp, sample_offset, _p(alb), _p(nrm))
        return alb, nrm

    def trace(self, rays, any_hit=False):
        rays = np.ascontiguousarray(rays, np.float32)
        hits = np.zeros((len(rays), 4), np.float32)
        self.L.oracle_trace_rays(self.h, _p(rays), len(rays), int(any_hit), _p(hits))
        return hits

    def trace_brute(self, rays):
        """trace() by brute force over every triangle (the walk's contract: smallest t, ties to the lower
        triangle index)"""
        rays = np.ascontiguousarray(rays, np.float32)
        hits = np.zeros((len(rays), 4), np.float32)
        self.L.oracle_trace_rays_brute(self.h, _p(rays), len(rays), _p(hits))
        return hits

    def path_rays(self, cfg, sdtree, pixel, sample, max_rays=4096):
        """The rays one path casts: (n x 11: kind 0 closest / 1 shadow, o, mint, d, maxt, t or occluded,
        prim bits), its clamped radiance, and its per-vertex records (n x 32, the kernels' PG_WATCH
        record: depth, triangle, p, T, alpha, guided, mode, woPdf, weight, wo, L, NEE contribution, NEE
        pdfs, RR q / survived, alive, shadow, b0, b1)"""
        out = np.zeros((max_rays, 11), np.float32)
        L = np.zeros(3, np.float32)
        vtx = np.zeros((256, 32), np.float32)
        nv = C.c_uint64()
        n = self.L.oracle_path_rays(self.h, C.byref(cfg), sdtree.h if sdtree else None, pixel, sample, _p(out),
                                    max_rays, _p(L), _p(vtx), 256, C.byref(nv))
        return out[:min(n, max_rays)], L, vtx[:min(nv.value, 256)]


class OracleSDTree:
    def __init__(self, oscene):
        self.L = oscene.L
        self.h = self.L.oracle_sdtree_create(oscene.h)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_sdtree_destroy(self.h)
            self.h = None

    def take_records(self, capi):
        n = self.L.oracle_sdtree_pending_count(self.h)
        buf = (capi.pg_record * max(1, n))()
        self.L.oracle_sdtree_take_pending(self.h, C.cast(buf, C.c_void_p), n)
        return np.frombuffer(buf, dtype=np.uint8, count=n * 32).copy().view(np.uint8)

    def splat_bytes(self, recbytes):
        recbytes = np.ascontiguousarray(recbytes, np.uint8)
        self.L.oracle_sdtree_splat(self.h, _p(recbytes), len(recbytes) // 32)

    def splat_pending(self):
        self.L.oracle_sdtree_splat_pending(self.h)

    def configure(self, cfg):
        """Learned BSDF-sampling fraction on or off (cfg.bsdf_fraction_bound == PG_FRACTION_LEARNED), as the
        device context does: the splat gathers its statistics, the refit learns.  render(record=True) and
        refit() call it; call it before splatting records that did not come from this oracle."""
        self.L.oracle_sdtree_configure(self.h, int(cfg.bsdf_fraction_bound == 3), cfg.bsdf_sampling_fraction)

    def refit(self, it, cfg):
        self.configure(cfg)
        self.L.oracle_sdtree_refit(self.h, it, cfg.s_tree_threshold, cfg.d_tree_threshold, cfg.d_tree_max_depth)

    def serialize(self):
        n = self.L.oracle_sdtree_serialize(self.h, None, 0)
        buf = np.zeros(n, np.uint8)
        self.L.oracle_sdtree_serialize(self.h, _p(buf), n)
        return buf

    def deserialize(self, buf):
        buf = np.ascontiguousarray(buf, np.uint8)
        if self.L.oracle_sdtree_deserialize(self.h, _p(buf), len(buf)) != 0:
            raise ValueError("bad SD-tree blob")

    def pdf(self, pos, d):
        pos = np.ascontiguousarray(pos, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        out = np.zeros(len(pos), np.float32)
        self.L.oracle_sdtree_pdf(self.h, _p(pos), _p(d), len(pos), _p(out))
        return out

    def sample(self, pos, u):
        pos = np.ascontiguousarray(pos, np.float32)
        u = np.ascontiguousarray(u, np.float32)
        d = np.zeros((len(pos), 3), np.float32)
        pdf = np.zeros(len(pos), np.float32)
        self.L.oracle_sdtree_sample(self.h, _p(pos), _p(u), len(pos), _p(d), _p(pdf))
        return d, pdf


def render(oscene, cfg, spp, sample_offset=0, record=False, sdtree=None, pixels=None, nthreads=0, film=None):
    """Returns (rgbw, sumsq, stats) arrays of shape (H, W, 4); accumulates into `film` if given."""
    sc = oscene.scene
    W, H = sc.width, sc.height
    if film is None:
        rgbw = np.zeros((H, W, 4), np.float32)
        sumsq = np.zeros((H, W, 4), np.float32)
    else:
        rgbw, sumsq = film
    stats = np.zeros(4, np.uint64)
    px = None if pixels is None else np.ascontiguousarray(pixels, np.uint32)
    oscene.L.oracle_render(oscene.h, C.byref(cfg), sdtree.h if sdtree else None, spp, sample_offset, int(record),
                           _p(px), 0 if px is None else len(px), nthreads, _p(rgbw), _p(sumsq), _p(stats))
    return rgbw, sumsq, stats


def bsdf_query(capi, mat, wi, u, wo_given=None):
    wi = np.ascontiguousarray(wi, np.float32)
    u = np.ascontiguousarray(u, np.float32)
    wg = None if wo_given is None else np.ascontiguousarray(wo_given, np.float32)
    out = np.zeros((len(wi), 12), np.float32)
    lib(capi).oracle_bsdf_query(C.byref(mat), _p(wi), _p(u), _p(wg), len(wi), _p(out))
    return out


def set_volpath_eager(capi, eager):
    lib(capi).oracle_set_volpath_eager(int(bool(eager)))


def hg_query(capi, g, wi, u, wo_given=None):
    """(wo.xyz, pdf, eval(wi, wo_given)) per query."""
    a = np.ascontiguousarray(np.concatenate([np.asarray(wi, np.float32), np.asarray(u, np.float32)], 1), np.float32)
    wg = None if wo_given is None else np.ascontiguousarray(wo_given, np.float32)
    out = np.zeros((len(a), 5), np.float32)
    lib(capi).oracle_hg_query(float(g), _p(a), _p(wg), len(a), _p(out))
    return out


def microfacet_query(capi, dist, au, av, wi, u, m_given=None):
    """(m.xyz, density of m, density of m_given) per query; wi all zero = sampleAll / pdfAll."""
    wi = np.ascontiguousarray(wi, np.float32)
    u = np.ascontiguousarray(u, np.float32)
    mg = None if m_given is None else np.ascontiguousarray(m_given, np.float32)
    out = np.zeros((len(wi), 5), np.float32)
    lib(capi).oracle_microfacet_query(int(dist), float(au), float(av), _p(wi), _p(u), _p(mg), len(wi), _p(out))
    return out


def material_type(capi, mat):
    return lib(capi).oracle_material_type(C.byref(mat))


def rough_transmittance(capi, distribution, alpha, eta):
    """Oracle roughplastic slices (orc_rtrans.h): (table[100], fdr_int)."""
    table = np.zeros(100, np.float32)
    fdr = np.zeros(1, np.float32)
    lib(capi).oracle_rough_transmittance(int(distribution), float(alpha), float(eta), _p(table), _p(fdr))
    return table, float(fdr[0])
