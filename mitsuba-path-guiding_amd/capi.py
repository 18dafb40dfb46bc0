"""ctypes mirror of include/pg_capi.h (the C-ABI boundary).

Struct layouts here must match the header byte for byte; tests/test_capi_abi.py checks the sizes
against the compiled library.  This module only describes types and loads a library; it does no
compute.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PG_LIB") or os.path.join(_HERE, "build", "libpgamd.so")  # PG_LIB: A/B builds (tools)

PG_OK, PG_ERR_INVALID, PG_ERR_HIP, PG_ERR_OOM, PG_ERR_STATE, PG_ERR_CANCELLED, PG_ERR_NO_DEVICE = range(7)
(PG_BSDF_DIFFUSE, PG_BSDF_CONDUCTOR, PG_BSDF_ROUGHCONDUCTOR, PG_BSDF_DIELECTRIC, PG_BSDF_ROUGHDIELECTRIC,
 PG_BSDF_PLASTIC, PG_BSDF_ROUGHPLASTIC, PG_BSDF_NULL) = range(8)
PG_MEDIUM_HETEROGENEOUS = 0
PG_INTEGRATOR_PATH, PG_INTEGRATOR_VOLPATH = 0, 1
PG_MAJORANT_GRID, PG_MAJORANT_GLOBAL = 0, 1
PG_FRACTION_FIXED, PG_FRACTION_ALBEDO, PG_FRACTION_THROUGHPUT, PG_FRACTION_LEARNED = 0, 1, 2, 3
MAJORANT_CELL = 16  # voxels per majorant-grid cell edge (pg_layout.h PG_MAJORANT_CELL / oracle/orc_medium.h)
PG_DIST_BECKMANN, PG_DIST_GGX = 0, 1
PG_MAT_TWOSIDED, PG_MAT_NONLINEAR, PG_MAT_SAMPLE_ALL = 1, 2, 4

# EBSDFType bits (include/mitsuba/render/bsdf.h:224-262)
ENull, EDiffuseReflection, EDiffuseTransmission, EGlossyReflection = 0x1, 0x2, 0x4, 0x8
EGlossyTransmission, EDeltaReflection, EDeltaTransmission = 0x10, 0x20, 0x40
EFrontSide, EBackSide = 0x8000, 0x10000
EDelta = EDeltaReflection | EDeltaTransmission
ESmooth = EDiffuseReflection | EDiffuseTransmission | EGlossyReflection | EGlossyTransmission

F4 = C.c_float * 4


class pg_material(C.Structure):
    _fields_ = [("type", C.c_uint32), ("distribution", C.c_uint32), ("flags", C.c_uint32), ("pad0", C.c_uint32),
                ("alpha_u", C.c_float), ("alpha_v", C.c_float), ("int_ior", C.c_float), ("ext_ior", C.c_float),
                ("diffuse_reflectance", F4), ("specular_reflectance", F4), ("specular_transmittance", F4),
                ("eta", F4), ("k", F4)]


class pg_shape(C.Structure):
    _fields_ = [("tri_begin", C.c_uint32), ("tri_count", C.c_uint32), ("material", C.c_uint32), ("emitter", C.c_int32),
                ("interior_medium", C.c_int32), ("exterior_medium", C.c_int32)]

    def __init__(self, tri_begin=0, tri_count=0, material=0, emitter=-1, interior_medium=-1, exterior_medium=-1):
        super().__init__(tri_begin, tri_count, material, emitter, interior_medium, exterior_medium)


class pg_medium(C.Structure):
    _fields_ = [("type", C.c_uint32), ("res", C.c_uint32 * 3), ("density", C.POINTER(C.c_float)),
                ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("scale", C.c_float),
                ("albedo", C.c_float * 3), ("g", C.c_float), ("pad0", C.c_uint32)]


class pg_emitter(C.Structure):
    _fields_ = [("shape", C.c_uint32), ("pad", C.c_uint32 * 3), ("radiance", F4)]


class pg_envmap(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgb", C.POINTER(C.c_float)),
                ("to_world", C.c_float * 9), ("scale", C.c_float), ("pad0", C.c_uint32), ("pad1", C.c_uint32)]


class pg_camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("target", C.c_float * 3), ("up", C.c_float * 3),
                ("fov_x_deg", C.c_float), ("near_clip", C.c_float), ("far_clip", C.c_float),
                ("width", C.c_uint32), ("height", C.c_uint32)]


class pg_scene_desc(C.Structure):
    _fields_ = [("num_vertices", C.c_uint32), ("num_triangles", C.c_uint32), ("num_shapes", C.c_uint32),
                ("num_materials", C.c_uint32), ("num_emitters", C.c_uint32), ("num_media", C.c_uint32),
                ("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("indices", C.POINTER(C.c_uint32)), ("shapes", C.POINTER(pg_shape)),
                ("materials", C.POINTER(pg_material)), ("emitters", C.POINTER(pg_emitter)),
                ("camera", pg_camera), ("media", C.POINTER(pg_medium)), ("camera_medium", C.c_int32),
                ("pad1", C.c_int32), ("envmap", C.POINTER(pg_envmap))]


class pg_config(C.Structure):
    _fields_ = [("device", C.c_int32), ("max_depth", C.c_int32), ("rr_depth", C.c_int32), ("use_nee", C.c_int32),
                ("hide_emitters", C.c_int32), ("strict_normals", C.c_int32), ("max_component_value", C.c_float),
                ("seed", C.c_uint32), ("guiding", C.c_int32), ("bsdf_sampling_fraction", C.c_float),
                ("s_tree_threshold", C.c_float), ("d_tree_threshold", C.c_float), ("d_tree_max_depth", C.c_int32),
                ("record_max_vertices", C.c_int32), ("rank", C.c_int32), ("world_size", C.c_int32),
                ("tile_size", C.c_uint32), ("max_paths_in_flight", C.c_uint32), ("gpu_depth_cap", C.c_int32),
                ("path_lanes", C.c_int32), ("integrator", C.c_int32), ("volume_majorant", C.c_int32),
                ("distance_guiding", C.c_float), ("aovs", C.c_int32), ("bsdf_fraction_bound", C.c_int32),
                ("kernel_timing", C.c_int32), ("volpath_exact_mis", C.c_int32),
                ("tail_paths", C.c_int32), ("glossy_prior", C.c_int32)]


class pg_record(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("dir", C.c_uint32), ("radiance", C.c_float), ("wo_pdf", C.c_float),
                ("product", C.c_float), ("weight", C.c_float)]


class pg_stats(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("segments", C.c_uint64), ("shadow_rays", C.c_uint64), ("records", C.c_uint64),
                ("trace_ms", C.c_double), ("shade_ms", C.c_double), ("shadow_ms", C.c_double), ("other_ms", C.c_double),
                ("trace_launches", C.c_uint64), ("stree_nodes", C.c_uint64), ("dtree_nodes", C.c_uint64),
                ("shade_launches", C.c_uint64), ("volume_ms", C.c_double), ("volume_launches", C.c_uint64),
                ("density_lookups", C.c_uint64), ("escaped", C.c_uint64), ("rays_ms", C.c_double),
                ("rays_launches", C.c_uint64), ("shadow_launches", C.c_uint64), ("tail_launches", C.c_uint64),
                # ABI 11: the volumetric wavefront's stages
                ("vol_flight_ms", C.c_double), ("vol_flight_launches", C.c_uint64), ("vol_flights", C.c_uint64),
                ("vol_flight_lookups", C.c_uint64), ("vol_vertex_ms", C.c_double),
                ("vol_vertex_launches", C.c_uint64), ("vol_vertices", C.c_uint64), ("vol_vertex_lookups", C.c_uint64),
                ("vol_nee_ms", C.c_double), ("vol_nee_launches", C.c_uint64), ("vol_nee_walks", C.c_uint64),
                ("vol_nee_lookups", C.c_uint64)]


def default_config(**overrides):
    """Mirror of pg_config_default() (kept in sync; tests compare both)."""
    c = pg_config()
    c.device = 0
    c.max_depth = -1
    c.rr_depth = 5
    c.use_nee = 1
    c.hide_emitters = 0
    c.strict_normals = 0
    c.max_component_value = float("inf")
    c.seed = 1337
    c.guiding = 0
    c.bsdf_sampling_fraction = 0.5
    c.s_tree_threshold = 12000.0
    c.d_tree_threshold = 0.01
    c.d_tree_max_depth = 20
    c.record_max_vertices = 32
    c.rank = 0
    c.world_size = 1
    c.tile_size = 32
    c.max_paths_in_flight = 0
    c.gpu_depth_cap = 1024
    c.path_lanes = 0
    c.integrator = PG_INTEGRATOR_PATH
    c.distance_guiding = 0.25
    c.aovs = 0
    c.bsdf_fraction_bound = PG_FRACTION_FIXED
    c.kernel_timing = 0
    c.volpath_exact_mis = 0
    c.tail_paths = 0
    c.glossy_prior = 0
    for k, v in overrides.items():
        if not hasattr(c, k):
            raise AttributeError(f"pg_config has no field {k!r}")
        setattr(c, k, v)
    return c


# (name, restype, argtypes) for every entry point declared in include/pg_capi.h
VP = C.c_void_p
SIGNATURES = [
    ("pg_config_default", C.c_int32, [C.POINTER(pg_config)]),
    ("pg_create", C.c_int32, [C.POINTER(pg_config), C.POINTER(VP)]),
    ("pg_destroy", C.c_int32, [VP]),
    ("pg_last_error", C.c_char_p, [VP]),
    ("pg_abi_version", C.c_int32, []),
    ("pg_cancel", C.c_int32, [VP]),
    ("pg_upload_scene", C.c_int32, [VP, C.POINTER(pg_scene_desc)]),
    ("pg_render_pass", C.c_int32, [VP, C.c_uint32, C.c_uint32, C.c_int32]),
    ("pg_render_time", C.c_int32, [VP, C.c_double, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("pg_get_record_count", C.c_int32, [VP, C.POINTER(C.c_uint64)]),
    ("pg_get_records", C.c_int32, [VP, VP, C.c_uint64, C.c_int32, C.POINTER(C.c_uint64)]),
    ("pg_splat_records", C.c_int32, [VP, VP, C.c_uint64, C.c_int32]),
    ("pg_splat_local_records", C.c_int32, [VP]),
    ("pg_refit", C.c_int32, [VP, C.c_uint32]),
    ("pg_get_sdtree", C.c_int32, [VP, VP, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("pg_put_sdtree", C.c_int32, [VP, VP, C.c_uint64]),
    ("pg_sdtree_pdf", C.c_int32, [VP, VP, VP, C.c_uint64, VP]),
    ("pg_sdtree_sample", C.c_int32, [VP, VP, VP, C.c_uint64, VP, VP]),
    ("pg_read_film", C.c_int32, [VP, VP, VP]),
    ("pg_reset_film", C.c_int32, [VP]),
    ("pg_read_aovs", C.c_int32, [VP, VP, VP]),
    ("pg_get_stats", C.c_int32, [VP, C.POINTER(pg_stats)]),
    ("pg_local_pixel_count", C.c_int32, [VP, C.POINTER(C.c_uint64)]),
    ("pg_trace_rays", C.c_int32, [VP, VP, C.c_uint64, C.c_int32, VP]),
    ("pg_hit_records", C.c_int32, [VP, VP, C.c_uint64, VP]),
    ("pg_bsdf_query", C.c_int32, [VP, C.c_uint32, VP, VP, VP, C.c_uint64, VP]),
    ("pg_phase_query", C.c_int32, [VP, C.c_uint32, VP, VP, C.c_uint64, VP]),
    ("pg_medium_query", C.c_int32, [VP, C.c_uint32, C.c_int32, VP, VP, C.c_uint64, VP]),
    ("pg_envmap_query", C.c_int32, [VP, C.c_int32, VP, C.c_uint64, VP]),
    ("pg_rough_transmittance", C.c_int32, [C.c_uint32, C.c_float, C.c_float, VP, VP]),
    ("pg_get_tree_stats", C.c_int32, [VP, VP, C.c_uint64, C.c_int32, VP]),
    ("pg_put_tree_stats", C.c_int32, [VP, VP, C.c_uint64, C.c_int32]),
    ("pg_comm_unique_id", C.c_int32, [VP]),
    ("pg_comm_init", C.c_int32, [VP, VP]),
    ("pg_comm_allreduce_tree_stats", C.c_int32, [VP]),
    ("pg_comm_reduce_film", C.c_int32, [VP, C.c_int32]),
    ("pg_comm_allreduce_f64", C.c_int32, [VP, VP, C.c_uint64]),
    ("pg_comm_allgather_records", C.c_int32, [VP, VP]),
]


PG_ABI_VERSION = 12  # include/pg_capi.h
PG_COMM_ID_BYTES = 128


def load_library(path=None):
    """Load libpgamd.so and attach prototypes.  Raises if it is missing or built against another
    ABI version (no fallback path)."""
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"HIP extension {path} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    lib = C.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pg_abi_version() != PG_ABI_VERSION:
        raise RuntimeError(f"{path} has ABI {lib.pg_abi_version()}, this package needs {PG_ABI_VERSION}: rebuild it")
    return lib
