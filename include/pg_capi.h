/*
 * pg_capi.h — the drop-in boundary of the MI355X guided path-tracing integrator.
 *
 * A thin C ABI (plain pointers, sizes and integer status codes; no C++ types, no exceptions)
 * between a host integrator plugin and the HIP/gfx950 hot path.  It replaces the CPU side of
 * the reference's progressive Monte-Carlo integrator for ONE job:
 *
 *   reference surface                                    replaced by
 *   ------------------------------------------------------------------------------------------
 *   Integrator::preprocess            include/mitsuba/render/integrator.h:61   pg_create + pg_upload_scene
 *   ProgressiveMonteCarloIntegrator::render / renderSamples
 *                                     src/librender/progressiveintegrator.cpp:65-114,170-220
 *                                                                              pg_render_pass (one progression)
 *   ProgressiveMonteCarloIntegrator::renderBlock (per-pixel sample loop, clamp, ImageBlock::put)
 *                                     src/librender/progressiveintegrator.cpp:222-282   (inside pg_render_pass)
 *   ProgressiveMIPathTracer::Li       src/integrators/path/progressive_path.cpp:133-314 (inside pg_render_pass)
 *   ProgressiveMonteCarloIntegrator::postprogression (guiding refit slot)
 *                                     src/librender/progressiveintegrator.cpp:314-317  pg_splat_* + pg_refit
 *   Integrator::cancel                integrator.h:84; progressiveintegrator.cpp:319-326  pg_cancel
 *   Film::develop / ImageBlock readback  src/librender/renderproc.cpp:142-149        pg_read_film
 *   Integrator::postprocess           integrator.h:96                             pg_get_stats + pg_destroy
 *
 * Every function returns a pg_status; on failure pg_last_error() holds a message (the Mitsuba
 * adapter turns it into Log(EError, ...), which throws: include/mitsuba/core/formatter.h:33).
 * All host arrays passed in are caller-owned and copied; all device memory is owned by the
 * context and released by pg_destroy.  One context per render job; calls come from one thread
 * except pg_cancel, which may be called from any thread.
 */
#ifndef PG_CAPI_H
#define PG_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PG_ABI_VERSION 12

typedef int32_t pg_status;
enum {
    PG_OK = 0,
    PG_ERR_INVALID = 1,    /* bad argument / inconsistent scene */
    PG_ERR_HIP = 2,        /* HIP runtime error */
    PG_ERR_OOM = 3,        /* device allocation failed */
    PG_ERR_STATE = 4,      /* call out of order (e.g. render before upload) */
    PG_ERR_CANCELLED = 5,  /* pg_cancel() was called */
    PG_ERR_NO_DEVICE = 6   /* no gfx950 device visible */
};

/* BSDF models (reference: EBSDFModel, include/mitsuba/render/bsdf.h:287-297; plugins in src/bsdfs/). */
enum {
    PG_BSDF_DIFFUSE = 0,          /* src/bsdfs/diffuse.cpp          */
    PG_BSDF_CONDUCTOR = 1,        /* src/bsdfs/conductor.cpp        */
    PG_BSDF_ROUGHCONDUCTOR = 2,   /* src/bsdfs/roughconductor.cpp   */
    PG_BSDF_DIELECTRIC = 3,       /* src/bsdfs/dielectric.cpp       */
    PG_BSDF_ROUGHDIELECTRIC = 4,  /* src/bsdfs/roughdielectric.cpp  */
    PG_BSDF_PLASTIC = 5,          /* src/bsdfs/plastic.cpp          */
    PG_BSDF_ROUGHPLASTIC = 6,     /* src/bsdfs/roughplastic.cpp     */
    PG_BSDF_NULL = 7,             /* src/bsdfs/null.cpp: index-matched medium boundary */
    PG_BSDF_COUNT = 8
};
/* Microfacet distributions (src/bsdfs/microfacet.h:48-58). */
enum { PG_DIST_BECKMANN = 0, PG_DIST_GGX = 1 };
/* Material flags. */
#define PG_MAT_TWOSIDED 1u    /* wrap in the 'twosided' adapter (src/bsdfs/twosided.cpp) */
#define PG_MAT_NONLINEAR 2u   /* plastic: 'nonlinear' (src/bsdfs/plastic.cpp) */
#define PG_MAT_SAMPLE_ALL 4u  /* microfacet: sampleVisible=false (microfacet.h:112) */

/* One material; 112 bytes.  Conductor eta/k are RGB and already divided by extEta
 * (roughconductor.cpp:173-188).  Dielectric/plastic use int_ior/ext_ior. */
typedef struct pg_material {
    uint32_t type;
    uint32_t distribution;
    uint32_t flags;
    uint32_t pad0;
    float alpha_u, alpha_v;
    float int_ior, ext_ior;
    float diffuse_reflectance[4];    /* diffuse.reflectance, plastic.diffuseReflectance */
    float specular_reflectance[4];
    float specular_transmittance[4];
    float eta[4];
    float k[4];
} pg_material;

/* A shape = a contiguous triangle range with one BSDF and optionally one area emitter
 * (reference: Shape/TriMesh + AreaLight, src/librender/trimesh.cpp, src/emitters/area.cpp). */
typedef struct pg_shape {
    uint32_t tri_begin;
    uint32_t tri_count;
    uint32_t material;
    int32_t emitter;          /* index into emitters, or -1 */
    int32_t interior_medium;  /* Shape::getInteriorMedium (shape.h), index into media or -1 */
    int32_t exterior_medium;  /* Shape::getExteriorMedium; the side is the geometric normal's */
} pg_shape;

/* Participating medium (volpath integrator only).  PG_MEDIUM_HETEROGENEOUS is
 * src/medium/heterogeneous.cpp with Woodcock tracking (the default 'method'): a float32 density
 * grid (src/volume/gridvolume.cpp, trilinear, the data AABB mapped onto [0, res-1]^3, zero outside),
 * density multiplier 'scale', constant albedo (constvolume) and a Henyey-Greenstein phase function
 * (src/phase/hg.cpp).  Densities must lie in [0, 1] (heterogeneous.cpp:236-239). */
enum { PG_MEDIUM_HETEROGENEOUS = 0 };
typedef struct pg_medium {
    uint32_t type;
    uint32_t res[3];
    const float *density;  /* res[0] * res[1] * res[2], x fastest; copied at upload */
    float aabb_min[3];
    float aabb_max[3];
    float scale;
    float albedo[3];
    float g;               /* HG mean cosine */
    uint32_t pad0;
} pg_medium;

/* Area emitter attached to a shape (src/emitters/area.cpp:158-183).  Sampling weight 1, so the
 * scene picks emitters uniformly (Scene::sampleEmitterDirect, src/librender/scene.cpp:871-895). */
typedef struct pg_emitter {
    uint32_t shape;
    uint32_t pad[3];
    float radiance[4];
} pg_emitter;

/* Environment emitter with Mitsuba 'envmap' semantics (src/emitters/envmap.cpp:100-677): a
 * latitude-longitude RGB image (x = phi, y = theta from +Y, texel (x, y) at rgb[3 * (y * width + x)]),
 * stored at half precision as the reference's MIP map does (SpectrumHalf, envmap.cpp:101-103;
 * negative texels are clamped, mipmap.h:232-240), bilinear lookups with repeat in x and clamp in y
 * (mipmap.h:503-596), importance sampling by the sin(theta)-weighted luminance CDFs of
 * EnvironmentMap::configure (envmap.cpp:260-329) with a tent-filtered in-pixel offset
 * (internalSampleDirection, :567-600).  to_world is the rotation part of the 'toWorld' transform,
 * row-major (world = R * local).  It is the last emitter of the uniform emitter pick
 * (Scene::sampleEmitterDirect, scene.cpp:871-895).  The volumetric integrator does not support it. */
typedef struct pg_envmap {
    uint32_t width;
    uint32_t height;
    const float *rgb;      /* width * height * 3, copied at upload */
    float to_world[9];
    float scale;           /* 'scale' (envmap.cpp:188) */
    uint32_t pad0;
    uint32_t pad1;
} pg_envmap;

/* Pinhole camera with Mitsuba 'perspective' semantics (src/sensors/perspective.cpp:271-298,
 * Transform::lookAt src/libcore/transform.cpp:191-214): fov along x, near/far clip. */
typedef struct pg_camera {
    float origin[3];
    float target[3];
    float up[3];
    float fov_x_deg;
    float near_clip;
    float far_clip;
    uint32_t width;
    uint32_t height;
} pg_camera;

/* Flattened scene (what a Mitsuba adapter extracts from Scene::getShapes()/getBSDFs()/emitters). */
typedef struct pg_scene_desc {
    uint32_t num_vertices;
    uint32_t num_triangles;
    uint32_t num_shapes;
    uint32_t num_materials;
    uint32_t num_emitters;
    uint32_t num_media;
    const float *positions;     /* 3 * num_vertices */
    const float *normals;       /* 3 * num_vertices, or NULL (face normals) */
    const uint32_t *indices;    /* 3 * num_triangles */
    const pg_shape *shapes;     /* shapes partition [0, num_triangles) */
    const pg_material *materials;
    const pg_emitter *emitters;
    pg_camera camera;
    const pg_medium *media;     /* num_media entries (may be NULL when 0) */
    int32_t camera_medium;      /* Sensor::getMedium, index into media or -1 */
    int32_t pad1;
    const pg_envmap *envmap;    /* Scene::getEnvironmentEmitter (scene.h), or NULL */
} pg_scene_desc;

/* Integrator parameters (MonteCarloIntegrator props: src/librender/integrator.cpp:195-230;
 * progressive: progressiveintegrator.cpp:296-300; useNee: progressive_path.cpp:117) plus the
 * SD-tree guiding parameters (Mueller et al. 2017) and the device/shard placement. */
typedef struct pg_config {
    int32_t device;               /* HIP device ordinal used by this context */
    int32_t max_depth;            /* -1 = unbounded (Mitsuba default) */
    int32_t rr_depth;             /* 5 */
    int32_t use_nee;              /* 1 */
    int32_t hide_emitters;        /* 0 */
    int32_t strict_normals;       /* 0 */
    float max_component_value;    /* +inf */
    uint32_t seed;                /* 1337 (deterministic.cpp salt) */
    int32_t guiding;              /* 0 = plain progressive path tracer, 1 = SD-tree guided */
    float bsdf_sampling_fraction; /* 0.5 */
    float s_tree_threshold;       /* 12000 */
    float d_tree_threshold;       /* 0.01 */
    int32_t d_tree_max_depth;     /* 20 */
    int32_t record_max_vertices;  /* 32: training-record vertices kept per path */
    int32_t rank;                 /* image-tile shard of this context */
    int32_t world_size;
    uint32_t tile_size;           /* 32 (Scene::setBlockSize default) */
    uint32_t max_paths_in_flight; /* paths per chunk; 0 = auto: 2^25, or four rounds of lanes (<= 2^27 paths a
                                     chunk) for a path-integrator pass of at least 3 x lanes x 2^26 paths; both
                                     capped to 70 % of the free device memory */
    int32_t gpu_depth_cap;        /* hard bounce cap on the device when max_depth < 0 (1024; the path integrator
                                     clamps it to 1098, and pg_create rejects a path-integrator max_depth above
                                     1097 with PG_ERR_INVALID; the volpath integrator honours both exactly) */
    int32_t path_lanes;           /* path chunks in flight on separate streams, 1..4 (0 = auto: 3) */
    int32_t integrator;           /* PG_INTEGRATOR_PATH (progressive_path) or _VOLPATH (progressive_volpath) */
    int32_t volume_majorant;      /* volpath free-flight / transmittance tracking: PG_MAJORANT_GRID (default:
                                     delta tracking against per-cell maxima of 8^3-voxel blocks, skipping empty
                                     cells) or PG_MAJORANT_GLOBAL (the reference's single majorant, scale * 1,
                                     heterogeneous.cpp:589-660).  Both sample the same distributions. */
    float distance_guiding;       /* volpath + guiding: mixing weight beta of guided free-flight sampling (weighted
                                     delta tracking toward the SD-tree's zero-variance collision probability,
                                     oracle/orc_volpath.h GuidedAccept); 0 = the reference's free flight. 0.25 */
    int32_t aovs;                 /* 1: accumulate the denoiser feature buffers (Denoiser::Sample albedo + normal,
                                     include/mitsuba/render/denoiser.h:12-16) of every camera sample's first hit;
                                     read with pg_read_aovs.  Path integrator only.  0 */
    int32_t bsdf_fraction_bound;  /* guided path integrator: how the one-sample-MIS BSDF fraction alpha of a vertex is
                                     chosen.  PG_FRACTION_FIXED: alpha = bsdf_sampling_fraction everywhere (Mueller et
                                     al. 2017).  PG_FRACTION_ALBEDO: alpha = max(bsdf_sampling_fraction, min(a, 0.95))
                                     with a = the max channel of BSDF::getAlbedo, which bounds the mixture weight
                                     f / (alpha p_bsdf + (1 - alpha) p_guide) <= (f / p_bsdf) / alpha by 1 for albedo
                                     bounded BSDF weights.  PG_FRACTION_THROUGHPUT: as ALBEDO with a scaled by the path
                                     throughput max(T), so a path may regain throughput it lost, but not grow past 1.
                                     PG_FRACTION_LEARNED: alpha per S-tree leaf, learned from the training records
                                     (after Mueller 2019: the candidate mixture in 0.05, 0.15 .. 0.95 with the largest
                                     estimated cross-entropy against f * L_i; bsdf_sampling_fraction
                                     until a leaf has 64 guided records).
                                     Any per-vertex choice independent of the sampled direction is unbiased.
                                     Default PG_FRACTION_FIXED (Mueller et al. 2017's fixed fraction). */
    int32_t kernel_timing;        /* 1: bracket every closest-hit, shading and shadow launch with HIP events and sum
                                     their device times into pg_stats trace_ms / shade_ms / shadow_ms.  Six event
                                     records per bounce cost ~2 % on C3, so 0 (the default) leaves
                                     those three statistics at 0. */
    int32_t volpath_exact_mis;    /* volpath: 0 (default) = the reference's MIS weight for an emitter reached through
                                     index-matched surfaces, whose emitter pdf uses the LAST segment's length
                                     (rayIntersectAndLookForEmitter + DirectSamplingRecord::setQuery,
                                     progressive_volpath.cpp:401-460, records.inl:170-178): biased, +34 % on
                                     data/tests/test_bidir_2.xml.  1 = the whole ray length: the MIS
                                     weights sum to one and the estimator is unbiased. */
    int32_t tail_paths;           /* path integrator: a chunk with at most this many live paths finishes in one launch
                                     (k_tail: each thread loops shade -> shadow -> closest hit) instead of one
                                     launch pair + count readback per bounce; bit-identical results.  0 = the
                                     default (131072, or the PG_TAIL_PATHS environment variable), < 0 = off. */
    int32_t glossy_prior;         /* guided path integrator: 1 = the BSDF's glossy sampling rate r
                                     (BSDF::getGlossySamplingRate, bsdf.h:365-381: 1 for roughconductor and
                                     roughdielectric, the glossy lobe's probability for roughplastic,
                                     roughplastic.cpp:323-345, 0 otherwise) raises the vertex's BSDF fraction
                                     to r + (1 - r) alpha; vertices with r = 1 are not guided, and only vertices
                                     with r = 0 feed the learned-fraction statistics.  0 = off (Mueller 2017). */
} pg_config;
enum { PG_FRACTION_FIXED = 0, PG_FRACTION_ALBEDO = 1, PG_FRACTION_THROUGHPUT = 2, PG_FRACTION_LEARNED = 3 };
enum { PG_INTEGRATOR_PATH = 0, PG_INTEGRATOR_VOLPATH = 1 };
enum { PG_MAJORANT_GRID = 0, PG_MAJORANT_GLOBAL = 1 };

/* Training record written per non-delta path vertex (SoA-free 32-byte AoS). */
typedef struct pg_record {
    float pos[3];
    uint32_t dir;      /* canonical (cos theta, phi) square coords as 2 x u16 */
    float radiance;    /* average incident radiance estimate along dir */
    float wo_pdf;      /* pdf the direction was sampled with (one-sample MIS) */
    float product;     /* guided vertex: f * L_i / wo_pdf, the BSDF-weighted contribution along dir divided
                          by the throughput before the vertex (channel average); 0 otherwise */
    float weight;      /* guided vertex: the D-tree pdf of dir (the mixture's p_guide); -1: not guided.
                          The learned fraction (PG_FRACTION_LEARNED) reads both in the splat. */
} pg_record;

typedef struct pg_stats {
    uint64_t paths;           /* camera paths traced since create */
    uint64_t segments;        /* path segments (extension rays) */
    uint64_t shadow_rays;
    uint64_t records;         /* training records written */
    double trace_ms;          /* device time of the closest-hit kernel (HIP events; lanes overlap; needs
                                 pg_config.kernel_timing) */
    double shade_ms;          /* device time of the shading kernels (all material classes) */
    double shadow_ms;
    double other_ms;
    uint64_t trace_launches;  /* closest-hit launches timed alone (the camera rays; every bounce with
                                 PG_NO_RAYS_FUSION) */
    uint64_t stree_nodes;
    uint64_t dtree_nodes;
    uint64_t shade_launches;  /* material-class shading launches */
    double volume_ms;         /* device time of the volumetric path kernel (integrator = volpath) */
    uint64_t volume_launches;
    uint64_t density_lookups; /* volpath: trilinear density-grid lookups (tentative collisions) */
    uint64_t escaped;         /* path integrator: segments whose ray left the scene (not shaded) */
    double rays_ms;           /* device time of the fused shadow + closest-hit launches (k_rays; kernel_timing) */
    uint64_t rays_launches;   /* k_rays launches (a bounce's shadow rays + the next bounce's closest hits) */
    uint64_t shadow_launches; /* unfused shadow-ray launches (PG_NO_RAYS_FUSION) */
    uint64_t tail_launches;   /* chunk tails finished in one launch (k_tail) */
    /* ABI 11: the volumetric wavefront's stages (integrator = volpath, PG_VOL_WAVEFRONT): device time
     * (HIP events; pg_config.kernel_timing), launches, items processed and density lookups made by the
     * free-flight launches (k_vflight) and the interaction launches (k_vvertex) */
    double vol_flight_ms;
    uint64_t vol_flight_launches;
    uint64_t vol_flights;
    uint64_t vol_flight_lookups;
    double vol_vertex_ms;
    uint64_t vol_vertex_launches; /* kernels: each interaction stage launches the medium and the surface kernel */
    uint64_t vol_vertices;
    uint64_t vol_vertex_lookups;
    /* ABI 12: the interactions' deferred transmittance walks (k_vnee: NEE shadow walks and emitter walks
     * through media, each on its own counter sub-stream): device time, launches, slots walked, lookups */
    double vol_nee_ms;
    uint64_t vol_nee_launches;
    uint64_t vol_nee_walks;
    uint64_t vol_nee_lookups;
} pg_stats;

/* ---- lifecycle ---------------------------------------------------------------------- */
pg_status pg_config_default(pg_config *cfg);
pg_status pg_create(const pg_config *cfg, void **ctx_out);
pg_status pg_destroy(void *ctx);
const char *pg_last_error(void *ctx);
int32_t pg_abi_version(void);
pg_status pg_cancel(void *ctx); /* thread-safe */

/* ---- scene ---------------------------------------------------------------------------- */
pg_status pg_upload_scene(void *ctx, const pg_scene_desc *scene);

/* ---- one progression (pass): spp samples per pixel of this rank's tiles,
 *      sample indices [sample_offset, sample_offset + spp).  record != 0 writes training
 *      records (only meaningful with guiding).  Accumulates into the film. ------------ */
pg_status pg_render_pass(void *ctx, uint32_t spp, uint32_t sample_offset, int32_t record);
/* Time-budget rendering (maxRenderTime; ProgressiveMonteCarloIntegrator::renderTime,
 * src/librender/progressiveintegrator.cpp:117-168,185,207-208): whole progressions of
 * spp_per_progression samples, sample indices from sample_offset on, until `seconds` of wall clock
 * have passed (checked after each batch of progressions) or max_spp samples are done (0 = no cap).
 * *spp_done = samples per pixel rendered (the reference's m_spp after renderTime).  No records. */
pg_status pg_render_time(void *ctx, double seconds, uint32_t spp_per_progression, uint32_t sample_offset,
                         uint32_t max_spp, uint32_t *spp_done);

/* ---- training records / SD-tree refit (the postprogression slot) ------------------------ */
pg_status pg_get_record_count(void *ctx, uint64_t *count);
/* Copy local records out: dst is host memory unless dst_is_device != 0. */
pg_status pg_get_records(void *ctx, void *dst, uint64_t max_records, int32_t dst_is_device, uint64_t *written);
/* Splat records (e.g. the all-gathered set of every rank) into the building SD-tree. */
pg_status pg_splat_records(void *ctx, const void *src, uint64_t count, int32_t src_is_device);
/* Splat this context's own records (single-GPU case). */
pg_status pg_splat_local_records(void *ctx);
/* Build sampling trees from the building trees, refine the S-tree for training iteration
 * `iteration`, reset the building trees; clears the local record buffer. */
pg_status pg_refit(void *ctx, uint32_t iteration);
/* Serialize / inject the SD-tree (golden-vector tests).  Query size with buf == NULL. */
pg_status pg_get_sdtree(void *ctx, void *buf, uint64_t capacity, uint64_t *size);
pg_status pg_put_sdtree(void *ctx, const void *buf, uint64_t size);
/* Evaluate / sample the sampling SD-tree on the device for host arrays (parity tests). */
pg_status pg_sdtree_pdf(void *ctx, const float *pos, const float *dir, uint64_t n, float *pdf_out);
pg_status pg_sdtree_sample(void *ctx, const float *pos, const float *u, uint64_t n, float *dir_out, float *pdf_out);

/* ---- film ------------------------------------------------------------------------------ */
/* rgbw: width*height*4 floats (sum r,g,b, sample count); sumsq: width*height*4 (sum r^2,g^2,b^2,0).
 * Pixels outside this rank's tiles are zero.  Either pointer may be NULL. */
pg_status pg_read_film(void *ctx, float *rgbw, float *sumsq);
pg_status pg_reset_film(void *ctx);
/* Denoiser feature buffers (pg_config.aovs = 1), the per-pixel inputs Denoiser::add averages
 * (src/librender/denoiser.cpp:138-144): albedo: width*height*4 floats (sum of BSDF::getAlbedo at the
 * first hit, r, g, b, sample count); normal: width*height*4 (sum of first-hit shading normals, world
 * space, 0).  A camera ray that escapes contributes Denoiser::Sample's defaults: albedo 0, normal
 * (0, 0, -1).  Cleared by pg_reset_film.  Either pointer may be NULL. */
pg_status pg_read_aovs(void *ctx, float *albedo, float *normal);
pg_status pg_get_stats(void *ctx, pg_stats *stats);
/* Number of pixels owned by this rank (tile shard). */
pg_status pg_local_pixel_count(void *ctx, uint64_t *count);

/* ---- unit-level device entry points used by the parity tests ---------------------------- */
/* rays: n x 8 floats (o.xyz, tmin, d.xyz, tmax).  hits: n x 4 (t, prim as float bits, u, v);
 * prim = 0xFFFFFFFF for a miss.  any_hit: hits[i*4] = 1 if occluded else 0. */
pg_status pg_trace_rays(void *ctx, const float *rays, uint64_t n, int32_t any_hit, float *hits);
/* The closest hit's full record as the shading kernels build it (fillIntersectionRecord<true>,
 * skdtree.h:343-430: barycentric position, face normal flipped to the shading normal's side, interpolated
 * shading normal, shading frame by computeShadingFrame(n, dpdu = p1 - p0), wi = toLocal(-d)); the unit KAT of
 * src/tests/test_dgeom.cpp:69-177.  rays: n x 8 as pg_trace_rays; out: n x 16 floats (p.xyz, t, geoN.xyz,
 * shN.xyz, shFrame.s.xyz, wi.xyz), all zero for a miss. */
pg_status pg_hit_records(void *ctx, const float *rays, uint64_t n, float *out);
/* BSDF queries on the device for material `material` of the uploaded scene.
 * wi: n x 3 local; u: n x 3 (2D sample + component sample); out per query 12 floats:
 * wo.xyz, pdf, weight.rgb, sampled_type, eval(wi,wo_given).rgb, pdf(wi,wo_given).
 * wo_given: n x 3 local directions for the eval/pdf part (may be NULL). */
pg_status pg_bsdf_query(void *ctx, uint32_t material, const float *wi, const float *u,
                        const float *wo_given, uint64_t n, float *out);
/* HG phase function of medium `medium` on the device (HGPhaseFunction::sample / eval, hg.cpp:74-106).
 * in: n x 5 (wi.xyz pointing back along the incident ray, 2D sample); out: n x 5 floats
 * wo.xyz, pdf, eval(wi, wo_given) (0 when wo_given is NULL). */
pg_status pg_phase_query(void *ctx, uint32_t medium, const float *in, const float *wo_given, uint64_t n, float *out);
/* Medium queries on the device for medium `medium` (heterogeneous.cpp:546-660, gridvolume.cpp:337-380).
 * op 0 (density): in n x 3 world points; out n floats = lookupFloat(p) (unscaled).
 * op 1 (free flight) / op 2 (transmittance): in n x 8 rays (o.xyz, mint, d.xyz, maxt) and keys n x 2
 * (rng key, sample): the draws are dimensions 1, 2, ... of that counter stream.  out n x 4:
 * op 1: (interaction 1/0, t, draws used, 0), op 2: (transmittance estimate, draws used, 0, 0).
 * op 3 / op 4: as op 1 / op 2 with PG_MAJORANT_GRID tracking (ops 1, 2 use the global majorant). */
pg_status pg_medium_query(void *ctx, uint32_t medium, int32_t op, const float *in, const uint32_t *keys, uint64_t n,
                          float *out);
/* Environment emitter of the uploaded scene on the device (envmap.cpp).
 * op 0 (EnvironmentMap::sampleDirect, :516-543, from the scene's bounding-sphere centre):
 *      in n x 2 samples; out n x 8 = d.xyz (world), pdf (solid angle), value / pdf (rgb), distance.
 *      pdf = 0 where the sample fails.
 * op 1 (pdfDirect, :545-556): in n x 3 world directions; out n floats (solid-angle pdf).
 * op 2 (evalEnvironment without ray differentials, :380-410): in n x 3 world ray directions;
 *      out n x 3 radiance. */
pg_status pg_envmap_query(void *ctx, int32_t op, const float *in, uint64_t n, float *out);

/* Rough dielectric transmittance slice of a roughplastic material, as RoughPlastic::configure
 * reduces it (roughplastic.cpp:283-299, src/bsdfs/rtrans.h setEta/setAlpha/evalDiffuse):
 * table[100] = transmittance at cos(theta) = (j/99)^4 (interpolated with Catmull-Rom in
 * cos^(1/4)), fdr_int = 1 - internal diffuse transmittance.  Computed on the host at scene upload
 * by quadrature instead of read from data/microfacet/ *.dat.  Needs no device or context. */
/* Building-tree statistics of the SD-tree, i.e. the additive state that splats produce: the u64
 * quadrant sums of every building node (4 per node, 2^-24 fixed point) followed by the record count
 * of every D-tree (u64), in the order of the serialized tree.  Summing these vectors over ranks
 * (an all-reduce) and putting the sum back equals splatting every rank's records into one tree,
 * bit for bit (replaces the record all-gather of postprogression).
 * dst == NULL: only *words is returned.  Between pg_refit calls the layout is fixed. */
pg_status pg_get_tree_stats(void *ctx, void *dst, uint64_t capacity_words, int32_t dst_is_device, uint64_t *words);
pg_status pg_put_tree_stats(void *ctx, const void *src, uint64_t words, int32_t src_is_device);

pg_status pg_rough_transmittance(uint32_t distribution, float alpha, float eta, float *table, float *fdr_int);

/* ---- multi-GPU inside the library: one RCCL communicator per context (RCCL over xGMI) --------
 * Replaces the reference's distributed rendering (the remote scheduler that ships work units and
 * merges image blocks, include/mitsuba/core/sched_remote.h:50-236) for one render job: one
 * process (or thread) per GPU, each with a context created with its rank / world_size (its tile
 * shard).  Rank 0 calls pg_comm_unique_id and hands the PG_COMM_ID_BYTES bytes to every rank by
 * any out-of-band channel (MPI_Bcast, a file, torch.distributed); then every rank calls
 * pg_comm_init.  The pg_comm_* calls below are collective: every rank makes them, in the same
 * order.  Postprogression slot: pg_splat_local_records; pg_comm_allreduce_tree_stats; pg_refit
 * (every rank then holds the tree one GPU builds from all records, bit for bit).  End of the
 * job: pg_comm_reduce_film(root), then the root's pg_read_film returns the whole image. */
#define PG_COMM_ID_BYTES 128
pg_status pg_comm_unique_id(void *id_out);
pg_status pg_comm_init(void *ctx, const void *id);
/* In-place sum over ranks of the building statistics (the pg_get_tree_stats vector) on the device. */
pg_status pg_comm_allreduce_tree_stats(void *ctx);
/* Sum of every rank's film (+ sums of squares, + feature buffers) into rank `root`'s film; the
 * shards are disjoint, so the root's film equals the single-GPU film bit for bit. */
pg_status pg_comm_reduce_film(void *ctx, int32_t root);
/* In-place sum over ranks of n host doubles (e.g. inverse-variance combination statistics). */
pg_status pg_comm_allreduce_f64(void *ctx, double *values, uint64_t n);
/* The record exchange SURVEY.md §5/§8e names (north_star: "RCCL all-gather of records"), the
 * alternative to pg_splat_local_records + pg_comm_allreduce_tree_stats in the postprogression slot:
 * every rank's record count (ncclAllGather of one u64), then every rank's records (ncclAllGather in
 * slices of at most 2^22 records per rank, padded to whole slices, into one reused buffer of
 * world_size slices), and every rank splats ALL records into its building tree, slice by slice in rank
 * order.  Integer splat sums commute, so every rank ends with the tree one GPU builds from all
 * records, bit for bit -- the same tree as the statistics all-reduce.  counts_out (may be NULL):
 * world_size record counts.  The local records stay until pg_refit. */
pg_status pg_comm_allgather_records(void *ctx, uint64_t *counts_out);

#ifdef __cplusplus
}
#endif
#endif /* PG_CAPI_H */
