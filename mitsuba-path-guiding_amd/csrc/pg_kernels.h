// Host-callable launchers for the gfx950 kernels (defined in pg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pg_layout.h"

struct SceneDev {
    const float4 *nodes;    // binary BVH (closest hit), PG_BVH_NODE_F4 float4 per node
    const float4 *tris;     // 3 float4 per BVH-order triangle
    const float4 *wnodes;   // 8-wide BVH (shadow rays), PG_WIDE_NODE_F4 float4 per node
    const float4 *wtris;    // the same triangle records as tris (both BVHs share one triangle order)
    const float4 *tshade;   // PG_TRI_SHADE_F4 float4 per BVH-order triangle
    const uint8_t *tclass;  // PG_CLASS_* of the triangle's material, per BVH-order triangle
    const GMat *mats;
    const GEmitter *ems;
    const float4 *emtri;    // PG_TRI_SHADE_F4 float4 per emitter triangle
    const float *emcdf;
    const GEnv *env;        // environment emitter (the last emitter), or nullptr
    uint32_t top_nodes;     // binary-BVH nodes [0, top_nodes) are the top levels (k_trace stages them in LDS)
};

// float4 per training vertex: (x, woPdf), (T after the vertex, packed canonical wo), (L snapshot, -),
// (T before the vertex, p_guide(wo) or -1 when the vertex was not guided)
#define PG_VTX_F4 4
struct PathDev {
    float4 *ray_o, *ray_d, *hit, *thr, *rad, *prev;
    uint4 *pinfo;
    float4 *sh_d, *sh_c;  // shadow ray (direction, tmax) and contribution; its origin is ray_o
    float4 *vtx;       // [max_vertices][P][PG_VTX_F4]
    uint32_t *stack_ovf;  // traversal-stack overflow ring, pg_stack_overflow_words(0) words
    uint32_t P;        // path-state capacity
    uint32_t vtxP;     // slot stride of vtx (recording passes)
    // denoiser features (pg_config.aovs), 1 per slot: the camera ray's hit record (t, tri | ~0, u, v),
    // written by the chunk's first k_trace; k_film turns it into albedo + normal sums.  nullptr: off.
    float4 *aov;
};

struct SDDev {
    const uint2 *snodes;
    const uint4 *meta;
    const float4 *qsum;        // sampling D-tree nodes, 32 B each: {float4 energies, uint4 children}
    const uint4 *qchild;       // (const uint4 *)(qsum + 1); node n at index 2n of both
    const uint4 *bchild;
    unsigned long long *bsum;  // 4 per building node
    unsigned long long *count;  // records per D-tree (u64, so the building statistics are one u64 vector)
    const uint32_t *jump;      // S-tree jump grid, (2^jump_bits)^3 node ids
    unsigned long long *frac;  // learned-fraction statistics, kFracStats (pg_sdtree.h) per D-tree
    float lo[3];
    float extent;
    int jump_bits;
    int built;
    int learned;               // pg_config.bsdf_fraction_bound == PG_FRACTION_LEARNED
    float alpha0;              // pg_config.bsdf_sampling_fraction: a leaf's fraction before it is learned
};

// Volumetric path tracing (pg_config.integrator == PG_INTEGRATOR_VOLPATH)
struct VolDev {
    const GMedium *media;
    const uint32_t *tmed;      // per BVH-order triangle: (interior + 1) | (exterior + 1) << 16, 0 = no transition
    int32_t cam_medium;        // -1: none
    uint32_t num_media;
    int32_t grid;              // 1: majorant-grid tracking, 0: the global majorant
    float4 *rad;               // per work item (layer-major: item = layer * npix + lp), radiance
    uint32_t *next;            // work counter (zeroed by the launcher)
    unsigned long long *stats; // [0] segments (closest-hit rays), [1] NEE transmittance queries, [2] density lookups;
                               // wavefront: [3] flights, [4] their lookups, [5] interactions, [6] their lookups,
                               // [7] deferred walk entries (k_vnee), [8] their lookups
    uint32_t *stack_ovf;       // pg_stack_overflow_words(0) words
    float4 *vtx;               // guided training vertices [max_vertices][vtx_P][PG_VTX_F4] (PathDev::vtx layout)
    uint32_t vtx_P;            // slot stride of vtx (>= items per launch)
    float dist_beta;           // pg_config.distance_guiding
    uint32_t refill_min;       // k_volpath refills a wave's finished lanes once at least this many are idle
    const uint8_t *tcheap;     // per BVH-order triangle: 1 = delta BSDF or emitter (the wavefront's cheap surface queue)
    uint32_t models;           // 1: every material is diffuse or null (surface launches compiled for those only)
};

// Volumetric wavefront (pg_volpath.hip k_vcam, k_vflight, k_vvertex, k_vtail): the megakernel's per-lane
// VPath + VRng as SoA per slot (slot = the chunk's work item), read and written by each stage
struct VolWave {
    float4 *o;   // (ray origin, its.t)
    float4 *d;   // (ray direction, its.u)
    uint4 *s;    // (bits(its.v), its.tri, (medium + 1) | valid << 16 | scattered << 17 | emission << 18, depth)
    float4 *T;   // (throughput, eta)
    float4 *L;   // (radiance, bits(training vertices written))
    uint4 *r;    // random stream (key, sample, next dimension, density lookups so far)
    float4 *mp;  // the medium interaction point of the current iteration's free flight
    // deferred transmittance walks of the current iteration's interactions (pg_volpath.hip VDefer, k_vnee):
    // NEE (shadow walk origin, dim), (emitter point, max crossings), (contribution, flags); emitter hit
    // (walk origin, mint), (direction, dim), (contribution, medium | crossings)
    float4 *n0, *n1, *n2, *h0, *h1, *h2;
    // (flags: which of them are valid, whether the path ended, its vertex (pg_volpath.hip deferFlags); the
    // path's rng key; its sample; 0): the walks' streams come from here, so k_vnee shares no memory with the
    // next iteration's k_vflight, which rewrites r[slot] on the other stream (PG_VOL_NEE_OVERLAP)
    uint4 *nflags;
};

// Sharded work queue of path slots: shard s holds items[s * stride, s * stride + counts[s]).
// Appends are wave-aggregated atomics on the shard's own counter: one counter per queue serialized
// every append of the chip (58k returning atomics on one address: 658 us; on 64 addresses: 18 us,
// tools/atomic_bench.hip).  A path keeps the shard the camera gave it until it terminates, so
// each queue's shard s is bounded by the camera queue's shard s (stride = pg_queue_stride(P)).
#define PG_QSHARDS 64
struct Queue {
    uint32_t *items;
    uint32_t *counts;  // PG_QSHARDS
    uint32_t stride;
    uint16_t *keys = nullptr;  // ray order keys of the entries (k_shade's output queue when rays are sorted)
};
// Ray order for the next closest-hit launch (pg_config: PG_RAY_SORT): key = direction octant (3 bits,
// major) then the Morton code of the origin's cell in an 8^3 grid over the SD-tree cube (9 bits)
#define PG_RAY_SORT_BINS 4096
// camera layout: slot -> shard (slot >> 6) & 63, entry ((slot >> 12) << 6) | (slot & 63)
// shard capacity for `capacity` paths: 64 x ceil(capacity / 4096) for the interleaved camera map, plus what the
// banded map (below) can add.  A band holds ceil(npix / 8) x nlayers <= n / 8 + 7 nlayers / 8 items and a shard
// at most 64 x ceil(band / 512) <= n / 64 + 7 nlayers / 64 + 64 of them; bands are used only for >= 4096 pixels,
// so nlayers <= capacity / 4096: the extra is <= 7 capacity / 2^18 + 64 entries
__host__ __device__ inline uint32_t pg_queue_stride(uint32_t capacity) {
    return 64u * ((capacity + 4095u) / 4096u + (uint32_t)(((uint64_t)capacity * 7u + (1u << 24) - 1u) >> 24) + 2u);
}
__host__ __device__ inline uint32_t pg_camera_shard_count(uint32_t n, uint32_t s) {
    int rem = (int)(n & 4095u) - 64 * (int)s;
    return 64u * (n >> 12) + (uint32_t)(rem < 0 ? 0 : rem > 64 ? 64 : rem);
}
// XCD-banded camera map (round 6, PG_CAMERA_BANDS): blocks b and b + 8 run on one XCD (MI355X_MICROARCH.md
// §Workgroup dispatch) and every sharded launch gives block b shard b % 64, so shards s and s + 8 share an XCD's
// L2 for the paths' whole lives.  The banded map deals the chunk's pixels in 8 contiguous bands (local pixel
// order: whole 32 x 32 tiles), band r to the 8 shards r, r + 8, ..., r + 56, so one XCD traces and shades the
// paths of one image region: their BVH nodes, triangles, materials and SD-tree cells are that region's.  Within
// a band, item k (layer-major) goes to shard r + 8 ((k >> 6) & 7) at ((k >> 9) << 6) | (k & 63).  Chunks of
// fewer than 4096 pixels keep the interleaved map (slot s -> shard (s >> 6) & 63).
constexpr uint32_t kBandMinPixels = 4096;
__host__ __device__ inline uint32_t pg_band_start(uint32_t r, uint32_t npix) {
    return (uint32_t)(((uint64_t)r * npix + 7u) / 8u);
}
__host__ __device__ inline uint32_t pg_banded_shard_count(uint32_t npix, uint32_t nlayers, uint32_t s) {
    const uint32_t r = s & 7u, j = s >> 3;
    const uint32_t m = (pg_band_start(r + 1, npix) - pg_band_start(r, npix)) * nlayers;
    const int rem = (int)(m & 511u) - 64 * (int)j;
    return 64u * (m >> 9) + (uint32_t)(rem < 0 ? 0 : rem > 64 ? 64 : rem);
}
__host__ __device__ inline bool pg_camera_banded(bool bands, uint32_t npix) { return bands && npix >= kBandMinPixels; }
__host__ __device__ inline uint32_t pg_camera_count(bool banded, uint32_t npix, uint32_t nlayers, uint32_t s) {
    return banded ? pg_banded_shard_count(npix, nlayers, s) : pg_camera_shard_count(npix * nlayers, s);
}
// the largest camera shard of a chunk (the bound every later queue of the chunk stays under)
inline uint32_t pg_camera_bound(bool banded, uint32_t npix, uint32_t nlayers) {
    uint32_t b = 0;
    for (uint32_t s = 0; s < 64; ++s) {
        const uint32_t c = pg_camera_count(banded, npix, nlayers, s);
        b = c > b ? c : b;
    }
    return b;
}

void pg_launch_camera(hipStream_t s, const GParams &g, const PathDev &p, const uint32_t *local_pixels,
                      uint32_t pix_begin, uint32_t npix, uint32_t nlayers, uint32_t sample_base, Queue q, bool banded);
// closest hit for the live queue, partitioned by the hit's material class: class c < PG_NUM_CLASSES
// goes to class_queues[c] (shard s -> shard s); escaped paths are only counted, in
// class_queues[PG_NUM_CLASSES].counts.  max_shard: upper bound of the largest shard count (sizes
// the grid; the kernels read the counts).
// first_bounce: the chunk's camera rays (their hit records are kept in p.aov when it is set)
void pg_launch_trace(hipStream_t s, const GParams &g, const SceneDev &sc, const PathDev &p, Queue q, uint32_t max_shard,
                     const Queue *class_queues, bool first_bounce);
void pg_launch_shade_class(hipStream_t s, int cls, const GParams &g, const SceneDev &sc, const SDDev &sd,
                           const PathDev &p, Queue in, uint32_t max_shard, Queue out, Queue shadow);
// every material class of a bounce in one launch (k_shade_all; scenes without an environment
// emitter): pg_launch_shade_class for each class c with max_shard[c] > 0
void pg_launch_shade_all(hipStream_t s, const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p,
                         const Queue *class_queues, const uint32_t *max_shard, Queue out, Queue shq);
// shadow rays of a bounce and the closest hits of the next in one launch (k_rays; scenes without an
// environment emitter): the pair pg_launch_shadow + pg_launch_trace without the aov hook
void pg_launch_rays(hipStream_t s, const GParams &g, const SceneDev &sc, const PathDev &p, Queue q, uint32_t max_shard,
                    const Queue *class_queues, Queue shq, uint32_t max_shadow_shard);
void pg_launch_shadow(hipStream_t s, const SceneDev &sc, const PathDev &p, Queue q, uint32_t max_shard);
// every remaining path of the queue `q` (its hits already traced) to its end in one launch, each thread
// looping shade -> shadow ray -> closest hit (k_tail); stats: 3 u64 (segments, escaped, shadow rays)
void pg_launch_tail(hipStream_t s, const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p, Queue q,
                    uint32_t max_shard, unsigned long long *stats);
// counting sort of every shard of `q` by its keys into sorted_items (same shard layout and counts):
// histogram, per-shard scan, scatter; hist: PG_QSHARDS * PG_RAY_SORT_BINS u32 of scratch (zeroed here)
void pg_launch_ray_sort(hipStream_t s, Queue q, uint32_t max_shard, uint32_t *sorted_items, uint32_t *hist,
                        uint32_t bins = PG_RAY_SORT_BINS);  // bins: PG_RAY_SORT_BINS or 512
// aov_albedo / aov_normal: per-pixel feature sums, read when p.aov is set
void pg_launch_film(hipStream_t s, const GParams &g, const SceneDev &sc, const PathDev &p, const uint32_t *local_pixels,
                    uint32_t pix_begin, uint32_t npix, uint32_t nlayers, float4 *film_rgbw, float4 *film_sumsq,
                    float4 *aov_albedo = nullptr, float4 *aov_normal = nullptr);
// unit-level environment-emitter queries (pg_envmap_query)
void pg_launch_envmap_query(hipStream_t s, const SceneDev &sc, int op, const float *in, uint32_t n, float *out);
// p.pinfo == nullptr: the vertex count of slot i is bits(p.rad[i].w) (volpath items)
// env_hits: surface path with an environment emitter (escape radiance in the hit record)
void pg_launch_commit(hipStream_t s, const PathDev &p, uint32_t nslots, int max_vertices, pg_record *records,
                      unsigned long long *rec_count, unsigned long long rec_capacity, int env_hits);
// S-tree jump grid (SDDev::jump) of the device S-tree: cell (x, y, z) of the 2^bits grid -> the node
// reached after 3 * bits axis-cycling midpoint decisions from the root (or the leaf met before)
void pg_launch_sd_jump(hipStream_t s, const uint32_t *snodes, int bits, uint32_t *jump);
void pg_launch_splat(hipStream_t s, const SDDev &sd, const pg_record *recs, unsigned long long n);
// one volpath sample per (pixel, layer) item of the chunk, written to v.rad[item]
void pg_launch_volpath(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                       const uint32_t *local_pixels, uint32_t pix_begin, uint32_t npix, uint32_t nlayers,
                       uint32_t sample_base);
// Volumetric wavefront, one chunk of npix * nlayers items (slot = item): the camera rays and first hits
// (paths in a medium -> flight, others -> surface queue); per iteration the free flights of `flight`
// (medium interactions -> med, flights reaching their surface -> surf) and the vertices of `med` and
// `surf` (surviving paths -> next_flight / next_surf by their medium); the tail finishes the paths
// of `flight` and `surf` one thread each.  max_*: upper bounds of the largest shard counts.
void pg_launch_vol_camera(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const VolWave &w,
                          const uint32_t *local_pixels, uint32_t pix_begin, uint32_t npix, uint32_t nlayers,
                          uint32_t sample_base, Queue flight, Queue surf, Queue dsurf);
// surf / dsurf: surface vertices on other / delta-class surfaces (and escaped rays), pg_volpath.hip PG_VOL_SPLIT_SURF
void pg_launch_vol_flight(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                          const VolWave &w, Queue flight, uint32_t max_flight, Queue med, Queue surf, Queue dsurf);
int pg_launch_vol_vertex(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                         const VolWave &w, Queue med, uint32_t max_med, Queue surf, uint32_t max_surf, Queue dsurf,
                         uint32_t max_dsurf, Queue next_flight, Queue next_surf, Queue next_dsurf, const Queue *nee);
// the interactions' deferred transmittance walks (k_vnee); max_nee bounds every shard of `nee`
void pg_launch_vol_nee(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const VolWave &w, Queue nee,
                       uint32_t max_nee);
void pg_launch_vol_tail(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                        const VolWave &w, Queue flight, uint32_t max_flight, Queue surf, uint32_t max_surf, Queue dsurf,
                        uint32_t max_dsurf);
void pg_launch_phase_query(hipStream_t s, const GMedium *medium, const float *in, const float *wog, uint32_t n,
                           float *out);
// corner-packed density of a linear grid (pg_layout.h PG_DENSITY_CORNERS); out: 8 floats per cell
void pg_launch_density_corners(hipStream_t s, const float *lin, uint32_t rx, uint32_t ry, uint32_t rz, float *out);
void pg_launch_medium_query(hipStream_t s, const GMedium *medium, int op, const float *in, const uint32_t *keys,
                            uint32_t n, float *out);
void pg_launch_trace_rays(hipStream_t s, const SceneDev &sc, const float *rays, uint32_t n, int any, float *hits,
                          uint32_t *ovf);
// words of traversal-stack overflow storage for a launch of max_threads (0 = persistent grid)
size_t pg_stack_overflow_words(uint64_t max_threads);
// threads pg_launch_trace_rays launches for n rays (size its overflow ring with this)
uint64_t pg_trace_rays_threads(uint64_t n);
void pg_launch_bsdf_query(hipStream_t s, const GMat *mat, const float *wi, const float *u, const float *wog,
                          uint32_t n, float *out);
void pg_launch_sd_pdf(hipStream_t s, const SDDev &sd, const float *pos, const float *dir, uint32_t n, float *out);
void pg_launch_sd_sample(hipStream_t s, const SDDev &sd, const float *pos, const float *u, uint32_t n, float *dir,
                         float *pdf);
