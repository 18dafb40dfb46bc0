// Host-callable launchers for the gfx950 kernels (defined in pg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pg_layout.h"

struct SceneDev {
    const float4 *nodes;    // BVH2, PG_BVH_NODE_F4 float4 per node
    const float4 *woop;     // 3 float4 per BVH-order triangle
    const float4 *tshade;   // PG_TRI_SHADE_F4 float4 per BVH-order triangle
    const GMat *mats;
    const GEmitter *ems;
    const float4 *emtri;    // PG_TRI_SHADE_F4 float4 per emitter triangle
    const float *emcdf;
};

struct PathDev {
    float4 *ray_o, *ray_d, *hit, *thr, *rad, *prev;
    uint4 *pinfo;
    float4 *sh_o, *sh_d, *sh_c;
    float4 *vtx;       // [max_vertices][P][3]
    uint32_t *stack_ovf;  // traversal-stack overflow ring, pg_stack_overflow_words(0) words
    uint32_t P;        // capacity (slot stride of vtx)
};

struct SDDev {
    const uint2 *snodes;
    const uint4 *meta;
    const float4 *qsum;
    const uint4 *qchild;
    const uint4 *bchild;
    unsigned long long *bsum;  // 4 per building node
    uint32_t *count;           // per D-tree
    const uint32_t *jump;      // S-tree jump grid, (2^jump_bits)^3 node ids
    float lo[3];
    float extent;
    int jump_bits;
    int built;
};

void pg_launch_camera(hipStream_t s, const GParams &g, const PathDev &p, const uint32_t *local_pixels,
                      uint32_t pix_begin, uint32_t npix, uint32_t nlayers, uint32_t sample_base, uint32_t *queue);
// fetch: FETCH_SHARDS (8) zeroed work counters for this launch
void pg_launch_trace(hipStream_t s, const SceneDev &sc, const PathDev &p, const uint32_t *queue,
                     const uint32_t *count, uint32_t max_count, uint32_t *fetch);
void pg_launch_shade(hipStream_t s, const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p,
                     const uint32_t *queue_in, const uint32_t *count_in, uint32_t max_count, uint32_t *queue_out,
                     uint32_t *count_out, uint32_t *shadow_queue, uint32_t *shadow_count);
void pg_launch_shadow(hipStream_t s, const SceneDev &sc, const PathDev &p, const uint32_t *queue,
                      const uint32_t *count, uint32_t max_count, uint32_t *fetch);
void pg_launch_film(hipStream_t s, const GParams &g, const PathDev &p, const uint32_t *local_pixels,
                    uint32_t pix_begin, uint32_t npix, uint32_t nlayers, float4 *film_rgbw, float4 *film_sumsq);
void pg_launch_commit(hipStream_t s, const PathDev &p, uint32_t nslots, int max_vertices, pg_record *records,
                      unsigned long long *rec_count, unsigned long long rec_capacity);
void pg_launch_splat(hipStream_t s, const SDDev &sd, const pg_record *recs, unsigned long long n);
void pg_launch_trace_rays(hipStream_t s, const SceneDev &sc, const float *rays, uint32_t n, int any, float *hits,
                          uint32_t *ovf);
// words of traversal-stack overflow storage for a launch of max_threads (0 = persistent grid)
size_t pg_stack_overflow_words(uint64_t max_threads);
void pg_launch_bsdf_query(hipStream_t s, const GMat *mat, const float *wi, const float *u, const float *wog,
                          uint32_t n, float *out);
void pg_launch_sd_pdf(hipStream_t s, const SDDev &sd, const float *pos, const float *dir, uint32_t n, float *out);
void pg_launch_sd_sample(hipStream_t s, const SDDev &sd, const float *pos, const float *u, uint32_t n, float *dir,
                         float *pdf);
