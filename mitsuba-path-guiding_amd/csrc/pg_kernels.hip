// gfx950 kernels of the guided path-tracing wavefront (DESIGN.md §"Kernels").
//
// One bounce of the reference's ProgressiveMIPathTracer::Li (progressive_path.cpp:133-314) is
// split into:  trace (closest hit over the live-path queue) -> shade (emission/MIS of the previous
// segment, Russian roulette, NEE sampling, BSDF / SD-tree one-sample-MIS direction sampling,
// training-vertex write, queue compaction by wave ballot) -> shadow (any hit; adds the NEE
// contribution).  Camera rays, film accumulation, record commit and SD-tree splat are separate
// kernels.  Path state is SoA float4/uint4 arrays indexed by path slot.
#include <algorithm>
#include <cstdlib>

#include "pg_trace.h"

// LDS staging of node and material tiles (measured, off by default: profiles/r02k_lds_ab/ -- C3
// within noise to -1 %: the top BVH levels and the few materials already hit in L1, and the block
// fill + barrier is paid by every short-lived shading block)
#ifndef SHADE_LDS_MATS
#define SHADE_LDS_MATS 0   // > 0: k_shade stages up to this many materials in LDS (64 = 8 KiB)
#endif
#ifndef PG_RAYS_LDS_TOP
#define PG_RAYS_LDS_TOP 0  // 1: k_rays' closest-hit blocks stage the 4-wide BVH's top levels in LDS (1.3 KiB)
#endif
// the LDS tile of the closest-hit BVH's top levels: node size and capacity of this build's BVH
#if PG_BVH4
#define PG_TOP_NODE_F4 PG_QNODE_F4
#define PG_TOP_TILE_F4 (PG_BVH4_TOP_NODES * PG_QNODE_F4)
#else
#define PG_TOP_NODE_F4 PG_BVH_NODE_F4
#define PG_TOP_TILE_F4 (PG_BVH_TOP_NODES * PG_BVH_NODE_F4)
#endif
#ifndef PG_TRACE_LDS_TOP
#define PG_TRACE_LDS_TOP 0  // 1: k_trace stages the BVH's top PG_BVH_TOP_LEVELS levels in LDS (2 KiB)
#endif

// =============================================================================================
// camera rays: PerspectiveCamera::sampleRay (perspective.cpp:271-298) for (pixel, sample) slots
__global__ __launch_bounds__(256) void k_camera(GParams g, PathDev p, const uint32_t *__restrict__ local_pixels,
                                                uint32_t pix_begin, uint32_t npix, uint32_t nlayers,
                                                uint32_t sample_base, Queue q, bool banded) {
    uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = npix * nlayers;
    if (slot < PG_QSHARDS) q.counts[slot] = pg_camera_count(banded, npix, nlayers, slot);
    if (slot >= n) return;
    uint32_t layer = slot / npix, lp = slot - layer * npix;
    uint32_t pix = local_pixels[pix_begin + lp];
    uint32_t sample = sample_base + layer;
    uint32_t key = rngKey(pix, g.seed);
    float jx, jy;
    rng2(key, sample, 0, jx, jy);
    float px = (float)(pix % g.width) + jx, py = (float)(pix / g.width) + jy;
    float sx = px / (float)g.width, sy = py / (float)g.height;
    f3 nearP = mk((1.0f - 2.0f * sx) * g.tan_half, (1.0f - 2.0f * sy) / g.aspect * g.tan_half, 1.0f);
    f3 d = normalize(nearP);
    float invZ = 1.0f / d.z;
    f3 left = mk(g.cam_left[0], g.cam_left[1], g.cam_left[2]);
    f3 up = mk(g.cam_up[0], g.cam_up[1], g.cam_up[2]);
    f3 dir = mk(g.cam_dir[0], g.cam_dir[1], g.cam_dir[2]);
    f3 wd = left * d.x + up * d.y + dir * d.z;
    stS(&p.ray_o[slot], make_float4(g.cam_o[0], g.cam_o[1], g.cam_o[2], g.near_clip * invZ));
    stS(&p.ray_d[slot], f4(wd, g.far_clip * invZ));
    // throughput (1, eta 1) and the previous vertex are implied by depth 1: the first bounce's readers
    // (shadeOne, envEscapeRadiance) do not load them.  L = 0 is stored: a camera ray that escapes is
    // never shaded and k_film reads its L.
    stS(&p.rad[slot], make_float4(0.f, 0.f, 0.f, 0.f));
    stS(&p.pinfo[slot], make_uint4(pix, sample, 1u | (PF_EMITTED_QUERY << 16), 0u));
    if (banded) {  // pg_kernels.h pg_banded_shard_count: band r of the local pixels -> shards r, r + 8, ...
        const uint32_t r = (uint32_t)(((uint64_t)lp * 8u) / npix);
        const uint32_t b0 = pg_band_start(r, npix), m = pg_band_start(r + 1, npix) - b0;
        const uint32_t k = layer * m + (lp - b0);
        q.items[(r + 8u * ((k >> 6) & 7u)) * q.stride + (((k >> 9) << 6) | (k & 63u))] = slot;
    } else {
        q.items[((slot >> 6) & 63u) * q.stride + (((slot >> 12) << 6) | (slot & 63u))] = slot;
    }
}

// BSDF::getAlbedo of the config BSDFs (diffuse.cpp:112, conductor.cpp:225, roughconductor.cpp:264,
// dielectric.cpp:230, roughdielectric.cpp:272, plastic.cpp:266, roughplastic.cpp:354; null: the
// BSDF default 0, bsdf.h:361).  twosided picks the nested BSDF by side, which is the same BSDF here.
__device__ __forceinline__ f3 bsdfAlbedo(const GMat &M) {
    const f3 diff = mk(M.diff[0], M.diff[1], M.diff[2]), spec = mk(M.spec[0], M.spec[1], M.spec[2]);
    const f3 trans = mk(M.trans[0], M.trans[1], M.trans[2]);
    switch (M.model) {
        case PG_BSDF_DIFFUSE: return diff;
        case PG_BSDF_CONDUCTOR:
        case PG_BSDF_ROUGHCONDUCTOR: return spec;
        case PG_BSDF_DIELECTRIC: return trans * 0.5f + spec * (1 - 0.5f);
        case PG_BSDF_ROUGHDIELECTRIC: return spec * 0.5f + trans * (1 - 0.5f);
        case PG_BSDF_PLASTIC: return diff * 0.5f + spec * (1 - 0.5f);
        case PG_BSDF_ROUGHPLASTIC: return spec * 0.5f + diff * (1 - 0.5f);
        default: return mk1(0.f);
    }
}

// A path whose extension ray escaped (progressive_path.cpp:150-158 for the camera ray, :252-267 +
// :276-284 after a bounce): the environment emitter's radiance, MIS-weighted against its NEE pdf.
// radiance an escaped path picks up from the environment emitter.  k_trace stores it in the path's
// hit record (t, u, v of a miss; the escape ends the path), and k_film / k_commit add it to L
// (envHitRadiance): the sum (L + NEE of the last vertex) + environment keeps its order while the
// last vertex's shadow ray may run in the same launch (k_rays)
__device__ __forceinline__ f3 envEscapeRadiance(const GParams &g, const SceneDev &sc, const PathDev &p, uint32_t slot,
                                                f3 rd) {
    const uint4 pi = p.pinfo[slot];
    const uint32_t depth = pi.z & 0xFFFFu, flags = pi.z >> 16;
    f3 add;
    if (depth == 1) {  // camera ray (throughput 1): the loop-top miss with EEmittedRadiance
        if (!(flags & PF_EMITTED_QUERY) || (g.hide_emitters && !(flags & PF_SCATTERED))) return mk1(0.f);
        add = envEval(*sc.env, rd);
    } else {
        const float4 T4 = p.thr[slot];
        if (g.hide_emitters && !(flags & PF_SCATTERED)) return mk1(0.f);
        const float4 pv = p.prev[slot];
        float w = 1.0f;
        if (g.use_nee) {
            const float lumPdf = (flags & PF_PREV_DELTA) ? 0.0f : envPdf(*sc.env, rd) * (1.0f / (float)g.num_emitters);
            w = miWeight(pv.w, lumPdf);
        }
        add = xyz(T4) * envEval(*sc.env, rd) * w;
    }
    return add;
}
// L of a finished path plus the environment radiance its escape left in the hit record
__device__ __forceinline__ float4 envHitRadiance(float4 L, float4 hv) {
    if (__float_as_uint(hv.y) == 0xFFFFFFFFu) {
        L.x += hv.x;
        L.y += hv.z;
        L.z += hv.w;
    }
    return L;
}


// closest hit for every queued path: hit[slot] = (t, BVH-order triangle | ~0, u, v).
// Grid-stride over the queue shard blockIdx % PG_QSHARDS.  (A persistent variant with dynamic
// ray fetch into finished lanes measured slower once traversal was made while-while.)
struct ClassQueues {
    Queue q[PG_NUM_CLASSES + 1];
};

// wave-aggregated append of `slot` to class queue `cls` (< 0: none), shard s: one atomic per class
// present in the wave; class PG_NUM_CLASSES (escaped paths) is counted only
__device__ __forceinline__ void classAppend(int cls, uint32_t slot, const ClassQueues &cqs, uint32_t s) {
    const int lane = threadIdx.x & 63;
    unsigned long long pending = __ballot(cls >= 0);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const int c = __shfl(cls, leader);
        const unsigned long long mine = __ballot(cls == c);
        const Queue &cq = cqs.q[c];
        uint32_t b = 0;
        if (lane == leader) b = atomicAdd(cq.counts + s, (uint32_t)__popcll(mine));
        b = __shfl(b, leader);
        if (cls == c && c < PG_NUM_CLASSES)
            cq.items[(size_t)s * cq.stride + b + __popcll(mine & ((1ull << lane) - 1ull))] = slot;
        pending &= ~mine;
    }
}

// closest hits of the rows of queue shard bid % PG_QSHARDS that block bid of nblk takes (a
// grid-stride loop: k_trace, or the trace blocks of k_rays).
// ENV: the scene has an environment emitter (escaped paths pick up its radiance)
// first: the camera rays' bounce with denoiser features on (pg_config.aovs): the hit record of every
// path also goes to p.aov, which k_film resolves into albedo and normal (nullptr: off)
// WIDE (PG_CLOSEST_WIDE, A/B): the closest hits walk the shadow rays' 8-wide quantised BVH (octant order,
// boxes culled at tmax; no slab padding) instead of the 4-wide nodes: k_rays 29.4 against 23.9 ms per
// calibration pass, C3 549-553 against 616-621 Mpaths/s (profiles/r05ag_closest_wide/): octant order
// visits more boxes than the 4-wide walk's sorted descent saves in node fetches
#ifndef PG_CLOSEST_WIDE
#define PG_CLOSEST_WIDE 0
#endif
template <bool ENV, bool LTOP, bool WIDE = false>
__device__ __forceinline__ void traceRows(const GParams &g, const SceneDev &sc, const PathDev &p, const Queue &q,
                                          const ClassQueues &cqs, float4 *first, uint32_t bid, uint32_t nblk,
                                          const TStack &stk, const float4 *top, int ntop) {
    const uint32_t s = bid & (PG_QSHARDS - 1);
    const uint32_t n = q.counts[s];
    const uint32_t *items = q.items + (size_t)s * q.stride;
    // block-uniform loop bound, so whole waves reach the class ballots together
    for (uint32_t base = (bid / PG_QSHARDS) * TRACE_BLOCK; base < n; base += nblk / PG_QSHARDS * TRACE_BLOCK) {
        const uint32_t i = base + threadIdx.x;
        int cls = -1;
        uint32_t slot = 0;
        if (i < n) {
            slot = items[i];
            float4 o = ldS(&p.ray_o[slot]), d = ldS(&p.ray_d[slot]);
            float tmax = d.w;
            uint32_t tri = 0xFFFFFFFFu;
            float u = 0, v = 0;
            bool h;
            if constexpr (WIDE)
                h = traverseWide<false>(sc.wnodes, sc.wtris, xyz(o), xyz(d), o.w, tmax, tri, u, v,
                                        WStack{stk.lds, stk.ovf, stk.ostride});
            else
                h = traverse<false, LTOP>(sc.nodes, sc.tris, xyz(o), xyz(d), o.w, tmax, tri, u, v, stk, top, ntop);
            float4 hr = make_float4(h ? tmax : 0.0f, __uint_as_float(h ? tri : 0xFFFFFFFFu), u, v);
            if (first) first[slot] = hr;
            if (ENV && !h) {
                const f3 e = envEscapeRadiance(g, sc, p, slot, xyz(d));
                hr = make_float4(e.x, hr.y, e.y, e.z);
            }
            stS(&p.hit[slot], hr);
            cls = h ? (int)sc.tclass[tri] : PG_NUM_CLASSES;
        }
        classAppend(cls, slot, cqs, s);
    }
}

// traceRows with persistent lanes (PG_TRACE_PERSIST, A/B, off): each wave takes a contiguous segment of its
// shard's queue and runs the closest-hit walk one while-while round at a time (pg_trace.h Walk4); once at least
// PG_TRACE_REFILL of its 64 lanes have finished their rays, they take the segment's next rays together (a lane
// refill costs the whole wave the ray loads and the walk setup, so refills are batched, as k_volpath's).  A
// finished lane writes its hit record and joins the class append of that round.  Every ray's walk is traverse4's,
// so hits, films and trees are the grid-stride kernel's bit for bit (tests/test_gpu_parity.py, _configs, _params:
// 90/90 with it on).  Measured slower (profiles/r06_persist/): C3 521-523 against 637 Mpaths/s, k_rays 31.6 against
// 22.6 ms and k_shade_all 26.7 against 22.2 ms per calibration pass.  With 8 waves per SIMD the idle lanes of one
// wave's while-while rounds are already covered by the other waves' issue, so the refill rounds only add their
// ballots and setup; and the class queues come out in completion order instead of queue order, which costs the
// shading kernel its ray coherence (6 waves per SIMD: 559-561, k_rays 27.0 ms).
#ifndef PG_TRACE_PERSIST
#define PG_TRACE_PERSIST 0
#endif
#ifndef PG_TRACE_REFILL
#define PG_TRACE_REFILL 24
#endif
template <bool ENV>
__device__ __forceinline__ void traceRowsPersist(const GParams &g, const SceneDev &sc, const PathDev &p, const Queue &q,
                                                 const ClassQueues &cqs, float4 *first, uint32_t bid, uint32_t nblk,
                                                 const TStack &stk) {
    const uint32_t s = bid & (PG_QSHARDS - 1);
    const uint32_t n = q.counts[s];
    const uint32_t *items = q.items + (size_t)s * q.stride;
    constexpr uint32_t kWavesPerBlock = TRACE_BLOCK / 64;
    const uint32_t waves = (nblk / PG_QSHARDS) * kWavesPerBlock;
    const uint32_t wv = (bid / PG_QSHARDS) * kWavesPerBlock + threadIdx.x / 64;
    const uint32_t per = (n + waves - 1) / waves;
    uint32_t cur = min(n, wv * per);
    const uint32_t end = min(n, cur + per);
    const int lane = threadIdx.x & 63;
    bool active = false;
    uint32_t slot = 0;
    Walk4 w;
    for (;;) {
        const unsigned long long act = __ballot(active);
        const uint32_t idle = 64u - (uint32_t)__popcll(act);
        if (cur < end && (idle >= PG_TRACE_REFILL || act == 0)) {  // batched refill of the idle lanes
            const uint32_t rank = (uint32_t)__popcll(~act & ((1ull << lane) - 1ull));
            if (!active && cur + rank < end) {
                slot = items[cur + rank];
                const float4 o = ldS(&p.ray_o[slot]), d = ldS(&p.ray_d[slot]);
                walk4Start(w, xyz(o), xyz(d), o.w, d.w);
                active = true;
            }
            cur += min(idle, end - cur);
        }
        if (__ballot(active) == 0) break;  // the segment is done (a refill above found no ray left)
        bool fin = false;
        if (active) fin = walk4Round(w, sc.nodes, sc.tris, stk);
        int cls = -1;
        if (fin) {
            const bool h = w.hitTri != 0xFFFFFFFFu;
            float4 hr = make_float4(h ? w.tmax : 0.0f, __uint_as_float(h ? w.hitTri : 0xFFFFFFFFu), w.hu, w.hv);
            if (first) first[slot] = hr;
            if (ENV && !h) {
                const f3 e = envEscapeRadiance(g, sc, p, slot, w.d);
                hr = make_float4(e.x, hr.y, e.y, e.z);
            }
            stS(&p.hit[slot], hr);
            cls = h ? (int)sc.tclass[w.hitTri] : PG_NUM_CLASSES;
            active = false;
        }
        classAppend(cls, slot, cqs, s);
    }
}

// traceRows with two rays per lane (PG_TRACE_PAIR, A/B): a block's grid-stride step takes 2 x TRACE_BLOCK rows
// of its shard, lane t rows base + t and base + TRACE_BLOCK + t, and walks both at once (pg_trace.h walk4Pair),
// so each lane has two rays' node fetches in flight; both class appends follow in row order.  The second
// walk's stack is a second LDS column block and a second band of the overflow ring (kPairRing rows on).
#ifndef PG_TRACE_PAIR
#define PG_TRACE_PAIR 0
#endif
constexpr uint32_t kPairRing = PG_QSTACK_DEPTH - LDS_STACK;
template <bool ENV>
__device__ __forceinline__ void finishWalk(const GParams &g, const SceneDev &sc, const PathDev &p, const Walk4 &w,
                                           uint32_t slot, float4 *first, int &cls) {
    const bool h = w.hitTri != 0xFFFFFFFFu;
    float4 hr = make_float4(h ? w.tmax : 0.0f, __uint_as_float(h ? w.hitTri : 0xFFFFFFFFu), w.hu, w.hv);
    if (first) first[slot] = hr;
    if (ENV && !h) {
        const f3 e = envEscapeRadiance(g, sc, p, slot, w.d);
        hr = make_float4(e.x, hr.y, e.y, e.z);
    }
    stS(&p.hit[slot], hr);
    cls = h ? (int)sc.tclass[w.hitTri] : PG_NUM_CLASSES;
}
template <bool ENV>
__device__ __forceinline__ void traceRowsPair(const GParams &g, const SceneDev &sc, const PathDev &p, const Queue &q,
                                              const ClassQueues &cqs, float4 *first, uint32_t bid, uint32_t nblk,
                                              const TStack &sa, const TStack &sb) {
    const uint32_t s = bid & (PG_QSHARDS - 1);
    const uint32_t n = q.counts[s];
    const uint32_t *items = q.items + (size_t)s * q.stride;
    for (uint32_t base = (bid / PG_QSHARDS) * 2 * TRACE_BLOCK; base < n; base += nblk / PG_QSHARDS * 2 * TRACE_BLOCK) {
        const uint32_t ia = base + threadIdx.x, ib = ia + TRACE_BLOCK;
        uint32_t slotA = 0, slotB = 0;
        Walk4 a, b;
        walk4Idle(a);
        walk4Idle(b);
        if (ia < n) {
            slotA = items[ia];
            const float4 o = ldS(&p.ray_o[slotA]), d = ldS(&p.ray_d[slotA]);
            walk4Start(a, xyz(o), xyz(d), o.w, d.w);
        }
        if (ib < n) {
            slotB = items[ib];
            const float4 o = ldS(&p.ray_o[slotB]), d = ldS(&p.ray_d[slotB]);
            walk4Start(b, xyz(o), xyz(d), o.w, d.w);
        }
        walk4Pair(a, b, sc.nodes, sc.tris, sa, sb);
        int ca = -1, cb = -1;
        if (ia < n) finishWalk<ENV>(g, sc, p, a, slotA, first, ca);
        if (ib < n) finishWalk<ENV>(g, sc, p, b, slotB, first, cb);
        classAppend(ca, slotA, cqs, s);
        classAppend(cb, slotB, cqs, s);
    }
}

template <bool ENV>
__global__ __launch_bounds__(TRACE_BLOCK) void k_trace(GParams g, SceneDev sc, PathDev p, Queue q, ClassQueues cqs,
                                                       float4 *first) {
    __shared__ uint32_t stack[LDS_STACK * TRACE_BLOCK];
    // the BVH's top levels (breadth first, pg_layout.h PG_BVH_TOP_NODES), staged in LDS once per block
    __shared__ float4 top[(PG_TRACE_LDS_TOP ? PG_TOP_TILE_F4 : 1)];
    const int ntop = PG_TRACE_LDS_TOP ? (int)sc.top_nodes : 0;
    if (PG_TRACE_LDS_TOP) {
        for (uint32_t k = threadIdx.x; k < (uint32_t)ntop * PG_TOP_NODE_F4; k += TRACE_BLOCK) top[k] = sc.nodes[k];
        __syncthreads();
    }
    traceRows<ENV, PG_TRACE_LDS_TOP != 0>(g, sc, p, q, cqs, first, blockIdx.x, gridDim.x, threadStack(stack, p.stack_ovf),
                                          top, ntop);
}

// shadow-ray mint at the shading point o (the extension ray's origin): Epsilon * max |o_i|
// (progressive_path.cpp via DirectSamplingRecord / Scene::sampleEmitterDirect's shadow ray)
__device__ __forceinline__ float shadowTmin(float4 o) {
    return kEpsilon * fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
}

// any hit for queued shadow rays; unoccluded -> add the NEE contribution to L (and to the
// training vertex's radiance snapshot, so its record excludes light arriving from elsewhere)
__device__ __forceinline__ void shadowRows(const SceneDev &sc, const PathDev &p, const Queue &q, uint32_t bid,
                                           uint32_t nblk, const WStack &stk) {
    const uint32_t s = bid & (PG_QSHARDS - 1);
    const uint32_t n = q.counts[s];
    const uint32_t *items = q.items + (size_t)s * q.stride;
    for (uint32_t i = (bid / PG_QSHARDS) * TRACE_BLOCK + threadIdx.x; i < n; i += nblk / PG_QSHARDS * TRACE_BLOCK) {
        uint32_t slot = items[i];
        // the shadow ray starts at the shading point, which is also the extension ray's origin
        float4 o = ldS(&p.ray_o[slot]), d = ldS(&p.sh_d[slot]);
        if (!occluded(sc, xyz(o), xyz(d), shadowTmin(o), d.w, stk)) {
            float4 c = ldS(&p.sh_c[slot]);
            float4 L = ldS(&p.rad[slot]);
            stS(&p.rad[slot], make_float4(L.x + c.x, L.y + c.y, L.z + c.z, L.w));
            uint32_t vi = __float_as_uint(c.w);
            if (vi != 0xFFFFFFFFu) {
                float4 *vl = p.vtx + ((size_t)vi * p.vtxP + slot) * PG_VTX_F4 + 2;
                float4 a = *vl;
                *vl = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w);
            }
        }
    }
}

__global__ __launch_bounds__(TRACE_BLOCK) void k_shadow(SceneDev sc, PathDev p, Queue q) {
    __shared__ uint32_t stack[2 * WIDE_LDS_STACK * TRACE_BLOCK];
    shadowRows(sc, p, q, blockIdx.x, gridDim.x, threadWideStack(stack, p.stack_ovf));
}

// a bounce's shadow rays and the next closest hits in one launch: blocks [0, shadow_blocks) run
// k_shadow's rows, the rest k_trace's (an escaped path's environment radiance goes to its hit
// record, not to L, so it cannot race with the same path's NEE add).  Both parts are grid-stride loops over their shards; the
// overflow ring holds two launches' worth of threads (2 x pg_stack_overflow_words(0)).
static_assert(2 * WIDE_LDS_STACK >= LDS_STACK, "k_rays / k_trace_rays share one LDS stack array");
#ifndef PG_RAYS_TRACE_FIRST
#define PG_RAYS_TRACE_FIRST 1
#endif
template <bool ENV>
#ifndef PG_RAYS_WAVES
#define PG_RAYS_WAVES 8
#endif
__global__ __launch_bounds__(TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(PG_RAYS_WAVES))) void k_rays(GParams g, SceneDev sc, PathDev p, Queue q, ClassQueues cqs,
                                                      Queue shq, uint32_t shadow_blocks) {
    // >= LDS_STACK words per thread (twice that for the paired walks)
    __shared__ uint32_t stack[(PG_TRACE_PAIR ? 2 : 1) * 2 * WIDE_LDS_STACK * TRACE_BLOCK];
#if PG_RAYS_TRACE_FIRST  // the costlier closest-hit blocks dispatched first (profiles/r03zg_rays_order_ab)
    const uint32_t trace_blocks = gridDim.x - shadow_blocks;
    if (blockIdx.x >= trace_blocks) {
        shadowRows(sc, p, shq, blockIdx.x - trace_blocks, shadow_blocks, threadWideStack(stack, p.stack_ovf));
    } else {
        // the 4-wide BVH's breadth-first top levels in LDS (PG_RAYS_LDS_TOP, A/B; round 5 re-measure of the
        // round-2 tile on the 64-B nodes)
        __shared__ float4 top[PG_RAYS_LDS_TOP ? PG_TOP_TILE_F4 : 1];
        const int ntop = PG_RAYS_LDS_TOP ? (int)sc.top_nodes : 0;
        if (PG_RAYS_LDS_TOP) {
            for (uint32_t k = threadIdx.x; k < (uint32_t)ntop * PG_TOP_NODE_F4; k += TRACE_BLOCK) top[k] = sc.nodes[k];
            __syncthreads();
        }
        const TStack sa = threadStack(stack, p.stack_ovf);
        if (PG_TRACE_PAIR && !PG_RAYS_LDS_TOP && !PG_CLOSEST_WIDE && PG_BVH4 && PG_QNODE_QUANT)
            traceRowsPair<ENV>(g, sc, p, q, cqs, nullptr, blockIdx.x, trace_blocks, sa,
                               TStack{sa.lds + LDS_STACK * TRACE_BLOCK, sa.ovf + (size_t)kPairRing * sa.ostride, sa.ostride});
        else if (PG_TRACE_PERSIST && !PG_RAYS_LDS_TOP && !PG_CLOSEST_WIDE && PG_BVH4 && PG_QNODE_QUANT)
            traceRowsPersist<ENV>(g, sc, p, q, cqs, nullptr, blockIdx.x, trace_blocks, sa);
        else
            traceRows<ENV, PG_RAYS_LDS_TOP != 0, PG_CLOSEST_WIDE != 0>(g, sc, p, q, cqs, nullptr, blockIdx.x, trace_blocks,
                                                 sa, top, ntop);
    }
#else
    if (blockIdx.x < shadow_blocks)
        shadowRows(sc, p, shq, blockIdx.x, shadow_blocks, threadWideStack(stack, p.stack_ovf));
    else
        traceRows<ENV, false>(g, sc, p, q, cqs, nullptr, blockIdx.x - shadow_blocks, gridDim.x - shadow_blocks,
                                threadStack(stack, p.stack_ovf), nullptr, 0);
#endif
}

// ray order key of a new extension ray (PG_RAY_SORT): direction octant, then the Morton code of the
// origin's cell in an 8^3 grid over the SD-tree cube (the scene bounds)
__device__ __forceinline__ uint32_t rayOrderKey(const SDDev &sd, f3 o, f3 d) {
    const float inv = 8.0f / sd.extent;
    const int cx = min(max((int)((o.x - sd.lo[0]) * inv), 0), 7);
    const int cy = min(max((int)((o.y - sd.lo[1]) * inv), 0), 7);
    const int cz = min(max((int)((o.z - sd.lo[2]) * inv), 0), 7);
    uint32_t m = 0;
    for (int b = 0; b < 3; ++b)
        m |= (((cx >> b) & 1) << (3 * b)) | (((cy >> b) & 1) << (3 * b + 1)) | (((cz >> b) & 1) << (3 * b + 2));
    const uint32_t oct = (d.x < 0 ? 1u : 0u) | (d.y < 0 ? 2u : 0u) | (d.z < 0 ? 4u : 0u);
    return (oct << 9) | m;
}

// PG_SD_PREFETCH (round 6): shadeOne issues the guided lookup's jump-grid and leaf-record loads from the ray's
// o + t d before the hit triangle and material resolve (the exact position decides; identical results)
#ifndef PG_SD_PREFETCH
#define PG_SD_PREFETCH 0
#endif
// PG_MAT_UNIFORM (round 6, A/B): shadeOne loads its material record once per distinct material of the wave, at a
// wave-uniform address (readfirstlane waterfall), instead of as a per-lane gather
#ifndef PG_MAT_UNIFORM
#define PG_MAT_UNIFORM 0
#endif
// one bounce of Li for every queued path (progressive_path.cpp:149-306 + guiding)
// MODEL >= 0 compiles only that BSDF model's code (material-class queues filled by k_trace);
// CAN_GUIDE = false drops the SD-tree code for classes that are never guided (delta lobes).
// ENV compiles in environment-emitter sampling for NEE (kept out of the other instantiations: it
// costs 4-8 VGPRs).
// one bounce of Li for the path in `slot` (progressive_path.cpp:149-306 + guiding): reads its state,
// writes the next one; alive = an extension ray was written, shadow = a shadow ray was written (sh_*)
// mats: the material table (global memory, or a block's LDS copy); wantKey: compute rkey (PG_RAY_SORT)
// the per-bounce half of a path's info record (depth | flags, vertex count): pixel and sample never
// change after k_camera, so an 8-B store replaces the 16-B rewrite
__device__ __forceinline__ void stPinfoZW(uint4 *p, uint32_t z, uint32_t w) {
    reinterpret_cast<uint2 *>(p)[1] = make_uint2(z, w);
}

#if PG_TRAV_STATS
extern "C" int pg_debug_trav_stats(unsigned long long *out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pgTravStats), 8 * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(pgTravStats), z, 8 * 8) != hipSuccess) return -1;
    }
    return 0;
}
#endif
// Debug build only (PG_WATCH=1, make watch -> build/libpgamd_watch.so; tools/diverge_c3.py): shadeOne
// logs every vertex of one (pixel, sample) path, the same record the oracle's Li writes (oracle.cpp
// g_vtxLog): depth, original triangle, p, T, alpha, guided, mode, woPdf, weight, wo, L, NEE
// contribution and pdfs, RR q / outcome, alive, shadow, b0, b1.  The product build has none of it.
#ifndef PG_WATCH
#define PG_WATCH 0
#endif
#if PG_WATCH
#define PG_WATCH_F 32
#define PG_WATCH_MAX 256
__device__ uint32_t pgWatch[3];  // pixel, sample, records written
__device__ float pgWatchLog[PG_WATCH_MAX * PG_WATCH_F];
extern "C" int pg_debug_watch(uint32_t pixel, uint32_t sample) {
    const uint32_t w[3] = {pixel, sample, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(pgWatch), w, sizeof(w)) == hipSuccess ? 0 : -1;
}
extern "C" int pg_debug_watch_read(float *out, uint32_t max, uint32_t *n) {
    uint32_t w[3];
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(w, HIP_SYMBOL(pgWatch), sizeof(w)) != hipSuccess) return -1;
    *n = w[2] < PG_WATCH_MAX ? w[2] : PG_WATCH_MAX;
    const uint32_t k = *n < max ? *n : max;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pgWatchLog), (size_t)k * PG_WATCH_F * 4) == hipSuccess ? 0 : -1;
}
#define WSET(i, v) (wr[i] = (float)(v))
#define WSET3(i, v) (wr[i] = (v).x, wr[(i) + 1] = (v).y, wr[(i) + 2] = (v).z)
#else
#define WSET(i, v) ((void)0)
#define WSET3(i, v) ((void)0)
#endif

template <int MODEL, bool CAN_GUIDE, bool ENV>
__device__ __forceinline__ void shadeOne(const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p,
                                         uint32_t slot, const GMat *mats, bool wantKey, bool &alive, bool &shadow,
                                         uint32_t &rkey) {
    bool dirtyL = false;
    f3 L = mk1(0.f);
#if PG_WATCH
    float wr[PG_WATCH_F];
    for (int i = 0; i < PG_WATCH_F; ++i) wr[i] = -1.0f;
    bool watched = false;
#endif
    do {
        uint4 pi = ldS(&p.pinfo[slot]);
        const uint32_t pix = pi.x, sample = pi.y;
#if PG_WATCH
        watched = pix == pgWatch[0] && sample == pgWatch[1];
#endif
        uint32_t depth = pi.z & 0xFFFFu, flags = pi.z >> 16, nv = pi.w;
        float4 hv = ldS(&p.hit[slot]);
        // a camera ray's state is implied (k_camera stores neither throughput nor prev)
        float4 T4 = depth == 1 ? make_float4(1.f, 1.f, 1.f, 1.f) : ldS(&p.thr[slot]);
        float4 L4 = depth == 1 ? make_float4(0.f, 0.f, 0.f, 0.f) : ldS(&p.rad[slot]);
        f3 T = xyz(T4);
        L = xyz(L4);
        float eta = T4.w;
        uint32_t tri = __float_as_uint(hv.y);
        if (tri == 0xFFFFFFFFu) break;  // escaped: no environment emitter
        const uint32_t key = rngKey(pix, g.seed);
        const float4 rd4 = ldS(&p.ray_d[slot]);
        f3 rd = xyz(rd4);
#if PG_SD_PREFETCH
        // the guided lookup's jump-grid cell and leaf record, fetched from the ray's o + t d while the triangle and
        // material gathers resolve; used only when the exact (barycentric) position lands in the same cell
        uint32_t jCell = 0xFFFFFFFFu, jSpec = 0;
        uint4 metaSpec = make_uint4(0, 0, 0, 0);
        if (CAN_GUIDE && g.guiding && sd.built) {
            const float4 ro = ldS(&p.ray_o[slot]);
            const SDView sv0 = sdv(sd);
            jCell = sdJumpCell(sv0, mk(ro.x + hv.x * rd.x, ro.y + hv.x * rd.y, ro.z + hv.x * rd.z));
            jSpec = sd.jump[jCell];
        }
#endif
        Hit h;
        fetchHit(sc, tri, hv.z, hv.w, rd, h);
#if PG_SD_PREFETCH
        // the leaf's record behind the triangle loads (index 0, a valid record, where the cell holds a node)
        if (CAN_GUIDE && g.guiding && sd.built) metaSpec = sd.meta[(jSpec & 0x80000000u) ? (jSpec & 0x7FFFFFFFu) : 0u];
#endif
        WSET(0, depth);
        WSET(1, __float_as_uint(sc.tshade[(size_t)PG_TRI_SHADE_STRIDE * tri + 2].w));
        WSET3(2, h.p);
        f3 Le = mk1(0.f);
        if (h.emitter >= 0 && dot(h.shN, -rd) > 0) {  // AreaLight::eval (area.cpp)
            const GEmitter &em = sc.ems[h.emitter];
            Le = mk(em.radiance[0], em.radiance[1], em.radiance[2]);
        }
        // ---- finish the previous bounce: emitter hit by the sampled direction (MIS), then RR
        if (depth > 1) {
            if (h.emitter >= 0) {
                float4 pv = ldS(&p.prev[slot]);
                float lumPdf = 0.0f;
                if (g.use_nee && !(flags & PF_PREV_DELTA)) {
                    f3 prevRefN = xyz(pv);
                    if (dot(rd, prevRefN) >= 0 && dot(rd, h.shN) < 0) {
                        const GEmitter &em = sc.ems[h.emitter];
                        lumPdf = em.inv_area * (hv.x * hv.x) / absDot(rd, h.shN) * (1.0f / (float)g.num_emitters);
                    }
                }
                float w = g.use_nee ? miWeight(pv.w, lumPdf) : 1.0f;
                L = L + T * Le * w;
                dirtyL = true;
            }
            if (depth - 1 >= (uint32_t)g.rr_depth) {
                float q = fminf(maxc(T) * eta * eta, 0.95f);
                WSET(26, q);
                WSET3(18, L);
                WSET3(5, T);
                WSET(27, 0);
                if (rng1(key, sample, dimOf(depth - 1, SLOT_RR)) >= q) break;
                WSET(27, 1);
                T = T / q;
            }
        }
        WSET3(5, T);
        if (depth > g.depth_cap) break;
#if PG_MAT_UNIFORM
        // one uniform (scalar-cache) load per distinct material of the wave instead of eight 16-B gathers per lane
        GMat M;
        for (;;) {
            const uint32_t u = __builtin_amdgcn_readfirstlane(h.mat);
            if (h.mat == u) {
                M = mats[u];
                break;
            }
        }
#else
        const GMat M = mats[h.mat];
#endif
        if ((flags & PF_EMITTED_QUERY) && h.emitter >= 0 && (!g.hide_emitters || (flags & PF_SCATTERED))) {
            L = L + T * Le;
            dirtyL = true;
        }
        if ((g.max_depth > 0 && (int)depth >= g.max_depth) ||
            (g.strict_normals && dot(rd, h.geoN) * h.wi.z >= 0))
            break;
        WSET3(18, L);
        const f3 refN = (M.type & (ETransmission | EBackSide)) == 0 ? h.shN : mk1(0.f);
        // glossy prior (pg_config.glossy_prior): r = BSDF::getGlossySamplingRate; r = 1 is not guided
        const float gRate = (CAN_GUIDE && g.glossy_prior) ? glossyRate<MODEL>(M, h.wi.z) : 0.0f;
        const bool guide = CAN_GUIDE && g.guiding && sd.built && (M.type & ESmooth) && !(M.type & EDelta) && gRate < 1.0f;
        const SDView sv = sdv(sd);
        uint4 meta = make_uint4(0, 0, 0, 0);
#if PG_SD_PREFETCH
        if (guide) {
            if ((jSpec & 0x80000000u) && sdJumpCell(sv, h.p) == jCell) meta = metaSpec;  // the same leaf
            else meta = sd.meta[sdLookup(sv, h.p)];
        }
#else
        if (guide) meta = sd.meta[sdLookup(sv, h.p)];
#endif
        // one-sample-MIS BSDF fraction of this vertex (pg_config.bsdf_fraction_bound; oracle guideFraction):
        // PG_FRACTION_LEARNED reads the leaf's learned fraction (meta.z; 0 = not learned yet)
        const float leafAlpha = __uint_as_float(meta.z);
        float alpha = g.fraction_bound == PG_FRACTION_LEARNED ? (leafAlpha > 0 ? leafAlpha : g.bsdf_fraction)
                                                               : guideFraction(g.fraction_bound, g.bsdf_fraction,
                                                                               M.wbound, maxc(T));
        if (gRate > 0.0f) {
#pragma clang fp contract(off)
            alpha = gRate + (1.0f - gRate) * alpha;
        }
        float pgWo = -1.0f;  // p_guide of the sampled direction at a guided vertex (training record)

        // ---- NEE (progressive_path.cpp:193-219); the shadow ray is deferred to k_shadow.  With
        // guiding, the D-tree pdf of the light direction is resolved below, in one lockstep walk
        // with the direction-sampling descent (sdDual).
        f3 neeC = mk1(0.f), neeD = mk1(0.f), neeV = mk1(0.f);
        float neeDist = 0, neeEmPdf = 0, neeBp = 0;
        bool neePending = false;
        if (g.use_nee && (M.type & ESmooth)) {
            float s0, s1;
            rng2(key, sample, dimOf(depth, SLOT_NEE), s0, s1);
            float emPdf;
            f3 value = sampleEmitter<ENV>(g, sc, h.p, refN, s0, s1, neeD, neeDist, emPdf);
            if (!isZero(value)) {
                f3 woL = h.sh.toLocal(neeD);
                f3 bsdfVal = bsdfEval<MODEL>(M, h.wi, woL);
                if (!isZero(bsdfVal) && (!g.strict_normals || dot(h.geoN, neeD) * woL.z > 0)) {
                    neeBp = bsdfPdf<MODEL>(M, h.wi, woL);
                    neeEmPdf = emPdf;
                    neeV = T * value * bsdfVal;
                    shadow = true;
                    if (guide) neePending = true;
                    else neeC = neeV * miWeight(emPdf, neeBp);
                }
            }
        }

        // ---- direction sampling: BSDF, or one-sample MIS between BSDF and the D-tree
        BS bs;
        f3 weight;
        float woPdf;
        bool ok = true;
        {
            float b0, b1;
            rng2(key, sample, dimOf(depth, SLOT_BSDF), b0, b1);
            float b2 = rng1(key, sample, dimOf(depth, SLOT_COMP));
            WSET(30, b0);
            WSET(31, b1);
            int mode = 0;  // D-tree walk of the sampled direction: 0 none, 1 pdf (BSDF sample), 2 sample
            float bu = 0, bw = 0;
            if (!guide) {
                weight = bsdfSample<MODEL>(M, h.wi, b0, b1, b2, bs);
                woPdf = bs.pdf;
            } else if (rng1(key, sample, dimOf(depth, SLOT_GUIDE_CHOICE)) < alpha) {
                weight = bsdfSample<MODEL>(M, h.wi, b0, b1, b2, bs);
                if (isZero(weight)) {
                    ok = false;
                } else {
                    mode = 1;
                    dirToCanonical(h.sh.toWorld(bs.wo), bu, bw);
                }
            } else {
                mode = 2;
                rng2(key, sample, dimOf(depth, SLOT_GUIDE), bu, bw);
            }
            if (guide) {
                float au = 0, aw = 0, aPdf, dPdf, cu, cv;
                if (neePending) dirToCanonical(neeD, au, aw);
                sdDual(sv, meta, neePending, au, aw, aPdf, mode != 0, mode == 2, bu, bw, cu, cv, dPdf);
                if (neePending) neeC = neeV * miWeight(neeEmPdf, alpha * neeBp + (1 - alpha) * aPdf);
                pgWo = dPdf;
                if (mode == 1) {
                    woPdf = alpha * bs.pdf + (1 - alpha) * dPdf;
                    weight = weight * (bs.pdf / woPdf);
                } else if (mode == 2) {
                    f3 dW = canonicalToDir(cu, cv);
                    f3 woL = h.sh.toLocal(dW);
                    f3 f = bsdfEval<MODEL>(M, h.wi, woL);
                    float bp = bsdfPdf<MODEL>(M, h.wi, woL);
                    woPdf = alpha * bp + (1 - alpha) * dPdf;
                    if (!(woPdf > 0) || isZero(f)) {
                        ok = false;
                    } else {
                        weight = f / woPdf;
                        bs.wo = woL;
                        bs.pdf = bp;
                        bool refl = h.wi.z * woL.z > 0;
                        bs.type = refl ? ((M.type & EDiffuseReflection) ? EDiffuseReflection : EGlossyReflection)
                                       : EGlossyTransmission;
                        bs.eta = refl ? 1.0f : (h.wi.z > 0 ? M.eta : M.invEta);
                    }
                }
            }
            WSET(10, mode + (ok ? 0 : 10));
        }
        uint32_t vtxIndex = 0xFFFFFFFFu;
        WSET(8, alpha);
        WSET(9, guide ? 1 : 0);
        WSET(11, woPdf);
        WSET3(12, weight);
        WSET3(15, h.sh.toWorld(bs.wo));
        WSET3(21, neeC);
        WSET(24, neeEmPdf);
        WSET(25, neeBp);
        if (ok && !isZero(weight)) {
            if (bs.type != ENull) flags |= PF_SCATTERED;
            f3 wo = h.sh.toWorld(bs.wo);
            if (!(g.strict_normals && dot(h.geoN, wo) * bs.wo.z <= 0)) {
                f3 Tn = T * weight;
                // training vertex: (x, wo, woPdf, T after this bounce, L snapshot)
                if (g.record && !(bs.type & EDelta) && nv < (uint32_t)g.max_vertices) {
                    float cu, cv;
                    dirToCanonical(wo, cu, cv);
                    float4 *vb = p.vtx + ((size_t)nv * p.vtxP + slot) * PG_VTX_F4;
                    stS(vb + 0, f4(h.p, woPdf));
                    stS(vb + 1, f4(Tn, __uint_as_float(packCanonical(cu, cv))));
                    stS(vb + 2, f4(L, 0.0f));
                    // learned-fraction statistics only from vertices whose fraction is the leaf's (r = 0)
                    stS(vb + 3, f4(T, guide && gRate == 0.0f ? pgWo : -1.0f));
                    vtxIndex = nv;
                    nv++;
                }
                float tmin = kEpsilon * fmaxf(fmaxf(fmaxf(fabsf(h.p.x), fabsf(h.p.y)), fabsf(h.p.z)), kEpsilon);
                stS(&p.ray_o[slot], f4(h.p, tmin));
                stS(&p.ray_d[slot], f4(wo, __int_as_float(0x7f800000)));
                stS(&p.thr[slot], f4(Tn, eta * bs.eta));
                stS(&p.prev[slot], f4(refN, woPdf));
                flags = (flags & ~(PF_EMITTED_QUERY | PF_PREV_DELTA)) | ((bs.type & EDelta) ? PF_PREV_DELTA : 0u);
                stPinfoZW(&p.pinfo[slot], (depth + 1) | (flags << 16), nv);
                alive = true;
                if (wantKey) rkey = rayOrderKey(sd, h.p, wo);
            }
        }
        if (shadow) {  // origin: ray_o (the extension ray's, written above when the path goes on)
            if (!alive) stS(&p.ray_o[slot], f4(h.p, 0.0f));
            stS(&p.sh_d[slot], f4(neeD, neeDist * (1 - kShadowEpsilon)));
            stS(&p.sh_c[slot], f4(neeC, __uint_as_float(vtxIndex)));
        }
        if (!alive && nv != pi.w) stPinfoZW(&p.pinfo[slot], pi.z, nv);
    } while (false);
    if (dirtyL) stS(&p.rad[slot], f4(L, 0.0f));
#if PG_WATCH
    if (watched) {
        wr[28] = alive ? 1.0f : 0.0f;
        wr[29] = shadow ? 1.0f : 0.0f;
        const uint32_t k = atomicAdd(&pgWatch[2], 1u);
        if (k < PG_WATCH_MAX)
            for (int i = 0; i < PG_WATCH_F; ++i) pgWatchLog[k * PG_WATCH_F + i] = wr[i];
    }
#endif
}

template <int MODEL, bool CAN_GUIDE, bool ENV>
__device__ __forceinline__ void shadeBlock(const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p,
                                           const Queue &in, const Queue &out, const Queue &shq, uint32_t bid) {
    // one item per thread (a grid-stride loop here cost ~45 VGPRs of hoisted invariants): block b
    // takes row b / PG_QSHARDS of shard b % PG_QSHARDS; rows past the shard's count exit at once
    const uint32_t s = bid & (PG_QSHARDS - 1);
    const uint32_t n = in.counts[s];
    {
    const uint32_t base = (bid / PG_QSHARDS) * SHADE_BLOCK;
    if (base >= n) return;
    const uint32_t i = base + threadIdx.x;
    bool alive = false, shadow = false;
    uint32_t slot = 0, rkey = 0;
    if (i < n) slot = in.items[(size_t)s * in.stride + i];
    // the material table, staged in LDS once per block (the material read sits on the dependent chain
    // hit -> triangle -> material of every shaded vertex); larger tables stay in global memory
    __shared__ float4 smat[(SHADE_LDS_MATS > 0 ? SHADE_LDS_MATS : 1) * (sizeof(GMat) / 16)];
    const bool ldsMats = SHADE_LDS_MATS > 0 && g.num_materials <= SHADE_LDS_MATS;
    if (ldsMats) {
        const float4 *src = reinterpret_cast<const float4 *>(sc.mats);
        for (uint32_t k = threadIdx.x; k < g.num_materials * (uint32_t)(sizeof(GMat) / 16); k += SHADE_BLOCK) smat[k] = src[k];
        __syncthreads();
    }
    if (i < n)
        shadeOne<MODEL, CAN_GUIDE, ENV>(g, sc, sd, p, slot, ldsMats ? reinterpret_cast<const GMat *>(smat) : sc.mats,
                                        out.keys != nullptr, alive, shadow, rkey);
    if (out.keys)
        waveAppendKey(alive, slot, (uint16_t)rkey, out.items + (size_t)s * out.stride, out.keys + (size_t)s * out.stride,
                      out.counts + s);
    else
        waveAppend(alive, slot, out.items + (size_t)s * out.stride, out.counts + s);
    waveAppend(shadow, slot, shq.items + (size_t)s * shq.stride, shq.counts + s);
    }
}

template <int MODEL, bool CAN_GUIDE, bool ENV>
__global__ __launch_bounds__(SHADE_BLOCK) void k_shade(GParams g, SceneDev sc, SDDev sd, PathDev p, Queue in,
                                                       Queue out, Queue shq) {
    shadeBlock<MODEL, CAN_GUIDE, ENV>(g, sc, sd, p, in, out, shq, blockIdx.x);
}

// every material class of a bounce in one launch (no environment emitter): blocks
// [end[c-1], end[c]) shade class c.  All class bodies fit 128 VGPRs, so the shared register budget
// keeps the 4 waves/SIMD each class kernel has alone.
struct ShadeRanges {
    uint32_t end[PG_NUM_CLASSES];
};
#ifndef PG_SHADE_WAVES
#define PG_SHADE_WAVES 4
#endif
__global__ __launch_bounds__(SHADE_BLOCK) __attribute__((amdgpu_waves_per_eu(PG_SHADE_WAVES))) void k_shade_all(
    GParams g, SceneDev sc, SDDev sd, PathDev p, ClassQueues in, Queue out, Queue shq, ShadeRanges r) {
    static_assert(PG_NUM_CLASSES == 6, "class ranges");
    const uint32_t b = blockIdx.x;
    if (b < r.end[0]) shadeBlock<PG_BSDF_DIFFUSE, true, false>(g, sc, sd, p, in.q[0], out, shq, b);
    else if (b < r.end[1]) shadeBlock<PG_BSDF_ROUGHCONDUCTOR, true, false>(g, sc, sd, p, in.q[1], out, shq, b - r.end[0]);
    else if (b < r.end[2]) shadeBlock<PG_BSDF_ROUGHDIELECTRIC, true, false>(g, sc, sd, p, in.q[2], out, shq, b - r.end[1]);
    else if (b < r.end[3]) shadeBlock<PG_BSDF_PLASTIC, false, false>(g, sc, sd, p, in.q[3], out, shq, b - r.end[2]);
    else if (b < r.end[4]) shadeBlock<PG_BSDF_ROUGHPLASTIC, true, false>(g, sc, sd, p, in.q[4], out, shq, b - r.end[3]);
    else shadeBlock<-1, false, false>(g, sc, sd, p, in.q[5], out, shq, b - r.end[4]);
}

// ---- counting sort of a queue's shards by ray order key (PG_RAY_SORT): the next closest-hit launch
// then traces each shard's rays grouped by direction octant and origin cell.  Within a key the order
// follows LDS/global atomics (nondeterministic), which is harmless: every path is a pure function of
// (pixel, sample), whatever the order its bounces are traced in.
#define RSORT_TILE 4096  // queue entries per block (256 threads x 16)
template <uint32_t BINS>
__global__ __launch_bounds__(256) void k_rsort_hist(Queue q, uint32_t *hist) {
    __shared__ uint32_t h[BINS];
    const uint32_t s = blockIdx.x & (PG_QSHARDS - 1), tile = blockIdx.x / PG_QSHARDS;
    const uint32_t n = q.counts[s], b0 = tile * RSORT_TILE;
    if (b0 >= n) return;
    for (uint32_t k = threadIdx.x; k < BINS; k += 256) h[k] = 0;
    __syncthreads();
    const uint16_t *keys = q.keys + (size_t)s * q.stride;
    const uint32_t e = min(n, b0 + RSORT_TILE);
    for (uint32_t i = b0 + threadIdx.x; i < e; i += 256) atomicAdd(&h[keys[i]], 1u);
    __syncthreads();
    uint32_t *g = hist + (size_t)s * BINS;
    for (uint32_t k = threadIdx.x; k < BINS; k += 256)
        if (h[k]) atomicAdd(&g[k], h[k]);
}
// exclusive scan of every shard's histogram in place (one block per shard)
template <uint32_t BINS>
__global__ __launch_bounds__(256) void k_rsort_scan(uint32_t *hist) {
    __shared__ uint32_t part[256];
    uint32_t *g = hist + (size_t)blockIdx.x * BINS;
    constexpr int PER = BINS / 256;
    uint32_t v[PER], sum = 0;
    for (int j = 0; j < PER; ++j) {
        v[j] = g[threadIdx.x * PER + j];
        sum += v[j];
    }
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {  // Hillis-Steele inclusive scan of the thread sums
        const uint32_t x = threadIdx.x >= (uint32_t)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (int j = 0; j < PER; ++j) {
        g[threadIdx.x * PER + j] = run;
        run += v[j];
    }
}
template <uint32_t BINS>
__global__ __launch_bounds__(256) void k_rsort_scatter(Queue q, uint32_t *hist, uint32_t *sorted) {
    __shared__ uint32_t cnt[BINS];
    const uint32_t s = blockIdx.x & (PG_QSHARDS - 1), tile = blockIdx.x / PG_QSHARDS;
    const uint32_t n = q.counts[s], b0 = tile * RSORT_TILE;
    if (b0 >= n) return;
    for (uint32_t k = threadIdx.x; k < BINS; k += 256) cnt[k] = 0;
    __syncthreads();
    const uint16_t *keys = q.keys + (size_t)s * q.stride;
    const uint32_t *items = q.items + (size_t)s * q.stride;
    const uint32_t e = min(n, b0 + RSORT_TILE);
    constexpr int PER = RSORT_TILE / 256;
    uint32_t rank[PER], key[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {  // fixed trip count: the per-thread arrays stay in registers
        const uint32_t i = b0 + threadIdx.x + 256u * j;
        key[j] = i < e ? keys[i] : 0u;
        rank[j] = i < e ? atomicAdd(&cnt[key[j]], 1u) : 0u;
    }
    __syncthreads();
    uint32_t *g = hist + (size_t)s * BINS;
    for (uint32_t k = threadIdx.x; k < BINS; k += 256)  // this tile's range of every key
        if (cnt[k]) cnt[k] = atomicAdd(&g[k], cnt[k]);
    __syncthreads();
    uint32_t *out = sorted + (size_t)s * q.stride;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t i = b0 + threadIdx.x + 256u * j;
        if (i < e) out[cnt[key[j]] + rank[j]] = items[i];
    }
}

// ---- the tail of a chunk: once few paths are alive, the host stops the per-bounce launches and
// count readbacks and one launch finishes every remaining path, each thread looping shade (the
// class's specialised body) -> shadow ray -> closest hit until its path ends.  Every step is the
// wavefront's own code on the path's own state and random numbers, in the same order (a path's NEE
// is added before its next vertex is shaded), so films, records and trees are bit-identical with
// the bounce-by-bounce loop.  Input: the queue of the bounce just traced (hits already in p.hit).
// stats: [0] traced segments, [1] escaped segments, [2] shadow rays (u64, device atomics).
template <bool ENV>
__device__ __forceinline__ void tailShade(const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p,
                                          uint32_t slot, uint32_t tri, bool &alive, bool &shadow) {
    uint32_t rk = 0;
    switch (sc.tclass[tri]) {
        case PG_CLASS_DIFFUSE: shadeOne<PG_BSDF_DIFFUSE, true, ENV>(g, sc, sd, p, slot, sc.mats, false, alive, shadow, rk); break;
        case PG_CLASS_ROUGHCONDUCTOR:
            shadeOne<PG_BSDF_ROUGHCONDUCTOR, true, ENV>(g, sc, sd, p, slot, sc.mats, false, alive, shadow, rk);
            break;
        case PG_CLASS_ROUGHDIELECTRIC:
            shadeOne<PG_BSDF_ROUGHDIELECTRIC, true, ENV>(g, sc, sd, p, slot, sc.mats, false, alive, shadow, rk);
            break;
        case PG_CLASS_PLASTIC: shadeOne<PG_BSDF_PLASTIC, false, ENV>(g, sc, sd, p, slot, sc.mats, false, alive, shadow, rk); break;
        case PG_CLASS_ROUGHPLASTIC:
            shadeOne<PG_BSDF_ROUGHPLASTIC, true, ENV>(g, sc, sd, p, slot, sc.mats, false, alive, shadow, rk);
            break;
        default: shadeOne<-1, false, ENV>(g, sc, sd, p, slot, sc.mats, false, alive, shadow, rk);
    }
}
template <bool ENV>
#ifndef PG_TAIL_WAVES
#define PG_TAIL_WAVES 0  // 0: the compiler's budget (A/B: 3)
#endif
__global__ __launch_bounds__(TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(PG_TAIL_WAVES > 0 ? PG_TAIL_WAVES : 1))) void k_tail(GParams g, SceneDev sc, SDDev sd, PathDev p, Queue q,
                                                      unsigned long long *stats) {
    __shared__ uint32_t stack[2 * WIDE_LDS_STACK * TRACE_BLOCK];  // >= LDS_STACK words per thread
    const TStack stk = threadStack(stack, p.stack_ovf);
    const WStack wstk = threadWideStack(stack, p.stack_ovf);
    const uint32_t s = blockIdx.x & (PG_QSHARDS - 1);
    const uint32_t rows = gridDim.x / PG_QSHARDS;  // grid capped at TRACE_MAX_BLOCKS: the overflow ring's size
    const uint32_t n = q.counts[s];
    uint32_t segs = 0, esc = 0, shadows = 0;
    for (uint32_t i = (blockIdx.x / PG_QSHARDS) * TRACE_BLOCK + threadIdx.x; i < n; i += rows * TRACE_BLOCK) {
        const uint32_t slot = q.items[(size_t)s * q.stride + i];
        uint32_t tri = __float_as_uint(ldS(&p.hit[slot]).y);
        while (tri != 0xFFFFFFFFu) {
            bool alive = false, shadow = false;
            tailShade<ENV>(g, sc, sd, p, slot, tri, alive, shadow);
            if (shadow) {  // shadowRows for this path
                ++shadows;
                const float4 o = ldS(&p.ray_o[slot]), d = ldS(&p.sh_d[slot]);
                if (!occluded(sc, xyz(o), xyz(d), shadowTmin(o), d.w, wstk)) {
                    const float4 c = ldS(&p.sh_c[slot]);
                    const float4 L = ldS(&p.rad[slot]);
                    stS(&p.rad[slot], make_float4(L.x + c.x, L.y + c.y, L.z + c.z, L.w));
                    const uint32_t vi = __float_as_uint(c.w);
                    if (vi != 0xFFFFFFFFu) {
                        float4 *vl = p.vtx + ((size_t)vi * p.vtxP + slot) * PG_VTX_F4 + 2;
                        const float4 a = *vl;
                        *vl = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, a.w);
                    }
                }
            }
            if (!alive) break;
            // traceRows for this path
            const float4 o = ldS(&p.ray_o[slot]), d = ldS(&p.ray_d[slot]);
            float tmax = d.w, u = 0, v = 0;
            tri = 0xFFFFFFFFu;
            const bool h = traverse<false>(sc.nodes, sc.tris, xyz(o), xyz(d), o.w, tmax, tri, u, v, stk);
            float4 hr = make_float4(h ? tmax : 0.0f, __uint_as_float(h ? tri : 0xFFFFFFFFu), u, v);
            if (ENV && !h) {
                const f3 e = envEscapeRadiance(g, sc, p, slot, xyz(d));
                hr = make_float4(e.x, hr.y, e.y, e.z);
            }
            stS(&p.hit[slot], hr);
            ++segs;
            if (!h) {
                ++esc;
                tri = 0xFFFFFFFFu;
            }
        }
    }
    // wave-summed counters
    unsigned long long a = segs, b = esc, c = shadows;
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
        c += __shfl_xor(c, off);
    }
    if ((threadIdx.x & 63) == 0 && (a | b | c)) {
        atomicAdd(stats + 0, a);
        atomicAdd(stats + 1, b);
        atomicAdd(stats + 2, c);
    }
}

// film: box-filtered accumulation of every layer's sample into its pixel, in sample order
// (ProgressiveMonteCarloIntegrator::renderBlock clamp + ImageBlock::put validity check)
__global__ __launch_bounds__(256) void k_film(GParams g, SceneDev sc, PathDev p, const uint32_t *__restrict__ local_pixels,
                                              uint32_t pix_begin, uint32_t npix, uint32_t nlayers,
                                              float4 *__restrict__ film, float4 *__restrict__ sumsq,
                                              float4 *__restrict__ aov_albedo, float4 *__restrict__ aov_normal) {
    uint32_t lp = blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= npix) return;
    uint32_t pix = local_pixels[pix_begin + lp];
    if (p.aov) {  // feature sums of every sample (Denoiser::add averages all of them, denoiser.cpp:138-144)
        float4 sa = aov_albedo[pix], sn = aov_normal[pix];
        for (uint32_t l = 0; l < nlayers; ++l) {
            const float4 hv = p.aov[(size_t)l * npix + lp];
            const uint32_t tri = __float_as_uint(hv.y);
            f3 a = mk1(0.f), n = mk(0.f, 0.f, -1.f);  // Denoiser::Sample defaults (denoiser.h:12-16): escaped ray
            if (tri != 0xFFFFFFFFu) {
                const float4 *r = sc.tshade + (size_t)PG_TRI_SHADE_STRIDE * tri;
                const float4 s1 = r[1], s3 = r[3], s4 = r[4];
                const float b0 = 1 - hv.z - hv.w;
                n = normalize(xyz(s3) * b0 + mk(s3.w, s4.x, s4.y) * hv.z + mk(s4.z, s4.w, s1.w) * hv.w);  // fetchHit's shN
                a = bsdfAlbedo(sc.mats[__float_as_uint(r[0].w) & 0xFFFFu]);
            }
            sa = make_float4(sa.x + a.x, sa.y + a.y, sa.z + a.z, sa.w + 1.0f);
            sn = make_float4(sn.x + n.x, sn.y + n.y, sn.z + n.z, 0.0f);
        }
        aov_albedo[pix] = sa;
        aov_normal[pix] = sn;
    }
    float4 a = film[pix], q = sumsq[pix];
    for (uint32_t l = 0; l < nlayers; ++l) {
        float4 L = p.rad[(size_t)l * npix + lp];
        if (sc.env && p.hit) L = envHitRadiance(L, p.hit[(size_t)l * npix + lp]);  // surface path (volpath: no hit)
        float m = fmaxf(L.x, fmaxf(L.y, L.z));
        if (m > g.max_component_value) {
            float s = g.max_component_value / m;
            L.x *= s;
            L.y *= s;
            L.z *= s;
        }
        bool okv = isfinite(L.x) && isfinite(L.y) && isfinite(L.z) && L.x >= 0 && L.y >= 0 && L.z >= 0;
        if (!okv) continue;
        a.x += L.x;
        a.y += L.y;
        a.z += L.z;
        a.w += 1.0f;
        q.x += L.x * L.x;
        q.y += L.y * L.y;
        q.z += L.z * L.z;
    }
    film[pix] = a;
    sumsq[pix] = q;
}

// training records of finished paths: radiance along wo_i = (L_final - L_i) / T_i (channel-wise)
// env_hits: the surface path of a scene with an environment emitter (envHitRadiance)
__global__ __launch_bounds__(256) void k_commit(PathDev p, uint32_t nslots, int maxV, pg_record *__restrict__ recs,
                                                unsigned long long *__restrict__ rec_count,
                                                unsigned long long capacity, int env_hits) {
    uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nv = 0;
    if (slot < nslots) nv = min(p.pinfo ? p.pinfo[slot].w : __float_as_uint(p.rad[slot].w), (uint32_t)maxV);
    // wave inclusive scan of nv
    int lane = threadIdx.x & 63;
    uint32_t incl = nv;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    uint32_t total = __shfl(incl, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(rec_count, (unsigned long long)total);
    base = __shfl(base, 63);
    if (nv == 0) return;
    unsigned long long o = base + (incl - nv);
    float4 L = p.rad[slot];
    if (env_hits) L = envHitRadiance(L, p.hit[slot]);
    for (uint32_t k = 0; k < nv; ++k, ++o) {
        if (o >= capacity) return;
        const float4 *vb = p.vtx + ((size_t)k * p.vtxP + slot) * PG_VTX_F4;
        float4 a = vb[0], b = vb[1], c = vb[2], e = vb[3];
        float woPdf = a.w;
        float lr = (b.x * woPdf > 1e-4f) ? (L.x - c.x) / b.x : 0.0f;
        float lg = (b.y * woPdf > 1e-4f) ? (L.y - c.y) / b.y : 0.0f;
        float lb = (b.z * woPdf > 1e-4f) ? (L.z - c.z) / b.z : 0.0f;
        // f L_i / woPdf per channel = (L_final - L_snapshot) / T_before (oracle: the same guards)
        float wr = (b.x * woPdf > 1e-4f) ? (L.x - c.x) / e.x : 0.0f;
        float wg = (b.y * woPdf > 1e-4f) ? (L.y - c.y) / e.y : 0.0f;
        float wb = (b.z * woPdf > 1e-4f) ? (L.z - c.z) / e.z : 0.0f;
        pg_record r;
        r.pos[0] = a.x;
        r.pos[1] = a.y;
        r.pos[2] = a.z;
        r.dir = __float_as_uint(b.w);
        r.radiance = (lr + lg + lb) * (1.0f / 3.0f);
        r.wo_pdf = woPdf;
        r.product = e.w >= 0.0f ? (wr + wg + wb) * (1.0f / 3.0f) : 0.0f;
        r.weight = e.w;
        float4 *dst = reinterpret_cast<float4 *>(recs + o);
        dst[0] = make_float4(r.pos[0], r.pos[1], r.pos[2], __uint_as_float(r.dir));
        dst[1] = make_float4(r.radiance, r.wo_pdf, r.product, r.weight);
    }
}

// SD-tree splat: records -> building-tree leaf quadrants (2^-24 fixed point, u64 atomics)
// Wave-aggregated atomic add: lanes with equal keys are summed in registers and one lane adds the
// sum.  Early training iterations splat ~1M records into a handful of D-tree nodes, where plain
// per-record atomics serialize on one address (53 ms for iteration 0).  Integer adds make the
// result independent of the grouping, so trees stay bit-identical.  Call with the whole wave active.
template <class T>
__device__ __forceinline__ void waveKeyedAdd(T *base, uint32_t key, T v, bool valid) {
    const int lane = threadIdx.x & 63;
    unsigned long long pending = __ballot(valid);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint32_t k = __shfl(key, leader);
        const bool mine = valid && key == k;
        const unsigned long long m = __ballot(mine);
        T sum = mine ? v : (T)0;
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
        if (lane == leader) atomicAdd(base + k, sum);
        pending &= ~m;
    }
}

// the learned-fraction statistics of a wave's guided records: per group of lanes with one D-tree,
// kFracCandidates wave-summed fixed-point values and the group's record count, added by its leader
__device__ __forceinline__ void waveKeyedFracAdd(unsigned long long *base, uint32_t key, float w, float pb, float pg,
                                                 float q0, bool valid) {
    const int lane = threadIdx.x & 63;
    unsigned long long pending = __ballot(valid);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint32_t k = __shfl(key, leader);
        const bool mine = valid && key == k;
        const unsigned long long m = __ballot(mine);
        unsigned long long *dst = base + (size_t)k * (kFracCandidates + 1);
        for (int c = 0; c < kFracCandidates; ++c) {
            unsigned long long v = mine ? fracStat(w, pb, pg, q0, c) : 0ull;
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            if (lane == leader) atomicAdd(dst + c, v);
        }
        if (lane == leader) atomicAdd(dst + kFracCandidates, (unsigned long long)__popcll(m));
        pending &= ~m;
    }
}

__global__ __launch_bounds__(256) void k_splat(SDDev sd, const pg_record *__restrict__ recs, unsigned long long n) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = i < n, found = false;
    unsigned long long fx = 0;
    uint32_t dt = 0, slot = 0;
    if (valid) {
        const float4 *src = reinterpret_cast<const float4 *>(recs + i);
        float4 a = src[0], b = src[1];
        float woPdf = b.y;
        float val = 0.0f;
        {
#pragma clang fp contract(off)
            if (woPdf > 0) val = b.x / woPdf;
        }
        valid = woPdf > 0 && val >= 0 && val < 1e30f;
        if (valid) {
            float s = val * 16777216.0f;
            // cap 2^48 (value <= 2^24; oracle kSplatCap).  A leaf quadrant's u64 atomic sum over all
            // records and ranks of an iteration wraps only past 2^40 value units (e.g. 2^16 records at
            // the cap); the host refit's interior sums saturate (pg_sdtree.cpp propagate)
            if (s >= 281474976710656.0f) s = 281474976710656.0f;
            fx = (unsigned long long)s;
            const SDView sv = sdv(sd);
            dt = sdLookup(sv, mk(a.x, a.y, a.z));
            uint32_t dirw = __float_as_uint(a.w);
            float u = ((float)(dirw & 0xFFFFu) + 0.5f) * (1.0f / 65536.0f);
            float v = ((float)(dirw >> 16) + 0.5f) * (1.0f / 65536.0f);
            uint32_t node = sd.meta[dt].y;
            for (int guard = 0; guard < 64; ++guard) {
                int q = childIndex(u, v);
                uint32_t c = c4(sd.bchild[node], q);
                if (c == 0) {
                    slot = 4 * node + q;
                    found = true;
                    break;
                }
                node = c;
            }
        }
    }
    waveKeyedAdd<unsigned long long>(sd.count, dt, 1ull, valid);
    waveKeyedAdd<unsigned long long>(sd.bsum, slot, fx, found);
    if (!sd.learned) return;
    // learned BSDF-sampling fraction (pg_device.h fracStat): a guided record (weight = p_guide >= 0)
    // with a contribution adds w log2(q_k / q0) for every candidate k, and 1 to its guided count.  p_bsdf
    // comes back from q0 = a0 p_bsdf + (1 - a0) p_guide with a0 the leaf's fraction that sampled it.
    bool stat = false;
    float w = 0, pb = 0, pg = 0, q0 = 0;
    if (valid) {
        const float4 b = reinterpret_cast<const float4 *>(recs + i)[1];
        pg = b.w;
        w = b.z;
        q0 = b.y;
        if (pg >= 0.0f && w > 0.0f && w < 1e30f) {
#pragma clang fp contract(off)
            const float la = __uint_as_float(sd.meta[dt].z);
            const float a0 = la > 0 ? la : sd.alpha0;
            pb = fmaxf((q0 - (1.0f - a0) * pg) / a0, 0.0f);
            stat = true;
        }
    }
    waveKeyedFracAdd(sd.frac, dt, w, pb, pg, q0, stat);
}

// Block-private splat (PG_SPLAT_LDS, default): a grid of at most ~1k blocks walks the records in
// block-strided rounds and sums the per-D-tree record counts and per-leaf-quadrant fixed-point values
// in two LDS hash tables (open addressing, 8 probes); keys that find no slot go straight to the global
// atomics.  Each block then adds its table entries to the global sums once.  A hot D-tree (one near
// the camera gets ~10 % of an iteration's records) thus costs one global atomic per block instead of
// one per wave.  Integer sums: the trees are bit-identical to the wave-aggregated k_splat.
// 1024 + 4096 entries (60 KiB, 2 blocks per CU): C3 W = 1 training 77 -> 70 ms against 512 + 2048
// (iteration 4's splat 7.5 -> 2.9 ms); 2048 + 8192 (1 block per CU) 74 ms (profiles/r03y_splat_tables_ab/)
#ifndef SPLAT_CNT_SLOTS
#define SPLAT_CNT_SLOTS 1024
#endif
#ifndef SPLAT_SUM_SLOTS
#define SPLAT_SUM_SLOTS 4096
#endif
#define SPLAT_EMPTY 0xFFFFFFFFu
__device__ __forceinline__ bool ldsTableAdd(uint32_t *keys, unsigned long long *vals, uint32_t mask, uint32_t key,
                                            unsigned long long v) {
    uint32_t h = (key * 2654435761u) >> 7;
    for (int probe = 0; probe < 8; ++probe, ++h) {
        h &= mask;
        uint32_t k = __atomic_load_n(&keys[h], __ATOMIC_RELAXED);
        if (k == SPLAT_EMPTY) k = atomicCAS(&keys[h], SPLAT_EMPTY, key);
        if (k == SPLAT_EMPTY || k == key) {
            atomicAdd(&vals[h], v);
            return true;
        }
    }
    return false;
}

__global__ __launch_bounds__(256) void k_splat_lds(SDDev sd, const pg_record *__restrict__ recs, unsigned long long n) {
    __shared__ uint32_t ckey[SPLAT_CNT_SLOTS], skey[SPLAT_SUM_SLOTS];
    __shared__ unsigned long long cval[SPLAT_CNT_SLOTS], sval[SPLAT_SUM_SLOTS];
    for (uint32_t e = threadIdx.x; e < SPLAT_SUM_SLOTS; e += blockDim.x) {
        skey[e] = SPLAT_EMPTY;
        sval[e] = 0;
        if (e < SPLAT_CNT_SLOTS) {
            ckey[e] = SPLAT_EMPTY;
            cval[e] = 0;
        }
    }
    __syncthreads();
    const SDView sv = sdv(sd);
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    // uniform trip count per block (waveKeyedFracAdd needs the whole wave)
    for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < n; base += stride) {
        const unsigned long long i = base + threadIdx.x;
        bool valid = i < n, found = false;
        unsigned long long fx = 0;
        uint32_t dt = 0, slot = 0;
        float4 b = make_float4(0, 0, 0, 0);
        if (valid) {
            const float4 *src = reinterpret_cast<const float4 *>(recs + i);
            const float4 a = src[0];
            b = src[1];
            const float woPdf = b.y;
            float val = 0.0f;
            {
#pragma clang fp contract(off)
                if (woPdf > 0) val = b.x / woPdf;
            }
            valid = woPdf > 0 && val >= 0 && val < 1e30f;
            if (valid) {
                float s = val * 16777216.0f;
                if (s >= 281474976710656.0f) s = 281474976710656.0f;  // cap 2^48, as k_splat
                fx = (unsigned long long)s;
                dt = sdLookup(sv, mk(a.x, a.y, a.z));
                const uint32_t dirw = __float_as_uint(a.w);
                float u = ((float)(dirw & 0xFFFFu) + 0.5f) * (1.0f / 65536.0f);
                float v = ((float)(dirw >> 16) + 0.5f) * (1.0f / 65536.0f);
                uint32_t node = sd.meta[dt].y;
                for (int guard = 0; guard < 64; ++guard) {
                    const int q = childIndex(u, v);
                    const uint32_t c = c4(sd.bchild[node], q);
                    if (c == 0) {
                        slot = 4 * node + q;
                        found = true;
                        break;
                    }
                    node = c;
                }
            }
        }
        if (valid && !ldsTableAdd(ckey, cval, SPLAT_CNT_SLOTS - 1, dt, 1ull)) atomicAdd(sd.count + dt, 1ull);
        if (found && fx && !ldsTableAdd(skey, sval, SPLAT_SUM_SLOTS - 1, slot, fx)) atomicAdd(sd.bsum + slot, fx);
        if (sd.learned) {  // learned-fraction statistics as in k_splat (wave-aggregated global atomics)
            bool stat = false;
            float w = 0, pb = 0, pg = 0, q0 = 0;
            if (valid) {
                pg = b.w;
                w = b.z;
                q0 = b.y;
                if (pg >= 0.0f && w > 0.0f && w < 1e30f) {
#pragma clang fp contract(off)
                    const float la = __uint_as_float(sd.meta[dt].z);
                    const float a0 = la > 0 ? la : sd.alpha0;
                    pb = fmaxf((q0 - (1.0f - a0) * pg) / a0, 0.0f);
                    stat = true;
                }
            }
            waveKeyedFracAdd(sd.frac, dt, w, pb, pg, q0, stat);
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < SPLAT_SUM_SLOTS; e += blockDim.x) {
        if (skey[e] != SPLAT_EMPTY && sval[e]) atomicAdd(sd.bsum + skey[e], sval[e]);
        if (e < SPLAT_CNT_SLOTS && ckey[e] != SPLAT_EMPTY) atomicAdd(sd.count + ckey[e], cval[e]);
    }
}

// ---- unit-level kernels used by the parity tests ---------------------------------------------
__global__ __launch_bounds__(TRACE_BLOCK) void k_trace_rays(SceneDev sc, const float *__restrict__ rays, uint32_t n,
                                                            int any, float *__restrict__ hits, uint32_t *ovf) {
    __shared__ uint32_t stack[2 * WIDE_LDS_STACK * TRACE_BLOCK];  // >= LDS_STACK words per thread
    const TStack stk = threadStack(stack, ovf);
    const WStack wstk = threadWideStack(stack, ovf);
    uint32_t i = blockIdx.x * TRACE_BLOCK + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + 8 * (size_t)i;
    f3 o = mk(r[0], r[1], r[2]), d = mk(r[4], r[5], r[6]);
    float tmax = r[7];
    uint32_t tri = 0xFFFFFFFFu;
    float u = 0, v = 0;
    float *h = hits + 4 * (size_t)i;
    if (any == 1) {
        bool occ = occluded(sc, o, d, r[3], tmax, wstk);
        h[0] = occ ? 1.0f : 0.0f;
        h[1] = h[2] = h[3] = 0.0f;
        return;
    }
    bool hit = traverse<false>(sc.nodes, sc.tris, o, d, r[3], tmax, tri, u, v, stk);
    if (any == 2) {  // pg_hit_records: the hit record the shading kernels build (fetchHit), 16 floats per ray
        float *q = hits + 16 * (size_t)i;
        if (!hit) {
            for (int k = 0; k < 16; ++k) q[k] = 0.0f;
            return;
        }
        Hit hr;
        fetchHit(sc, tri, u, v, d, hr);
        const float rec[16] = {hr.p.x,    hr.p.y,    hr.p.z,    tmax,       hr.geoN.x, hr.geoN.y, hr.geoN.z, hr.shN.x,
                               hr.shN.y,  hr.shN.z,  hr.sh.s.x, hr.sh.s.y,  hr.sh.s.z, hr.wi.x,   hr.wi.y,   hr.wi.z};
        for (int k = 0; k < 16; ++k) q[k] = rec[k];
        return;
    }
    uint32_t orig = hit ? __float_as_uint(sc.tshade[(size_t)PG_TRI_SHADE_STRIDE * tri + 2].w) : 0xFFFFFFFFu;
    h[0] = hit ? tmax : 0.0f;
    h[1] = __uint_as_float(orig);
    h[2] = u;
    h[3] = v;
}

__global__ __launch_bounds__(256) void k_bsdf_query(const GMat *mat, const float *wi, const float *u, const float *wog,
                                                    uint32_t n, float *out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GMat M = *mat;
    f3 w = mk(wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]);
    BS bs;
    f3 wt = bsdfSample(M, w, u[3 * i], u[3 * i + 1], u[3 * i + 2], bs);
    float *o = out + 12 * (size_t)i;
    bool z = isZero(wt);
    o[0] = bs.wo.x;
    o[1] = bs.wo.y;
    o[2] = bs.wo.z;
    o[3] = z ? 0.0f : bs.pdf;
    o[4] = wt.x;
    o[5] = wt.y;
    o[6] = wt.z;
    o[7] = z ? 0.0f : (float)bs.type;
    if (wog) {
        f3 g = mk(wog[3 * i], wog[3 * i + 1], wog[3 * i + 2]);
        f3 e = bsdfEval(M, w, g);
        o[8] = e.x;
        o[9] = e.y;
        o[10] = e.z;
        o[11] = bsdfPdf(M, w, g);
    } else {
        o[8] = o[9] = o[10] = o[11] = 0.0f;
    }
}

__global__ __launch_bounds__(256) void k_sd_pdf(SDDev sd, const float *pos, const float *dir, uint32_t n, float *out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SDView sv = sdv(sd);
    uint4 meta = sd.meta[sdLookup(sv, mk(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]))];
    out[i] = sdPdf(sv, meta, mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]));
}

__global__ __launch_bounds__(256) void k_sd_sample(SDDev sd, const float *pos, const float *u, uint32_t n, float *dir,
                                                   float *pdf) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SDView sv = sdv(sd);
    uint4 meta = sd.meta[sdLookup(sv, mk(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]))];
    float cu, cv, pd;
    sdSampleCanon(sv, meta, u[2 * i], u[2 * i + 1], cu, cv, pd);
    f3 d = canonicalToDir(cu, cv);
    dir[3 * i] = d.x;
    dir[3 * i + 1] = d.y;
    dir[3 * i + 2] = d.z;
    pdf[i] = pd;
}

// =============================================================================================
static inline uint32_t blocks(uint64_t n, uint32_t b) { return (uint32_t)((n + b - 1) / b); }

size_t pg_stack_overflow_words(uint64_t max_threads) {
    if (max_threads == 0) max_threads = (uint64_t)TRACE_MAX_BLOCKS * TRACE_BLOCK;
    const size_t words = std::max<size_t>(std::max(STACK_DEPTH, PG_BVH4 ? PG_QSTACK_DEPTH : 0) - LDS_STACK,
                                          2 * (STACK_DEPTH - WIDE_LDS_STACK)) +
                         (PG_TRACE_PAIR ? kPairRing : 0);  // the paired walks' second band
    return words * max_threads;
}
// threads k_trace_rays launches for n rays: its overflow stride is gridDim.x * TRACE_BLOCK
uint64_t pg_trace_rays_threads(uint64_t n) { return (uint64_t)blocks(n, TRACE_BLOCK) * TRACE_BLOCK; }

void pg_launch_camera(hipStream_t s, const GParams &g, const PathDev &p, const uint32_t *local_pixels,
                      uint32_t pix_begin, uint32_t npix, uint32_t nlayers, uint32_t sample_base, Queue q, bool banded) {
    uint64_t n = (uint64_t)npix * nlayers;
    if (!n) return;
    hipLaunchKernelGGL(k_camera, dim3(blocks(n, 256)), dim3(256), 0, s, g, p, local_pixels, pix_begin, npix, nlayers,
                       sample_base, q, pg_camera_banded(banded, npix));
}
// grid of a sharded launch: PG_QSHARDS x rows (rows capped for persistent grid-stride kernels)
static inline dim3 shardGrid(uint32_t max_shard, uint32_t block, uint32_t max_rows) {
    const uint32_t rows = blocks(max_shard, block);
    return dim3(PG_QSHARDS * (rows < max_rows ? rows : max_rows));
}
void pg_launch_trace(hipStream_t s, const GParams &g, const SceneDev &sc, const PathDev &p, Queue q, uint32_t max_shard,
                     const Queue *class_queues, bool first_bounce) {
    if (!max_shard) return;
    ClassQueues cq;
    for (int c = 0; c <= PG_NUM_CLASSES; ++c) cq.q[c] = class_queues[c];
    const dim3 grid = shardGrid(max_shard, TRACE_BLOCK, TRACE_MAX_BLOCKS / PG_QSHARDS);
    float4 *first = first_bounce ? p.aov : nullptr;
    if (sc.env) hipLaunchKernelGGL(k_trace<true>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, p, q, cq, first);
    else hipLaunchKernelGGL(k_trace<false>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, p, q, cq, first);
}
template <bool ENV>
static void launchShade(hipStream_t s, int cls, dim3 grid, const GParams &g, const SceneDev &sc, const SDDev &sd,
                        const PathDev &p, Queue in, Queue out, Queue shq) {
    const dim3 block(SHADE_BLOCK);
    switch (cls) {
        case PG_CLASS_DIFFUSE:
            hipLaunchKernelGGL((k_shade<PG_BSDF_DIFFUSE, true, ENV>), grid, block, 0, s, g, sc, sd, p, in, out, shq);
            break;
        case PG_CLASS_ROUGHCONDUCTOR:
            hipLaunchKernelGGL((k_shade<PG_BSDF_ROUGHCONDUCTOR, true, ENV>), grid, block, 0, s, g, sc, sd, p, in, out, shq);
            break;
        case PG_CLASS_ROUGHDIELECTRIC:
            hipLaunchKernelGGL((k_shade<PG_BSDF_ROUGHDIELECTRIC, true, ENV>), grid, block, 0, s, g, sc, sd, p, in, out, shq);
            break;
        case PG_CLASS_PLASTIC:
            hipLaunchKernelGGL((k_shade<PG_BSDF_PLASTIC, false, ENV>), grid, block, 0, s, g, sc, sd, p, in, out, shq);
            break;
        case PG_CLASS_ROUGHPLASTIC:
            hipLaunchKernelGGL((k_shade<PG_BSDF_ROUGHPLASTIC, true, ENV>), grid, block, 0, s, g, sc, sd, p, in, out, shq);
            break;
        default:  // delta lobes: conductor, dielectric (runtime switch, never guided)
            hipLaunchKernelGGL((k_shade<-1, false, ENV>), grid, block, 0, s, g, sc, sd, p, in, out, shq);
    }
}
void pg_launch_shade_class(hipStream_t s, int cls, const GParams &g, const SceneDev &sc, const SDDev &sd,
                           const PathDev &p, Queue in, uint32_t max_shard, Queue out, Queue shq) {
    if (!max_shard) return;
    const dim3 grid = shardGrid(max_shard, SHADE_BLOCK, 0xFFFFFFFFu);
    if (sc.env) launchShade<true>(s, cls, grid, g, sc, sd, p, in, out, shq);
    else launchShade<false>(s, cls, grid, g, sc, sd, p, in, out, shq);
}
void pg_launch_shade_all(hipStream_t s, const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p,
                         const Queue *class_queues, const uint32_t *max_shard, Queue out, Queue shq) {
    ClassQueues cq;
    ShadeRanges r;
    uint32_t total = 0;
    for (int c = 0; c < PG_NUM_CLASSES; ++c) {
        cq.q[c] = class_queues[c];
        total += max_shard[c] ? shardGrid(max_shard[c], SHADE_BLOCK, 0xFFFFFFFFu).x : 0;
        r.end[c] = total;
    }
    cq.q[PG_NUM_CLASSES] = class_queues[PG_NUM_CLASSES];
    if (!total) return;
    hipLaunchKernelGGL(k_shade_all, dim3(total), dim3(SHADE_BLOCK), 0, s, g, sc, sd, p, cq, out, shq, r);
}
void pg_launch_rays(hipStream_t s, const GParams &g, const SceneDev &sc, const PathDev &p, Queue q, uint32_t max_shard,
                    const Queue *class_queues, Queue shq, uint32_t max_shadow_shard) {
    ClassQueues cq;
    for (int c = 0; c <= PG_NUM_CLASSES; ++c) cq.q[c] = class_queues[c];
    const uint32_t sb = max_shadow_shard ? shardGrid(max_shadow_shard, TRACE_BLOCK, TRACE_MAX_BLOCKS / PG_QSHARDS).x : 0;
    const uint32_t tb =
        max_shard ? shardGrid(max_shard, (PG_TRACE_PAIR ? 2 : 1) * TRACE_BLOCK, TRACE_MAX_BLOCKS / PG_QSHARDS).x : 0;
    if (sb + tb == 0) return;
    if (tb == 0) {  // no trace rows: k_rays needs at least one trace block per shard to stay sharded
        hipLaunchKernelGGL(k_shadow, dim3(sb), dim3(TRACE_BLOCK), 0, s, sc, p, shq);
        return;
    }
    if (sc.env) hipLaunchKernelGGL(k_rays<true>, dim3(sb + tb), dim3(TRACE_BLOCK), 0, s, g, sc, p, q, cq, shq, sb);
    else hipLaunchKernelGGL(k_rays<false>, dim3(sb + tb), dim3(TRACE_BLOCK), 0, s, g, sc, p, q, cq, shq, sb);
}
void pg_launch_shadow(hipStream_t s, const SceneDev &sc, const PathDev &p, Queue q, uint32_t max_shard) {
    if (!max_shard) return;
    hipLaunchKernelGGL(k_shadow, shardGrid(max_shard, TRACE_BLOCK, TRACE_MAX_BLOCKS / PG_QSHARDS), dim3(TRACE_BLOCK), 0,
                       s, sc, p, q);
}
void pg_launch_tail(hipStream_t s, const GParams &g, const SceneDev &sc, const SDDev &sd, const PathDev &p, Queue q,
                    uint32_t max_shard, unsigned long long *stats) {
    if (!max_shard) return;
    // at most TRACE_MAX_BLOCKS blocks (a grid-stride loop over each shard): the traversal stacks' overflow
    // ring (threadStack / threadWideStack, stride gridDim.x * TRACE_BLOCK) holds that many threads
    const dim3 grid = shardGrid(max_shard, TRACE_BLOCK, TRACE_MAX_BLOCKS / PG_QSHARDS);
    if (sc.env) hipLaunchKernelGGL(k_tail<true>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, sd, p, q, stats);
    else hipLaunchKernelGGL(k_tail<false>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, sd, p, q, stats);
}
template <uint32_t BINS>
static void raySort(hipStream_t s, Queue q, uint32_t max_shard, uint32_t *sorted_items, uint32_t *hist) {
    (void)hipMemsetAsync(hist, 0, (size_t)PG_QSHARDS * BINS * 4, s);
    const dim3 grid(PG_QSHARDS * blocks(max_shard, RSORT_TILE));
    hipLaunchKernelGGL(k_rsort_hist<BINS>, grid, dim3(256), 0, s, q, hist);
    hipLaunchKernelGGL(k_rsort_scan<BINS>, dim3(PG_QSHARDS), dim3(256), 0, s, hist);
    hipLaunchKernelGGL(k_rsort_scatter<BINS>, grid, dim3(256), 0, s, q, hist, sorted_items);
}
void pg_launch_ray_sort(hipStream_t s, Queue q, uint32_t max_shard, uint32_t *sorted_items, uint32_t *hist,
                        uint32_t bins) {
    if (!max_shard) return;
    if (bins == 512) raySort<512>(s, q, max_shard, sorted_items, hist);
    else raySort<PG_RAY_SORT_BINS>(s, q, max_shard, sorted_items, hist);
}
void pg_launch_film(hipStream_t s, const GParams &g, const SceneDev &sc, const PathDev &p, const uint32_t *local_pixels, uint32_t pix_begin,
                    uint32_t npix, uint32_t nlayers, float4 *film_rgbw, float4 *film_sumsq, float4 *aov_albedo,
                    float4 *aov_normal) {
    if (!npix) return;
    hipLaunchKernelGGL(k_film, dim3(blocks(npix, 256)), dim3(256), 0, s, g, sc, p, local_pixels, pix_begin, npix, nlayers,
                       film_rgbw, film_sumsq, aov_albedo, aov_normal);
}

// op 0: sampleDirect from the bounding-sphere centre (in: n x 2 samples; out n x 8: d, pdf, value/pdf, dist)
// op 1: pdfDirect (in: n x 3 world directions; out n); op 2: evalEnvironment (in n x 3; out n x 3)
__global__ __launch_bounds__(256) void k_envmap_query(SceneDev sc, int op, const float *in, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !sc.env) return;
    const GEnv &e = *sc.env;
    if (op == 0) {
        f3 d = mk1(0.f);
        float dist = 0, pdf;
        const f3 v = envSampleDirect(e, mk(e.center[0], e.center[1], e.center[2]), in[2 * i], in[2 * i + 1], d, dist, pdf);
        float *o = out + 8 * (size_t)i;
        o[0] = d.x;
        o[1] = d.y;
        o[2] = d.z;
        o[3] = pdf;
        o[4] = v.x;
        o[5] = v.y;
        o[6] = v.z;
        o[7] = dist;
    } else if (op == 1) {
        out[i] = envPdf(e, mk(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
    } else {
        const f3 v = envEval(e, mk(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
        out[3 * (size_t)i] = v.x;
        out[3 * (size_t)i + 1] = v.y;
        out[3 * (size_t)i + 2] = v.z;
    }
}
void pg_launch_envmap_query(hipStream_t s, const SceneDev &sc, int op, const float *in, uint32_t n, float *out) {
    if (!n) return;
    hipLaunchKernelGGL(k_envmap_query, dim3(blocks(n, 256)), dim3(256), 0, s, sc, op, in, n, out);
}
void pg_launch_commit(hipStream_t s, const PathDev &p, uint32_t nslots, int max_vertices, pg_record *records,
                      unsigned long long *rec_count, unsigned long long rec_capacity, int env_hits) {
    if (!nslots) return;
    hipLaunchKernelGGL(k_commit, dim3(blocks(nslots, 256)), dim3(256), 0, s, p, nslots, max_vertices, records, rec_count,
                       rec_capacity, env_hits);
}
// the host's fillJump (pg_sdtree.cpp) per cell: level d splits axis d % 3 by bit (bits - 1 - d / 3) of
// the cell's coordinate on that axis
__global__ __launch_bounds__(256) void k_sd_jump(const uint2 *__restrict__ snodes, int bits, uint32_t *__restrict__ jump) {
    const uint32_t R = 1u << bits, cell = blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= R * R * R) return;
    const uint32_t xyz[3] = {cell % R, (cell / R) % R, cell / (R * R)};
    uint32_t n = 0;
    for (int d = 0; d < 3 * bits; ++d) {
        const uint2 nd = snodes[n];
        if (nd.x == 0xFFFFFFFFu) break;
        n = ((xyz[d % 3] >> (bits - 1 - d / 3)) & 1u) ? nd.y : nd.x;
    }
    // a cell inside one leaf holds the leaf's D-tree id, flagged (pg_device.h sdLookup: one load, not two)
    const uint2 nd = snodes[n];
    jump[cell] = nd.x == 0xFFFFFFFFu ? (0x80000000u | nd.y) : n;
}
void pg_launch_sd_jump(hipStream_t s, const uint32_t *snodes, int bits, uint32_t *jump) {
    const uint32_t n = 1u << (3 * bits);
    hipLaunchKernelGGL(k_sd_jump, dim3((n + 255) / 256), dim3(256), 0, s, reinterpret_cast<const uint2 *>(snodes), bits,
                       jump);
}
void pg_launch_splat(hipStream_t s, const SDDev &sd, const pg_record *recs, unsigned long long n) {
    if (!n) return;
    static const bool lds = [] {
        const char *e = std::getenv("PG_SPLAT_LDS");
        return !e || std::atoi(e) != 0;
    }();
    if (lds) {  // ~16 records per thread, at most 1024 blocks (4 per CU)
        const unsigned long long nb = std::min<unsigned long long>(1024, std::max<unsigned long long>(1, n / 4096));
        hipLaunchKernelGGL(k_splat_lds, dim3((uint32_t)nb), dim3(256), 0, s, sd, recs, n);
    } else {
        hipLaunchKernelGGL(k_splat, dim3(blocks(n, 256)), dim3(256), 0, s, sd, recs, n);
    }
}
void pg_launch_trace_rays(hipStream_t s, const SceneDev &sc, const float *rays, uint32_t n, int any, float *hits,
                          uint32_t *ovf) {
    if (!n) return;
    hipLaunchKernelGGL(k_trace_rays, dim3(blocks(n, TRACE_BLOCK)), dim3(TRACE_BLOCK), 0, s, sc, rays, n, any, hits, ovf);
}
void pg_launch_bsdf_query(hipStream_t s, const GMat *mat, const float *wi, const float *u, const float *wog, uint32_t n,
                          float *out) {
    if (!n) return;
    hipLaunchKernelGGL(k_bsdf_query, dim3(blocks(n, 256)), dim3(256), 0, s, mat, wi, u, wog, n, out);
}
void pg_launch_sd_pdf(hipStream_t s, const SDDev &sd, const float *pos, const float *dir, uint32_t n, float *out) {
    if (!n) return;
    hipLaunchKernelGGL(k_sd_pdf, dim3(blocks(n, 256)), dim3(256), 0, s, sd, pos, dir, n, out);
}
void pg_launch_sd_sample(hipStream_t s, const SDDev &sd, const float *pos, const float *u, uint32_t n, float *dir,
                         float *pdf) {
    if (!n) return;
    hipLaunchKernelGGL(k_sd_sample, dim3(blocks(n, 256)), dim3(256), 0, s, sd, pos, u, n, dir, pdf);
}
