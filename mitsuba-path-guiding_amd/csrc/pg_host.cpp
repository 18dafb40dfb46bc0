// Host driver behind the C-ABI (include/pg_capi.h): device context, scene flattening/upload,
// the progressive pass driver (ProgressiveMonteCarloIntegrator::renderSamples/renderBlock,
// src/librender/progressiveintegrator.cpp:65-114,222-282, re-expressed as a GPU wavefront loop),
// training-record management and the SD-tree refit hook (postprogression, :314-317).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../include/pg_capi.h"
#include "pg_bvh.h"
#include "pg_envmap.h"
#include "pg_kernels.h"
#include "pg_layout.h"
#include "pg_rtrans.h"
#include "pg_sdtree.h"

namespace {

constexpr uint32_t kStackDepth = 48;  // must match STACK_DEPTH in pg_kernels.hip
constexpr uint32_t kMaxBounces = 1100;     // > gpu_depth_cap default (1024) + 2
// per-bounce device counters (words): [0, 64) shard counts of the live queue entering the bounce,
// [64, 128) shadow-queue shard counts, [128, 512) shard counts of the PG_NUM_CLASSES material-class
// queues followed by the escaped-path counts
constexpr uint32_t kBounceWords = 640;
constexpr uint32_t kShadowCounts = PG_QSHARDS, kClassCounts = 2 * PG_QSHARDS;
static_assert(kClassCounts + (PG_NUM_CLASSES + 1) * PG_QSHARDS <= kBounceWords, "counter layout");
constexpr uint32_t kCounterWords = kBounceWords * (kMaxBounces + 1);
// the device's bounce cap (GParams::depth_cap): max_depth + 1 or gpu_depth_cap.  The surface path keeps
// one counter block per bounce, so its cap is at most kMaxBounces - 2 (pg_create rejects a larger
// max_depth and clamps gpu_depth_cap there), and the bounce-by-bounce loop (maxBounces = depth_cap + 2 <=
// kMaxBounces) and k_tail, which loops until shadeOne's depth_cap test ends the path, stop at the same
// bounce.  The volumetric path has no per-bounce buffer and honours max_depth exactly.
static uint32_t deviceDepthCap(const pg_config &cfg) {
    const int64_t cap = cfg.max_depth > 0 ? (int64_t)cfg.max_depth + 1 : (int64_t)cfg.gpu_depth_cap;
    if (cfg.integrator == PG_INTEGRATOR_VOLPATH) return (uint32_t)std::min<int64_t>(cap, 0x7fffffff);
    return (uint32_t)std::min<int64_t>(cap, (int64_t)kMaxBounces - 2);
}

// shading-queue class of a BSDF model (one specialised k_shade per class)
int materialClass(uint32_t model) {
    switch (model) {
        case PG_BSDF_DIFFUSE: return PG_CLASS_DIFFUSE;
        case PG_BSDF_ROUGHCONDUCTOR: return PG_CLASS_ROUGHCONDUCTOR;
        case PG_BSDF_ROUGHDIELECTRIC: return PG_CLASS_ROUGHDIELECTRIC;
        case PG_BSDF_PLASTIC: return PG_CLASS_PLASTIC;
        case PG_BSDF_ROUGHPLASTIC: return PG_CLASS_ROUGHPLASTIC;
        default: return PG_CLASS_DELTA;
    }
}

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t alloc(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        release();
        if (n == 0) return hipSuccess;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        else p = nullptr;
        return e;
    }
    // growth with headroom, for buffers re-sized every training iteration (SD-tree): freeing and
    // re-allocating device memory per refit stalled the next stream operation by up to ~20 ms
    hipError_t grow(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        return alloc(std::max(n, bytes + bytes / 2));
    }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// Pinned host staging buffer (reused): pageable-memory copies are pinned on demand by the runtime.
struct PinnedBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        n = std::max(n, (size_t)1 << 20);
        n += n / 2;
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e == hipSuccess) bytes = n;
        return e;
    }
};

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
};
// what a timed launch ran (pg_stats buckets)
enum LaunchKind { KT_TRACE = 0, KT_SHADE = 1, KT_SHADOW = 2, KT_RAYS = 3 };

// One in-flight chunk of paths: its own stream, path state, queues and counters.  pg_render_pass
// interleaves pg_config.path_lanes lanes, so while the host waits for one lane's per-bounce class counts the
// GPU runs the other lane's kernels (and a lane's sparse late bounces overlap the other's).
#define PG_MAX_LANES 4
#ifndef PG_SMALL_PASS
#define PG_SMALL_PASS (1u << 21)  // paths: passes up to this size run as one chunk (0: always one per lane)
#endif
// the same threshold at run time (A/B: PG_SMALL_PASS_PATHS overrides)
uint64_t smallPass() {
    static const uint64_t n = [] {
        const char *e = std::getenv("PG_SMALL_PASS_PATHS");
        return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)PG_SMALL_PASS;
    }();
    return n;
}
#ifndef PG_PIXEL_BLOCK
#define PG_PIXEL_BLOCK 8  // local pixel order inside a tile: 8x8 blocks (0: row-major)
#endif
#define PG_DEFAULT_LANES 3
struct Lane {
    hipStream_t stream = nullptr;
    uint32_t P = 0;
    int vtx_slots = 0;
    uint32_t vtxP = 0;  // slot stride of vtx (recording passes only allocate it)
    DevBuf ray_o, ray_d, hit, thr, rad, prev, pinfo, sh_d, sh_c, vtx, q0, q1, qs, class_q, counters, stack_ovf;
    DevBuf qkey, qsorted, rsort_hist;  // ray-sorted trace queues (PG_RAY_SORT): keys, sorted entries, histograms
    bool sorted = false;               // the queue of the next trace launch is qsorted
    DevBuf tail_stats;                 // k_tail counters of the running chunk (3 u64), copied to h_tail
    uint64_t *h_tail = nullptr;        // pinned: k_tail counters of the last finished chunk
    DevBuf aov;  // denoiser features per slot (pg_config.aovs), 2 x float4
    uint32_t *h_counts = nullptr;  // pinned: per-bounce class counts of the running chunk
    uint32_t *h_stats = nullptr;   // pinned: counters of the last finished chunk
    std::vector<EventPair> ev[2];  // kernel-timing events: running chunk / last finished chunk
    std::vector<uint8_t> evkind[2];  // LaunchKind of each used pair
    size_t evused[2] = {0, 0};
    int evcur = 0;
    hipEvent_t ready = nullptr;    // class counts of the current bounce are on the host
    hipEvent_t done = nullptr;     // last finished chunk's statistics copy
    bool stats_pending = false;
    uint32_t stats_bounces = 0;
    // PG_DEBUG_COUNTS: per-bounce segment totals the host read (running chunk / last finished chunk),
    // checked against the device counters of the finished chunk
    std::vector<uint64_t> used_cur, used_prev;
    // running chunk
    bool active = false;
    bool traced = false;  // every path of the chunk terminated; film waits for its turn
    uint32_t chunk = 0;   // chunk index within the pass (films accumulate in this order)
    uint32_t b = 0, bound = 0, n = 0, pb = 0, np = 0, nl = 0, layer0 = 0;
};

// One in-flight chunk of the volumetric wavefront (renderVolpath): its own stream, SoA path state
// (VolWave, 7 x 16 B per slot), five sharded queues (flight / surface for two iterations, medium
// vertices) with their counters and host copy, per-item radiance and stack overflow ring.  Several
// lanes overlap one chunk's sparse late iterations and k_vtail with the next chunk's full ones.
struct VolLane {
    hipStream_t stream = nullptr;
    hipEvent_t ready = nullptr;  // the counters' host copy landed
    // the deferred transmittance walks (k_vnee) on a stream of their own, overlapping the next iteration's
    // free flights (PG_VOL_NEE_OVERLAP): vdone = this iteration's interactions done, ndone = its walks done
    hipStream_t nstream = nullptr;
    hipEvent_t vdone = nullptr, ndone = nullptr;
    bool npending = false;
    DevBuf state, items, counts, rad, ovf;
    DevBuf keys, sorted, hist;  // flight order keys of both flight queues, a sorted copy, histograms (PG_VOL_SORT)
    PinnedBuf host;
    uint32_t cap = 0;
    int stateF4 = 0;  // float4 arrays per slot in `state` (7, or 14 with the k_vnee stage's records)
    // the chunk in flight
    bool active = false, waved = false;  // waved: its paths are done, its film waits for its turn
    uint32_t chunk = 0, pb = 0, np = 0, nl = 0, sample_base = 0;
    int it = 0;
    EventPair span;                      // chunk start .. film (pg_stats volume_ms; moved to the pass's list)
};

struct Ctx {
    pg_config cfg{};
    std::string err;
    std::atomic<bool> cancel{false};
    hipStream_t stream = nullptr;
    // scene
    bool has_scene = false;
    GParams g{};
    DevBuf nodes, tris, wnodes, tshade, tclass, mats, rtab, ems, emtri, emcdf;  // tris: both BVHs' triangles
    DevBuf env, envtex, envtab;  // environment emitter: GEnv record, texels, CDFs + row weights
    bool has_env = false;
    // media (volpath)
    DevBuf media, density, tmed, majorant, tcheap;
    bool diffuse_null = false;  // every material diffuse or null: VolDev::models (PG_VOL_MODELS=0 turns it off)
    int32_t cam_medium = -1;
    uint32_t num_media = 0;
    DevBuf vol_rad, vol_ovf, vol_work;  // per-item radiance, traversal-stack overflow, counter + stats
    DevBuf vol_vtx;                     // guided volpath training vertices (48 B each)
    uint64_t vol_vtx_cap = 0;
    // volumetric wavefront (PG_VOL_WAVEFRONT) lanes
    VolLane vlanes[PG_MAX_LANES];
    hipEvent_t vw_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // stage timing (kernel_timing)
    uint32_t vol_cap = 0;
    uint32_t num_tris = 0, num_mats = 0;
    uint32_t bvh_top_nodes = 0;  // breadth-first top levels of the binary BVH (staged in LDS by k_trace)
    std::vector<GMat> host_mats;
    float scene_lo[3] = {0, 0, 0}, scene_hi[3] = {0, 0, 0};
    // shard
    std::vector<uint32_t> local_pixels;
    DevBuf d_local_pixels;
    DevBuf d_band_pixels;  // the surface path's order of the same pixels (cameraBands)
    // path state
    Lane lanes[PG_MAX_LANES];
    int nlanes = PG_DEFAULT_LANES;
    hipEvent_t film_order = nullptr;  // last chunk's film + record commit (keeps them in chunk order)
    hipEvent_t pass_start = nullptr;
    uint64_t rec_bound = 0;           // upper bound of the device-side record count
    EventPair timing;                 // context-stream kernel timing (splat)
    // film
    DevBuf film, film_sq;
    DevBuf aov_albedo, aov_normal;  // per-pixel denoiser feature sums (pg_config.aovs)
    // records
    DevBuf records, rec_count;
    uint64_t rec_capacity = 0;
    uint64_t rec_host_count = 0;
    DevBuf ext_records;
    // sd-tree
    pgh::SdTree sd;
    // the device SD-tree lives in one allocation (uploadSd): snodes | meta | qnode {energies, children} |
    // bchild | bsum | count | frac | jump.  bsum, count and frac are contiguous -- the pg_get_tree_stats
    // vector -- so the statistics move in one copy (download, all-reduce in place), the host-built
    // part in one upload, and the jump grid is built on the device from the S-tree.
    DevBuf sd_blob;
    struct {
        uint32_t *snodes = nullptr, *meta = nullptr, *qnode = nullptr, *bchild = nullptr, *jump = nullptr;
        uint64_t *bsum = nullptr, *count = nullptr, *frac = nullptr;  // frac: pgh::kFracStats u64 per leaf
    } sdp;
    int sd_jump_bits = 0;
    PinnedBuf sd_stage;
    bool sd_dirty = true;
    // multi-GPU: RCCL communicator over the job's ranks (pg_comm_init), one per context/device
    ncclComm_t comm = nullptr;
    // stats
    pg_stats stats{};
};

thread_local std::string g_tls_err;

pg_status fail(Ctx *c, pg_status code, const std::string &msg) {
    if (c) c->err = msg;
    else g_tls_err = msg;
    return code;
}

#define HIPC(c, expr)                                                                                              \
    do {                                                                                                           \
        hipError_t e_ = (expr);                                                                                    \
        if (e_ != hipSuccess)                                                                                      \
            return fail((c), e_ == hipErrorOutOfMemory ? PG_ERR_OOM : PG_ERR_HIP,                                  \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                                        \
    } while (0)

inline float luminance(const float *c) { return c[0] * 0.212671f + c[1] * 0.715160f + c[2] * 0.072169f; }

// fresnelDielectricExt (util.cpp:653-683), host copy for BSDF::configure()-time constants
float fresnelDielectricExtH(float cosThetaI_, float eta) {
    if (eta == 1) return 0.0f;
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta;
    float cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) return 1.0f;
    float cosThetaI = std::fabs(cosThetaI_);
    float cosThetaT = std::sqrt(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    return 0.5f * (Rs * Rs + Rp * Rp);
}
// fresnelDiffuseReflectance(eta, fast=false) (util.cpp:816-870): 2 * int_0^1 F(sqrt(xi)) dxi ... as
// the integral of F over the cosine-weighted hemisphere, by composite Simpson in double.
float fresnelDiffuseReflectanceH(float eta) {
    const int N = 2000;
    double h = 1.0 / N, acc = 0;
    for (int i = 0; i <= N; ++i) {
        double w = (i == 0 || i == N) ? 1 : ((i & 1) ? 4 : 2);
        acc += w * fresnelDielectricExtH((float)std::sqrt(i * h), eta);
    }
    return (float)(acc * h / 3.0);
}

// BSDF::configure(): type bits and derived constants of each plugin
GMat makeGMat(const pg_material &m) {
    GMat g{};
    g.model = m.type;
    g.dist = m.distribution;
    g.flags = m.flags;
    g.alpha_u = std::max(m.alpha_u, 1e-4f);  // MicrofacetDistribution clamps alpha (microfacet.h:70-72)
    g.alpha_v = std::max(m.alpha_v, 1e-4f);
    g.eta = m.int_ior / m.ext_ior;
    g.invEta = 1.0f / g.eta;
    g.invEta2 = 1.0f / (g.eta * g.eta);
    for (int i = 0; i < 4; ++i) {
        g.diff[i] = m.diffuse_reflectance[i];
        g.spec[i] = m.specular_reflectance[i];
        g.trans[i] = m.specular_transmittance[i];
        g.ceta[i] = m.eta[i];
        g.ck[i] = m.k[i];
    }
    uint32_t sides = 0x8000u;  // EFrontSide
    switch (m.type) {
        case PG_BSDF_DIFFUSE: g.type = 0x2; break;                       // EDiffuseReflection
        case PG_BSDF_CONDUCTOR: g.type = 0x20; break;                    // EDeltaReflection
        case PG_BSDF_ROUGHCONDUCTOR: g.type = 0x8; break;                // EGlossyReflection
        case PG_BSDF_DIELECTRIC: g.type = 0x20 | 0x40; sides |= 0x10000u; break;
        case PG_BSDF_ROUGHDIELECTRIC: g.type = 0x8 | 0x10; sides |= 0x10000u; break;
        case PG_BSDF_PLASTIC: {
            g.type = 0x20 | 0x2;
            g.fdrInt = fresnelDiffuseReflectanceH(1 / g.eta);
            float dAvg = luminance(m.diffuse_reflectance), sAvg = luminance(m.specular_reflectance);
            g.specWeight = sAvg / (dAvg + sAvg);
            break;
        }
        case PG_BSDF_NULL: g.type = 0x1; sides |= 0x10000u; break;  // ENull, both sides (null.cpp:40)
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:258-307; table + fdrInt set by the caller
            g.type = 0x8 | 0x2;         // EGlossyReflection | EDiffuseReflection
            float dAvg = luminance(m.diffuse_reflectance), sAvg = luminance(m.specular_reflectance);
            g.specWeight = sAvg / (dAvg + sAvg);
            break;
        }
        default: g.type = 0;
    }
    if (m.flags & PG_MAT_TWOSIDED) sides |= 0x10000u;
    g.type |= sides;
    {  // BSDF::getAlbedo (as bsdfAlbedo in pg_kernels.hip), max channel: the guide-fraction bound
        float a[3];
        for (int i = 0; i < 3; ++i) {
            const float d = g.diff[i], s = g.spec[i], t = g.trans[i];
            switch (m.type) {
                case PG_BSDF_DIFFUSE: a[i] = d; break;
                case PG_BSDF_CONDUCTOR:
                case PG_BSDF_ROUGHCONDUCTOR: a[i] = s; break;
                case PG_BSDF_DIELECTRIC: a[i] = t * 0.5f + s * 0.5f; break;
                case PG_BSDF_ROUGHDIELECTRIC: a[i] = s * 0.5f + t * 0.5f; break;
                case PG_BSDF_PLASTIC: a[i] = d * 0.5f + s * 0.5f; break;
                case PG_BSDF_ROUGHPLASTIC: a[i] = s * 0.5f + d * 0.5f; break;
                default: a[i] = 0.0f;
            }
        }
        g.wbound = std::max(std::max(a[0], a[1]), a[2]);
    }
    return g;
}

// Shading record of triangle t (pg_layout.h PG_TRI_SHADE_F4)
void packShade(float *o, const float *P, const float *N, const uint32_t *I, uint32_t t, uint32_t bits, uint32_t orig) {
    const uint32_t i0 = I[3 * (size_t)t], i1 = I[3 * (size_t)t + 1], i2 = I[3 * (size_t)t + 2];
    const float *p0 = P + 3 * (size_t)i0, *p1 = P + 3 * (size_t)i1, *p2 = P + 3 * (size_t)i2;
    float n0[3], n1[3], n2[3];
    if (N) {
        for (int a = 0; a < 3; ++a) {
            n0[a] = N[3 * (size_t)i0 + a];
            n1[a] = N[3 * (size_t)i1 + a];
            n2[a] = N[3 * (size_t)i2 + a];
        }
    } else {  // face normal (TriMesh without vertex normals)
        float e1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
        float e2[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
        float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        float l = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        for (int a = 0; a < 3; ++a) n0[a] = n1[a] = n2[a] = l > 0 ? c[a] / l : 0.0f;
    }
    float b, o2;
    std::memcpy(&b, &bits, 4);
    std::memcpy(&o2, &orig, 4);
    float rec[20] = {p0[0], p0[1], p0[2], b,     p1[0], p1[1], p1[2], n2[2], p2[0], p2[1],
                     p2[2], o2,    n0[0], n0[1], n0[2], n1[0], n1[1], n1[2], n2[0], n2[1]};
    std::memcpy(o, rec, sizeof rec);
}

template <class T>
pg_status upload(Ctx *c, DevBuf &b, const std::vector<T> &v) {
    size_t n = std::max<size_t>(v.size() * sizeof(T), 16);
    HIPC(c, b.alloc(n));
    if (!v.empty()) HIPC(c, hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return PG_OK;
}

SceneDev sceneView(const Ctx *c) {
    return SceneDev{c->nodes.as<float4>(), c->tris.as<float4>(), c->wnodes.as<float4>(), c->tris.as<float4>(),
                    c->tshade.as<float4>(), c->tclass.as<uint8_t>(),
                    c->mats.as<GMat>(),
                    c->ems.as<GEmitter>(), c->emtri.as<float4>(), c->emcdf.as<float>(),
                    c->has_env ? c->env.as<GEnv>() : nullptr, c->bvh_top_nodes};
}
SDDev sdView(const Ctx *c) {
    SDDev s{};
    s.snodes = reinterpret_cast<const uint2 *>(c->sdp.snodes);
    s.meta = reinterpret_cast<const uint4 *>(c->sdp.meta);
    s.qsum = reinterpret_cast<const float4 *>(c->sdp.qnode);
    s.qchild = reinterpret_cast<const uint4 *>(reinterpret_cast<const float4 *>(c->sdp.qnode) + 1);
    s.bchild = reinterpret_cast<const uint4 *>(c->sdp.bchild);
    s.bsum = reinterpret_cast<unsigned long long *>(c->sdp.bsum);
    s.count = reinterpret_cast<unsigned long long *>(c->sdp.count);
    s.jump = c->sdp.jump;
    s.frac = reinterpret_cast<unsigned long long *>(c->sdp.frac);
    s.jump_bits = c->sd_jump_bits;
    s.learned = c->cfg.bsdf_fraction_bound == PG_FRACTION_LEARNED ? 1 : 0;
    s.alpha0 = c->cfg.bsdf_sampling_fraction;
    for (int a = 0; a < 3; ++a) s.lo[a] = c->sd.lo[a];
    s.extent = c->sd.extent;
    s.built = c->sd.built ? 1 : 0;
    return s;
}
PathDev pathView(const Lane *c) {
    return PathDev{c->ray_o.as<float4>(), c->ray_d.as<float4>(), c->hit.as<float4>(), c->thr.as<float4>(),
                   c->rad.as<float4>(),   c->prev.as<float4>(),  c->pinfo.as<uint4>(),
                   c->sh_d.as<float4>(),  c->sh_c.as<float4>(),  c->vtx.as<float4>(), c->stack_ovf.as<uint32_t>(),
                   c->P,                  c->vtxP,               c->aov.as<float4>()};
}

pg_status uploadSd(Ctx *c) {
    // the device layout (Ctx::sd_blob) is written straight into the pinned staging buffer at the same
    // offsets, then copied in one piece; the jump grid is derived on the device from the S-tree
    const pgh::SdTree &t = c->sd;
    const size_t R = (size_t)1 << pgh::SdTree::kJumpBits;
    const size_t nl = t.leaves.size(), ns = t.samplingNodes(), nb = t.buildingNodes();
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t oMeta = up(4 * t.snode.size()), oQ = oMeta + up(16 * nl), oB = oQ + up(32 * ns);
    const size_t oStats = oB + up(16 * nb), statBytes = 32 * nb + 8 * nl + 8 * pgh::kFracStats * nl;
    const size_t oJump = oStats + up(statBytes), total = oJump + 4 * R * R * R;
    HIPC(c, c->sd_stage.reserve(oJump));
    uint8_t *h = (uint8_t *)c->sd_stage.p;
    uint64_t *hs = (uint64_t *)(h + oStats);
    t.flattenInto(pgh::SdTree::Layout{(uint32_t *)h, (uint32_t *)(h + oMeta), (uint32_t *)(h + oQ),
                                      (uint32_t *)(h + oB), hs, hs + 4 * nb, nullptr, hs + 4 * nb + nl});
    HIPC(c, c->sd_blob.grow(total));
    uint8_t *d = (uint8_t *)c->sd_blob.p;
    c->sdp.snodes = (uint32_t *)d;
    c->sdp.meta = (uint32_t *)(d + oMeta);
    c->sdp.qnode = (uint32_t *)(d + oQ);
    c->sdp.bchild = (uint32_t *)(d + oB);
    c->sdp.bsum = (uint64_t *)(d + oStats);
    c->sdp.count = c->sdp.bsum + 4 * nb;
    c->sdp.frac = c->sdp.count + nl;
    c->sdp.jump = (uint32_t *)(d + oJump);
    HIPC(c, hipMemcpyAsync(d, h, oJump, hipMemcpyHostToDevice, c->stream));
    pg_launch_sd_jump(c->stream, c->sdp.snodes, pgh::SdTree::kJumpBits, c->sdp.jump);
    HIPC(c, hipGetLastError());
    HIPC(c, hipStreamSynchronize(c->stream));
    c->stats.stree_nodes = t.snode.size() / 2;
    c->stats.dtree_nodes = ns;
    c->sd_jump_bits = pgh::SdTree::kJumpBits;
    c->sd_dirty = false;
    return PG_OK;
}

// pull device-side building sums + counts (+ fraction statistics) into the host tree: one copy
pg_status downloadSd(Ctx *c) {
    const size_t nb = c->sd.buildingNodes(), nl = c->sd.leaves.size();
    const size_t bytes = 32 * nb + 8 * nl + 8 * pgh::kFracStats * nl;
    HIPC(c, c->sd_stage.reserve(bytes));
    uint64_t *bsum = (uint64_t *)c->sd_stage.p, *cnt = bsum + 4 * nb, *frac = cnt + nl;
    HIPC(c, hipMemcpyAsync(bsum, c->sdp.bsum, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> cnt32(nl);
    for (size_t i = 0; i < nl; ++i) cnt32[i] = (uint32_t)std::min<uint64_t>(cnt[i], 0xFFFFFFFFu);
    c->sd.absorb(bsum, cnt32.data(), frac);
    return PG_OK;
}

EventPair nextEvents(Lane *l, LaunchKind kind) {
    std::vector<EventPair> &pool = l->ev[l->evcur];
    std::vector<uint8_t> &kinds = l->evkind[l->evcur];
    kinds.resize(l->evused[l->evcur] + 1);
    kinds[l->evused[l->evcur]] = (uint8_t)kind;
    if (l->evused[l->evcur] == pool.size()) {
        EventPair e;
        (void)hipEventCreate(&e.a);
        (void)hipEventCreate(&e.b);
        pool.push_back(e);
    }
    return pool[l->evused[l->evcur]++];
}

// ray-sorted trace queues (A/B switch PG_RAY_SORT=1): k_shade writes a ray order key per queued path and
// a counting sort groups every shard of the next closest-hit queue by direction octant + origin cell
bool raySortEnabled() {
    static const bool on = [] {
        const char *e = std::getenv("PG_RAY_SORT");
        return e && std::atoi(e) != 0;
    }();
    return on;
}
constexpr uint32_t kRaySortMinShard = 1024;  // smaller bounces trace unsorted (the sort's launches cost more)

// the tail of a chunk (k_tail): at most this many live paths left -> one launch finishes them all
// instead of one launch pair + count readback per bounce (PG_TAIL_PATHS overrides; 0 = off)
uint32_t tailPaths() {
    static const uint32_t n = [] {
        const char *e = std::getenv("PG_TAIL_PATHS");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : (uint32_t)1 << 17;  // profiles/r03n_*: 2^17 vs 2^16 +0.3 %
    }();
    return n;
}

// training-vertex slots per path of a pass (only recording passes write training vertices)
int vertexSlots(const Ctx *c, bool rec) { return rec ? std::max(0, std::min(c->cfg.record_max_vertices, 64)) : 0; }

// release every lane's path state (streams, events and counters stay)
void releasePaths(Ctx *c) {
    for (int li = 0; li < c->nlanes; ++li) {
        Lane &l = c->lanes[li];
        for (DevBuf *b : {&l.ray_o, &l.ray_d, &l.hit, &l.thr, &l.rad, &l.prev, &l.pinfo, &l.sh_d, &l.sh_c,
                          &l.vtx, &l.q0, &l.q1, &l.qs, &l.class_q, &l.aov, &l.qkey, &l.qsorted})
            b->release();
        l.P = 0;
        l.vtx_slots = 0;
        l.vtxP = 0;
    }
}

// path-state capacity of every lane for chunks of up to `want` paths; recording passes also need
// vertex slots for `want` paths (a non-recording pass never allocates them: the 2^25-path chunks of
// a final render would need ~51 GB per lane)
pg_status ensurePaths(Ctx *c, uint32_t want, bool rec) {
    const int vslots = vertexSlots(c, rec);
    for (int li = 0; li < c->nlanes; ++li) {
        Lane &l = c->lanes[li];
        if (!l.stream) {
            HIPC(c, hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking));
            HIPC(c, hipEventCreateWithFlags(&l.ready, hipEventDisableTiming));
            HIPC(c, hipEventCreateWithFlags(&l.done, hipEventDisableTiming));
            HIPC(c, hipHostMalloc((void **)&l.h_counts, kCounterWords * 4, hipHostMallocDefault));
            HIPC(c, hipHostMalloc((void **)&l.h_stats, kCounterWords * 4, hipHostMallocDefault));
            HIPC(c, l.counters.alloc(kCounterWords * 4));
            HIPC(c, l.stack_ovf.alloc(2 * pg_stack_overflow_words(0) * 4));  // k_rays: two launches' worth
            HIPC(c, l.tail_stats.alloc(32));
            HIPC(c, hipHostMalloc((void **)&l.h_tail, 32, hipHostMallocDefault));
        }
        const bool aovMissing = c->cfg.aovs && !l.aov.p;
        if (vslots > 0 && (vslots > l.vtx_slots || want > l.vtxP)) {
            const int vs = std::max(vslots, l.vtx_slots);
            const uint32_t vp = std::max(want, l.vtxP);
            HIPC(c, l.vtx.alloc((size_t)vs * vp * 16 * PG_VTX_F4));
            l.vtx_slots = vs;
            l.vtxP = vp;
        }
        if (want <= l.P && !aovMissing) continue;
        const uint32_t P = std::max(want, l.P);
        size_t f4 = (size_t)P * 16;
        HIPC(c, l.ray_o.alloc(f4));
        HIPC(c, l.ray_d.alloc(f4));
        HIPC(c, l.hit.alloc(f4));
        HIPC(c, l.thr.alloc(f4));
        HIPC(c, l.rad.alloc(f4));
        HIPC(c, l.prev.alloc(f4));
        HIPC(c, l.pinfo.alloc(f4));
        HIPC(c, l.sh_d.alloc(f4));
        HIPC(c, l.sh_c.alloc(f4));
        const size_t qbytes = (size_t)PG_QSHARDS * pg_queue_stride(P) * 4;
        HIPC(c, l.q0.alloc(qbytes));
        HIPC(c, l.q1.alloc(qbytes));
        HIPC(c, l.qs.alloc(qbytes));
        HIPC(c, l.class_q.alloc((size_t)PG_NUM_CLASSES * qbytes));
        if (c->cfg.aovs) HIPC(c, l.aov.alloc((size_t)P * 16));
        if (raySortEnabled()) {
            HIPC(c, l.qkey.alloc(qbytes / 2));
            HIPC(c, l.qsorted.alloc(qbytes));
            HIPC(c, l.rsort_hist.alloc((size_t)PG_QSHARDS * PG_RAY_SORT_BINS * 4));
        }
        l.P = P;
    }
    return PG_OK;
}

pg_status ensureRecords(Ctx *c, uint64_t want) {
    if (want <= c->rec_capacity) return PG_OK;
    uint64_t cap = std::max<uint64_t>(want + want / 2, 1u << 20);
    DevBuf nb;
    HIPC(c, nb.alloc(cap * sizeof(pg_record)));
    if (c->rec_host_count)
        HIPC(c, hipMemcpyAsync(nb.p, c->records.p, c->rec_host_count * sizeof(pg_record), hipMemcpyDeviceToDevice,
                               c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    std::swap(c->records.p, nb.p);
    std::swap(c->records.bytes, nb.bytes);
    c->rec_capacity = cap;
    return PG_OK;
}

}  // namespace

extern "C" {

int32_t pg_abi_version(void) { return PG_ABI_VERSION; }

// HeterogeneousMedium / GridDataSource preconditions (heterogeneous.cpp:227-242: densities in
// [0, 1]; hg.cpp:47-50: |g| < 1).  The optical-depth bound keeps one Woodcock walk across the
// grid box below ~1e7 steps (the reference has no bound; a thicker medium is rejected).
pg_status validateMedium(Ctx *c, const pg_medium &pm, uint32_t m) {
    const std::string id = "pg_upload_scene: medium " + std::to_string(m) + ": ";
    if (pm.type != PG_MEDIUM_HETEROGENEOUS) return fail(c, PG_ERR_INVALID, id + "unknown type");
    if (!pm.density || pm.res[0] < 1 || pm.res[1] < 1 || pm.res[2] < 1 ||
        (uint64_t)pm.res[0] * pm.res[1] * pm.res[2] > (1ull << 30))
        return fail(c, PG_ERR_INVALID, id + "bad density grid");
    double diag2 = 0;
    for (int a = 0; a < 3; ++a) {
        if (!(pm.aabb_max[a] > pm.aabb_min[a]) || !std::isfinite(pm.aabb_min[a]) || !std::isfinite(pm.aabb_max[a]))
            return fail(c, PG_ERR_INVALID, id + "empty or non-finite AABB");
        diag2 += (double)(pm.aabb_max[a] - pm.aabb_min[a]) * (pm.aabb_max[a] - pm.aabb_min[a]);
        if (!(pm.albedo[a] >= 0) || !std::isfinite(pm.albedo[a])) return fail(c, PG_ERR_INVALID, id + "bad albedo");
    }
    if (!(pm.scale > 0) || !std::isfinite(pm.scale)) return fail(c, PG_ERR_INVALID, id + "scale must be finite and > 0");
    if (pm.scale * std::sqrt(diag2) > 1e7) return fail(c, PG_ERR_INVALID, id + "optical depth too large");
    if (!(pm.g > -1 && pm.g < 1)) return fail(c, PG_ERR_INVALID, id + "HG g must lie in (-1, 1)");
    const size_t n = (size_t)pm.res[0] * pm.res[1] * pm.res[2];
    for (size_t i = 0; i < n; ++i)
        if (!(pm.density[i] >= 0.0f && pm.density[i] <= 1.0f)) return fail(c, PG_ERR_INVALID, id + "density outside [0, 1]");
    return PG_OK;
}

// per-cell maxima of the density grid (cell c covers voxels [c * CELL - 1, (c + 1) * CELL + 1] per
// axis, clamped), times scale; appended to `out` in cell order (x fastest)
void buildMajorants(const pg_medium &pm, const GMedium &gm, std::vector<float> &out) {
    const int C = PG_MAJORANT_CELL;
    const int r[3] = {(int)pm.res[0], (int)pm.res[1], (int)pm.res[2]}, n[3] = {(int)gm.mx, (int)gm.my, (int)gm.mz};
    // separable running maxima: along x, then y, then z, each over the cell's voxel window
    auto win = [&](int a, int cidx, int &lo, int &hi) {
        lo = std::max(0, cidx * C - 1);
        hi = std::min(r[a] - 1, (cidx + 1) * C + 1);
    };
    std::vector<float> ax((size_t)n[0] * r[1] * r[2]), ay((size_t)n[0] * n[1] * r[2]);
    for (int z = 0; z < r[2]; ++z)
        for (int y = 0; y < r[1]; ++y) {
            const float *row = pm.density + ((size_t)z * r[1] + y) * r[0];
            for (int cx = 0; cx < n[0]; ++cx) {
                int lo, hi;
                win(0, cx, lo, hi);
                float m = 0;
                for (int x = lo; x <= hi; ++x) m = std::max(m, row[x]);
                ax[((size_t)z * r[1] + y) * n[0] + cx] = m;
            }
        }
    for (int z = 0; z < r[2]; ++z)
        for (int cy = 0; cy < n[1]; ++cy) {
            int lo, hi;
            win(1, cy, lo, hi);
            for (int cx = 0; cx < n[0]; ++cx) {
                float m = 0;
                for (int y = lo; y <= hi; ++y) m = std::max(m, ax[((size_t)z * r[1] + y) * n[0] + cx]);
                ay[((size_t)z * n[1] + cy) * n[0] + cx] = m;
            }
        }
    const size_t base = out.size();
    out.resize(base + (size_t)n[0] * n[1] * n[2]);
    for (int cz = 0; cz < n[2]; ++cz) {
        int lo, hi;
        win(2, cz, lo, hi);
        for (int cy = 0; cy < n[1]; ++cy)
            for (int cx = 0; cx < n[0]; ++cx) {
                float m = 0;
                for (int z = lo; z <= hi; ++z) m = std::max(m, ay[((size_t)z * n[1] + cy) * n[0] + cx]);
                out[base + ((size_t)cz * n[1] + cy) * n[0] + cx] = m * pm.scale;
            }
    }
}

pg_status pg_config_default(pg_config *c) {
    if (!c) return PG_ERR_INVALID;
    std::memset(c, 0, sizeof *c);
    c->device = 0;
    c->max_depth = -1;
    c->rr_depth = 5;
    c->use_nee = 1;
    c->hide_emitters = 0;
    c->strict_normals = 0;
    c->max_component_value = std::numeric_limits<float>::infinity();
    c->seed = 1337;
    c->guiding = 0;
    c->bsdf_sampling_fraction = 0.5f;
    c->s_tree_threshold = 12000.0f;
    c->d_tree_threshold = 0.01f;
    c->d_tree_max_depth = 20;
    c->record_max_vertices = 32;
    c->rank = 0;
    c->world_size = 1;
    c->tile_size = 32;
    c->max_paths_in_flight = 0;
    c->gpu_depth_cap = 1024;
    c->path_lanes = 0;
    c->integrator = PG_INTEGRATOR_PATH;
    c->distance_guiding = 0.25f;
    c->bsdf_fraction_bound = PG_FRACTION_FIXED;
    c->kernel_timing = 0;
    c->volpath_exact_mis = 0;
    c->tail_paths = 0;
    c->glossy_prior = 0;
    return PG_OK;
}

const char *pg_last_error(void *ctx) {
    if (!ctx) return g_tls_err.c_str();
    return ((Ctx *)ctx)->err.c_str();
}

pg_status pg_create(const pg_config *cfg, void **out) {
    if (!cfg || !out) return fail(nullptr, PG_ERR_INVALID, "pg_create: null argument");
    *out = nullptr;
    if (cfg->world_size < 1 || cfg->rank < 0 || cfg->rank >= cfg->world_size)
        return fail(nullptr, PG_ERR_INVALID, "pg_create: bad rank/world_size");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(nullptr, PG_ERR_NO_DEVICE, "pg_create: no HIP device visible");
    if (cfg->device < 0 || cfg->device >= n) return fail(nullptr, PG_ERR_INVALID, "pg_create: bad device ordinal");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess)
        return fail(nullptr, PG_ERR_HIP, "pg_create: hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, PG_ERR_NO_DEVICE, std::string("pg_create: device is ") + prop.gcnArchName + ", need gfx950");
    Ctx *c = new Ctx();
    c->cfg = *cfg;
    if (c->cfg.tile_size == 0) c->cfg.tile_size = 32;
    if (c->cfg.gpu_depth_cap <= 0) c->cfg.gpu_depth_cap = 1024;
    if (c->cfg.integrator == PG_INTEGRATOR_PATH) {  // the surface wavefront's per-bounce counter blocks
        if (c->cfg.gpu_depth_cap > (int32_t)kMaxBounces - 2) c->cfg.gpu_depth_cap = (int32_t)kMaxBounces - 2;
        if (c->cfg.max_depth > (int32_t)kMaxBounces - 3) {
            delete c;
            return fail(nullptr, PG_ERR_INVALID,
                        "pg_create: max_depth above " + std::to_string(kMaxBounces - 3) +
                            " is not supported by the path integrator (use -1 for unbounded paths)");
        }
    }
    if (c->cfg.path_lanes < 0 || c->cfg.path_lanes > PG_MAX_LANES) {
        delete c;
        return fail(nullptr, PG_ERR_INVALID, "pg_create: path_lanes must be 0..4");
    }
    c->nlanes = c->cfg.path_lanes ? c->cfg.path_lanes : PG_DEFAULT_LANES;
    if (c->cfg.integrator != PG_INTEGRATOR_PATH && c->cfg.integrator != PG_INTEGRATOR_VOLPATH) {
        delete c;
        return fail(nullptr, PG_ERR_INVALID, "pg_create: unknown integrator");
    }
    if (c->cfg.bsdf_fraction_bound < PG_FRACTION_FIXED || c->cfg.bsdf_fraction_bound > PG_FRACTION_LEARNED) {
        delete c;
        return fail(nullptr, PG_ERR_INVALID, "pg_create: unknown bsdf_fraction_bound");
    }
    if (c->cfg.volume_majorant != PG_MAJORANT_GRID && c->cfg.volume_majorant != PG_MAJORANT_GLOBAL) {
        delete c;
        return fail(nullptr, PG_ERR_INVALID, "pg_create: unknown volume_majorant");
    }
    if (c->cfg.aovs && c->cfg.integrator != PG_INTEGRATOR_PATH) {
        delete c;
        return fail(nullptr, PG_ERR_INVALID, "pg_create: aovs need the path integrator");
    }
    if (!(c->cfg.distance_guiding >= 0.0f && c->cfg.distance_guiding < 1.0f)) {
        delete c;
        return fail(nullptr, PG_ERR_INVALID, "pg_create: distance_guiding must be in [0, 1)");
    }
    if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->film_order, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->pass_start, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return fail(nullptr, PG_ERR_HIP, "pg_create: stream/pinned allocation failed");
    }
    *out = c;
    return PG_OK;
}

pg_status pg_destroy(void *ctx) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return PG_OK;
    (void)hipSetDevice(c->cfg.device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t &e : c->vw_ev)
        if (e) (void)hipEventDestroy(e);
    for (VolLane &l : c->vlanes) {
        if (l.nstream) (void)hipStreamSynchronize(l.nstream);
        if (l.stream) (void)hipStreamSynchronize(l.stream);
        if (l.ready) (void)hipEventDestroy(l.ready);
        if (l.vdone) (void)hipEventDestroy(l.vdone);
        if (l.ndone) (void)hipEventDestroy(l.ndone);
        if (l.nstream) (void)hipStreamDestroy(l.nstream);
        if (l.stream) (void)hipStreamDestroy(l.stream);
    }
    for (Lane &l : c->lanes) {
        if (l.stream) (void)hipStreamSynchronize(l.stream);
        for (auto &pool : l.ev)
            for (auto &e : pool) {
                (void)hipEventDestroy(e.a);
                (void)hipEventDestroy(e.b);
            }
        if (l.ready) (void)hipEventDestroy(l.ready);
        if (l.done) (void)hipEventDestroy(l.done);
        if (l.h_counts) (void)hipHostFree(l.h_counts);
        if (l.h_stats) (void)hipHostFree(l.h_stats);
        if (l.h_tail) (void)hipHostFree(l.h_tail);
        if (l.stream) (void)hipStreamDestroy(l.stream);
    }
    if (c->timing.a) (void)hipEventDestroy(c->timing.a);
    if (c->timing.b) (void)hipEventDestroy(c->timing.b);
    if (c->film_order) (void)hipEventDestroy(c->film_order);
    if (c->pass_start) (void)hipEventDestroy(c->pass_start);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return PG_OK;
}

pg_status pg_cancel(void *ctx) {
    if (!ctx) return PG_ERR_INVALID;
    ((Ctx *)ctx)->cancel.store(true);
    return PG_OK;
}

// the camera's XCD-banded shard map (pg_kernels.h pg_banded_shard_count) over PG_CAMERA_BANDS bands of the local
// pixels (0: the interleaved map): band g goes to XCD group g % 8, so with more than 8 bands each XCD takes
// every 8th band (the surface path's pixel order d_band_pixels groups them).  Paths are pure functions of
// (pixel, sample), so films and trees do not depend on it
uint32_t cameraBands() {
    const char *e = std::getenv("PG_CAMERA_BANDS");
    return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
}

pg_status pg_upload_scene(void *ctx, const pg_scene_desc *d) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !d) return fail(c, PG_ERR_INVALID, "pg_upload_scene: null argument");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!d->positions || !d->indices || !d->shapes || !d->materials || d->num_triangles == 0)
        return fail(c, PG_ERR_INVALID, "pg_upload_scene: empty scene");
    if (d->camera.width == 0 || d->camera.height == 0) return fail(c, PG_ERR_INVALID, "pg_upload_scene: empty film");
    const uint32_t nt = d->num_triangles;
    for (uint64_t i = 0; i < 3ull * nt; ++i)
        if (d->indices[i] >= d->num_vertices) return fail(c, PG_ERR_INVALID, "pg_upload_scene: index out of range");
    if (d->num_materials > 65535 || d->num_emitters > 65534 || d->num_media > 65534)
        return fail(c, PG_ERR_INVALID, "pg_upload_scene: too many materials/emitters/media");
    for (uint32_t m = 0; m < d->num_materials; ++m)
        if (d->materials[m].type >= PG_BSDF_COUNT || d->materials[m].distribution > PG_DIST_GGX)
            return fail(c, PG_ERR_INVALID, "pg_upload_scene: bad material type");
    if (d->num_media && !d->media) return fail(c, PG_ERR_INVALID, "pg_upload_scene: media missing");
    if (d->camera_medium < -1 || d->camera_medium >= (int32_t)d->num_media)
        return fail(c, PG_ERR_INVALID, "pg_upload_scene: bad camera medium");
    if (d->envmap && c->cfg.integrator != PG_INTEGRATOR_PATH)
        return fail(c, PG_ERR_INVALID, "pg_upload_scene: the volumetric integrator does not support an environment emitter");
    std::vector<GMedium> gmed;
    std::vector<size_t> denOff;
    size_t denTotal = 0;
    for (uint32_t m = 0; m < d->num_media; ++m) {
        const pg_medium &pm = d->media[m];
        if (pg_status vs = validateMedium(c, pm, m)) return vs;
        GMedium gm{};
        gm.resx = pm.res[0];
        gm.resy = pm.res[1];
        gm.resz = pm.res[2];
        gm.scale = pm.scale;
        gm.invMax = 1.0f / (pm.scale * 1.0f);  // maxDensity = scale * getMaximumFloatValue() = scale
        gm.g = pm.g;
        for (int a = 0; a < 3; ++a) {
            gm.lo[a] = pm.aabb_min[a];
            gm.hi[a] = pm.aabb_max[a];
            gm.gs[a] = (float)(pm.res[a] - 1) / (pm.aabb_max[a] - pm.aabb_min[a]);
            gm.go[a] = gm.gs[a] * -pm.aabb_min[a];
            gm.albedo[a] = pm.albedo[a];
        }
        denOff.push_back(denTotal);
        denTotal += (size_t)pm.res[0] * pm.res[1] * pm.res[2];
        gm.mx = std::max(1u, (pm.res[0] - 1 + PG_MAJORANT_CELL - 1) / PG_MAJORANT_CELL);
        gm.my = std::max(1u, (pm.res[1] - 1 + PG_MAJORANT_CELL - 1) / PG_MAJORANT_CELL);
        gm.mz = std::max(1u, (pm.res[2] - 1 + PG_MAJORANT_CELL - 1) / PG_MAJORANT_CELL);
        gmed.push_back(gm);
    }
    // per-triangle (material | emitter+1 << 16) from the shape partition
    std::vector<uint32_t> triBits(nt, 0xFFFFFFFFu);
    for (uint32_t s = 0; s < d->num_shapes; ++s) {
        const pg_shape &sh = d->shapes[s];
        if ((uint64_t)sh.tri_begin + sh.tri_count > nt || sh.material >= d->num_materials ||
            (sh.emitter >= 0 && (uint32_t)sh.emitter >= d->num_emitters) || sh.interior_medium < -1 ||
            sh.interior_medium >= (int32_t)d->num_media || sh.exterior_medium < -1 ||
            sh.exterior_medium >= (int32_t)d->num_media)
            return fail(c, PG_ERR_INVALID, "pg_upload_scene: bad shape");
        uint32_t bits = sh.material | ((uint32_t)(sh.emitter + 1) << 16);
        for (uint32_t t = 0; t < sh.tri_count; ++t) triBits[sh.tri_begin + t] = bits;
    }
    for (uint32_t t = 0; t < nt; ++t)
        if (triBits[t] == 0xFFFFFFFFu) return fail(c, PG_ERR_INVALID, "pg_upload_scene: triangle without a shape");

    pgh::BvhOut bvh;
    if (!pgh::buildBvh(d->positions, d->indices, nt, kStackDepth, bvh))
        return fail(c, PG_ERR_INVALID, "pg_upload_scene: BVH deeper than the traversal stack");
    std::vector<float> shade((size_t)4 * PG_TRI_SHADE_STRIDE * nt, 0.0f);
    std::vector<uint8_t> tclass(nt), tcheap(nt);
    c->diffuse_null = true;
    for (uint32_t i = 0; i < d->num_materials; ++i)
        if (d->materials[i].type != PG_BSDF_DIFFUSE && d->materials[i].type != PG_BSDF_NULL) c->diffuse_null = false;
    for (uint32_t k = 0; k < nt; ++k) {
        uint32_t t = bvh.order[k];
        packShade(&shade[4 * PG_TRI_SHADE_STRIDE * (size_t)k], d->positions, d->normals, d->indices, t, triBits[t], t);
        tclass[k] = (uint8_t)materialClass(d->materials[triBits[t] & 0xFFFFu].type);
        // volumetric wavefront: surfaces whose interaction skips the shadow walk through media (delta
        // BSDFs) or ends the path at once (emitters: black in the scenes here) -- VolDev::tcheap
        tcheap[k] = tclass[k] == PG_CLASS_DELTA || (triBits[t] >> 16) != 0;
    }
    // per BVH-order triangle: the shape's medium transition, (interior + 1) | (exterior + 1) << 16
    std::vector<uint32_t> tmed(nt, 0);
    {
        std::vector<uint32_t> shapeMed(nt, 0);
        for (uint32_t sidx = 0; sidx < d->num_shapes; ++sidx) {
            const pg_shape &sh = d->shapes[sidx];
            const uint32_t bits = (uint32_t)(sh.interior_medium + 1) | ((uint32_t)(sh.exterior_medium + 1) << 16);
            for (uint32_t t = 0; t < sh.tri_count; ++t) shapeMed[sh.tri_begin + t] = bits;
        }
        for (uint32_t k = 0; k < nt; ++k) tmed[k] = shapeMed[bvh.order[k]];
    }
    // emitters: compact triangle array + area CDF (double accumulation of fp32 areas)
    std::vector<GEmitter> ems;
    std::vector<float> emtri, emcdf;
    for (uint32_t e = 0; e < d->num_emitters; ++e) {
        const pg_emitter &pe = d->emitters[e];
        if (pe.shape >= d->num_shapes) return fail(c, PG_ERR_INVALID, "pg_upload_scene: emitter without shape");
        const pg_shape &sh = d->shapes[pe.shape];
        GEmitter g{};
        g.tri_begin = (uint32_t)(emtri.size() / 20);
        g.tri_count = sh.tri_count;
        g.cdf_begin = (uint32_t)emcdf.size();
        std::vector<double> cum(sh.tri_count + 1, 0.0);
        double acc = 0;
        for (uint32_t i = 0; i < sh.tri_count; ++i) {
            uint32_t t = sh.tri_begin + i;
            const float *a = d->positions + 3 * (size_t)d->indices[3 * (size_t)t];
            const float *b = d->positions + 3 * (size_t)d->indices[3 * (size_t)t + 1];
            const float *cc = d->positions + 3 * (size_t)d->indices[3 * (size_t)t + 2];
            float u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, v[3] = {cc[0] - a[0], cc[1] - a[1], cc[2] - a[2]};
            float x[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
            float area = 0.5f * std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
            acc += (double)area;
            cum[i + 1] = acc;
            size_t o = emtri.size();
            emtri.resize(o + 20);
            packShade(&emtri[o], d->positions, d->normals, d->indices, t, 0, t);
        }
        if (!(acc > 0)) return fail(c, PG_ERR_INVALID, "pg_upload_scene: emitter with zero area");
        for (uint32_t i = 0; i < sh.tri_count; ++i) emcdf.push_back((float)(cum[i] / acc));
        emcdf.push_back(1.0f);
        g.inv_area = 1.0f / (float)acc;
        for (int k = 0; k < 4; ++k) g.radiance[k] = pe.radiance[k];
        ems.push_back(g);
    }
    c->host_mats.clear();
    for (uint32_t m = 0; m < d->num_materials; ++m) c->host_mats.push_back(makeGMat(d->materials[m]));
    // roughplastic: rough-transmittance slice + internal diffuse Fresnel per material
    // (RoughPlastic::configure, roughplastic.cpp:283-299; ranges of rtrans.h checkEta/checkAlpha)
    std::vector<float> rtab;
    std::vector<std::pair<uint32_t, size_t>> rtabOf;
    for (uint32_t m = 0; m < d->num_materials; ++m) {
        const pg_material &pm = d->materials[m];
        if (pm.type != PG_BSDF_ROUGHPLASTIC) continue;
        GMat &gm = c->host_mats[m];
        if (pm.alpha_u != pm.alpha_v)
            return fail(c, PG_ERR_INVALID, "pg_upload_scene: roughplastic does not support anisotropic roughness");
        const float e = gm.eta < 1 ? 1 / gm.eta : gm.eta;
        if (!(e >= 1.0001f && e <= 4.0f) || !(gm.alpha_u <= 4.0f))
            return fail(c, PG_ERR_INVALID, "pg_upload_scene: roughplastic IOR or roughness outside the tabulated range");
        const size_t off = rtab.size();
        rtab.resize(off + pgh::kRoughTransSamples);
        pgh::roughTransmittance((int)pm.distribution, gm.alpha_u, gm.eta, &rtab[off], &gm.fdrInt);
        rtabOf.push_back({m, off});
    }

    pg_status s;
    if ((s = upload(c, c->rtab, rtab))) return s;
    for (auto &mo : rtabOf) c->host_mats[mo.first].rtrans = c->rtab.as<float>() + mo.second;
    c->bvh_top_nodes = std::min<uint32_t>(bvh.top_nodes, PG_BVH4 ? PG_BVH4_TOP_NODES : PG_BVH_TOP_NODES);
    if ((s = upload(c, c->nodes, bvh.nodes)) || (s = upload(c, c->tris, bvh.tris)) ||
        (s = upload(c, c->wnodes, bvh.wnodes)) || (s = upload(c, c->tshade, shade)) ||
        (s = upload(c, c->tclass, tclass)) ||
        (s = upload(c, c->mats, c->host_mats)) || (s = upload(c, c->ems, ems)) || (s = upload(c, c->emtri, emtri)) ||
        (s = upload(c, c->emcdf, emcdf)) || (s = upload(c, c->tmed, tmed)) || (s = upload(c, c->tcheap, tcheap)))
        return s;
    // densities: one buffer, each grid 256-B aligned (bricked, see pg_layout.h GMedium)
    {
        size_t words = 0, linMax = 0;
        std::vector<size_t> at;
        std::vector<float> stage;
        // corner-packed grids (pg_layout.h PG_DENSITY_CORNERS); a grid with a dimension of 1 has no
        // cell (every lookup is 0) and keeps no density
        for (uint32_t m = 0; m < d->num_media; ++m) {
            const pg_medium &pm = d->media[m];
            at.push_back(words);
            gmed[m].bx = (pm.res[0] + 3) / 4;
            gmed[m].by = (pm.res[1] + 3) / 4;
            const size_t lin = (size_t)pm.res[0] * pm.res[1] * pm.res[2];
            const size_t cells = (size_t)(pm.res[0] - 1) * (pm.res[1] - 1) * (pm.res[2] - 1);
            const size_t n = PG_DENSITY_BRICKS ? (size_t)gmed[m].bx * gmed[m].by * ((pm.res[2] + 3) / 4) * 64
                             : PG_DENSITY_CORNERS ? cells * 8 : lin;
            if (PG_DENSITY_CORNERS && cells) linMax = std::max(linMax, lin);
            words += (n + 63) & ~(size_t)63;
        }
        {
            // corner packing takes 8x the grid's memory plus a linear staging copy (pg_layout.h)
            const hipError_t e = c->density.grow(std::max<size_t>(words * 4, 256));
            if (e != hipSuccess)
                return fail(c, e == hipErrorOutOfMemory ? PG_ERR_OOM : PG_ERR_HIP,
                            "pg_upload_scene: cannot allocate " + std::to_string(words * 4) + " B of density" +
                                (PG_DENSITY_CORNERS ? " (corner-packed: 8 floats per cell)" : "") + ": " +
                                hipGetErrorString(e));
        }
        DevBuf linTmp;  // the linear grid of a corner-packed medium, expanded on the device
        if (linMax) HIPC(c, linTmp.alloc(linMax * 4));
        for (uint32_t m = 0; m < d->num_media; ++m) {
            const pg_medium &pm = d->media[m];
            const size_t n = (size_t)pm.res[0] * pm.res[1] * pm.res[2];
            if (PG_DENSITY_CORNERS) {
                HIPC(c, hipMemcpyAsync(linTmp.p, pm.density, n * 4, hipMemcpyHostToDevice, c->stream));
                pg_launch_density_corners(c->stream, linTmp.as<float>(), pm.res[0], pm.res[1], pm.res[2],
                                          c->density.as<float>() + at[m]);
                HIPC(c, hipGetLastError());
                HIPC(c, hipStreamSynchronize(c->stream));  // linTmp is reused by the next medium
            } else if (PG_DENSITY_BRICKS) {
                const uint32_t bx = gmed[m].bx, by = gmed[m].by, bz = (pm.res[2] + 3) / 4;
                stage.assign((size_t)bx * by * bz * 64, 0.0f);
                for (uint32_t z = 0; z < pm.res[2]; ++z)
                    for (uint32_t y = 0; y < pm.res[1]; ++y)
                        for (uint32_t x = 0; x < pm.res[0]; ++x)
                            stage[(((size_t)(z >> 2) * by + (y >> 2)) * bx + (x >> 2)) * 64 + (z & 3) * 16 + (y & 3) * 4 +
                                  (x & 3)] = pm.density[((size_t)z * pm.res[1] + y) * pm.res[0] + x];
                HIPC(c, hipMemcpy(c->density.as<float>() + at[m], stage.data(), stage.size() * 4, hipMemcpyHostToDevice));
            } else {
                HIPC(c, hipMemcpyAsync(c->density.as<float>() + at[m], pm.density, n * 4, hipMemcpyHostToDevice, c->stream));
            }
            gmed[m].density = c->density.as<float>() + at[m];
        }
        // majorant grids (PG_MAJORANT_GRID tracking): one buffer, per-medium offsets
        std::vector<float> maj;
        std::vector<size_t> majAt;
        for (uint32_t m = 0; m < d->num_media; ++m) {
            majAt.push_back(maj.size());
            buildMajorants(d->media[m], gmed[m], maj);
        }
        if ((s = upload(c, c->majorant, maj))) return s;
        for (uint32_t m = 0; m < d->num_media; ++m) gmed[m].maj = c->majorant.as<float>() + majAt[m];
        HIPC(c, hipStreamSynchronize(c->stream));  // the host density arrays are caller-owned
        if ((s = upload(c, c->media, gmed))) return s;
        c->num_media = d->num_media;
        c->cam_medium = d->camera_medium;
    }

    // camera (Transform::lookAt, transform.cpp:191-214) and integrator constants
    GParams &g = c->g;
    std::memset(&g, 0, sizeof g);
    const pg_camera &cam = d->camera;
    float dir[3] = {cam.target[0] - cam.origin[0], cam.target[1] - cam.origin[1], cam.target[2] - cam.origin[2]};
    float l = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    for (int a = 0; a < 3; ++a) dir[a] /= l;
    const float *up = cam.up;
    float left[3] = {up[1] * dir[2] - up[2] * dir[1], up[2] * dir[0] - up[0] * dir[2], up[0] * dir[1] - up[1] * dir[0]};
    l = std::sqrt(left[0] * left[0] + left[1] * left[1] + left[2] * left[2]);
    for (int a = 0; a < 3; ++a) left[a] /= l;
    float nup[3] = {dir[1] * left[2] - dir[2] * left[1], dir[2] * left[0] - dir[0] * left[2],
                    dir[0] * left[1] - dir[1] * left[0]};
    for (int a = 0; a < 3; ++a) {
        g.cam_o[a] = cam.origin[a];
        g.cam_left[a] = left[a];
        g.cam_up[a] = nup[a];
        g.cam_dir[a] = dir[a];
    }
    g.tan_half = std::tan(cam.fov_x_deg * 3.14159265358979323846f / 360.0f);
    g.aspect = (float)cam.width / (float)cam.height;
    g.near_clip = cam.near_clip;
    g.far_clip = cam.far_clip;
    g.width = cam.width;
    g.height = cam.height;
    g.num_emitters = d->num_emitters + (d->envmap ? 1u : 0u);
    g.num_materials = d->num_materials;

    // tile shard of this rank: 32x32 tiles dealt round-robin
    const uint32_t T = c->cfg.tile_size, tx = (cam.width + T - 1) / T, ty = (cam.height + T - 1) / T;
    c->local_pixels.clear();
    for (uint32_t t = 0; t < tx * ty; ++t) {
        if ((int32_t)(t % (uint32_t)c->cfg.world_size) != c->cfg.rank) continue;
        uint32_t x0 = (t % tx) * T, y0 = (t / tx) * T;
        const uint32_t x1 = std::min(x0 + T, cam.width), y1 = std::min(y0 + T, cam.height);
        // within a tile, PG_PIXEL_BLOCK^2 pixel blocks (one wave of camera rays per 8x8 block) in
        // row-major block order; 0 = plain row-major.  Per-pixel results do not depend on the order.
        const uint32_t B = PG_PIXEL_BLOCK > 0 ? PG_PIXEL_BLOCK : T;
        for (uint32_t by = y0; by < y1; by += B)
            for (uint32_t bx = x0; bx < x1; bx += B)
                for (uint32_t y = by; y < std::min(by + B, y1); ++y)
                    for (uint32_t x = bx; x < std::min(bx + B, x1); ++x) c->local_pixels.push_back(y * cam.width + x);
    }
    if ((s = upload(c, c->d_local_pixels, c->local_pixels))) return s;
    {  // the surface path's pixel order: bands {r, r + 8, r + 16, ...} of the local pixels as the r-th eighth
        const uint32_t nb = cameraBands(), np = (uint32_t)c->local_pixels.size();
        std::vector<uint32_t> bp;
        bp.reserve(np);
        if (nb > 8 && np >= kBandMinPixels) {
            for (uint32_t r = 0; r < 8; ++r)
                for (uint32_t gb = r; gb < nb; gb += 8)
                    for (uint32_t i = (uint32_t)((uint64_t)gb * np / nb); i < (uint32_t)((uint64_t)(gb + 1) * np / nb); ++i)
                        bp.push_back(c->local_pixels[i]);
        } else {
            bp = c->local_pixels;
        }
        if ((s = upload(c, c->d_band_pixels, bp))) return s;
    }
    size_t fb = (size_t)cam.width * cam.height * 16;
    HIPC(c, c->film.alloc(fb));
    HIPC(c, c->film_sq.alloc(fb));
    HIPC(c, hipMemsetAsync(c->film.p, 0, fb, c->stream));
    HIPC(c, hipMemsetAsync(c->film_sq.p, 0, fb, c->stream));
    if (c->cfg.aovs) {
        HIPC(c, c->aov_albedo.alloc(fb));
        HIPC(c, c->aov_normal.alloc(fb));
        HIPC(c, hipMemsetAsync(c->aov_albedo.p, 0, fb, c->stream));
        HIPC(c, hipMemsetAsync(c->aov_normal.p, 0, fb, c->stream));
    }
    HIPC(c, c->rec_count.alloc(16));
    HIPC(c, hipMemsetAsync(c->rec_count.p, 0, 16, c->stream));
    c->rec_host_count = 0;
    c->num_tris = nt;
    c->num_mats = d->num_materials;
    // Scene::getAABB(): the kd-tree's slightly enlarged bounds (gkdtree.h:1213-1220,
    // MTS_KD_AABB_EPSILON = 1e-3); the SD-tree covers this box
    for (int a = 0; a < 3; ++a) {
        const float eps = 1e-3f;
        float lo = bvh.lo[a], hi = bvh.hi[a];
        lo = lo - ((hi - lo) * eps + eps);
        hi = hi + ((hi - lo) * eps + eps);
        c->scene_lo[a] = lo;
        c->scene_hi[a] = hi;
    }
    // environment emitter (EnvironmentMap::configure + createShape, envmap.cpp:260-356)
    c->has_env = false;
    if (d->envmap) {
        pgh::EnvTables et;
        std::string err;
        if (!pgh::buildEnvTables(*d->envmap, c->scene_lo, c->scene_hi, et, err))
            return fail(c, PG_ERR_INVALID, "pg_upload_scene: " + err);
        std::vector<float> tab;  // cdf_rows | cdf_cols | row_weights, each 16-B aligned
        auto put = [&](const std::vector<float> &v) {
            const size_t at = tab.size();
            tab.insert(tab.end(), v.begin(), v.end());
            tab.resize((tab.size() + 3) & ~(size_t)3, 0.0f);
            return at;
        };
        const size_t oRows = put(et.cdf_rows), oCols = put(et.cdf_cols), oW = put(et.row_weights);
        if ((s = upload(c, c->envtex, et.texels)) || (s = upload(c, c->envtab, tab))) return s;
        GEnv ge{};
        ge.texels = c->envtex.as<float>();
        ge.cdf_rows = c->envtab.as<float>() + oRows;
        ge.cdf_cols = c->envtab.as<float>() + oCols;
        ge.row_weights = c->envtab.as<float>() + oW;
        ge.width = et.width;
        ge.height = et.height;
        ge.scale = et.scale;
        ge.normalization = et.normalization;
        ge.pixel_size[0] = et.pixel_size[0];
        ge.pixel_size[1] = et.pixel_size[1];
        ge.radius = et.radius;
        for (int a = 0; a < 3; ++a) ge.center[a] = et.center[a];
        for (int k = 0; k < 9; ++k) ge.R[k] = et.R[k];
        if ((s = upload(c, c->env, std::vector<GEnv>{ge}))) return s;
        c->has_env = true;
    }
    c->sd.reset(c->scene_lo, c->scene_hi);
    // pinned staging for the tree transfers, sized once for a large tree here (growing it inside a
    // training loop re-pins memory, ~10-20 ms per growth)
    HIPC(c, c->sd_stage.reserve((size_t)48 << 20));
    if ((s = uploadSd(c))) return s;
    HIPC(c, hipStreamSynchronize(c->stream));
    c->has_scene = true;
    return PG_OK;
}

// The volumetric path as a wavefront (pg_volpath.hip k_vcam / k_vflight / k_vvertex / k_vtail) or as the
// persistent megakernel k_volpath (PG_VOL_WAVEFRONT=0): the same per-path arithmetic and random
// streams, so the same films and trees
// (read per chunk, so tests can compare both in one process)
bool volWavefront() {
    const char *e = std::getenv("PG_VOL_WAVEFRONT");
    return e && *e ? std::atoi(e) != 0 : true;
}
// the interactions' transmittance walks (NEE shadow walks, emitter walks through media) as a stage of their
// own (k_vnee, after each k_vvertex; PG_VOL_NEE_STAGE=1) or inline at the end of each k_vvertex interaction
// (default): both give the same films and trees (the walks draw from their own sub-streams either way).  The
// stage takes the walks out of k_vvertex (medium interactions at 3 waves/SIMD, 166 VGPRs, no scratch) but the
// walks then run 45 % slower on their own: C5 328.8 / 326.4 Mpaths/s as a stage, 334.7 / 335.6 with the stage
// overlapping the next iteration's flights, 373.7 / 373.9 inline on one box (profiles/r05c_vol_nee_stage/)
bool volNeeStage() {
    const char *e = std::getenv("PG_VOL_NEE_STAGE");
    return e && *e ? std::atoi(e) != 0 : false;
}
// VolLane path state: VolWave's 14 float4 per slot (7 path columns, 6 deferred-walk columns and their flags /
// key / sample column; the first 7 when the walks run inline); its queues (pg_volpath.hip)
constexpr int kVolStateF4 = 14, kVolStateF4Inline = 7, kVolQueues = 8;
// k_vnee of iteration i on the lane's second stream, concurrent with iteration i + 1's k_vflight (which reads
// no state the walks write); k_vvertex of i + 1 waits for it.  PG_VOL_NEE_OVERLAP=0: on the lane's stream
bool volNeeOverlap() {
    const char *e = std::getenv("PG_VOL_NEE_OVERLAP");
    return e && *e ? std::atoi(e) != 0 : true;
}
// below this many live paths a chunk's remaining paths finish in one k_vtail launch (PG_VOL_TAIL_PATHS): 2^17
// with three lanes (C5 398.7 / 399.4 against 396.6 / 397.5 at 2^18, profiles/r04al_vol_tail/)
uint32_t volTailPaths() {
    const char *e = std::getenv("PG_VOL_TAIL_PATHS");
    return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : (uint32_t)1 << 17;
}


// chunks of a volumetric pass: np pixels from pb, nl sample layers from sample_base
struct VChunk {
    uint32_t pb, np, nl, sample_base;
};
// flight queues sorted by the 16^3 cell of the flight's start before k_vflight, for shards of at least this
// many flights (PG_VOL_SORT; 0 = off, the default since round 5).  Round 4: C5 351.5 / 350.0 against
// 346.3 / 345.7 Mpaths/s unsorted (profiles/r04s_vol_sort/, r04t_vol_ab/).  With round 5's 3-wave interaction
// launches the sort no longer pays: 442.9 / 442.5 sorted (4096) against 445.0 / 445.8 unsorted, k_vflight
// 45.3 against 48.9 ms per calibration pass but k_vvertex 136.4 against 133.8 (its state reads no longer
// scattered) plus the sort kernels (profiles/r05t_vol_tune/)
uint32_t volSortMin() {
    const char *e = std::getenv("PG_VOL_SORT");
    return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
}
// volumetric wavefront lanes in flight: pg_config.path_lanes (default 3, as for the path integrator; C5 at
// the round-4 kernels: 393.7 / 397.0 / 389.7 Mpaths/s with 2 / 3 / 4 lanes, profiles/r04aj_vol_lanes/);
// PG_VOL_LANES overrides (A/B)
int volLanes(const Ctx *c) {
    const char *e = std::getenv("PG_VOL_LANES");
    const int n = e && *e ? std::atoi(e) : c->nlanes;
    return std::max(1, std::min(PG_MAX_LANES, n));
}

// The chunks of one pass through the wavefront: per chunk the camera rays, then per iteration the
// free flights and the interactions, until at most volTailPaths() paths live; the tail finishes them.
// The host reads a chunk's queue counters once per iteration (grid sizes; the kernels read the counts)
// and advances whichever lane's counters have landed, so one chunk's readback and sparse last
// iterations overlap another's full ones.  Films (and record commits) run in chunk order, so every
// pixel's float sums are those of one lane.  Recording passes use two lanes (each with its own region of
// training vertices), per-stage timing one.
pg_status volWavefrontPass(Ctx *c, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                           const PathDev &pv, const std::vector<VChunk> &chunks, uint32_t want, int maxV,
                           uint32_t vtxLanes, std::vector<EventPair> &evs) {
    const bool evt = c->cfg.kernel_timing != 0;
    const int nl = evt ? 1 : std::min<int>(g.record ? (int)vtxLanes : volLanes(c), (int)chunks.size());
    // training vertices of lane li (recording passes): region li of vtxLanes, want items each
    auto laneVtx = [&](const VolLane &l) -> float4 * {
        return v.vtx ? v.vtx + (size_t)(&l - c->vlanes) * want * (size_t)maxV * PG_VTX_F4 : nullptr;
    };
    const size_t cbytes = (size_t)PG_QSHARDS * 4 * kVolQueues;
    const bool neeStage = volNeeStage(), neeOverlap = neeStage && volNeeOverlap() && !evt;
    auto joinNee = [&](VolLane &l) -> pg_status {  // the lane's stream waits for its pending walks
        if (l.npending) {
            HIPC(c, hipStreamWaitEvent(l.stream, l.ndone, 0));
            l.npending = false;
        }
        return PG_OK;
    };
    const uint32_t sortMin = volSortMin();
    HIPC(c, hipEventRecord(c->pass_start, c->stream));  // lanes start after the context stream's work
    for (int li = 0; li < nl; ++li) {
        VolLane &l = c->vlanes[li];
        if (!l.stream) {
            HIPC(c, hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking));
            HIPC(c, hipEventCreateWithFlags(&l.ready, hipEventDisableTiming));
        }
        // the second stream only when the overlapped k_vnee stage runs: HIP maps a process's streams onto
        // GPU_MAX_HW_QUEUES (4) hardware queues, and with one more stream per lane two lanes shared a queue
        // and serialized (C5 380 against 400 Mpaths/s, profiles/r05h_vol_streams/)
        if (neeOverlap && !l.nstream) {
            HIPC(c, hipStreamCreateWithFlags(&l.nstream, hipStreamNonBlocking));
            HIPC(c, hipEventCreateWithFlags(&l.vdone, hipEventDisableTiming));
            HIPC(c, hipEventCreateWithFlags(&l.ndone, hipEventDisableTiming));
        }
        l.npending = false;
        const int f4 = neeStage ? kVolStateF4 : kVolStateF4Inline;  // the stage's records only when it runs
        if (l.cap < want || l.stateF4 != f4) {
            const uint32_t lc = std::max(want, l.cap);
            HIPC(c, l.state.alloc((size_t)lc * 16 * f4));
            l.stateF4 = f4;
            HIPC(c, l.items.alloc((size_t)pg_queue_stride(lc) * PG_QSHARDS * 4 * kVolQueues));
            HIPC(c, l.rad.alloc((size_t)lc * 16));
            l.cap = lc;
        }
        HIPC(c, l.counts.alloc(cbytes));
        HIPC(c, l.host.reserve(cbytes));
        if (sortMin) {
            const size_t qstride = (size_t)pg_queue_stride(l.cap) * PG_QSHARDS;
            HIPC(c, l.keys.alloc(qstride * 2 * 2));
            HIPC(c, l.sorted.alloc(qstride * 4));
            HIPC(c, l.hist.alloc((size_t)PG_QSHARDS * PG_RAY_SORT_BINS * 4));
        }
        if (!l.ovf.p) HIPC(c, l.ovf.alloc(pg_stack_overflow_words(0) * 4));
        HIPC(c, hipStreamWaitEvent(l.stream, c->pass_start, 0));
        l.active = l.waved = false;
    }
    HIPC(c, hipEventRecord(c->film_order, c->stream));
    const uint32_t tail = volTailPaths();
    uint32_t next = 0, filmNext = 0;
    auto views = [&](VolLane &l, VolDev &lv, VolWave &w, Queue *q) {  // q: kVolQueues queues
        lv = v;
        lv.rad = l.rad.as<float4>();
        lv.stack_ovf = l.ovf.as<uint32_t>();
        lv.vtx = laneVtx(l);
        float4 *st = l.state.as<float4>();
        const size_t cap = l.cap;
        w = VolWave{st, st + cap, reinterpret_cast<uint4 *>(st + 2 * cap), st + 3 * cap, st + 4 * cap,
                    reinterpret_cast<uint4 *>(st + 5 * cap), st + 6 * cap};
        if (l.stateF4 == kVolStateF4) {  // the k_vnee stage's deferred-walk records
            w.n0 = st + 7 * cap;
            w.n1 = st + 8 * cap;
            w.n2 = st + 9 * cap;
            w.h0 = st + 10 * cap;
            w.h1 = st + 11 * cap;
            w.h2 = st + 12 * cap;
            w.nflags = reinterpret_cast<uint4 *>(st + 13 * cap);
        }
        // queues 0/1: flight of even / odd iterations, 2/3: surface, 4: medium vertices, 5/6: delta surface,
        // 7: deferred transmittance walks (k_vnee)
        const size_t qstride = (size_t)pg_queue_stride(l.cap) * PG_QSHARDS;
        const uint32_t stride = pg_queue_stride(l.np * l.nl);
        for (int k = 0; k < kVolQueues; ++k)
            q[k] = Queue{l.items.as<uint32_t>() + k * qstride, l.counts.as<uint32_t>() + k * PG_QSHARDS, stride};
        if (sortMin)
            for (int k = 0; k < 2; ++k) q[k].keys = l.keys.as<uint16_t>() + k * qstride;
    };
    auto readback = [&](VolLane &l) -> pg_status {
        HIPC(c, hipMemcpyAsync(l.host.p, l.counts.p, cbytes, hipMemcpyDeviceToHost, l.stream));
        HIPC(c, hipEventRecord(l.ready, l.stream));
        return PG_OK;
    };
    auto start = [&](VolLane &l) -> pg_status {
        if (next >= chunks.size()) {
            l.active = false;
            return PG_OK;
        }
        const VChunk &ch = chunks[next];
        l.chunk = next++;
        l.pb = ch.pb, l.np = ch.np, l.nl = ch.nl, l.sample_base = ch.sample_base;
        l.it = 0;
        l.active = true;
        l.waved = false;
        HIPC(c, hipEventCreate(&l.span.a));
        HIPC(c, hipEventCreate(&l.span.b));
        HIPC(c, hipEventRecord(l.span.a, l.stream));
        VolDev lv;
        VolWave w;
        Queue q[kVolQueues];
        views(l, lv, w, q);
        HIPC(c, hipMemsetAsync(l.counts.p, 0, cbytes, l.stream));
        pg_launch_vol_camera(l.stream, g, sc, lv, w, c->d_local_pixels.as<uint32_t>(), l.pb, l.np, l.nl, l.sample_base,
                             q[0], q[2], q[5]);
        HIPC(c, hipGetLastError());
        return readback(l);
    };
    // record commit + film of a chunk whose paths are done (its turn in chunk order), then its next chunk
    auto finish = [&](VolLane &l) -> pg_status {
        HIPC(c, hipStreamWaitEvent(l.stream, c->film_order, 0));
        PathDev lp = pv;
        lp.rad = l.rad.as<float4>();
        lp.vtx = laneVtx(l);
        if (g.record) {
            const uint64_t items = (uint64_t)l.np * l.nl, add = items * (uint64_t)maxV;
            if (c->rec_bound + add > c->rec_capacity) {
                unsigned long long rc = 0;
                HIPC(c, hipStreamSynchronize(l.stream));
                HIPC(c, hipMemcpy(&rc, c->rec_count.p, 8, hipMemcpyDeviceToHost));
                c->stats.records += rc - c->rec_host_count;
                c->rec_host_count = c->rec_bound = rc;
                pg_status st;
                if ((st = ensureRecords(c, rc + add))) return st;
            }
            c->rec_bound += add;
            pg_launch_commit(l.stream, lp, (uint32_t)items, maxV, c->records.as<pg_record>(),
                             c->rec_count.as<unsigned long long>(), c->rec_capacity, 0);
        }
        pg_launch_film(l.stream, g, sc, lp, c->d_local_pixels.as<uint32_t>(), l.pb, l.np, l.nl, c->film.as<float4>(),
                       c->film_sq.as<float4>());
        HIPC(c, hipGetLastError());
        HIPC(c, hipEventRecord(c->film_order, l.stream));
        HIPC(c, hipEventRecord(l.span.b, l.stream));
        evs.push_back(l.span);
        l.span = EventPair{};
        c->stats.paths += (uint64_t)l.np * l.nl;
        return start(l);
    };
    // one iteration of lane l (its counters are on the host)
    auto advance = [&](VolLane &l) -> pg_status {
        if (c->cancel.load()) return fail(c, PG_ERR_CANCELLED, "cancelled");
        const uint32_t *hc = reinterpret_cast<const uint32_t *>(l.host.p);
        auto maxShard = [&](int k) {
            uint32_t m = 0, t = 0;
            for (int i = 0; i < PG_QSHARDS; ++i) {
                m = std::max(m, hc[k * PG_QSHARDS + i]);
                t += hc[k * PG_QSHARDS + i];
            }
            return std::make_pair(m, t);
        };
        VolDev lv;
        VolWave w;
        Queue q[kVolQueues];
        views(l, lv, w, q);
        const int cur = l.it & 1, nxt = cur ^ 1;
        const auto f = maxShard(cur), su = maxShard(2 + cur), sdl = maxShard(5 + cur);
        if (f.second + su.second + sdl.second <= tail) {
            if (pg_status js = joinNee(l)) return js;
            if (f.second + su.second + sdl.second) {
                pg_launch_vol_tail(l.stream, g, sc, lv, sd, w, q[cur], f.first, q[2 + cur], su.first, q[5 + cur],
                                   sdl.first);
                HIPC(c, hipGetLastError());
            }
            l.waved = true;
            // finish this chunk and every waiting one whose turn comes after it
            for (bool progress = true; progress;) {
                progress = false;
                for (int k = 0; k < nl; ++k) {
                    VolLane &o = c->vlanes[k];
                    if (o.active && o.waved && o.chunk == filmNext) {
                        ++filmNext;
                        pg_status st = finish(o);
                        if (st) return st;
                        progress = true;
                    }
                }
            }
            return PG_OK;
        }
        // the next iteration's output queues and the medium queue start empty
        HIPC(c, hipMemsetAsync(q[nxt].counts, 0, PG_QSHARDS * 4, l.stream));
        HIPC(c, hipMemsetAsync(q[2 + nxt].counts, 0, PG_QSHARDS * 4, l.stream));
        HIPC(c, hipMemsetAsync(q[4].counts, 0, PG_QSHARDS * 4, l.stream));
        HIPC(c, hipMemsetAsync(q[5 + nxt].counts, 0, PG_QSHARDS * 4, l.stream));
        // per-stage device time (pg_config.kernel_timing, one lane): events around each launch
        if (evt && !c->vw_ev[0])
            for (hipEvent_t &e : c->vw_ev) HIPC(c, hipEventCreate(&e));
        Queue fq = q[cur];
        if (sortMin && f.first >= sortMin) {  // the flights in cell order (same shards and counts)
            pg_launch_ray_sort(l.stream, fq, f.first, l.sorted.as<uint32_t>(), l.hist.as<uint32_t>(), PG_VOL_SORT_BINS);
            fq.items = l.sorted.as<uint32_t>();
        }
        if (evt) HIPC(c, hipEventRecord(c->vw_ev[0], l.stream));
        pg_launch_vol_flight(l.stream, g, sc, lv, sd, w, fq, f.first, q[4], q[2 + cur], q[5 + cur]);
        if (evt) HIPC(c, hipEventRecord(c->vw_ev[1], l.stream));
        // shard bounds without a readback: a medium vertex came from a flight; a surface vertex from a
        // flight or from the previous iteration's interactions; no shard exceeds the queue stride
        const uint32_t mm = f.first, ms = std::min(q[0].stride, f.first + su.first + sdl.first);
        // the previous iteration's walks write L: done before this iteration's interactions read it
        if (pg_status js = joinNee(l)) return js;
        if (neeStage) HIPC(c, hipMemsetAsync(q[7].counts, 0, PG_QSHARDS * 4, l.stream));
        const int vk = pg_launch_vol_vertex(l.stream, g, sc, lv, sd, w, q[4], mm, q[2 + cur], ms, q[5 + cur], ms,
                                            q[nxt], q[2 + nxt], q[5 + nxt], neeStage ? &q[7] : nullptr);
        if (evt) HIPC(c, hipEventRecord(c->vw_ev[2], l.stream));
        // the deferred walks: at most one entry per path live in this iteration (<= ms per shard)
        if (neeOverlap) {
            HIPC(c, hipEventRecord(l.vdone, l.stream));
            HIPC(c, hipStreamWaitEvent(l.nstream, l.vdone, 0));
            pg_launch_vol_nee(l.nstream, g, sc, lv, w, q[7], ms);
            HIPC(c, hipEventRecord(l.ndone, l.nstream));
            l.npending = true;
        } else if (neeStage) {
            pg_launch_vol_nee(l.stream, g, sc, lv, w, q[7], ms);
        }
        if (evt) {
            HIPC(c, hipEventRecord(c->vw_ev[3], l.stream));
            HIPC(c, hipEventSynchronize(c->vw_ev[3]));
            float a = 0, b = 0, e = 0;
            if (f.first) {
                HIPC(c, hipEventElapsedTime(&a, c->vw_ev[0], c->vw_ev[1]));
                c->stats.vol_flight_ms += a;
                c->stats.vol_flight_launches++;
            }
            HIPC(c, hipEventElapsedTime(&b, c->vw_ev[1], c->vw_ev[2]));
            c->stats.vol_vertex_ms += b;
            c->stats.vol_vertex_launches += vk;  // kernels, not stages: the medium and surface launches
            if (neeStage) {
                HIPC(c, hipEventElapsedTime(&e, c->vw_ev[2], c->vw_ev[3]));
                c->stats.vol_nee_ms += e;
                c->stats.vol_nee_launches++;
            }
        }
        HIPC(c, hipGetLastError());
        ++l.it;
        return readback(l);
    };
    pg_status s;
    for (int li = 0; li < nl; ++li)
        if ((s = start(c->vlanes[li]))) return s;
    // advance whichever lane has its counters first
    for (uint32_t rr = 0;; ++rr) {
        int active = 0, picked = -1;
        for (int k = 0; k < nl; ++k) {
            VolLane &l = c->vlanes[(rr + k) % nl];
            if (!l.active) continue;
            ++active;
            if (l.waved) continue;  // waiting for an earlier chunk's film
            const hipError_t qr = hipEventQuery(l.ready);
            if (qr == hipSuccess) {
                picked = (int)((rr + k) % nl);
                break;
            }
            if (qr != hipErrorNotReady) HIPC(c, qr);
        }
        if (!active) break;
        if (picked >= 0 && (s = advance(c->vlanes[picked]))) return s;
    }
    for (int li = 0; li < nl; ++li) HIPC(c, hipStreamSynchronize(c->vlanes[li].stream));
    return PG_OK;
}

// progressive_volpath: chunks of (pixel, sample) items through the wavefront or k_volpath, films in chunk order
pg_status renderVolpath(Ctx *c, uint32_t spp, uint32_t sample_offset, bool rec) {
    const uint32_t npix = (uint32_t)c->local_pixels.size();
    // 2^25 items per launch: fewer persistent-kernel tails (C5 guided: 177.8 -> 189.8 Mpaths/s
    // against 2^22, profiles/r01h_c5_*.log); 50 GB of training vertices when guided
    const uint32_t cap = c->cfg.max_paths_in_flight ? c->cfg.max_paths_in_flight : (1u << 25);
    const uint64_t total = (uint64_t)npix * spp;
    uint32_t want = (uint32_t)std::min<uint64_t>(total, cap);
    const bool wave = volWavefront();  // the wavefront's lanes hold their own radiance and overflow rings
    const int maxV = std::min(std::max(c->cfg.record_max_vertices, 0), 64);
    // a recording pass through the wavefront runs as (at least) two chunks on two lanes, each lane with
    // its own region of training vertices (indexed by item within the chunk): the same vertex memory as
    // one chunk of the whole pass
    const char *rl = std::getenv("PG_VOL_REC_LANES");  // 1: one lane (A/B)
    const uint32_t vtxLanes = (wave && rec && maxV > 0 && !c->cfg.kernel_timing && volLanes(c) >= 2 && total > 1 &&
                               !(rl && std::atoi(rl) == 1)) ? 2u : 1u;
    if (vtxLanes == 2) want = (uint32_t)std::min<uint64_t>(want, (total + 1) / 2);
    if (!wave && c->vol_cap < want) {
        HIPC(c, c->vol_rad.alloc((size_t)want * 16));
        c->vol_cap = want;
    }
    if (rec && maxV > 0 && c->vol_vtx_cap < (uint64_t)want * maxV * vtxLanes) {
        HIPC(c, c->vol_vtx.alloc((size_t)want * maxV * vtxLanes * 16 * PG_VTX_F4));
        c->vol_vtx_cap = (uint64_t)want * maxV * vtxLanes;
    }
    if (!wave && !c->vol_ovf.p) HIPC(c, c->vol_ovf.alloc(pg_stack_overflow_words(0) * 4));
    HIPC(c, c->vol_work.alloc(128));  // work counter, then 7 u64 statistics from byte 16
    HIPC(c, hipMemsetAsync(c->vol_work.p, 0, 128, c->stream));
    GParams g = c->g;
    g.max_depth = c->cfg.max_depth;
    g.rr_depth = c->cfg.rr_depth;
    g.use_nee = c->cfg.use_nee;
    g.hide_emitters = c->cfg.hide_emitters;
    g.strict_normals = c->cfg.strict_normals;
    g.max_component_value = c->cfg.max_component_value;
    g.seed = c->cfg.seed;
    g.depth_cap = deviceDepthCap(c->cfg);
    g.guiding = c->cfg.guiding;
    g.bsdf_fraction = c->cfg.bsdf_sampling_fraction;
    g.fraction_bound = c->cfg.bsdf_fraction_bound;
    g.exact_mis = c->cfg.volpath_exact_mis;
    g.record = rec && maxV > 0;
    g.max_vertices = maxV;
    const SceneDev sc = sceneView(c);
    const SDDev sd = sdView(c);
    VolDev v{};
    v.grid = c->cfg.volume_majorant == PG_MAJORANT_GRID ? 1 : 0;
    v.media = c->media.as<GMedium>();
    v.tmed = c->tmed.as<uint32_t>();
    v.tcheap = c->tcheap.as<uint8_t>();
    {  // the surface launches specialised to diffuse / null materials (read per pass: tests A/B it in-process)
        const char *e = std::getenv("PG_VOL_MODELS");
        v.models = c->diffuse_null && !(e && *e && std::atoi(e) == 0) ? 1u : 0u;
    }
    v.cam_medium = c->cam_medium;
    v.num_media = c->num_media;
    v.rad = c->vol_rad.as<float4>();
    v.next = c->vol_work.as<uint32_t>();
    v.stats = (unsigned long long *)(c->vol_work.as<uint8_t>() + 16);
    v.stack_ovf = c->vol_ovf.as<uint32_t>();
    v.vtx = g.record ? c->vol_vtx.as<float4>() : nullptr;
    v.vtx_P = want;
    v.dist_beta = c->cfg.distance_guiding;
    {  // refill threshold of the persistent volumetric kernel: C5 198 / 212 / 227 / 243 / 248 / 247 / 242 /
       // 211 Mpaths/s at 1 / 8 / 16 / 32 / 40 / 48 / 56 / 64 idle lanes (profiles/r03p_vol_refill/);
       // PG_VOL_REFILL overrides (A/B)
        const char *e = std::getenv("PG_VOL_REFILL");
        v.refill_min = e ? (uint32_t)std::max(1, std::min(64, std::atoi(e))) : 40u;
    }
    PathDev pv{};
    pv.rad = v.rad;
    pv.vtx = v.vtx;
    pv.P = want;
    pv.vtxP = want;
    pv.pinfo = nullptr;  // k_commit reads the vertex count from rad[item].w
    const uint32_t layersPer = std::max<uint32_t>(1, want / npix), pixPer = std::min(npix, want);
    std::vector<VChunk> chunks;
    for (uint32_t layer = 0; layer < spp;) {
        const uint32_t nl = npix > want ? 1 : std::min(layersPer, spp - layer);
        for (uint32_t pb = 0; pb < npix; pb += pixPer)
            chunks.push_back(VChunk{pb, std::min(pixPer, npix - pb), nl, sample_offset + layer});
        layer += nl;
    }
    std::vector<EventPair> evs;
    struct EventsGuard {  // the chunk spans, on every exit (an error or cancellation returns early)
        std::vector<EventPair> &v;
        ~EventsGuard() {
            for (EventPair &e : v) {
                (void)hipEventDestroy(e.a);
                (void)hipEventDestroy(e.b);
            }
        }
    } evsGuard{evs};
    if (wave) {
        pg_status ws = volWavefrontPass(c, g, sc, v, sd, pv, chunks, want, maxV, vtxLanes, evs);
        if (ws) return ws;
    }
    for (size_t ci = 0; !wave && ci < chunks.size(); ++ci) {  // the persistent megakernel
        if (c->cancel.load()) return fail(c, PG_ERR_CANCELLED, "cancelled");
        const uint32_t pb = chunks[ci].pb, np = chunks[ci].np, nl = chunks[ci].nl;
        EventPair e;
        HIPC(c, hipEventCreate(&e.a));
        HIPC(c, hipEventCreate(&e.b));
        evs.push_back(e);
        HIPC(c, hipEventRecord(e.a, c->stream));
        pg_launch_volpath(c->stream, g, sc, v, sd, c->d_local_pixels.as<uint32_t>(), pb, np, nl, chunks[ci].sample_base);
        HIPC(c, hipEventRecord(e.b, c->stream));
        if (g.record) {
            const uint64_t items = (uint64_t)np * nl, add = items * (uint64_t)maxV;
            if (c->rec_bound + add > c->rec_capacity) {
                unsigned long long rc = 0;
                HIPC(c, hipStreamSynchronize(c->stream));
                HIPC(c, hipMemcpy(&rc, c->rec_count.p, 8, hipMemcpyDeviceToHost));
                c->stats.records += rc - c->rec_host_count;
                c->rec_host_count = c->rec_bound = rc;
                pg_status st;
                if ((st = ensureRecords(c, rc + add))) return st;
            }
            c->rec_bound += add;
            pg_launch_commit(c->stream, pv, (uint32_t)items, maxV, c->records.as<pg_record>(),
                             c->rec_count.as<unsigned long long>(), c->rec_capacity, 0);
        }
        pg_launch_film(c->stream, g, sc, pv, c->d_local_pixels.as<uint32_t>(), pb, np, nl, c->film.as<float4>(),
                       c->film_sq.as<float4>());
        HIPC(c, hipGetLastError());
        c->stats.paths += (uint64_t)np * nl;
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    unsigned long long st[9];
    HIPC(c, hipMemcpy(st, c->vol_work.as<uint8_t>() + 16, 72, hipMemcpyDeviceToHost));
    c->stats.vol_nee_walks += st[7];
    c->stats.vol_nee_lookups += st[8];
    c->stats.vol_flights += st[3];
    c->stats.vol_flight_lookups += st[4];
    c->stats.vol_vertices += st[5];
    c->stats.vol_vertex_lookups += st[6];
    c->stats.segments += st[0];
    c->stats.shadow_rays += st[1];
    c->stats.density_lookups += st[2];
    if (g.record) {
        unsigned long long rc = 0;
        HIPC(c, hipMemcpy(&rc, c->rec_count.p, 8, hipMemcpyDeviceToHost));
        c->stats.records += rc - c->rec_host_count;
        c->rec_host_count = c->rec_bound = rc;
    }
    for (EventPair &e : evs) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e.a, e.b);
        c->stats.volume_ms += ms;
        c->stats.volume_launches++;
    }
    return PG_OK;
}

// Every exit of a pass that did not complete (cancellation, a HIP error): the lane streams are created
// non-blocking, so nothing queued later on c->stream (pg_read_film, pg_reset_film) orders after them.
// Wait for them, so that no lane kernel still writes the film or the records once pg_render_pass has
// returned, and release the chunk span events a volumetric lane had not handed over yet.
static void drainLanes(Ctx *c) {
    for (int li = 0; li < c->nlanes; ++li)
        if (c->lanes[li].stream) (void)hipStreamSynchronize(c->lanes[li].stream);
    for (VolLane &l : c->vlanes) {
        if (l.nstream) (void)hipStreamSynchronize(l.nstream);
        if (l.stream) (void)hipStreamSynchronize(l.stream);
        l.npending = false;
        if (l.span.a) (void)hipEventDestroy(l.span.a);
        if (l.span.b) (void)hipEventDestroy(l.span.b);
        l.span = EventPair{};
        l.active = l.waved = false;
    }
    if (c->stream) (void)hipStreamSynchronize(c->stream);
}

static pg_status renderPass(Ctx *c, uint32_t spp, uint32_t sample_offset, int32_t record);

pg_status pg_render_pass(void *ctx, uint32_t spp, uint32_t sample_offset, int32_t record) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_render_pass: null context");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_render_pass: no scene uploaded");
    if (c->cancel.load()) return fail(c, PG_ERR_CANCELLED, "cancelled");
    HIPC(c, hipSetDevice(c->cfg.device));
    const pg_status s = renderPass(c, spp, sample_offset, record);
    if (s) drainLanes(c);
    return s;
}

static pg_status renderPass(Ctx *c, uint32_t spp, uint32_t sample_offset, int32_t record) {
    const uint32_t npix = (uint32_t)c->local_pixels.size();
    if (npix == 0 || spp == 0) return PG_OK;
    if (c->cfg.integrator == PG_INTEGRATOR_VOLPATH) return renderVolpath(c, spp, sample_offset, record && c->cfg.guiding);
    const bool rec = record && c->cfg.guiding;
    // 2^25 paths per chunk by default: bigger chunks mean fewer sparse tail bounces (each costs a
    // class-count readback) per path.  C3 with 3 lanes: 2^22 491, 2^23 552, 2^24 569, 2^25 587
    // Mpaths/s (DESIGN.md "Lanes"; round 2: 2^26 / 2^27 within noise, profiles/r02zq_chunk_ab).  Round 6, with
    // the faster kernels, C3's final render (943.7 M paths, 3 lanes) by chunk count: 30 (2^25) 633-644, 15
    // (2^26) 646-650, 12 655-660, 9 (2^27) 637-648 Mpaths/s (profiles/r06_chunk/, r06_chunk2/).  So a pass of at
    // least 3 x lanes x 2^26 paths is cut into four rounds of lanes (whole sample layers, at most 2^27 paths a
    // chunk); smaller passes (training, an N-GPU shard) keep 2^25 so every lane still gets several chunks.
    // A non-recording lane holds ~6.6 GB per 2^25 paths; recording lanes add 32 training vertices per path.
    const uint64_t total = (uint64_t)npix * spp;
    uint32_t cap = c->cfg.max_paths_in_flight ? c->cfg.max_paths_in_flight : (1u << 25);
    if (!c->cfg.max_paths_in_flight && total >= 3ull * (uint64_t)c->nlanes * (1ull << 26)) {
        const uint32_t rounds = 4u * (uint32_t)c->nlanes;
        cap = (uint32_t)std::min<uint64_t>((uint64_t)((spp + rounds - 1) / rounds) * npix, 1ull << 27);
    }
    if (!c->cfg.max_paths_in_flight) {
        // ... but at most 70 % of the device memory this context can use for path state (free memory
        // plus what its lanes already hold), e.g. when several contexts or ranks share one GPU
        size_t freeB = 0, totalB = 0;
        if (hipMemGetInfo(&freeB, &totalB) == hipSuccess && freeB > 0) {
            size_t held = 0;
            for (int li = 0; li < c->nlanes; ++li) {
                const Lane &l = c->lanes[li];
                for (const DevBuf *b : {&l.ray_o, &l.ray_d, &l.hit, &l.thr, &l.rad, &l.prev, &l.pinfo,
                                        &l.sh_d, &l.sh_c, &l.vtx, &l.q0, &l.q1, &l.qs, &l.class_q, &l.aov})
                    held += b->bytes;
            }
            const int vs = vertexSlots(c, rec);
            const double perPath = 9.0 * 16 + (3 + PG_NUM_CLASSES) * 4.0 + vs * 16.0 * PG_VTX_F4 + (c->cfg.aovs ? 16.0 : 0.0);
            const double fit = 0.7 * (double)(freeB + held) / (perPath * c->nlanes);
            if (fit < (double)cap) cap = std::max<uint32_t>(1u << 20, (uint32_t)fit & ~4095u);
        }
    }
    uint32_t want;
    pg_status s;
    for (;;) {
        // chunk count rounded up to whole rounds of lanes, so that the last round keeps every lane busy
        // (a rank of an N-GPU job may get only a few chunks of the final render); small passes split
        // into one chunk per lane
        uint64_t chunks = std::max<uint64_t>(1, (total + cap - 1) / cap);
        chunks = (chunks + c->nlanes - 1) / c->nlanes * c->nlanes;
        // a small pass (early training iterations, a rank's shard of them) runs as ONE chunk: three
        // lanes would each pay the whole bounce tail of launches and count readbacks for a third of
        // the paths.  Per-pixel sums keep their layer order either way.
        if (total <= smallPass()) chunks = 1;
        if ((uint64_t)npix * chunks <= total) {  // whole sample layers per chunk
            const uint64_t layers = (spp + chunks - 1) / chunks;
            want = (uint32_t)std::min<uint64_t>(layers * npix, cap);
        } else {
            want = (uint32_t)std::min<uint64_t>((total + chunks - 1) / chunks, cap);
        }
        s = ensurePaths(c, want, rec);
        if (s != PG_ERR_OOM || cap <= (1u << 20)) break;
        // out of device memory (e.g. contexts sharing a GPU sized their chunks from the same free
        // memory): release the lanes and retry with half the chunk size, down to 2^20 paths
        releasePaths(c);
        (void)hipGetLastError();
        cap = std::max<uint32_t>(1u << 20, (cap / 2) & ~4095u);
    }
    if (s) return s;
    GParams g = c->g;
    g.max_depth = c->cfg.max_depth;
    g.rr_depth = c->cfg.rr_depth;
    g.use_nee = c->cfg.use_nee;
    g.hide_emitters = c->cfg.hide_emitters;
    g.strict_normals = c->cfg.strict_normals;
    g.guiding = c->cfg.guiding;
    g.record = rec ? 1 : 0;
    g.max_vertices = rec ? std::min(vertexSlots(c, rec), c->lanes[0].vtx_slots) : 0;
    g.max_component_value = c->cfg.max_component_value;
    g.bsdf_fraction = c->cfg.bsdf_sampling_fraction;
    g.fraction_bound = c->cfg.bsdf_fraction_bound;
    g.glossy_prior = c->cfg.glossy_prior;
    g.seed = c->cfg.seed;
    g.depth_cap = deviceDepthCap(c->cfg);
    const SceneDev sc = sceneView(c);
    const SDDev sd = sdView(c);
    const uint32_t maxBounces = std::min<uint32_t>(g.depth_cap + 2, kMaxBounces);
    const bool evt = c->cfg.kernel_timing != 0;  // per-launch HIP events (pg_stats trace/shade/shadow_ms)
    // the fused launches (k_rays: shadow rays + next closest hits; k_shade_all: every material class)
    // are what a render runs; with kernel_timing they are timed as launched (pg_stats rays_ms /
    // shade_ms), so a one-lane calibration context measures the shipped kernels
    const bool fuseRays = !std::getenv("PG_NO_RAYS_FUSION");
    const bool bands = cameraBands() > 0;
    const bool fuseShade = !c->has_env && !std::getenv("PG_NO_SHADE_FUSION");
    // chunks: whole sample layers over the local pixels when they fit, else pixel ranges
    const uint32_t layersPer = std::max<uint32_t>(1, want / npix);
    const uint32_t pixPer = std::min(npix, want);
    uint32_t nextLayer = 0, nextPix = 0, nextChunk = 0;  // chunk cursor
    uint32_t filmNext = 0;  // chunk whose film is next: films run in chunk order, so the float sums
                            // of a pixel do not depend on which lane finishes first
    // the lanes start after everything already queued on the context stream (film reset, uploads)
    HIPC(c, hipEventRecord(c->pass_start, c->stream));
    HIPC(c, hipEventRecord(c->film_order, c->stream));
    c->rec_bound = c->rec_host_count;

    auto lqueue = [](const Lane &l, uint32_t *items, uint32_t *counts) {
        return Queue{items, counts, pg_queue_stride(l.P)};
    };
    auto classQueues = [&](const Lane &l, uint32_t *cb, Queue *cls) {
        for (int k = 0; k <= PG_NUM_CLASSES; ++k)
            cls[k] = lqueue(l, k < PG_NUM_CLASSES ? l.class_q.as<uint32_t>() + (size_t)k * PG_QSHARDS * pg_queue_stride(l.P)
                                                 : nullptr,
                            cb + kClassCounts + k * PG_QSHARDS);
    };
    // trace of bounce l.b (closest hit + material-class partition), then the class counts to the host;
    // shq: the previous bounce's shadow queue, traced in the same launch (k_rays)
    auto launchTrace = [&](Lane &l, const Queue *shq) -> pg_status {
        uint32_t *cb = l.counters.as<uint32_t>() + (size_t)kBounceWords * l.b;
        Queue cls[PG_NUM_CLASSES + 1];
        classQueues(l, cb, cls);
        EventPair et{};
        if (evt) et = nextEvents(&l, shq ? KT_RAYS : KT_TRACE);
        if (evt) HIPC(c, hipEventRecord(et.a, l.stream));
        const Queue tq = lqueue(l, l.sorted ? l.qsorted.as<uint32_t>() : (l.b & 1) ? l.q1.as<uint32_t>() : l.q0.as<uint32_t>(),
                                cb);
        if (shq) pg_launch_rays(l.stream, g, sc, pathView(&l), tq, l.bound, cls, *shq, l.bound);
        else pg_launch_trace(l.stream, g, sc, pathView(&l), tq, l.bound, cls, l.b == 0);
        if (evt) HIPC(c, hipEventRecord(et.b, l.stream));
        HIPC(c, hipMemcpyAsync(l.h_counts + (size_t)kBounceWords * l.b + kClassCounts, cb + kClassCounts,
                               (PG_NUM_CLASSES + 1) * PG_QSHARDS * 4, hipMemcpyDeviceToHost, l.stream));
        HIPC(c, hipEventRecord(l.ready, l.stream));
        return PG_OK;
    };
    // fold the last finished chunk's shadow counts and kernel times into the statistics
    auto collectStats = [&](Lane &l) -> pg_status {
        if (!l.stats_pending) return PG_OK;
        HIPC(c, hipEventSynchronize(l.done));
        for (uint32_t k = 0; k < l.stats_bounces; ++k)
            for (int sh = 0; sh < PG_QSHARDS; ++sh)
                c->stats.shadow_rays += l.h_stats[(size_t)kBounceWords * k + kShadowCounts + sh];
        c->stats.segments += l.h_tail[0];  // the chunk's tail (k_tail)
        c->stats.escaped += l.h_tail[1];
        c->stats.shadow_rays += l.h_tail[2];
        if (std::getenv("PG_DEBUG_COUNTS")) {
            for (uint32_t k = 0; k < l.stats_bounces && k < l.used_prev.size(); ++k) {
                uint64_t t = 0;
                for (int w = 0; w < (PG_NUM_CLASSES + 1) * PG_QSHARDS; ++w)
                    t += l.h_stats[(size_t)kBounceWords * k + kClassCounts + w];
                if (t != l.used_prev[k])
                    std::fprintf(stderr, "PG_DEBUG_COUNTS: chunk bounce %u: host read %llu segments, device %llu\n", k,
                                 (unsigned long long)l.used_prev[k], (unsigned long long)t);
            }
        }
        const int prev = l.evcur ^ 1;
        std::vector<EventPair> &pool = l.ev[prev];
        for (size_t e = 0; e < l.evused[prev]; ++e) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, pool[e].a, pool[e].b);
            switch (l.evkind[prev][e]) {
                case KT_TRACE: c->stats.trace_ms += ms; c->stats.trace_launches++; break;
                case KT_SHADE: c->stats.shade_ms += ms; break;
                case KT_SHADOW: c->stats.shadow_ms += ms; c->stats.shadow_launches++; break;
                default: c->stats.rays_ms += ms; c->stats.rays_launches++;
            }
        }
        l.evused[prev] = 0;
        l.stats_pending = false;
        return PG_OK;
    };
    // start the next chunk on lane l (false: no chunks left)
    auto startChunk = [&](Lane &l) -> pg_status {
        l.active = false;
        if (nextLayer >= spp) return PG_OK;
        if (c->cancel.load()) return fail(c, PG_ERR_CANCELLED, "cancelled");
        uint32_t nl = std::min(layersPer, spp - nextLayer);
        if (npix > want) nl = 1;
        const uint32_t pb = nextPix, np = std::min(pixPer, npix - pb);
        l.layer0 = nextLayer;
        l.pb = pb;
        l.np = np;
        l.nl = nl;
        l.n = np * nl;
        nextPix += np;
        if (nextPix >= npix) {
            nextPix = 0;
            nextLayer += nl;
        }
        l.b = 0;
        l.sorted = false;  // camera rays: their queue order is already coherent
        l.bound = pg_camera_bound(pg_camera_banded(bands, l.np), l.np, l.nl);
        l.active = true;
        l.traced = false;
        l.chunk = nextChunk++;
        HIPC(c, hipStreamWaitEvent(l.stream, c->pass_start, 0));
        HIPC(c, hipMemsetAsync(l.counters.p, 0, (size_t)kBounceWords * (maxBounces + 1) * 4, l.stream));
        HIPC(c, hipMemsetAsync(l.tail_stats.p, 0, 24, l.stream));
        pg_launch_camera(l.stream, g, pathView(&l), c->d_band_pixels.as<uint32_t>(), l.pb, l.np, l.nl,
                         sample_offset + l.layer0, lqueue(l, l.q0.as<uint32_t>(), l.counters.as<uint32_t>()), bands);
        return launchTrace(l, nullptr);
    };
    // film + record commit (in chunk order across lanes), statistics copy; then the next chunk
    auto finishChunk = [&](Lane &l) -> pg_status {
        pg_status st;
        if ((st = collectStats(l))) return st;
        const PathDev pv = pathView(&l);
        HIPC(c, hipMemcpyAsync(l.h_stats, l.counters.p, (size_t)kBounceWords * l.b * 4, hipMemcpyDeviceToHost, l.stream));
        HIPC(c, hipMemcpyAsync(l.h_tail, l.tail_stats.p, 24, hipMemcpyDeviceToHost, l.stream));
        HIPC(c, hipStreamWaitEvent(l.stream, c->film_order, 0));
        pg_launch_film(l.stream, g, sc, pv, c->d_band_pixels.as<uint32_t>(), l.pb, l.np, l.nl, c->film.as<float4>(),
                       c->film_sq.as<float4>(), c->aov_albedo.as<float4>(), c->aov_normal.as<float4>());
        if (rec) {
            // every slot can emit at most max_vertices records; grow the buffer (lanes idle) when the
            // bound could overflow it
            const uint64_t add = (uint64_t)l.n * g.max_vertices;
            if (c->rec_bound + add > c->rec_capacity) {
                for (int li = 0; li < c->nlanes; ++li) HIPC(c, hipStreamSynchronize(c->lanes[li].stream));
                unsigned long long rc = 0;
                HIPC(c, hipMemcpy(&rc, c->rec_count.p, 8, hipMemcpyDeviceToHost));
                c->stats.records += rc - c->rec_host_count;
                c->rec_host_count = c->rec_bound = rc;
                if ((st = ensureRecords(c, rc + add))) return st;
            }
            c->rec_bound += add;
            pg_launch_commit(l.stream, pv, l.n, g.max_vertices, c->records.as<pg_record>(),
                             c->rec_count.as<unsigned long long>(), c->rec_capacity, c->has_env ? 1 : 0);
        }
        HIPC(c, hipEventRecord(c->film_order, l.stream));
        HIPC(c, hipEventRecord(l.done, l.stream));
        HIPC(c, hipGetLastError());
        l.stats_pending = true;
        l.stats_bounces = l.b;
        l.used_prev.swap(l.used_cur);
        l.used_cur.clear();
        l.evcur ^= 1;
        c->stats.paths += l.n;
        return startChunk(l);
    };
    // one bounce's shading + shadow rays + next trace on lane l (class counts already on the host)
    auto advance = [&](Lane &l) -> pg_status {
        HIPC(c, hipEventSynchronize(l.ready));
        uint32_t *cb = l.counters.as<uint32_t>() + (size_t)kBounceWords * l.b;
        const uint32_t *hc = l.h_counts + (size_t)kBounceWords * l.b + kClassCounts;
        uint32_t clsMax[PG_NUM_CLASSES], shardLive[PG_QSHARDS] = {};
        uint64_t nlive = 0;
        for (int k = 0; k <= PG_NUM_CLASSES; ++k) {
            uint32_t m = 0;
            for (int sh = 0; sh < PG_QSHARDS; ++sh) {
                const uint32_t v = hc[k * PG_QSHARDS + sh];
                c->stats.segments += v;
                if (k == PG_NUM_CLASSES) {
                    c->stats.escaped += v;
                    continue;
                }
                m = std::max(m, v);
                shardLive[sh] += v;
                nlive += v;
            }
            if (k < PG_NUM_CLASSES) clsMax[k] = m;
        }
        {
            uint64_t t = 0;
            for (int w = 0; w < (PG_NUM_CLASSES + 1) * PG_QSHARDS; ++w) t += hc[w];
            l.used_cur.push_back(t);
        }
        ++l.b;
        const uint32_t tailMax = c->cfg.tail_paths < 0 ? 0u : c->cfg.tail_paths > 0 ? (uint32_t)c->cfg.tail_paths : tailPaths();
        const bool tail = nlive > 0 && nlive <= tailMax && l.b < maxBounces;
        if (tail) {  // one launch finishes every remaining path (shading starts at the hits just traced)
            const uint32_t *cbt = l.counters.as<uint32_t>() + (size_t)kBounceWords * (l.b - 1);
            const Queue tq = lqueue(l, l.sorted ? l.qsorted.as<uint32_t>()
                                                : ((l.b - 1) & 1) ? l.q1.as<uint32_t>() : l.q0.as<uint32_t>(),
                                    const_cast<uint32_t *>(cbt));
            pg_launch_tail(l.stream, g, sc, sd, pathView(&l), tq, l.bound, l.tail_stats.as<unsigned long long>());
            c->stats.tail_launches += 1;
        }
        if (nlive == 0 || tail || l.b >= maxBounces) {
            l.traced = true;
            // finish this lane and every waiting lane whose turn comes after it, in chunk order
            for (bool progress = true; progress;) {
                progress = false;
                for (Lane &o : c->lanes)
                    if (o.active && o.traced && o.chunk == filmNext) {
                        ++filmNext;
                        pg_status st = finishChunk(o);
                        if (st) return st;
                        progress = true;
                    }
            }
            return PG_OK;
        }
        Queue cls[PG_NUM_CLASSES + 1];
        classQueues(l, cb, cls);
        const PathDev pv = pathView(&l);
        Queue next = lqueue(l, (l.b & 1) ? l.q1.as<uint32_t>() : l.q0.as<uint32_t>(), cb + kBounceWords);
        const Queue shq = lqueue(l, l.qs.as<uint32_t>(), cb + kShadowCounts);
        const uint32_t nextBound = *std::max_element(shardLive, shardLive + PG_QSHARDS);
        const bool sortNext = raySortEnabled() && nextBound >= kRaySortMinShard;
        if (sortNext) next.keys = l.qkey.as<uint16_t>();
        EventPair es{}, ew{};
        if (evt) es = nextEvents(&l, KT_SHADE);
        if (evt) HIPC(c, hipEventRecord(es.a, l.stream));
        if (fuseShade) {  // one launch for every class present
            pg_launch_shade_all(l.stream, g, sc, sd, pv, cls, clsMax, next, shq);
            c->stats.shade_launches += 1;
        } else {
            for (int k = 0; k < PG_NUM_CLASSES; ++k) {
                pg_launch_shade_class(l.stream, k, g, sc, sd, pv, cls[k], clsMax[k], next, shq);
                c->stats.shade_launches += clsMax[k] ? 1 : 0;
            }
        }
        if (evt) HIPC(c, hipEventRecord(es.b, l.stream));
        l.bound = nextBound;
        if (sortNext)  // group every shard of the next closest-hit queue by ray order key
            pg_launch_ray_sort(l.stream, next, l.bound, l.qsorted.as<uint32_t>(), l.rsort_hist.as<uint32_t>());
        l.sorted = sortNext;
        // without per-launch timing the shadow rays share the next trace's launch
        if (fuseRays) return launchTrace(l, &shq);
        if (evt) ew = nextEvents(&l, KT_SHADOW);
        if (evt) HIPC(c, hipEventRecord(ew.a, l.stream));
        pg_launch_shadow(l.stream, sc, pv, shq, l.bound);
        if (evt) HIPC(c, hipEventRecord(ew.b, l.stream));
        return launchTrace(l, nullptr);
    };

    for (int li = 0; li < c->nlanes; ++li)
        if ((s = startChunk(c->lanes[li]))) return s;
    // advance whichever lane has its counts first (waiting on a fixed lane order leaves the GPU idle
    // whenever the other lane is already ready)
    for (uint32_t rr = 0;; ++rr) {
        int active = 0, picked = -1;
        for (int k = 0; k < c->nlanes; ++k) {
            Lane &l = c->lanes[(rr + k) % c->nlanes];
            if (!l.active) continue;
            ++active;
            if (l.traced) continue;  // waiting for an earlier chunk's film
            const hipError_t q = hipEventQuery(l.ready);
            if (q == hipSuccess) {
                picked = (int)((rr + k) % c->nlanes);
                break;
            }
            if (q != hipErrorNotReady) HIPC(c, q);
        }
        if (!active) break;
        if (picked >= 0 && (s = advance(c->lanes[picked]))) return s;
    }
    for (int li = 0; li < c->nlanes; ++li) {
        Lane &l = c->lanes[li];
        HIPC(c, hipStreamSynchronize(l.stream));
        if ((s = collectStats(l))) return s;
    }
    if (rec) {
        unsigned long long rc = 0;
        HIPC(c, hipMemcpy(&rc, c->rec_count.p, 8, hipMemcpyDeviceToHost));
        c->stats.records += rc - c->rec_host_count;
        c->rec_host_count = c->rec_bound = rc;
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

// ProgressiveMonteCarloIntegrator::renderTime (progressiveintegrator.cpp:117-168): whole
// progressions until the wall-clock budget is spent.  The reference checks the timer after every
// progression of a 128-progression batch and cancels the rest; here consecutive progressions are
// merged into one pg_render_pass (the film adds samples in sample order, so a merged pass equals
// its progressions bit for bit), each merge covering at most half the remaining budget at the
// measured rate, so the overshoot stays below one progression plus one readback.  Only whole
// progressions reach the film: every pixel holds the same sample count (the reference may cancel
// a progression midway, leaving some blocks with one progression more).
pg_status pg_render_time(void *ctx, double seconds, uint32_t spp_per_progression, uint32_t sample_offset,
                         uint32_t max_spp, uint32_t *spp_done) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !spp_done) return fail(c, PG_ERR_INVALID, "pg_render_time: null argument");
    *spp_done = 0;
    if (!(seconds > 0) || spp_per_progression == 0)
        return fail(c, PG_ERR_INVALID, "pg_render_time: need seconds > 0 and spp_per_progression > 0");
    const uint32_t limit = max_spp ? max_spp : 0x7FFFFFFFu;
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t done = 0, batch = std::min(spp_per_progression, limit);
    while (done < limit) {
        pg_status s = pg_render_pass(ctx, batch, sample_offset + done, 0);
        if (s) return s;
        done += batch;
        *spp_done = done;
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el >= seconds) break;
        const double perProg = el / (done / spp_per_progression);
        const double progs = std::floor(0.5 * (seconds - el) / std::max(perProg, 1e-9));
        const uint64_t want = (uint64_t)std::max(1.0, std::min(progs, 1e6)) * spp_per_progression;
        batch = (uint32_t)std::min<uint64_t>(want, limit - done);
        batch -= batch % spp_per_progression;  // whole progressions
        if (batch == 0) break;
    }
    return PG_OK;
}

pg_status pg_rough_transmittance(uint32_t distribution, float alpha, float eta, float *table, float *fdr_int) {
    if (!table || !fdr_int) return fail(nullptr, PG_ERR_INVALID, "pg_rough_transmittance: null argument");
    if (distribution > PG_DIST_GGX || !(alpha >= 0) || !(eta > 0) || eta == 1.0f)
        return fail(nullptr, PG_ERR_INVALID, "pg_rough_transmittance: bad distribution, alpha or eta");
    pgh::roughTransmittance((int)distribution, std::max(alpha, 1e-4f), eta, table, fdr_int);
    return PG_OK;
}

pg_status pg_get_record_count(void *ctx, uint64_t *count) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !count) return fail(c, PG_ERR_INVALID, "pg_get_record_count: null argument");
    *count = c->rec_host_count;
    return PG_OK;
}

pg_status pg_get_records(void *ctx, void *dst, uint64_t max_records, int32_t dst_is_device, uint64_t *written) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!dst && max_records)) return fail(c, PG_ERR_INVALID, "pg_get_records: null argument");
    HIPC(c, hipSetDevice(c->cfg.device));
    uint64_t n = std::min(max_records, c->rec_host_count);
    if (n)
        HIPC(c, hipMemcpyAsync(dst, c->records.p, n * sizeof(pg_record),
                               dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    if (written) *written = n;
    return PG_OK;
}

pg_status pg_splat_records(void *ctx, const void *src, uint64_t count, int32_t src_is_device) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!src && count)) return fail(c, PG_ERR_INVALID, "pg_splat_records: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_splat_records: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!count) return PG_OK;
    const pg_record *dsrc = (const pg_record *)src;
    if (!src_is_device) {
        HIPC(c, c->ext_records.alloc(count * sizeof(pg_record)));
        HIPC(c, hipMemcpyAsync(c->ext_records.p, src, count * sizeof(pg_record), hipMemcpyHostToDevice, c->stream));
        dsrc = c->ext_records.as<pg_record>();
    }
    EventPair &e = c->timing;
    if (!e.a) {
        HIPC(c, hipEventCreate(&e.a));
        HIPC(c, hipEventCreate(&e.b));
    }
    HIPC(c, hipEventRecord(e.a, c->stream));
    pg_launch_splat(c->stream, sdView(c), dsrc, count);
    HIPC(c, hipEventRecord(e.b, c->stream));
    HIPC(c, hipGetLastError());
    HIPC(c, hipStreamSynchronize(c->stream));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e.a, e.b);
    c->stats.other_ms += ms;
    return PG_OK;
}

pg_status pg_splat_local_records(void *ctx) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_splat_local_records: null context");
    if (c->rec_host_count == 0) return PG_OK;
    return pg_splat_records(ctx, c->records.p, c->rec_host_count, 1);
}

pg_status pg_refit(void *ctx, uint32_t iteration) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_refit: null context");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_refit: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    pg_status s;
    const auto t0 = std::chrono::steady_clock::now();
    if ((s = downloadSd(c))) return s;
    const auto t1 = std::chrono::steady_clock::now();
    c->sd.refit(iteration, c->cfg.s_tree_threshold, c->cfg.d_tree_threshold, c->cfg.d_tree_max_depth,
                c->cfg.bsdf_fraction_bound == PG_FRACTION_LEARNED);
    const auto t2 = std::chrono::steady_clock::now();
    if ((s = uploadSd(c))) return s;
    HIPC(c, hipMemsetAsync(c->rec_count.p, 0, 8, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    if (std::getenv("PG_DEBUG_REFIT")) {
        const auto t3 = std::chrono::steady_clock::now();
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "refit %u: download %.2f ms, refit %.2f ms, upload %.2f ms (%zu D-trees, %zu / %zu nodes)\n",
                     iteration, ms(t0, t1), ms(t1, t2), ms(t2, t3), c->sd.leaves.size(), c->sd.samplingNodes(),
                     c->sd.buildingNodes());
    }
    c->rec_host_count = 0;
    return PG_OK;
}

pg_status pg_get_tree_stats(void *ctx, void *dst, uint64_t capacity_words, int32_t dst_is_device, uint64_t *words) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !words) return fail(c, PG_ERR_INVALID, "pg_get_tree_stats: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_get_tree_stats: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    const size_t nb = c->sd.buildingNodes(), nl = c->sd.leaves.size();
    *words = 4 * nb + nl + pgh::kFracStats * nl;
    if (!dst) return PG_OK;
    if (capacity_words < *words) return fail(c, PG_ERR_INVALID, "pg_get_tree_stats: buffer too small");
    const hipMemcpyKind k = dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    HIPC(c, hipMemcpyAsync(dst, c->sdp.bsum, 8 * *words, k, c->stream));  // bsum | count | frac, contiguous
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_put_tree_stats(void *ctx, const void *src, uint64_t words, int32_t src_is_device) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !src) return fail(c, PG_ERR_INVALID, "pg_put_tree_stats: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_put_tree_stats: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    const size_t nb = c->sd.buildingNodes(), nl = c->sd.leaves.size();
    if (words != 4 * nb + nl + pgh::kFracStats * nl)
        return fail(c, PG_ERR_INVALID, "pg_put_tree_stats: size does not match the tree");
    const hipMemcpyKind k = src_is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    HIPC(c, hipMemcpyAsync(c->sdp.bsum, src, 8 * words, k, c->stream));  // bsum | count | frac, contiguous
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

// ---- multi-GPU inside the library (RCCL over xGMI).  Replaces what the reference's remote
// scheduler does for a distributed render (include/mitsuba/core/sched_remote.h:50-236: ship work
// units to other machines, merge their image blocks): here every rank renders its tile shard, and
// the only exchanges are the postprogression statistics all-reduce and the final film reduce.
#define NCCLC(c, expr)                                                                            \
    do {                                                                                          \
        ncclResult_t _r = (expr);                                                                 \
        if (_r != ncclSuccess) return fail(c, PG_ERR_HIP, std::string("RCCL: ") + #expr + ": " + \
                                                              ncclGetErrorString(_r));              \
    } while (0)

static_assert(PG_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "pg_comm id size");

pg_status pg_comm_unique_id(void *id_out) {
    if (!id_out) return fail(nullptr, PG_ERR_INVALID, "pg_comm_unique_id: null argument");
    ncclUniqueId id;
    NCCLC(nullptr, ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return PG_OK;
}

pg_status pg_comm_init(void *ctx, const void *id) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !id) return fail(c, PG_ERR_INVALID, "pg_comm_init: null argument");
    if (c->comm) return fail(c, PG_ERR_STATE, "pg_comm_init: communicator already initialised");
    if (c->cfg.world_size < 1 || c->cfg.rank < 0 || c->cfg.rank >= c->cfg.world_size)
        return fail(c, PG_ERR_INVALID, "pg_comm_init: rank / world_size of the config are inconsistent");
    HIPC(c, hipSetDevice(c->cfg.device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    NCCLC(c, ncclCommInitRank(&c->comm, c->cfg.world_size, uid, c->cfg.rank));
    return PG_OK;
}

pg_status pg_comm_allreduce_tree_stats(void *ctx) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_comm_allreduce_tree_stats: null context");
    if (!c->comm) return fail(c, PG_ERR_STATE, "pg_comm_allreduce_tree_stats: no communicator (pg_comm_init)");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_comm_allreduce_tree_stats: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    // the reduced vector IS the pg_get_tree_stats vector (u64 quadrant sums, per-D-tree record counts,
    // fraction statistics), which the device keeps contiguous: summed over ranks in place -- the
    // multi-rank arithmetic the torch.distributed / gloo exchange tests check.  Integer sums: every
    // rank ends with identical statistics.
    uint64_t words = 0;
    pg_status st;
    if ((st = pg_get_tree_stats(ctx, nullptr, 0, 1, &words))) return st;
    if (words) NCCLC(c, ncclAllReduce(c->sdp.bsum, c->sdp.bsum, words, ncclUint64, ncclSum, c->comm, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_comm_reduce_film(void *ctx, int32_t root) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_comm_reduce_film: null context");
    if (!c->comm) return fail(c, PG_ERR_STATE, "pg_comm_reduce_film: no communicator (pg_comm_init)");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_comm_reduce_film: no scene");
    if (root < 0 || root >= c->cfg.world_size) return fail(c, PG_ERR_INVALID, "pg_comm_reduce_film: bad root");
    HIPC(c, hipSetDevice(c->cfg.device));
    const size_t nf = (size_t)c->g.width * c->g.height * 4;
    // disjoint tile shards: every pixel has one non-zero contributor, so the f32 sum is exact
    NCCLC(c, ncclGroupStart());
    NCCLC(c, ncclReduce(c->film.p, c->film.p, nf, ncclFloat32, ncclSum, root, c->comm, c->stream));
    NCCLC(c, ncclReduce(c->film_sq.p, c->film_sq.p, nf, ncclFloat32, ncclSum, root, c->comm, c->stream));
    if (c->aov_albedo.p) {
        NCCLC(c, ncclReduce(c->aov_albedo.p, c->aov_albedo.p, nf, ncclFloat32, ncclSum, root, c->comm, c->stream));
        NCCLC(c, ncclReduce(c->aov_normal.p, c->aov_normal.p, nf, ncclFloat32, ncclSum, root, c->comm, c->stream));
    }
    NCCLC(c, ncclGroupEnd());
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_comm_allreduce_f64(void *ctx, double *values, uint64_t n) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!values && n)) return fail(c, PG_ERR_INVALID, "pg_comm_allreduce_f64: null argument");
    if (!c->comm) return fail(c, PG_ERR_STATE, "pg_comm_allreduce_f64: no communicator (pg_comm_init)");
    if (!n) return PG_OK;
    HIPC(c, hipSetDevice(c->cfg.device));
    DevBuf b;
    HIPC(c, b.alloc(n * 8));
    HIPC(c, hipMemcpyAsync(b.p, values, n * 8, hipMemcpyHostToDevice, c->stream));
    NCCLC(c, ncclAllReduce(b.p, b.p, n, ncclFloat64, ncclSum, c->comm, c->stream));
    HIPC(c, hipMemcpyAsync(values, b.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_comm_allgather_records(void *ctx, uint64_t *counts_out) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_comm_allgather_records: null context");
    if (!c->comm) return fail(c, PG_ERR_STATE, "pg_comm_allgather_records: no communicator (pg_comm_init)");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_comm_allgather_records: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    const int W = c->cfg.world_size;
    // 1. every rank's record count
    DevBuf cnt;
    HIPC(c, cnt.alloc((size_t)(W + 1) * 8));
    const uint64_t mine = c->rec_host_count;
    HIPC(c, hipMemcpyAsync(cnt.as<uint64_t>() + W, &mine, 8, hipMemcpyHostToDevice, c->stream));
    NCCLC(c, ncclAllGather(cnt.as<uint64_t>() + W, cnt.p, 1, ncclUint64, c->comm, c->stream));
    std::vector<uint64_t> counts(W);
    HIPC(c, hipMemcpyAsync(counts.data(), cnt.p, (size_t)W * 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    const uint64_t maxn = *std::max_element(counts.begin(), counts.end());
    if (counts_out) std::copy(counts.begin(), counts.end(), counts_out);
    if (maxn == 0) return PG_OK;
    // 2. the records, all-gathered in slices of at most kGatherSlice records per rank: round k gathers
    //    every rank's records [k S, (k + 1) S) (the local record buffer, padded to whole slices, is the
    //    send buffer) into ext_records (W S records, allocated once and reused by every round and every
    //    iteration), and every rank's valid part of the round is splatted, in rank order, before the next
    //    round overwrites it (same stream).  A single padded all-gather would need W x the largest count:
    //    ~13.6 GB per rank, re-allocated each iteration, for C3's 16-spp pass at W = 8.  Integer sums:
    //    the tree does not depend on the splat order.
    uint64_t slice = 1ull << 22;  // 128 MiB of records per rank and round
    if (const char *e = std::getenv("PG_GATHER_SLICE")) slice = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));  // tests
    const uint64_t S = std::min<uint64_t>(maxn, slice), rounds = (maxn + S - 1) / S;
    pg_status st;
    if ((st = ensureRecords(c, rounds * S))) return st;
    HIPC(c, c->ext_records.alloc((size_t)W * S * sizeof(pg_record)));
    const SDDev sd = sdView(c);
    for (uint64_t k = 0; k < rounds; ++k) {
        NCCLC(c, ncclAllGather(c->records.as<pg_record>() + k * S, c->ext_records.p, S * sizeof(pg_record), ncclUint8,
                               c->comm, c->stream));
        for (int r = 0; r < W; ++r) {
            const uint64_t lo = k * S, n = counts[r] > lo ? std::min(S, counts[r] - lo) : 0;
            if (n) pg_launch_splat(c->stream, sd, c->ext_records.as<pg_record>() + (size_t)r * S, n);
        }
        HIPC(c, hipGetLastError());
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_get_sdtree(void *ctx, void *buf, uint64_t capacity, uint64_t *size) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !size) return fail(c, PG_ERR_INVALID, "pg_get_sdtree: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_get_sdtree: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    pg_status s;
    if ((s = downloadSd(c))) return s;
    std::vector<uint8_t> blob = c->sd.serialize();
    *size = blob.size();
    if (buf) {
        if (capacity < blob.size()) return fail(c, PG_ERR_INVALID, "pg_get_sdtree: buffer too small");
        std::memcpy(buf, blob.data(), blob.size());
    }
    return PG_OK;
}

pg_status pg_put_sdtree(void *ctx, const void *buf, uint64_t size) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !buf) return fail(c, PG_ERR_INVALID, "pg_put_sdtree: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_put_sdtree: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    pgh::SdTree t;
    if (!t.deserialize((const uint8_t *)buf, size)) return fail(c, PG_ERR_INVALID, "pg_put_sdtree: malformed blob");
    c->sd = std::move(t);
    return uploadSd(c);
}

pg_status pg_sdtree_pdf(void *ctx, const float *pos, const float *dir, uint64_t n, float *out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !pos || !dir || !out) return fail(c, PG_ERR_INVALID, "pg_sdtree_pdf: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_sdtree_pdf: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    DevBuf a, b, o;
    HIPC(c, a.alloc(n * 12 + 16));
    HIPC(c, b.alloc(n * 12 + 16));
    HIPC(c, o.alloc(n * 4 + 16));
    HIPC(c, hipMemcpyAsync(a.p, pos, n * 12, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(b.p, dir, n * 12, hipMemcpyHostToDevice, c->stream));
    pg_launch_sd_pdf(c->stream, sdView(c), a.as<float>(), b.as<float>(), (uint32_t)n, o.as<float>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(out, o.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_sdtree_sample(void *ctx, const float *pos, const float *u, uint64_t n, float *dir_out, float *pdf_out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !pos || !u || !dir_out || !pdf_out) return fail(c, PG_ERR_INVALID, "pg_sdtree_sample: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_sdtree_sample: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    DevBuf a, b, d, p;
    HIPC(c, a.alloc(n * 12 + 16));
    HIPC(c, b.alloc(n * 8 + 16));
    HIPC(c, d.alloc(n * 12 + 16));
    HIPC(c, p.alloc(n * 4 + 16));
    HIPC(c, hipMemcpyAsync(a.p, pos, n * 12, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(b.p, u, n * 8, hipMemcpyHostToDevice, c->stream));
    pg_launch_sd_sample(c->stream, sdView(c), a.as<float>(), b.as<float>(), (uint32_t)n, d.as<float>(), p.as<float>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(dir_out, d.p, n * 12, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(pdf_out, p.p, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_read_film(void *ctx, float *rgbw, float *sumsq) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_read_film: null context");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_read_film: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    size_t fb = (size_t)c->g.width * c->g.height * 16;
    if (rgbw) HIPC(c, hipMemcpyAsync(rgbw, c->film.p, fb, hipMemcpyDeviceToHost, c->stream));
    if (sumsq) HIPC(c, hipMemcpyAsync(sumsq, c->film_sq.p, fb, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_reset_film(void *ctx) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_reset_film: null context");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_reset_film: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    size_t fb = (size_t)c->g.width * c->g.height * 16;
    HIPC(c, hipMemsetAsync(c->film.p, 0, fb, c->stream));
    HIPC(c, hipMemsetAsync(c->film_sq.p, 0, fb, c->stream));
    if (c->aov_albedo.p) {
        HIPC(c, hipMemsetAsync(c->aov_albedo.p, 0, fb, c->stream));
        HIPC(c, hipMemsetAsync(c->aov_normal.p, 0, fb, c->stream));
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_read_aovs(void *ctx, float *albedo, float *normal) {
    Ctx *c = (Ctx *)ctx;
    if (!c) return fail(nullptr, PG_ERR_INVALID, "pg_read_aovs: null context");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_read_aovs: no scene");
    if (!c->cfg.aovs) return fail(c, PG_ERR_STATE, "pg_read_aovs: the context was created with aovs = 0");
    HIPC(c, hipSetDevice(c->cfg.device));
    size_t fb = (size_t)c->g.width * c->g.height * 16;
    if (albedo) HIPC(c, hipMemcpyAsync(albedo, c->aov_albedo.p, fb, hipMemcpyDeviceToHost, c->stream));
    if (normal) HIPC(c, hipMemcpyAsync(normal, c->aov_normal.p, fb, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_envmap_query(void *ctx, int32_t op, const float *in, uint64_t n, float *out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!in && n) || (!out && n)) return fail(c, PG_ERR_INVALID, "pg_envmap_query: null argument");
    if (op < 0 || op > 2) return fail(c, PG_ERR_INVALID, "pg_envmap_query: bad op");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_envmap_query: no scene");
    if (!c->has_env) return fail(c, PG_ERR_STATE, "pg_envmap_query: the scene has no environment emitter");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!n) return PG_OK;
    const size_t inBytes = n * (op == 0 ? 8 : 12), outBytes = n * (op == 0 ? 32 : op == 1 ? 4 : 12);
    DevBuf a, o;
    HIPC(c, a.alloc(inBytes));
    HIPC(c, o.alloc(outBytes));
    HIPC(c, hipMemcpyAsync(a.p, in, inBytes, hipMemcpyHostToDevice, c->stream));
    pg_launch_envmap_query(c->stream, sceneView(c), op, a.as<float>(), (uint32_t)n, o.as<float>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(out, o.p, outBytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_get_stats(void *ctx, pg_stats *st) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !st) return fail(c, PG_ERR_INVALID, "pg_get_stats: null argument");
    *st = c->stats;
    return PG_OK;
}

pg_status pg_local_pixel_count(void *ctx, uint64_t *count) {
    Ctx *c = (Ctx *)ctx;
    if (!c || !count) return fail(c, PG_ERR_INVALID, "pg_local_pixel_count: null argument");
    *count = c->local_pixels.size();
    return PG_OK;
}

pg_status pg_trace_rays(void *ctx, const float *rays, uint64_t n, int32_t any_hit, float *hits) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!rays && n) || (!hits && n)) return fail(c, PG_ERR_INVALID, "pg_trace_rays: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_trace_rays: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!n) return PG_OK;
    DevBuf r, h, ovf;
    HIPC(c, r.alloc(n * 32));
    HIPC(c, h.alloc(n * 16));
    HIPC(c, ovf.alloc(pg_stack_overflow_words(pg_trace_rays_threads(n)) * 4));
    HIPC(c, hipMemcpyAsync(r.p, rays, n * 32, hipMemcpyHostToDevice, c->stream));
    pg_launch_trace_rays(c->stream, sceneView(c), r.as<float>(), (uint32_t)n, any_hit ? 1 : 0, h.as<float>(),
                         ovf.as<uint32_t>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(hits, h.p, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_hit_records(void *ctx, const float *rays, uint64_t n, float *out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!rays && n) || (!out && n)) return fail(c, PG_ERR_INVALID, "pg_hit_records: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_hit_records: no scene");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!n) return PG_OK;
    DevBuf r, h, ovf;
    HIPC(c, r.alloc(n * 32));
    HIPC(c, h.alloc(n * 64));
    HIPC(c, ovf.alloc(pg_stack_overflow_words(pg_trace_rays_threads(n)) * 4));
    HIPC(c, hipMemcpyAsync(r.p, rays, n * 32, hipMemcpyHostToDevice, c->stream));
    pg_launch_trace_rays(c->stream, sceneView(c), r.as<float>(), (uint32_t)n, 2, h.as<float>(), ovf.as<uint32_t>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(out, h.p, n * 64, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_bsdf_query(void *ctx, uint32_t material, const float *wi, const float *u, const float *wo_given, uint64_t n,
                        float *out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!wi && n) || (!u && n) || (!out && n)) return fail(c, PG_ERR_INVALID, "pg_bsdf_query: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_bsdf_query: no scene");
    if (material >= c->num_mats) return fail(c, PG_ERR_INVALID, "pg_bsdf_query: bad material");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!n) return PG_OK;
    DevBuf a, b, g, o;
    HIPC(c, a.alloc(n * 12));
    HIPC(c, b.alloc(n * 12));
    HIPC(c, o.alloc(n * 48));
    HIPC(c, hipMemcpyAsync(a.p, wi, n * 12, hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(b.p, u, n * 12, hipMemcpyHostToDevice, c->stream));
    if (wo_given) {
        HIPC(c, g.alloc(n * 12));
        HIPC(c, hipMemcpyAsync(g.p, wo_given, n * 12, hipMemcpyHostToDevice, c->stream));
    }
    pg_launch_bsdf_query(c->stream, c->mats.as<GMat>() + material, a.as<float>(), b.as<float>(),
                         wo_given ? g.as<float>() : nullptr, (uint32_t)n, o.as<float>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(out, o.p, n * 48, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_phase_query(void *ctx, uint32_t medium, const float *in, const float *wo_given, uint64_t n, float *out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!in && n) || (!out && n)) return fail(c, PG_ERR_INVALID, "pg_phase_query: null argument");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_phase_query: no scene");
    if (medium >= c->num_media) return fail(c, PG_ERR_INVALID, "pg_phase_query: bad medium");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!n) return PG_OK;
    DevBuf a, g, o;
    HIPC(c, a.alloc(n * 20));
    HIPC(c, o.alloc(n * 20));
    HIPC(c, hipMemcpyAsync(a.p, in, n * 20, hipMemcpyHostToDevice, c->stream));
    if (wo_given) {
        HIPC(c, g.alloc(n * 12));
        HIPC(c, hipMemcpyAsync(g.p, wo_given, n * 12, hipMemcpyHostToDevice, c->stream));
    }
    pg_launch_phase_query(c->stream, c->media.as<GMedium>() + medium, a.as<float>(), wo_given ? g.as<float>() : nullptr,
                          (uint32_t)n, o.as<float>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(out, o.p, n * 20, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

pg_status pg_medium_query(void *ctx, uint32_t medium, int32_t op, const float *in, const uint32_t *keys, uint64_t n,
                          float *out) {
    Ctx *c = (Ctx *)ctx;
    if (!c || (!in && n) || (!out && n) || (op != 0 && !keys && n))
        return fail(c, PG_ERR_INVALID, "pg_medium_query: null argument");
    if (op < 0 || op > 4) return fail(c, PG_ERR_INVALID, "pg_medium_query: bad op");
    if (!c->has_scene) return fail(c, PG_ERR_STATE, "pg_medium_query: no scene");
    if (medium >= c->num_media) return fail(c, PG_ERR_INVALID, "pg_medium_query: bad medium");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!n) return PG_OK;
    const size_t inBytes = n * (op == 0 ? 12 : 32), outBytes = n * (op == 0 ? 4 : 16);
    DevBuf a, k, o;
    HIPC(c, a.alloc(inBytes));
    HIPC(c, o.alloc(outBytes));
    HIPC(c, hipMemcpyAsync(a.p, in, inBytes, hipMemcpyHostToDevice, c->stream));
    if (op != 0) {
        HIPC(c, k.alloc(n * 8));
        HIPC(c, hipMemcpyAsync(k.p, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    }
    pg_launch_medium_query(c->stream, c->media.as<GMedium>() + medium, op, a.as<float>(),
                           op != 0 ? k.as<uint32_t>() : nullptr, (uint32_t)n, o.as<float>());
    HIPC(c, hipGetLastError());
    HIPC(c, hipMemcpyAsync(out, o.p, outBytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return PG_OK;
}

}  // extern "C"
