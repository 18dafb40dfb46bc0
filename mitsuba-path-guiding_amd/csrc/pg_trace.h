// Device-side ray casting and hit/emitter helpers shared by the wavefront kernels (pg_kernels.hip)
// and the volumetric megakernel (pg_volpath.hip).  Included once per translation unit.
#pragma once
#include "pg_device.h"
#include "pg_kernels.h"

using namespace pgd;

// block sizes (C3, profiles/r02zj_block_ab: shading 128 / traversal 256 beat 256 / 128 by 1.7 %)
#ifndef TRACE_BLOCK
#define TRACE_BLOCK 256
#endif
#define STACK_DEPTH 48  // total traversal stack entries (the BVH builder bounds the depth below this)
#ifndef LDS_STACK
#define LDS_STACK 16    // binary BVH: top entries in LDS (4 B each: 16 KiB per block), deeper ones spill
#endif
#ifndef WIDE_LDS_STACK
#define WIDE_LDS_STACK 8  // wide BVH: top group entries in LDS (8 B each: 16 KiB per block)
#endif
#ifndef SHADE_BLOCK
#define SHADE_BLOCK 128
#endif
// persistent grid-stride launches: enough blocks to fill 256 CUs at full occupancy
#ifndef TRACE_MAX_BLOCKS
#define TRACE_MAX_BLOCKS (256 * 16)
#endif

namespace {

// Path-state accesses (every SoA record is read once and written once per bounce).  Non-temporal
// loads/stores here measured +1 % on C3 but made results timing-dependent with three lanes in flight
// (2 outcomes in 12 runs of tools/det_kitchen.py, 1 in 20 without), so they are plain.
// PG_NT_STATE=1 (A/B builds): the non-temporal variant again (round 5, VERDICT r04 item 2: keep the streamed
// state out of the XCD's L2 so the BVH and TriAccel working set stays).
#ifndef PG_NT_STATE
#define PG_NT_STATE 0
#endif
#if PG_NT_STATE
typedef float pgF4v __attribute__((ext_vector_type(4)));
typedef unsigned int pgU4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldS(const float4 *p) {
    const pgF4v v = __builtin_nontemporal_load(reinterpret_cast<const pgF4v *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ldS(const uint4 *p) {
    const pgU4v v = __builtin_nontemporal_load(reinterpret_cast<const pgU4v *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stS(float4 *p, float4 a) {
    const pgF4v v = {a.x, a.y, a.z, a.w};
    __builtin_nontemporal_store(v, reinterpret_cast<pgF4v *>(p));
}
__device__ __forceinline__ void stS(uint4 *p, uint4 a) {
    const pgU4v v = {a.x, a.y, a.z, a.w};
    __builtin_nontemporal_store(v, reinterpret_cast<pgU4v *>(p));
}
#else
__device__ __forceinline__ float4 ldS(const float4 *p) { return *p; }
__device__ __forceinline__ uint4 ldS(const uint4 *p) { return *p; }
__device__ __forceinline__ void stS(float4 *p, float4 a) { *p = a; }
__device__ __forceinline__ void stS(uint4 *p, uint4 a) { *p = a; }
#endif

// Traversal statistics (debug build PG_TRAV_STATS=1, make travstats; tools/r06_trav_stats.py): per walk kind
// (0 closest, 1 any hit) the walks, node visits, triangle tests and executed node-test iterations of whole waves
#ifndef PG_TRAV_STATS
#define PG_TRAV_STATS 0
#endif
#if PG_TRAV_STATS
__device__ unsigned long long pgTravStats[8];
#define PG_TSTAT(i, v) atomicAdd(&pgTravStats[i], (unsigned long long)(v))
#endif

// ---------------------------------------------------------------------------------------------
// BVH traversal.  Replaces ShapeKDTree::rayIntersect / rayIntersectHavran (skdtree.cpp:112-142,
// sahkdtree3.h:178-308) with the same contract: closest t in [tmin, tmax] (any hit for shadow
// rays).  Closest-hit rays walk the 4-wide BVH (128-B nodes; the binary BVH's 64-B nodes in PG_BVH4 = 0
// builds), shadow rays the 8-wide BVH with quantised boxes (80-B nodes); all test the 48-B triangle records
// of pg_layout.h PG_TRIACCEL (the reference's TriAccel).
// Stacks: entries [0, LDS) in LDS (columns per thread, stride TRACE_BLOCK: conflict-free), deeper
// entries in a per-thread column of a global overflow ring (stride = launched threads).
struct TStack {
    uint32_t *lds;
    uint32_t *ovf;
    uint32_t ostride;
    __device__ __forceinline__ void put(int i, uint32_t v) const {
        if (i < LDS_STACK) lds[i * TRACE_BLOCK] = v;
        else ovf[(size_t)(i - LDS_STACK) * ostride] = v;
    }
    __device__ __forceinline__ uint32_t get(int i) const {
        return i < LDS_STACK ? lds[i * TRACE_BLOCK] : ovf[(size_t)(i - LDS_STACK) * ostride];
    }
};
// group entries (base index, hit mask) of the wide traversal
struct WStack {
    uint32_t *lds;
    uint32_t *ovf;
    uint32_t ostride;
    __device__ __forceinline__ void put(int i, uint2 v) const {
        if (i < WIDE_LDS_STACK) {
            lds[(2 * i) * TRACE_BLOCK] = v.x;
            lds[(2 * i + 1) * TRACE_BLOCK] = v.y;
        } else {
            ovf[(size_t)(2 * (i - WIDE_LDS_STACK)) * ostride] = v.x;
            ovf[(size_t)(2 * (i - WIDE_LDS_STACK) + 1) * ostride] = v.y;
        }
    }
    __device__ __forceinline__ uint2 get(int i) const {
        if (i < WIDE_LDS_STACK) return make_uint2(lds[(2 * i) * TRACE_BLOCK], lds[(2 * i + 1) * TRACE_BLOCK]);
        return make_uint2(ovf[(size_t)(2 * (i - WIDE_LDS_STACK)) * ostride],
                          ovf[(size_t)(2 * (i - WIDE_LDS_STACK) + 1) * ostride]);
    }
};

// Triangle test of every walk (pg_layout.h PG_TRIACCEL): a hit at t in [tmin, tmax] with (bu, bv) the
// barycentric weights of p1 and p2.  TriAccel::rayIntersect (triaccel.h:96-157) with the reference's
// expression order and no contraction: the oracle's t, u, v bit for bit.
// PG_TRI_PRELOAD=1: the record's three rows loaded together up front instead of rows 1 and 2 only for the
// lanes whose earlier tests pass (the later rows are cache hits of the same lines): k_rays 23.72-23.83
// against 23.82-23.91 ms per calibration pass, C3 609-613 against 613-621 Mpaths/s (profiles/r05af_tri_preload/);
// off by default
#ifndef PG_TRI_PRELOAD
#define PG_TRI_PRELOAD 0
#endif
// triHitRow0: the test with the record's first row already loaded (the paired walk issues both rays' rows first)
__device__ __forceinline__ bool triHitRow0(const float4 r0, const float4 *__restrict__ tris, uint32_t tr, f3 o, f3 d,
                                           float tmin, float tmax, float &tt, float &bu, float &bv) {
#pragma clang fp contract(off)
#if PG_TRI_PRELOAD
    const float4 r1 = tris[PG_TRI_ROW(tr, 1)];
    const float2 r2 = *reinterpret_cast<const float2 *>(tris + PG_TRI_ROW(tr, 2));
#endif
    const uint32_t k = __float_as_uint(r0.w);  // projection axis; (u, v) = the next two axes cyclically
    const float ou = k == 0 ? o.y : (k == 1 ? o.z : o.x), ov = k == 0 ? o.z : (k == 1 ? o.x : o.y);
    const float ok = k == 0 ? o.x : (k == 1 ? o.y : o.z);
    const float du = k == 0 ? d.y : (k == 1 ? d.z : d.x), dv = k == 0 ? d.z : (k == 1 ? d.x : d.y);
    const float dk = k == 0 ? d.x : (k == 1 ? d.y : d.z);
    tt = (r0.z - ou * r0.x - ov * r0.y - ok) / (du * r0.x + dv * r0.y + dk);
    if (!(tt >= tmin && tt <= tmax)) return false;
#if !PG_TRI_PRELOAD
    const float4 r1 = tris[PG_TRI_ROW(tr, 1)];
#endif
    const float hu = ou + tt * du - r1.x, hv = ov + tt * dv - r1.y;
    const float u = hv * r1.z + hu * r1.w;
    if (!(u >= 0.0f)) return false;
#if !PG_TRI_PRELOAD
    const float2 r2 = *reinterpret_cast<const float2 *>(tris + PG_TRI_ROW(tr, 2));
#endif
    const float v = hu * r2.x + hv * r2.y;
    if (!(v >= 0.0f && u + v <= 1.0f)) return false;
    bu = u;
    bv = v;
    return true;
}
__device__ __forceinline__ bool triHit(const float4 *__restrict__ tris, uint32_t tr, f3 o, f3 d, float tmin, float tmax,
                                       float &tt, float &bu, float &bv) {
#if PG_TRIACCEL
    return triHitRow0(tris[PG_TRI_ROW(tr, 0)], tris, tr, o, d, tmin, tmax, tt, bu, bv);
#else
    const float4 w0 = tris[PG_TRI_ROW(tr, 0)];
    float dz = d.x * w0.x + d.y * w0.y + d.z * w0.z;
    float oz = w0.w - (o.x * w0.x + o.y * w0.y + o.z * w0.z);
    tt = oz / dz;
    if (!(tt >= tmin && tt <= tmax)) return false;
    const float4 w1 = tris[PG_TRI_ROW(tr, 1)];
    float a = (w1.w + o.x * w1.x + o.y * w1.y + o.z * w1.z) + tt * (d.x * w1.x + d.y * w1.y + d.z * w1.z);
    if (!(a >= 0.0f && a <= 1.0f)) return false;
    const float4 w2 = tris[PG_TRI_ROW(tr, 2)];
    float b = (w2.w + o.x * w2.x + o.y * w2.y + o.z * w2.z) + tt * (d.x * w2.x + d.y * w2.y + d.z * w2.z);
    if (!(b >= 0.0f && a + b <= 1.0f)) return false;
    bu = b;             // weight of p1
    bv = 1.0f - a - b;  // weight of p2
    return true;
#endif
}

// Closest-hit accept rule of every walk: a smaller t, or an equal t (shared edges, coplanar triangles)
// on the lower ORIGINAL triangle index (TriAccel row 2, .z; pg_bvh.cpp triAccelRecord), the oracle's
// rule (orc_scene.h Scene::traverse / bruteForce), so a tie resolves the same way on both sides and
// whatever the BVH order.  The ids are loaded only on a tie.
__device__ __forceinline__ bool acceptHit(const float4 *__restrict__ tris, float tt, float tmax, uint32_t tr,
                                          uint32_t hitTri) {
    if (tt < tmax || hitTri == 0xFFFFFFFFu) return true;
#if PG_TRIACCEL
    return __float_as_uint(tris[PG_TRI_ROW(tr, 2)].z) < __float_as_uint(tris[PG_TRI_ROW(hitTri, 2)].z);
#else
    return tr < hitTri;  // Woop rows carry no original id: BVH order (A/B builds only)
#endif
}

__device__ __forceinline__ float qbyte(uint32_t lo, uint32_t hi, int s) {
    return (float)(((s < 4 ? lo : hi) >> (8 * (s & 3))) & 0xFFu);
}
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float min3f(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// bit s of m moves to bit s ^ x (x < 8): three conditional swaps of bit groups
__device__ __forceinline__ uint32_t permuteXor8(uint32_t m, uint32_t x) {
    if (x & 1u) m = ((m & 0x55u) << 1) | ((m >> 1) & 0x55u);
    if (x & 2u) m = ((m & 0x33u) << 2) | ((m >> 2) & 0x33u);
    if (x & 4u) m = ((m & 0x0Fu) << 4) | ((m >> 4) & 0x0Fu);
    return m;
}

// PG_NODE_PK (round 6, default): a slot's near- and far-plane distances of one axis as one packed fma
// (v_pk_fma_f32 computes two fp32 lanes per instruction at the VALU's full rate), the same fmas bit for bit
#ifndef PG_NODE_PK
#define PG_NODE_PK 0
#endif
typedef float pgf2 __attribute__((ext_vector_type(2)));

// PG_LEAF_PAIRS (default): leaf triangles are taken two at a time with both first rows loaded before either
// test (the tests, and so the accepted hit, stay in triangle order): closest hits k_rays 22.1 against 22.5 ms
// per calibration pass, C3 634-635 against 625-626 Mpaths/s (profiles/r06_leafpairs/).  PG_LEAF_PAIRS=3 / 4 take
// three / four per step: k_rays 22.13 / 22.42 against 22.02 ms (profiles/r06_leafgroup/)
#ifndef PG_LEAF_PAIRS
#define PG_LEAF_PAIRS 1
#endif
// the same for the 8-wide walk's triangle groups (shadow rays): k_rays 21.75 against 22.21 ms, C3 653 against
// 649 Mpaths/s (profiles/r06_wideleafpairs/)
#ifndef PG_WIDE_LEAF_PAIRS
#define PG_WIDE_LEAF_PAIRS 1
#endif
// Traversal of the 8-wide BVH (after Ylitie, Karras & Laine 2017): the current node group
// G = (child_base, hit bits 24..31 in octant order | imask bits 0..7) and triangle group
// T = (tri_base, hit bits 0..23); one node is opened per step, its remaining siblings stay on the
// stack as one group entry.  (Postponing triangle groups while few lanes have triangle work, as
// in the paper, measured slower here: 20.0 vs 17.4 ms per pass.)
template <bool ANY>
__device__ __forceinline__ bool traverseWide(const float4 *__restrict__ nodes, const float4 *__restrict__ tris, f3 o,
                                             f3 d, float tmin, float &tmax, uint32_t &hitTri, float &hu, float &hv,
                                             const WStack &stk) {
    const float eps = 1e-30f;
    const f3 idir = mk(1.0f / (fabsf(d.x) > eps ? d.x : copysignf(eps, d.x)),
                       1.0f / (fabsf(d.y) > eps ? d.y : copysignf(eps, d.y)),
                       1.0f / (fabsf(d.z) > eps ? d.z : copysignf(eps, d.z)));
    // 7 - octant: bit a set where the direction is non-negative along axis a
    const uint32_t octinv = (d.x < 0 ? 0u : 1u) | (d.y < 0 ? 0u : 2u) | (d.z < 0 ? 0u : 4u);
    uint2 G = make_uint2(0u, 0x80000000u);  // the root, as a one-node group
    uint2 T = make_uint2(0u, 0u);
    int sp = 0;
    bool found = false;
#if PG_TRAV_STATS
    PG_TSTAT(4, 1);
#endif
    for (;;) {
        if (G.y > 0x00FFFFFFu) {
#if PG_TRAV_STATS
            PG_TSTAT(5, 1);
#endif
            const int bit = 31 - __clz(G.y);
            const uint32_t slot = (uint32_t)(bit - 24) ^ octinv;
            const uint32_t ni = G.x + __popc(G.y & 0xFFu & ((1u << slot) - 1u));
            G.y &= ~(1u << bit);
            if (G.y > 0x00FFFFFFu) stk.put(sp++, G);
            const float4 n0 = nodes[PG_WIDE_NODE_F4 * ni + 0];
            const float4 n1 = nodes[PG_WIDE_NODE_F4 * ni + 1];
            const float4 n2 = nodes[PG_WIDE_NODE_F4 * ni + 2];
            const float4 n3 = nodes[PG_WIDE_NODE_F4 * ni + 3];
            const float4 n4 = nodes[PG_WIDE_NODE_F4 * ni + 4];
            const uint32_t e = __float_as_uint(n0.w);
            // t = q * (2^e * idir) + (p - o) * idir per axis; the near plane of each axis is the lo
            // byte for a non-negative direction and the hi byte otherwise (chosen once per node)
            const float ax = __uint_as_float((e & 0xFFu) << 23) * idir.x, bx = (n0.x - o.x) * idir.x;
            const float ay = __uint_as_float(((e >> 8) & 0xFFu) << 23) * idir.y, by = (n0.y - o.y) * idir.y;
            const float az = __uint_as_float(((e >> 16) & 0xFFu) << 23) * idir.z, bz = (n0.z - o.z) * idir.z;
            const uint32_t imask = e >> 24;
            const bool px = octinv & 1u, py = octinv & 2u, pz = octinv & 4u;
            const uint32_t loX0 = __float_as_uint(n2.x), loX1 = __float_as_uint(n2.y);
            const uint32_t loY0 = __float_as_uint(n2.z), loY1 = __float_as_uint(n2.w);
            const uint32_t loZ0 = __float_as_uint(n3.x), loZ1 = __float_as_uint(n3.y);
            const uint32_t hiX0 = __float_as_uint(n3.z), hiX1 = __float_as_uint(n3.w);
            const uint32_t hiY0 = __float_as_uint(n4.x), hiY1 = __float_as_uint(n4.y);
            const uint32_t hiZ0 = __float_as_uint(n4.z), hiZ1 = __float_as_uint(n4.w);
            const uint32_t nX0 = px ? loX0 : hiX0, nX1 = px ? loX1 : hiX1, fX0 = px ? hiX0 : loX0, fX1 = px ? hiX1 : loX1;
            const uint32_t nY0 = py ? loY0 : hiY0, nY1 = py ? loY1 : hiY1, fY0 = py ? hiY0 : loY0, fY1 = py ? hiY1 : loY1;
            const uint32_t nZ0 = pz ? loZ0 : hiZ0, nZ1 = pz ? loZ1 : hiZ1, fZ0 = pz ? hiZ0 : loZ0, fZ1 = pz ? hiZ1 : loZ1;
            uint32_t hitSlots = 0;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
#if PG_NODE_PK  // (near, far) of an axis as one packed fma (pg_trace.h traverse4)
                const pgf2 tx = __builtin_elementwise_fma(pgf2{qbyte(nX0, nX1, s), qbyte(fX0, fX1, s)}, pgf2{ax, ax}, pgf2{bx, bx});
                const pgf2 ty = __builtin_elementwise_fma(pgf2{qbyte(nY0, nY1, s), qbyte(fY0, fY1, s)}, pgf2{ay, ay}, pgf2{by, by});
                const pgf2 tz = __builtin_elementwise_fma(pgf2{qbyte(nZ0, nZ1, s), qbyte(fZ0, fZ1, s)}, pgf2{az, az}, pgf2{bz, bz});
                const float cmin = max3f(tx.x, ty.x, fmaxf(tz.x, tmin));
                const float cmax = min3f(tx.y, ty.y, fminf(tz.y, tmax));
#else
                const float tnx = fmaf(qbyte(nX0, nX1, s), ax, bx), tfx = fmaf(qbyte(fX0, fX1, s), ax, bx);
                const float tny = fmaf(qbyte(nY0, nY1, s), ay, by), tfy = fmaf(qbyte(fY0, fY1, s), ay, by);
                const float tnz = fmaf(qbyte(nZ0, nZ1, s), az, bz), tfz = fmaf(qbyte(fZ0, fZ1, s), az, bz);
                const float cmin = max3f(tnx, tny, fmaxf(tnz, tmin));
                const float cmax = min3f(tfx, tfy, fminf(tfz, tmax));
#endif
                hitSlots |= (cmin <= cmax ? 1u : 0u) << s;
            }
            const uint32_t nodeHits = permuteXor8(hitSlots & imask, octinv) << 24;
            uint32_t triHits = 0;
            const uint32_t meta0 = __float_as_uint(n1.z), meta1 = __float_as_uint(n1.w);
            for (uint32_t leaves = hitSlots & ~imask; leaves; leaves &= leaves - 1u) {
                const int s = __ffs(leaves) - 1;
                const uint32_t meta = ((s < 4 ? meta0 : meta1) >> (8 * (s & 3))) & 0xFFu;
                triHits |= ((1u << (meta >> 5)) - 1u) << (meta & 31u);
            }
            G = make_uint2(__float_as_uint(n1.x), nodeHits | imask);
            T = make_uint2(__float_as_uint(n1.y), triHits);
        }
#if PG_WIDE_LEAF_PAIRS && PG_TRIACCEL && !PG_TRAV_STATS
        while (T.y != 0) {  // two triangles per step, both first rows loaded up front
            const uint32_t ta = T.x + (uint32_t)(__ffs(T.y) - 1);
            T.y &= T.y - 1u;
            const bool two = T.y != 0;
            const uint32_t tb = two ? T.x + (uint32_t)(__ffs(T.y) - 1) : ta;
            if (two) T.y &= T.y - 1u;
            const float4 ra = tris[PG_TRI_ROW(ta, 0)], rb = tris[PG_TRI_ROW(tb, 0)];
            float tt, bu, bv;
            if (triHitRow0(ra, tris, ta, o, d, tmin, tmax, tt, bu, bv) && acceptHit(tris, tt, tmax, ta, hitTri)) {
                found = true;
                if (ANY) return true;
                tmax = tt;
                hitTri = ta;
                hu = bu;
                hv = bv;
            }
            if (two && triHitRow0(rb, tris, tb, o, d, tmin, tmax, tt, bu, bv) && acceptHit(tris, tt, tmax, tb, hitTri)) {
                found = true;
                if (ANY) return true;
                tmax = tt;
                hitTri = tb;
                hu = bu;
                hv = bv;
            }
        }
#else
        while (T.y != 0) {
            const uint32_t tr = T.x + (uint32_t)(__ffs(T.y) - 1);
            T.y &= T.y - 1u;
#if PG_TRAV_STATS
            PG_TSTAT(6, 1);
#endif
            float tt, bu, bv;
            if (triHit(tris, tr, o, d, tmin, tmax, tt, bu, bv) && acceptHit(tris, tt, tmax, tr, hitTri)) {
                found = true;
                if (ANY) return true;
                tmax = tt;
                hitTri = tr;
                hu = bu;
                hv = bv;
            }
        }
#endif
        if (G.y <= 0x00FFFFFFu) {
            if (sp == 0) break;
            G = stk.get(--sp);
        }
    }
    return found;
}

// Postponed-leaf triangle tests shared by the binary and the 4-wide closest-hit walks: every
// triangle of leaf ref `leaf` (< 0: ~leaf = first << 4 | count) against the ray.
template <bool ANY>
__device__ __forceinline__ bool leafTest(const float4 *__restrict__ tris, int leaf, f3 o, f3 d, float tmin,
                                         float &tmax, uint32_t &hitTri, float &hu, float &hv, bool &found) {
    const uint32_t lr = ~(uint32_t)leaf;
    const uint32_t first = lr >> 4, cnt = lr & 15u;
#if PG_LEAF_PAIRS && PG_TRIACCEL
    constexpr uint32_t G = PG_LEAF_PAIRS > 1 ? PG_LEAF_PAIRS : 2;  // triangles per step
    for (uint32_t k = 0; k < cnt; k += G) {
        float4 r[G];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) r[j] = tris[PG_TRI_ROW(first + min(k + j, cnt - 1), 0)];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) {
            const uint32_t tr = first + k + j;
            float tt, bu, bv;
            if (k + j < cnt && triHitRow0(r[j], tris, tr, o, d, tmin, tmax, tt, bu, bv) && acceptHit(tris, tt, tmax, tr, hitTri)) {
                found = true;
                if (ANY) return true;
                tmax = tt;
                hitTri = tr;
                hu = bu;
                hv = bv;
            }
        }
    }
#else
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint32_t tr = first + k;
        float tt, bu, bv;
        // equal distances: the lower original triangle index (acceptHit)
        if (triHit(tris, tr, o, d, tmin, tmax, tt, bu, bv) && acceptHit(tris, tt, tmax, tr, hitTri)) {
            found = true;
            if (ANY) return true;
            tmax = tt;
            hitTri = tr;
            hu = bu;
            hv = bv;
        }
    }
#endif
    return false;
}

// ascending compare-exchange of (key, ref) pairs
__device__ __forceinline__ void cxch(float &ka, int &ra, float &kb, int &rb) {
    const bool s = kb < ka;
    const float k = s ? kb : ka;
    kb = s ? ka : kb;
    ka = k;
    const int r = s ? rb : ra;
    rb = s ? ra : rb;
    ra = r;
}

// Per-ray slab-test setup of the closest-hit walks.  t = fma(plane, idir, add) per axis; with
// PG_ROBUST_BOX (default) the addends move each axis's near plane earlier and its far plane later by
// 2^-21 |o_a idir_a| -- a spatial padding of 2^-21 |o_a| along that axis, which bounds the rounding of
// o * idir and of the fma -- and box intervals are compared as cmin <= cmax (1 + 2^-21) for the
// rounding relative to t.  Without it a ray clipping a box edge far from the origin could see its
// rounded interval come out empty while it hits the triangle inside (tests/test_bvh4_build.py, a
// strip of triangles spanning 1 to 1.6e5: 0.55 % of the rays).  It costs one multiply per box; a
// global slack of 1e-6 max|o idir| instead made the kitchen's traversal 2.8x slower (near-axis rays).
#ifndef PG_ROBUST_BOX
#define PG_ROBUST_BOX 1
#endif
struct SlabRay {
    f3 idir, addLo, addHi;
    float tslack;  // culling-distance slack (tie rule): a few ulps of the largest |o_a idir_a|
};
constexpr float kBoxRel = PG_ROBUST_BOX ? 1.000000477f : 1.0f;  // 1 + 2^-21
__device__ __forceinline__ SlabRay slabRay(f3 o, f3 d) {
    const float eps = 1e-30f;
    SlabRay r;
    r.idir = mk(1.0f / (fabsf(d.x) > eps ? d.x : copysignf(eps, d.x)), 1.0f / (fabsf(d.y) > eps ? d.y : copysignf(eps, d.y)),
                1.0f / (fabsf(d.z) > eps ? d.z : copysignf(eps, d.z)));
    const f3 ood = o * r.idir;
    r.tslack = 1e-6f * fmaxf(fmaxf(fabsf(ood.x), fabsf(ood.y)), fabsf(ood.z));
    const float k = PG_ROBUST_BOX ? 4.76837158e-7f : 0.0f;  // 2^-21
    const f3 se = mk(copysignf(k * fabsf(ood.x), r.idir.x), copysignf(k * fabsf(ood.y), r.idir.y),
                     copysignf(k * fabsf(ood.z), r.idir.z));
    r.addLo = -ood - se;  // the lo plane is the near one for idir >= 0
    r.addHi = -ood + se;
    return r;
}

// Closest-hit walk of the 4-wide BVH (PG_BVH4): one 128-B node per visit instead of two 64-B binary
// nodes, its hit children visited nearest first (a 5-exchange sorting network on the entry
// distances; the others pushed far to near), with the binary walk's while-while loop, postponed
// leaves, tie rule and widened culling distance, so it returns the same hit.
// LTOP: nodes [0, ntop) are read from `lnodes` (the breadth-first top levels, staged in LDS by the caller)
// PG_NODE_NEARFAR (round 6, default): each axis's near and far planes chosen once per node by the ray's
// direction sign (the lo plane is the near one for idir >= 0), so a slot's entry and exit distances are one
// max3 / min3 each instead of a min and a max per axis.  The same distances and comparisons as the min/max
// form bit for bit: for a non-empty slot lo <= hi and the padded addends keep their order, so min(lo-plane t,
// hi-plane t) IS the near plane's t (empty slots are rejected by their ref either way).  The walk is VALU-bound
// (~4 cycles x 1.0 M VALU wave-instructions per SIMD per k_rays launch against its ~4.8 M cycles)
#ifndef PG_NODE_NEARFAR
#define PG_NODE_NEARFAR 1
#endif
template <bool ANY, bool LTOP = false>
__device__ __forceinline__ bool traverse4(const float4 *__restrict__ nodes, const float4 *__restrict__ tris, f3 o, f3 d,
                                          float tmin, float &tmax, uint32_t &hitTri, float &hu, float &hv,
                                          const TStack &stk, const float4 *lnodes = nullptr, int ntop = 0) {
    const int DONE = 0x7fffffff;
    const float INF = __builtin_huge_valf();
    const SlabRay sr = slabRay(o, d);
    const f3 idir = sr.idir, aLo = sr.addLo, aHi = sr.addHi;
    const float tslack = sr.tslack;
#if PG_QNODE_QUANT && PG_NODE_NEARFAR
    const bool negx = idir.x < 0.0f, negy = idir.y < 0.0f, negz = idir.z < 0.0f;
    const f3 aN = mk(negx ? aHi.x : aLo.x, negy ? aHi.y : aLo.y, negz ? aHi.z : aLo.z);
    const f3 aF = mk(negx ? aLo.x : aHi.x, negy ? aLo.y : aHi.y, negz ? aLo.z : aHi.z);
#endif
    int sp = 0;
    int node = 0;
    int leaf = 0;
    bool found = false;
#if PG_TRAV_STATS
    uint32_t nVisit = 0, nTri = 0;
#endif
    while (node != DONE) {
        const float tcull = tmax * 1.000001f + tslack;
        while (node >= 0 && node != DONE) {
#if PG_TRAV_STATS
            nVisit++;
#endif
            const float4 *np = nodes + (size_t)PG_QNODE_F4 * node;
            float k[4];
            int r[4];
#if PG_QNODE_QUANT
            // planes origin + q 2^e: t = q (2^e idir) + (origin - o) idir, the latter padded outward by
            // slabRay's addends and by 2^-22 |origin idir| (its own rounding)
            float4 n0, rf, q0, q1;
            if (LTOP && node < ntop) {  // LDS loads for the staged top levels, global loads below them
                const float4 *lp = lnodes + (size_t)PG_QNODE_F4 * node;
                n0 = lp[0];
                rf = lp[1];
                q0 = lp[2];
                q1 = lp[3];
            } else {
                n0 = np[0];
                rf = np[1];
                q0 = np[2];
                q1 = np[3];
            }
            const uint32_t e = __float_as_uint(n0.w);
            const float sx = __uint_as_float((e & 0xFFu) << 23) * idir.x;
            const float sy = __uint_as_float(((e >> 8) & 0xFFu) << 23) * idir.y;
            const float sz = __uint_as_float(((e >> 16) & 0xFFu) << 23) * idir.z;
#if PG_NODE_NEARFAR
            // |padding| per axis; near addend - it, far addend + it (the sign-carrying form below, unrolled)
            const float ax = 2.38418579e-7f * fabsf(n0.x * idir.x);
            const float ay = 2.38418579e-7f * fabsf(n0.y * idir.y);
            const float az = 2.38418579e-7f * fabsf(n0.z * idir.z);
#if !PG_NODE_PK
            const float bnx = fmaf(n0.x, idir.x, aN.x) - ax, bfx = fmaf(n0.x, idir.x, aF.x) + ax;
            const float bny = fmaf(n0.y, idir.y, aN.y) - ay, bfy = fmaf(n0.y, idir.y, aF.y) + ay;
            const float bnz = fmaf(n0.z, idir.z, aN.z) - az, bfz = fmaf(n0.z, idir.z, aF.z) + az;
#endif
            const uint32_t wnx = __float_as_uint(negx ? q0.y : q0.x), wfx = __float_as_uint(negx ? q0.x : q0.y);
            const uint32_t wny = __float_as_uint(negy ? q0.w : q0.z), wfy = __float_as_uint(negy ? q0.z : q0.w);
            const uint32_t wnz = __float_as_uint(negz ? q1.y : q1.x), wfz = __float_as_uint(negz ? q1.x : q1.y);
#if PG_NODE_PK
            // (near, far) of an axis as one packed fma (v_pk_fma_f32: two lanes of fp32 per instruction)
            const pgf2 sx2 = {sx, sx}, sy2 = {sy, sy}, sz2 = {sz, sz};
            const pgf2 bx2 = __builtin_elementwise_fma(pgf2{n0.x, n0.x}, pgf2{idir.x, idir.x}, pgf2{aN.x, aF.x}) + pgf2{-ax, ax};
            const pgf2 by2 = __builtin_elementwise_fma(pgf2{n0.y, n0.y}, pgf2{idir.y, idir.y}, pgf2{aN.y, aF.y}) + pgf2{-ay, ay};
            const pgf2 bz2 = __builtin_elementwise_fma(pgf2{n0.z, n0.z}, pgf2{idir.z, idir.z}, pgf2{aN.z, aF.z}) + pgf2{-az, az};
#define PG_QB(w, i) ((float)(((w) >> (8 * (i))) & 0xFFu))
#define PG_Q4_SLOT(i, c)                                                                              \
    {                                                                                                 \
        const pgf2 tx = __builtin_elementwise_fma(pgf2{PG_QB(wnx, i), PG_QB(wfx, i)}, sx2, bx2);        \
        const pgf2 ty = __builtin_elementwise_fma(pgf2{PG_QB(wny, i), PG_QB(wfy, i)}, sy2, by2);        \
        const pgf2 tz = __builtin_elementwise_fma(pgf2{PG_QB(wnz, i), PG_QB(wfz, i)}, sz2, bz2);        \
        const float cmin = fmaxf(fmaxf(tx.x, ty.x), fmaxf(tz.x, tmin));                               \
        const float cmax = fminf(fminf(tx.y, ty.y), fminf(tz.y, tcull));                              \
        r[i] = __float_as_int(rf.c);                                                                  \
        k[i] = (cmin <= cmax * kBoxRel && r[i] != PG_QNODE_EMPTY) ? cmin : INF;                       \
    }
#else
#define PG_QB(w, i) ((float)(((w) >> (8 * (i))) & 0xFFu))
#define PG_Q4_SLOT(i, c)                                                                              \
    {                                                                                                 \
        const float tnx = fmaf(PG_QB(wnx, i), sx, bnx), tfx = fmaf(PG_QB(wfx, i), sx, bfx);           \
        const float tny = fmaf(PG_QB(wny, i), sy, bny), tfy = fmaf(PG_QB(wfy, i), sy, bfy);           \
        const float tnz = fmaf(PG_QB(wnz, i), sz, bnz), tfz = fmaf(PG_QB(wfz, i), sz, bfz);           \
        const float cmin = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, tmin));                                  \
        const float cmax = fminf(fminf(tfx, tfy), fminf(tfz, tcull));                                 \
        r[i] = __float_as_int(rf.c);                                                                  \
        k[i] = (cmin <= cmax * kBoxRel && r[i] != PG_QNODE_EMPTY) ? cmin : INF;                       \
    }
#endif
#else
            const float px = copysignf(2.38418579e-7f * fabsf(n0.x * idir.x), idir.x);
            const float py = copysignf(2.38418579e-7f * fabsf(n0.y * idir.y), idir.y);
            const float pz = copysignf(2.38418579e-7f * fabsf(n0.z * idir.z), idir.z);
            const float bxl = fmaf(n0.x, idir.x, aLo.x) - px, bxh = fmaf(n0.x, idir.x, aHi.x) + px;
            const float byl = fmaf(n0.y, idir.y, aLo.y) - py, byh = fmaf(n0.y, idir.y, aHi.y) + py;
            const float bzl = fmaf(n0.z, idir.z, aLo.z) - pz, bzh = fmaf(n0.z, idir.z, aHi.z) + pz;
            const uint32_t wlx = __float_as_uint(q0.x), whx = __float_as_uint(q0.y), wly = __float_as_uint(q0.z),
                           why = __float_as_uint(q0.w), wlz = __float_as_uint(q1.x), whz = __float_as_uint(q1.y);
#define PG_QB(w, i) ((float)(((w) >> (8 * (i))) & 0xFFu))
#define PG_Q4_SLOT(i, c)                                                                              \
    {                                                                                                 \
        const float x0 = fmaf(PG_QB(wlx, i), sx, bxl), x1 = fmaf(PG_QB(whx, i), sx, bxh);              \
        const float y0 = fmaf(PG_QB(wly, i), sy, byl), y1 = fmaf(PG_QB(why, i), sy, byh);              \
        const float z0 = fmaf(PG_QB(wlz, i), sz, bzl), z1 = fmaf(PG_QB(whz, i), sz, bzh);              \
        const float cmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), tmin));    \
        const float cmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tcull));   \
        r[i] = __float_as_int(rf.c);                                                                  \
        k[i] = (cmin <= cmax * kBoxRel && r[i] != PG_QNODE_EMPTY) ? cmin : INF;                       \
    }
#endif
#else
            const float4 *fp = (LTOP && node < ntop) ? lnodes + (size_t)PG_QNODE_F4 * node : np;
            const float4 lx = fp[0], hx = fp[1], ly = fp[2], hy = fp[3], lz = fp[4], hz = fp[5];
            const float4 rf = fp[6];
#define PG_Q4_SLOT(i, c)                                                                              \
    {                                                                                                 \
        const float x0 = fmaf(lx.c, idir.x, aLo.x), x1 = fmaf(hx.c, idir.x, aHi.x);                   \
        const float y0 = fmaf(ly.c, idir.y, aLo.y), y1 = fmaf(hy.c, idir.y, aHi.y);                   \
        const float z0 = fmaf(lz.c, idir.z, aLo.z), z1 = fmaf(hz.c, idir.z, aHi.z);                   \
        const float cmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), tmin));    \
        const float cmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tcull));   \
        r[i] = __float_as_int(rf.c);                                                                  \
        k[i] = (cmin <= cmax * kBoxRel && r[i] != PG_QNODE_EMPTY) ? cmin : INF;                       \
    }
#endif
            PG_Q4_SLOT(0, x) PG_Q4_SLOT(1, y) PG_Q4_SLOT(2, z) PG_Q4_SLOT(3, w)
#undef PG_Q4_SLOT
#undef PG_QB
            cxch(k[0], r[0], k[1], r[1]);
            cxch(k[2], r[2], k[3], r[3]);
            cxch(k[0], r[0], k[2], r[2]);
            cxch(k[1], r[1], k[3], r[3]);
            cxch(k[1], r[1], k[2], r[2]);
            if (k[0] == INF) {
                node = sp > 0 ? (int)stk.get(--sp) : DONE;
            } else {
                node = r[0];
                if (k[3] != INF && sp < PG_QSTACK_DEPTH) stk.put(sp++, (uint32_t)r[3]);
                if (k[2] != INF && sp < PG_QSTACK_DEPTH) stk.put(sp++, (uint32_t)r[2]);
                if (k[1] != INF && sp < PG_QSTACK_DEPTH) stk.put(sp++, (uint32_t)r[1]);
            }
            if (node < 0 && leaf >= 0) {
                leaf = node;
                node = sp > 0 ? (int)stk.get(--sp) : DONE;
            }
            if (!__any(leaf >= 0)) break;
        }
        while (leaf < 0) {
#if PG_TRAV_STATS
            nTri += (~(uint32_t)leaf) & 15u;
#endif
            if (leafTest<ANY>(tris, leaf, o, d, tmin, tmax, hitTri, hu, hv, found)) return true;
            leaf = node;
            if (node < 0) node = sp > 0 ? (int)stk.get(--sp) : DONE;
        }
    }
#if PG_TRAV_STATS
    PG_TSTAT(0, 1);
    PG_TSTAT(1, nVisit);
    PG_TSTAT(2, nTri);
#endif
    return found;
}

// ---- the 4-wide closest-hit walk as a resumable state (PG_TRACE_PERSIST, pg_kernels.hip traceRowsPersist) ----
// The same per-ray constants, node test, sorting network, postponed leaf, tie rule and culling distance as
// traverse4's default configuration (PG_QNODE_QUANT, PG_NODE_NEARFAR), split so a lane can run one round of
// the while-while loop at a time: between rounds, lanes whose ray finished take a new ray, so the wave's lanes
// stay busy instead of waiting for the round's longest ray.  Each ray's own sequence of node visits and leaf
// tests is traverse4's, so it returns the same hit.
struct Walk4 {
    f3 o, d, idir, aN, aF;
    float tmin, tmax, tslack, hu, hv;
    uint32_t hitTri;
    int node, leaf, sp;
    bool negx, negy, negz;
};
__device__ __forceinline__ void walk4Start(Walk4 &w, f3 o, f3 d, float tmin, float tmax) {
    const SlabRay sr = slabRay(o, d);
    w.o = o;
    w.d = d;
    w.idir = sr.idir;
    w.tslack = sr.tslack;
    w.negx = sr.idir.x < 0.0f;
    w.negy = sr.idir.y < 0.0f;
    w.negz = sr.idir.z < 0.0f;
    w.aN = mk(w.negx ? sr.addHi.x : sr.addLo.x, w.negy ? sr.addHi.y : sr.addLo.y, w.negz ? sr.addHi.z : sr.addLo.z);
    w.aF = mk(w.negx ? sr.addLo.x : sr.addHi.x, w.negy ? sr.addLo.y : sr.addHi.y, w.negz ? sr.addLo.z : sr.addHi.z);
    w.tmin = tmin;
    w.tmax = tmax;
    w.hitTri = 0xFFFFFFFFu;
    w.hu = w.hv = 0.0f;
    w.node = 0;
    w.leaf = 0;
    w.sp = 0;
}
// one node of the 4-wide BVH (quantised: origin + exponents, child refs, near/far byte planes)
struct QNode4 {
    float4 n0, rf, q0, q1;
};
__device__ __forceinline__ QNode4 walk4Fetch(const float4 *__restrict__ nodes, int node) {
    const float4 *np = nodes + (size_t)PG_QNODE_F4 * node;
    return QNode4{np[0], np[1], np[2], np[3]};
}
// one node visit of traverse4 on fetched node data: w.node becomes the nearest hit child (the others pushed
// far to near) or the popped entry, and a leaf is parked in w.leaf when that slot is free
__device__ __forceinline__ void walk4Visit(Walk4 &w, const QNode4 &nd, float tcull, const TStack &stk) {
    const int DONE = 0x7fffffff;
    const float INF = __builtin_huge_valf();
    const float4 n0 = nd.n0, rf = nd.rf, q0 = nd.q0, q1 = nd.q1;
    const f3 idir = w.idir;
    const uint32_t e = __float_as_uint(n0.w);
    const float sx = __uint_as_float((e & 0xFFu) << 23) * idir.x;
    const float sy = __uint_as_float(((e >> 8) & 0xFFu) << 23) * idir.y;
    const float sz = __uint_as_float(((e >> 16) & 0xFFu) << 23) * idir.z;
    const float ax = 2.38418579e-7f * fabsf(n0.x * idir.x);
    const float ay = 2.38418579e-7f * fabsf(n0.y * idir.y);
    const float az = 2.38418579e-7f * fabsf(n0.z * idir.z);
    const float bnx = fmaf(n0.x, idir.x, w.aN.x) - ax, bfx = fmaf(n0.x, idir.x, w.aF.x) + ax;
    const float bny = fmaf(n0.y, idir.y, w.aN.y) - ay, bfy = fmaf(n0.y, idir.y, w.aF.y) + ay;
    const float bnz = fmaf(n0.z, idir.z, w.aN.z) - az, bfz = fmaf(n0.z, idir.z, w.aF.z) + az;
    const uint32_t wnx = __float_as_uint(w.negx ? q0.y : q0.x), wfx = __float_as_uint(w.negx ? q0.x : q0.y);
    const uint32_t wny = __float_as_uint(w.negy ? q0.w : q0.z), wfy = __float_as_uint(w.negy ? q0.z : q0.w);
    const uint32_t wnz = __float_as_uint(w.negz ? q1.y : q1.x), wfz = __float_as_uint(w.negz ? q1.x : q1.y);
    float k[4];
    int r[4];
#define PG_QB(w_, i) ((float)(((w_) >> (8 * (i))) & 0xFFu))
#define PG_W4_SLOT(i, c)                                                                              \
    {                                                                                                 \
        const float tnx = fmaf(PG_QB(wnx, i), sx, bnx), tfx = fmaf(PG_QB(wfx, i), sx, bfx);           \
        const float tny = fmaf(PG_QB(wny, i), sy, bny), tfy = fmaf(PG_QB(wfy, i), sy, bfy);           \
        const float tnz = fmaf(PG_QB(wnz, i), sz, bnz), tfz = fmaf(PG_QB(wfz, i), sz, bfz);           \
        const float cmin = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, w.tmin));                                \
        const float cmax = fminf(fminf(tfx, tfy), fminf(tfz, tcull));                                 \
        r[i] = __float_as_int(rf.c);                                                                  \
        k[i] = (cmin <= cmax * kBoxRel && r[i] != PG_QNODE_EMPTY) ? cmin : INF;                       \
    }
    PG_W4_SLOT(0, x) PG_W4_SLOT(1, y) PG_W4_SLOT(2, z) PG_W4_SLOT(3, w)
#undef PG_W4_SLOT
#undef PG_QB
    cxch(k[0], r[0], k[1], r[1]);
    cxch(k[2], r[2], k[3], r[3]);
    cxch(k[0], r[0], k[2], r[2]);
    cxch(k[1], r[1], k[3], r[3]);
    cxch(k[1], r[1], k[2], r[2]);
    if (k[0] == INF) {
        w.node = w.sp > 0 ? (int)stk.get(--w.sp) : DONE;
    } else {
        w.node = r[0];
        if (k[3] != INF && w.sp < PG_QSTACK_DEPTH) stk.put(w.sp++, (uint32_t)r[3]);
        if (k[2] != INF && w.sp < PG_QSTACK_DEPTH) stk.put(w.sp++, (uint32_t)r[2]);
        if (k[1] != INF && w.sp < PG_QSTACK_DEPTH) stk.put(w.sp++, (uint32_t)r[1]);
    }
    if (w.node < 0 && w.leaf >= 0) {
        w.leaf = w.node;
        w.node = w.sp > 0 ? (int)stk.get(--w.sp) : DONE;
    }
}
// after a parked leaf's triangles: the next parked entry (traverse4's leaf loop step)
__device__ __forceinline__ void walk4NextLeaf(Walk4 &w, const TStack &stk) {
    const int DONE = 0x7fffffff;
    w.leaf = w.node;
    if (w.node < 0) w.node = w.sp > 0 ? (int)stk.get(--w.sp) : DONE;
}
// one round of traverse4's outer loop (the inner node loop until every lane of the round holds a leaf, then
// the postponed leaves); returns true when the walk is over (w.hitTri = ~0: no hit)
__device__ __forceinline__ bool walk4Round(Walk4 &w, const float4 *__restrict__ nodes, const float4 *__restrict__ tris,
                                           const TStack &stk) {
    const int DONE = 0x7fffffff;
    bool found = false;
    const float tcull = w.tmax * 1.000001f + w.tslack;
    while (w.node >= 0 && w.node != DONE) {
        walk4Visit(w, walk4Fetch(nodes, w.node), tcull, stk);
        if (!__any(w.leaf >= 0)) break;
    }
    while (w.leaf < 0) {
        leafTest<false>(tris, w.leaf, w.o, w.d, w.tmin, w.tmax, w.hitTri, w.hu, w.hv, found);
        walk4NextLeaf(w, stk);
    }
    return w.node == DONE;
}

// ---- two closest-hit walks per lane, interleaved (PG_TRACE_PAIR, pg_kernels.hip traceRowsPair) ----
// Each step issues both rays' node (or triangle) loads before either ray's test, so a lane keeps two
// dependent chains' requests in flight.  Each walk is traverse4's while-while walk (the inner loop runs
// while a descending ray of the wave has a free leaf slot; then every parked leaf is tested), so the hits
// are traverse4's: the closest (t, original index) over the visited boxes, whatever the visit order.
__device__ __forceinline__ void walk4Idle(Walk4 &w) {
    w.node = 0x7fffffff;
    w.leaf = 0;
    w.sp = 0;
    w.hitTri = 0xFFFFFFFFu;
    w.tmax = 0.0f;
    w.hu = w.hv = 0.0f;
}
// one triangle of a parked leaf, its first row already loaded (triHitRow0: triHit's test bit for bit)
__device__ __forceinline__ void walk4Tri(Walk4 &w, const float4 *__restrict__ tris, uint32_t tr, float4 r0) {
    float tt, bu, bv;
    if (triHitRow0(r0, tris, tr, w.o, w.d, w.tmin, w.tmax, tt, bu, bv) && acceptHit(tris, tt, w.tmax, tr, w.hitTri)) {
        w.tmax = tt;
        w.hitTri = tr;
        w.hu = bu;
        w.hv = bv;
    }
}
__device__ __forceinline__ void walk4Pair(Walk4 &a, Walk4 &b, const float4 *__restrict__ nodes,
                                          const float4 *__restrict__ tris, const TStack &sa, const TStack &sb) {
    const int DONE = 0x7fffffff;
    while (a.node != DONE || b.node != DONE) {
        const float ca = a.tmax * 1.000001f + a.tslack, cb = b.tmax * 1.000001f + b.tslack;
        for (;;) {
            const bool da = a.node >= 0 && a.node != DONE, db = b.node >= 0 && b.node != DONE;
            if (!(da || db)) break;
            QNode4 na, nb;
            if (da) na = walk4Fetch(nodes, a.node);
            if (db) nb = walk4Fetch(nodes, b.node);
            if (da) walk4Visit(a, na, ca, sa);
            if (db) walk4Visit(b, nb, cb, sb);
            const bool free = (a.leaf >= 0 && a.node >= 0 && a.node != DONE) || (b.leaf >= 0 && b.node >= 0 && b.node != DONE);
            if (!__any(free)) break;
        }
        for (;;) {
            const bool la = a.leaf < 0, lb = b.leaf < 0;
            if (!(la || lb)) break;
            const uint32_t ra = la ? ~(uint32_t)a.leaf : 0u, rb = lb ? ~(uint32_t)b.leaf : 0u;
            const uint32_t fa = ra >> 4, na = ra & 15u, fb = rb >> 4, nb = rb & 15u;
            for (uint32_t k = 0; k < na || k < nb; ++k) {
                float4 ta, tb;
                if (k < na) ta = tris[PG_TRI_ROW(fa + k, 0)];
                if (k < nb) tb = tris[PG_TRI_ROW(fb + k, 0)];
                if (k < na) walk4Tri(a, tris, fa + k, ta);
                if (k < nb) walk4Tri(b, tris, fb + k, tb);
            }
            if (la) walk4NextLeaf(a, sa);
            if (lb) walk4NextLeaf(b, sb);
        }
    }
}

// While-while traversal with postponed leaves (Aila & Laine 2009): lanes keep descending inner
// nodes until every lane of the wave holds a leaf, then all lanes test triangles together.  This
// keeps the 64-wide wave in one code path most of the time (if-if traversal measured 23 % lane
// utilisation on gfx950).
// LTOP: nodes [0, ntop) are read from `lnodes` (the top levels, staged in LDS by the caller).
template <bool ANY, bool LTOP = false>
__device__ __forceinline__ bool traverseBin(const float4 *__restrict__ nodes, const float4 *__restrict__ tris, f3 o, f3 d,
                                            float tmin, float &tmax, uint32_t &hitTri, float &hu, float &hv,
                                            const TStack &stk, const float4 *lnodes = nullptr, int ntop = 0) {
    const int DONE = 0x7fffffff;
    const SlabRay sr = slabRay(o, d);
    const f3 idir = sr.idir, aLo = sr.addLo, aHi = sr.addHi;
    // rounding of the slab distances fma(plane, idir, -o * idir) is bounded by a few ulps of |o * idir|
    const float tslack = sr.tslack;
    int sp = 0;
    int node = 0;   // >= 0 inner node, < 0 leaf ref, DONE
    int leaf = 0;   // postponed leaf ref (< 0) or none (>= 0)
    bool found = false;
    while (node != DONE) {
        // boxes are culled against tmax widened by the slab-distance rounding: a triangle that ties
        // with the current hit (shared edge, coplanar) can sit in a box whose rounded entry distance
        // lands just past tmax, and skipping it would make the tie-break (lower index) depend on
        // traversal order, i.e. on which paths share the wave (box intervals: slabRay)
        const float tcull = tmax * 1.000001f + tslack;
        while (node >= 0 && node != DONE) {
            float4 n0, n1, n2, n3;
            if (LTOP && node < ntop) {
                n0 = lnodes[4 * node + 0];
                n1 = lnodes[4 * node + 1];
                n2 = lnodes[4 * node + 2];
                n3 = lnodes[4 * node + 3];
            } else {
                n0 = nodes[4 * node + 0];
                n1 = nodes[4 * node + 1];
                n2 = nodes[4 * node + 2];
                n3 = nodes[4 * node + 3];
            }
            float a0 = fmaf(n0.x, idir.x, aLo.x), a1 = fmaf(n0.y, idir.x, aHi.x);
            float a2 = fmaf(n0.z, idir.y, aLo.y), a3 = fmaf(n0.w, idir.y, aHi.y);
            float a4 = fmaf(n2.x, idir.z, aLo.z), a5 = fmaf(n2.y, idir.z, aHi.z);
            float c0min = fmaxf(fmaxf(fminf(a0, a1), fminf(a2, a3)), fmaxf(fminf(a4, a5), tmin));
            float c0max = fminf(fminf(fmaxf(a0, a1), fmaxf(a2, a3)), fminf(fmaxf(a4, a5), tcull));
            float b0 = fmaf(n1.x, idir.x, aLo.x), b1 = fmaf(n1.y, idir.x, aHi.x);
            float b2 = fmaf(n1.z, idir.y, aLo.y), b3 = fmaf(n1.w, idir.y, aHi.y);
            float b4 = fmaf(n2.z, idir.z, aLo.z), b5 = fmaf(n2.w, idir.z, aHi.z);
            float c1min = fmaxf(fmaxf(fminf(b0, b1), fminf(b2, b3)), fmaxf(fminf(b4, b5), tmin));
            float c1max = fminf(fminf(fmaxf(b0, b1), fmaxf(b2, b3)), fminf(fmaxf(b4, b5), tcull));
            const bool h0 = c0min <= c0max * kBoxRel, h1 = c1min <= c1max * kBoxRel;
            const int ch0 = __float_as_int(n3.x), ch1 = __float_as_int(n3.y);
            if (!h0 && !h1) {
                node = sp > 0 ? (int)stk.get(--sp) : DONE;
            } else {
                node = h0 ? ch0 : ch1;
                if (h0 && h1) {
                    int farC = ch1;
                    if (c1min < c0min) {
                        node = ch1;
                        farC = ch0;
                    }
                    if (sp < STACK_DEPTH) stk.put(sp++, (uint32_t)farC);
                }
            }
            // first leaf found: postpone it and keep descending
            if (node < 0 && leaf >= 0) {
                leaf = node;
                node = sp > 0 ? (int)stk.get(--sp) : DONE;
            }
            if (!__any(leaf >= 0)) break;  // every lane still here holds a leaf
        }
        while (leaf < 0) {
            const uint32_t lr = ~(uint32_t)leaf;
            const uint32_t first = lr >> 4, cnt = lr & 15u;
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t tr = first + k;
                float tt, bu, bv;
                // equal distances (shared edges, coplanar triangles) go to the lower original triangle
                // index (acceptHit), so the closest hit depends neither on the BVH nor on the order in
                // which the wave's postponed leaves are visited (and thus on which paths share the wave)
                if (triHit(tris, tr, o, d, tmin, tmax, tt, bu, bv) && acceptHit(tris, tt, tmax, tr, hitTri)) {
                    found = true;
                    if (ANY) return true;
                    tmax = tt;
                    hitTri = tr;
                    hu = bu;  // weight of p1
                    hv = bv;  // weight of p2
                }
            }
            // another postponed leaf (in node)?  process it too
            leaf = node;
            if (node < 0) node = sp > 0 ? (int)stk.get(--sp) : DONE;
        }
    }
    return found;
}

// the closest-hit walk of this build's closest-hit BVH (SceneDev::nodes)
template <bool ANY, bool LTOP = false>
__device__ __forceinline__ bool traverse(const float4 *__restrict__ nodes, const float4 *__restrict__ tris, f3 o, f3 d,
                                         float tmin, float &tmax, uint32_t &hitTri, float &hu, float &hv,
                                         const TStack &stk, const float4 *lnodes = nullptr, int ntop = 0) {
#if PG_BVH4
    return traverse4<ANY, LTOP>(nodes, tris, o, d, tmin, tmax, hitTri, hu, hv, stk, lnodes, ntop);
#else
    return traverseBin<ANY, LTOP>(nodes, tris, o, d, tmin, tmax, hitTri, hu, hv, stk, lnodes, ntop);
#endif
}

// shadow-ray any hit: the 8-wide BVH, or the 4-wide closest-hit BVH in PG_SHADOW4 builds (A/B; the
// 4-wide walk's stack is the wide stack's storage, >= LDS_STACK LDS words + the shared overflow ring)
#ifndef PG_SHADOW4
#define PG_SHADOW4 0
#endif
__device__ __forceinline__ bool occluded(const SceneDev &sc, f3 o, f3 d, float tmin, float tmax, const WStack &w) {
    uint32_t tri = 0xFFFFFFFFu;
    float u, v;
#if PG_BVH4 && PG_SHADOW4
    return traverse4<true>(sc.nodes, sc.tris, o, d, tmin, tmax, tri, u, v, TStack{w.lds, w.ovf, w.ostride});
#else
    return traverseWide<true>(sc.wnodes, sc.wtris, o, d, tmin, tmax, tri, u, v, w);
#endif
}

__device__ __forceinline__ float miWeight(float a, float b) {
    a *= a;
    b *= b;
    return a / (a + b);
}

// BSDF fraction alpha of one guided vertex's one-sample MIS (pg_config.bsdf_fraction_bound).  The
// mixture weight f / (alpha p_bsdf + (1 - alpha) p_guide) is at most (f / p_bsdf) / alpha, so
// raising alpha to the BSDF's albedo keeps it <= 1 and the path throughput cannot compound upward
// over bounces where the D-tree has no density.  Oracle: guideFraction (oracle/oracle.cpp).
__device__ __forceinline__ float guideFraction(int mode, float alpha, float wbound, float maxT) {
    if (mode == PG_FRACTION_ALBEDO) return fmaxf(alpha, fminf(wbound, 0.95f));
    if (mode == PG_FRACTION_THROUGHPUT) return fmaxf(alpha, fminf(wbound * maxT, 0.95f));
    return alpha;
}

// wave-aggregated append of `pred` lanes' values into q (one atomic per wave)
__device__ __forceinline__ void waveAppend(bool pred, uint32_t value, uint32_t *q, uint32_t *count) {
    unsigned long long m = __ballot(pred);
    if (m == 0) return;
    int lane = threadIdx.x & 63;
    int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (pred) {
        unsigned long long below = m & ((1ull << lane) - 1ull);
        q[base + __popcll(below)] = value;
    }
}
// waveAppend that also stores each entry's order key (counting-sorted by pg_launch_ray_sort)
__device__ __forceinline__ void waveAppendKey(bool pred, uint32_t value, uint16_t key, uint32_t *q, uint16_t *keys,
                                              uint32_t *count) {
    unsigned long long m = __ballot(pred);
    if (m == 0) return;
    int lane = threadIdx.x & 63;
    int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (pred) {
        const uint32_t at = base + __popcll(m & ((1ull << lane) - 1ull));
        q[at] = value;
        keys[at] = key;
    }
}

__device__ __forceinline__ SDView sdv(const SDDev &sd) {
    return SDView{sd.snodes, sd.meta, sd.qsum, sd.qchild, sd.jump, make_float3(sd.lo[0], sd.lo[1], sd.lo[2]),
                  sd.extent, sd.jump_bits, sd.built};
}

struct Hit {
    f3 p, geoN, shN;
    Frame sh;
    f3 wi;
    uint32_t mat;
    int emitter;
};

__device__ __forceinline__ void fetchHit(const SceneDev &sc, uint32_t tri, float u, float v, f3 rd, Hit &h) {
    const float4 *r = sc.tshade + (size_t)PG_TRI_SHADE_STRIDE * tri;
    float4 s0 = r[0], s1 = r[1], s2 = r[2], s3 = r[3], s4 = r[4];
    uint32_t bits = __float_as_uint(s0.w);
    h.mat = bits & 0xFFFFu;
    h.emitter = (int)(bits >> 16) - 1;
    float b0 = 1 - u - v;
    f3 p0 = xyz(s0), p1 = xyz(s1), p2 = xyz(s2);
    f3 n0 = xyz(s3), n1 = mk(s3.w, s4.x, s4.y), n2 = mk(s4.z, s4.w, s1.w);
    // fillIntersectionRecord<true> (skdtree.h:343-430); the position without contraction, as the
    // oracle's Scene::fill computes it (with the TriAccel barycentrics, the same point bit for bit)
    {  // scalar expressions: the f3 operators' bodies lie outside this pragma's scope
#pragma clang fp contract(off)
        h.p = mk(p0.x * b0 + p1.x * u + p2.x * v, p0.y * b0 + p1.y * u + p2.y * v, p0.z * b0 + p1.z * u + p2.z * v);
    }
    f3 side1 = p1 - p0, side2 = p2 - p0;
    f3 fn = cross(side1, side2);
    float l = len(fn);
    if (!isZero(fn)) fn = fn / l;
    f3 shn = normalize(n0 * b0 + n1 * u + n2 * v);
    if (dot(fn, shn) < 0) fn = -fn;
    h.geoN = fn;
    h.shN = shn;
    h.sh = shadingFrame(shn, side1);
    h.wi = h.sh.toLocal(-rd);
}

// ---------------------------------------------------------------------------------------------
// Environment emitter (src/emitters/envmap.cpp).  Texel lookups follow TMIPMap::evalTexel at level 0
// (mipmap.h:503-563: repeat in x, clamp in y); the summation orders of evalBilinear (mipmap.h:575-596)
// and internalSampleDirection / internalPdfDirection (envmap.cpp:567-633) are kept as written.
constexpr float kInvTwoPi = 0.15915494309189533577f;
__device__ __forceinline__ f3 envTexel(const GEnv &e, int x, int y) {
    const int w = (int)e.width, h = (int)e.height;
    if (x < 0 || x >= w) {  // math::modulo
        x %= w;
        if (x < 0) x += w;
    }
    y = min(max(y, 0), h - 1);
    const float4 t = reinterpret_cast<const float4 *>(e.texels)[(size_t)y * (uint32_t)w + (uint32_t)x];
    return mk(t.x, t.y, t.z);
}
__device__ __forceinline__ float envLum(f3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; }
// Transform::inverse()(v) of the rotation (R^T v) and Transform::operator()(v) (R v)
__device__ __forceinline__ f3 envToLocal(const GEnv &e, f3 d) {
    return mk(e.R[0] * d.x + e.R[3] * d.y + e.R[6] * d.z, e.R[1] * d.x + e.R[4] * d.y + e.R[7] * d.z,
              e.R[2] * d.x + e.R[5] * d.y + e.R[8] * d.z);
}
__device__ __forceinline__ f3 envToWorld(const GEnv &e, f3 d) {
    return mk(e.R[0] * d.x + e.R[1] * d.y + e.R[2] * d.z, e.R[3] * d.x + e.R[4] * d.y + e.R[5] * d.z,
              e.R[6] * d.x + e.R[7] * d.y + e.R[8] * d.z);
}
__device__ __forceinline__ float safeAcos(float v) { return acosf(fminf(1.0f, fmaxf(-1.0f, v))); }

// EnvironmentMap::evalEnvironment without ray differentials (envmap.cpp:380-410)
__device__ __forceinline__ f3 envEval(const GEnv &e, f3 dWorld) {
#pragma clang fp contract(off)
    const f3 v = envToLocal(e, dWorld);
    const float ux = atan2f(v.x, -v.z) * kInvTwoPi, uy = safeAcos(v.y) * kInvPi;
    if (!isfinite(ux) || !isfinite(uy)) return mk1(0.f);
    const float u = ux * (float)e.width - 0.5f, w = uy * (float)e.height - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(w);
    const float dx1 = u - (float)xPos, dx2 = 1.0f - dx1, dy1 = w - (float)yPos, dy2 = 1.0f - dy1;
    const f3 r = envTexel(e, xPos, yPos) * dx2 * dy2 + envTexel(e, xPos, yPos + 1) * dx2 * dy1 +
                 envTexel(e, xPos + 1, yPos) * dx1 * dy2 + envTexel(e, xPos + 1, yPos + 1) * dx1 * dy1;
    return r * e.scale;
}

// internalPdfDirection (envmap.cpp:603-633) of a local direction
__device__ __forceinline__ float envPdfLocal(const GEnv &e, f3 d) {
#pragma clang fp contract(off)
    const float ux = atan2f(d.x, -d.z) * kInvTwoPi, uy = safeAcos(d.y) * kInvPi;
    if (!isfinite(ux) || !isfinite(uy)) return 0.0f;
    const float u = ux * (float)e.width - 0.5f, w = uy * (float)e.height - 0.5f;
    const int xPos = (int)floorf(u), yPos = (int)floorf(w);
    const float dx1 = u - (float)xPos, dx2 = 1.0f - dx1, dy1 = w - (float)yPos, dy2 = 1.0f - dy1;
    const f3 v1 = envTexel(e, xPos, yPos) * dx2 * dy2 + envTexel(e, xPos + 1, yPos) * dx1 * dy2;
    const f3 v2 = envTexel(e, xPos, yPos + 1) * dx2 * dy1 + envTexel(e, xPos + 1, yPos + 1) * dx1 * dy1;
    const int h = (int)e.height;
    const float sinTheta = safe_sqrt(1 - d.y * d.y);
    return (envLum(v1) * e.row_weights[min(max(yPos, 0), h - 1)] +
            envLum(v2) * e.row_weights[min(max(yPos + 1, 0), h - 1)]) *
           e.normalization / fmaxf(fabsf(sinTheta), kEpsilon);
}
// EnvironmentMap::pdfDirect for a solid-angle record (envmap.cpp:545-556)
__device__ __forceinline__ float envPdf(const GEnv &e, f3 dWorld) { return envPdfLocal(e, envToLocal(e, dWorld)); }

// EnvironmentMap::sampleReuse (envmap.cpp:658-663): lower_bound over cdf[0..size]
__device__ __forceinline__ uint32_t envSampleReuse(const float *cdf, uint32_t size, float &s) {
    uint32_t lo = 0, hi = size + 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < s) lo = mid + 1; else hi = mid;
    }
    const uint32_t index = min((uint32_t)max((int)lo - 1, 0), size - 1);
    s = (s - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}
// warp::squareToTent's intervalToTent (warp.cpp:143-155)
__device__ __forceinline__ float intervalToTent(float s) {
    float sign;
    if (s < 0.5f) {
        sign = 1;
        s *= 2;
    } else {
        sign = -1;
        s = 2 * (s - 0.5f);
    }
    return sign * (1 - sqrtf(s));
}
// internalSampleDirection (envmap.cpp:567-600): local direction, value (incl. scale) and pdf
__device__ __forceinline__ f3 envSampleLocal(const GEnv &e, float sx, float sy, f3 &value, float &pdf) {
#pragma clang fp contract(off)
    const uint32_t row = envSampleReuse(e.cdf_rows, e.height, sy);
    const uint32_t col = envSampleReuse(e.cdf_cols + (size_t)row * (e.width + 1), e.width, sx);
    const float px = (float)col + intervalToTent(sx), py = (float)row + intervalToTent(sy);
    const int xPos = (int)floorf(px), yPos = (int)floorf(py);
    const float dx1 = px - (float)xPos, dx2 = 1.0f - dx1, dy1 = py - (float)yPos, dy2 = 1.0f - dy1;
    const f3 v1 = envTexel(e, xPos, yPos) * dx2 * dy2 + envTexel(e, xPos + 1, yPos) * dx1 * dy2;
    const f3 v2 = envTexel(e, xPos, yPos + 1) * dx2 * dy1 + envTexel(e, xPos + 1, yPos + 1) * dx1 * dy1;
    value = (v1 + v2) * e.scale;
    const int h = (int)e.height;
    pdf = (envLum(v1) * e.row_weights[min(max(yPos, 0), h - 1)] +
           envLum(v2) * e.row_weights[min(max(yPos + 1, 0), h - 1)]) *
          e.normalization;
    float sinPhi, cosPhi, sinTheta, cosTheta;
    sincosf(e.pixel_size[0] * (px + 0.5f), &sinPhi, &cosPhi);
    sincosf(e.pixel_size[1] * (py + 0.5f), &sinTheta, &cosTheta);
    pdf /= fmaxf(fabsf(sinTheta), kEpsilon);
    return mk(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
}
// EnvironmentMap::sampleDirect (envmap.cpp:516-543): value / pdf, with the far intersection of the
// scene's bounding sphere as the light distance (BSphere::rayIntersect + solveQuadratic, util.cpp)
__device__ __forceinline__ f3 envSampleDirect(const GEnv &e, f3 ref, float sx, float sy, f3 &dOut, float &dist,
                                              float &pdfOut) {
    f3 value;
    float pdf;
    const f3 d = envToWorld(e, envSampleLocal(e, sx, sy, value, pdf));
    pdfOut = 0;
    if (isZero(value) || pdf == 0) return mk1(0.f);
    const f3 o = ref - mk(e.center[0], e.center[1], e.center[2]);
    const float A = dot(d, d), B = 2 * dot(o, d), C = dot(o, o) - e.radius * e.radius;
    const float disc = B * B - 4.0f * A * C;
    if (disc < 0) return mk1(0.f);
    const float sq = sqrtf(disc), temp = (B < 0) ? -0.5f * (B - sq) : -0.5f * (B + sq);
    float x0 = temp / A, x1 = C / temp;
    if (x0 > x1) {
        const float t = x0;
        x0 = x1;
        x1 = t;
    }
    if (x0 >= 0 || x1 <= 0) return mk1(0.f);
    dOut = d;
    dist = x1;
    pdfOut = pdf;
    return value / pdf;
}

// Scene::sampleEmitterDirect without the visibility test (scene.cpp:871-895 + area.cpp:158-171 +
// shape.cpp:102-115 + trimesh.cpp:412-423 + triangle.cpp:24-45); returns radiance/pdf.  With an
// environment emitter (sc.env; compiled in with ENV only), it is emitter g.num_emitters - 1.
template <bool ENV = false>
__device__ __forceinline__ f3 sampleEmitter(const GParams &g, const SceneDev &sc, f3 ref, f3 refN, float sx, float sy,
                                            f3 &dOut, float &dist, float &pdfOut, f3 *pOut = nullptr) {
    uint32_t ne = g.num_emitters;
    pdfOut = 0;
    if (ne == 0) return mk1(0.f);
    uint32_t ei = min((uint32_t)(sx * (float)ne), ne - 1);
    sx = sx * (float)ne - (float)ei;
    if (ENV && ei == ne - 1) {
        float pdf;
        const f3 v = envSampleDirect(*sc.env, ref, sx, sy, dOut, dist, pdf);
        if (pdf == 0) return mk1(0.f);
        const float emPdf = 1.0f / (float)ne;
        pdfOut = pdf * emPdf;
        if (pOut) *pOut = ref + dOut * dist;
        return v / emPdf;
    }
    const GEmitter em = sc.ems[ei];
    // DiscreteDistribution::sampleReuse over the area CDF (lower_bound)
    const float *cdf = sc.emcdf + em.cdf_begin;
    uint32_t lo = 0, hi = em.tri_count + 1;  // first index with cdf[i] >= sy
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] < sy) lo = mid + 1; else hi = mid;
    }
    int e = (int)lo - 1;
    uint32_t idx = (uint32_t)min((int)em.tri_count - 1, max(0, e));
    while (cdf[idx + 1] - cdf[idx] == 0 && idx < em.tri_count - 1) ++idx;
    sy = (sy - cdf[idx]) / (cdf[idx + 1] - cdf[idx]);
    const float4 *r = sc.emtri + (size_t)PG_TRI_SHADE_F4 * (em.tri_begin + idx);
    float4 s0 = r[0], s1 = r[1], s2 = r[2], s3 = r[3], s4 = r[4];
    f3 p0 = xyz(s0), p1 = xyz(s1), p2 = xyz(s2);
    float a = safe_sqrt(1.0f - sx);
    float bx = 1 - a, by = a * sy;
    f3 sideA = p1 - p0, sideB = p2 - p0;
    f3 p = p0 + (sideA * bx) + (sideB * by);
    f3 n0 = xyz(s3), n1 = mk(s3.w, s4.x, s4.y), n2 = mk(s4.z, s4.w, s1.w);
    f3 n = normalize(n0 * (1.0f - bx - by) + n1 * bx + n2 * by);
    float pdf = em.inv_area;
    f3 d = p - ref;
    float distSq = dot(d, d);
    dist = sqrtf(distSq);
    d = d / dist;
    float dp = absDot(d, n);
    pdf *= dp != 0 ? (distSq / dp) : 0.0f;
    dOut = d;
    if (pOut) *pOut = p;
    if (dot(d, refN) >= 0 && dot(d, n) < 0 && pdf != 0) {
        float emPdf = 1.0f / (float)ne;
        pdfOut = pdf * emPdf;
        return mk(em.radiance[0], em.radiance[1], em.radiance[2]) / pdf / emPdf;
    }
    return mk1(0.f);
}

__device__ __forceinline__ TStack threadStack(uint32_t *lds, uint32_t *ovf) {
    const uint32_t gtid = blockIdx.x * TRACE_BLOCK + threadIdx.x;
    return TStack{lds + threadIdx.x, ovf + gtid, gridDim.x * TRACE_BLOCK};
}
__device__ __forceinline__ WStack threadWideStack(uint32_t *lds, uint32_t *ovf) {
    const uint32_t gtid = blockIdx.x * TRACE_BLOCK + threadIdx.x;
    return WStack{lds + threadIdx.x, ovf + gtid, gridDim.x * TRACE_BLOCK};
}

}  // namespace
