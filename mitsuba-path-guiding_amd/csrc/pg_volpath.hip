// gfx950 volumetric path tracer: ProgressiveVolumetricPathTracer::Li
// (src/integrators/path/progressive_volpath.cpp:98-374) with heterogeneous media
// (src/medium/heterogeneous.cpp, Woodcock tracking), grid densities (src/volume/gridvolume.cpp)
// and the HG phase function (src/phase/hg.cpp).  DESIGN.md §"Volumes".
//
// One persistent megakernel: every lane owns one camera path at a time and runs the reference's
// loop one iteration per step; a lane whose path ended takes the next (pixel, sample) item from a
// wave-aggregated work counter, so long paths (dense media) do not idle the rest of the wave.
// Each item's radiance goes to rad[item]; k_film then accumulates items in sample order, so the
// image is independent of which lane ran which item.  Random numbers: one sequential counter
// stream per path (dimension 0 = pixel jitter, then one dimension per next1D / next2D), the same
// stream the CPU oracle (oracle/orc_volpath.h) draws from.
#include "pg_trace.h"

// Index checks of the megakernel (debug build PG_VOL_CHECK=1, make volcheck): VCHK(cond, code, value)
// is `cond` in the product build (a guard the code keeps) and, in the check build, also counts
// violations and keeps the first one's code and value (pg_debug_volcheck_read).  Codes: 1 the emitter
// walk's transmittance re-walk missed a surface the first walk hit, 2 a shadow walk's medium
// transition on an invalid triangle, 3 rad[item] out of range, 4 a training vertex out of range,
// 5 a majorant cell out of range, 6 a density cell out of range.
#ifndef PG_VOL_CHECK
#define PG_VOL_CHECK 0
#endif
#if PG_VOL_CHECK
__device__ uint32_t pgVolCheck[12];  // count, first code, first value, per-code counts [3 + code - 1]
__device__ __forceinline__ bool volCheck(bool ok, uint32_t code, uint32_t value) {
    if (!ok && atomicAdd(&pgVolCheck[0], 1u) == 0) {
        pgVolCheck[1] = code;
        pgVolCheck[2] = value;
    }
    if (!ok) atomicAdd(&pgVolCheck[2 + code], 1u);  // per-code counts in [3, 8] (codes 1..6)
    return ok;
}
extern "C" int pg_debug_volcheck_read(uint32_t *out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pgVolCheck), 12 * 4) == hipSuccess ? 0 : -1;
}
#define VCHK(cond, code, value) volCheck((cond), (code), (uint32_t)(value))
#else
#define VCHK(cond, code, value) (cond)
#endif

namespace {

#define VOL_BLOCK TRACE_BLOCK  // the traversal stack columns assume TRACE_BLOCK threads per block
#ifndef PG_VOL_WAVES
#define PG_VOL_WAVES 2  // min waves per SIMD: caps the megakernel at 256 VGPRs (occupancy 2)
#endif

// Sampler::next1D / next2D over the counter RNG
struct VRng {
    uint32_t key, sample, dim;
    uint32_t lookups;  // density-grid lookups of this path (statistics)
    __device__ __forceinline__ float next1() { return rng1(key, sample, dim++); }
    __device__ __forceinline__ void next2(float &a, float &b) { rng2(key, sample, dim++, a, b); }
};

// Transmittance sub-streams (oracle/orc_volpath.h subStream): the NEE shadow walk (kind 0) and the
// re-walk of a sampled ray that found a lit emitter through media (kind 1) draw from a Philox stream keyed
// by key ^ 0x9E3779B9 (2 dim + kind + 1), dim = the main-stream dimension at which the interaction drew its
// light sample / started its emitter walk, at dimensions 0x80000000 + j (the main stream's stay below
// 2^31).  The key map is a bijection of (dim, kind) for dim < 2^31, so no two walks of a path share
// numbers however long the path or the walk (round 6; until then dim and kind were bit-packed into the
// dimension and aliased from dim = 2^15 or j = 2^15 on).  The main stream does not depend on the walks, so
// the wavefront runs them as a stage of their own (k_vnee).
__device__ __forceinline__ VRng subStream(uint32_t key, uint32_t sample, uint32_t dim, uint32_t kind) {
    return VRng{key ^ (0x9E3779B9u * (2u * dim + kind + 1u)), sample, 0x80000000u, 0};
}

// What an interaction leaves for its transmittance walks (k_vnee in the wavefront, resolveDeferred
// right after the step in k_vtail / k_volpath): the emitter hit's contribution before the transmittance
// of its walk (hit) and the NEE's contribution before the shadow walk's transmittance (nee), added to L
// in that order; the NEE also joins the training snapshot of the interaction's vertex k.
struct VDefer {
    f3 nC, n1, n2;  // NEE: contribution, shadow walk from n1 to the emitter point n2
    int nMedium, nMaxInter;
    uint32_t nDim;
    bool nee, nOnSurface;
    f3 hC, hO, hD;  // emitter hit: contribution, the walk's first ray (origin, direction, mint)
    float hMint;
    int hMedium, hInter;  // the walk's starting medium and null-surface crossings
    uint32_t hDim;
    bool hit;
    int k;  // training vertex of the interaction (-1: none)
};

// ---- HG phase function (hg.cpp:74-106) --------------------------------------------------------
__device__ __forceinline__ float hgEval(float g, f3 wi, f3 wo) {
    float temp = 1.0f + g * g + 2.0f * g * dot(wi, wo);
    return kInvFourPi * (1 - g * g) / (temp * sqrtf(temp));
}
// Frame(n) by coordinateSystem (util.cpp:594-603): s = cross(c, n), t = c
__device__ __forceinline__ f3 frameToWorld(f3 a, f3 v) {
    f3 c;
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        c = mk(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        c = mk(0.0f, a.z * invLen, -a.y * invLen);
    }
    return cross(c, a) * v.x + c * v.y + a * v.z;
}
__device__ __forceinline__ f3 hgSample(float g, f3 wi, float sx, float sy, float &pdf) {
    float cosTheta;
    if (fabsf(g) < kEpsilon) {
        cosTheta = 1 - 2 * sx;
    } else {
        float sqrTerm = (1 - g * g) / (1 - g + 2 * g * sx);
        cosTheta = (1 + g * g - sqrTerm * sqrTerm) / (2 * g);
    }
    float sinTheta = safe_sqrt(1.0f - cosTheta * cosTheta);
    float sinPhi, cosPhi;
    sincosf(2 * kPi * sy, &sinPhi, &cosPhi);
    f3 wo = frameToWorld(-wi, mk(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta));
    pdf = hgEval(g, wi, wo);
    return wo;
}

// ---- heterogeneous medium (heterogeneous.cpp:546-660, gridvolume.cpp:337-380) -----------------
struct MedView {
    const float *density;
    const float *maj;
    int rx, ry, rz;
    int bx, by;
    int mx, my, mz;
    f3 gs, go, lo, hi;
    float scale, invMax;
};
__device__ __forceinline__ MedView medView(const GMedium *media, int m) {
    const GMedium &G = media[m];
    MedView v;
    v.density = G.density;
    v.rx = (int)G.resx;
    v.ry = (int)G.resy;
    v.rz = (int)G.resz;
    v.gs = mk(G.gs[0], G.gs[1], G.gs[2]);
    v.go = mk(G.go[0], G.go[1], G.go[2]);
    v.lo = mk(G.lo[0], G.lo[1], G.lo[2]);
    v.hi = mk(G.hi[0], G.hi[1], G.hi[2]);
    v.scale = G.scale;
    v.invMax = G.invMax;
    v.maj = G.maj;
    v.bx = (int)G.bx;
    v.by = (int)G.by;
    v.mx = (int)G.mx;
    v.my = (int)G.my;
    v.mz = (int)G.mz;
    return v;
}
// lookupFloat: trilinear, zero unless all 8 corners are inside the grid
__device__ __forceinline__ float lookupDensity(const MedView &M, f3 p) {
    const float px = p.x * M.gs.x + M.go.x, py = p.y * M.gs.y + M.go.y, pz = p.z * M.gs.z + M.go.z;
    const int x1 = (int)floorf(px), y1 = (int)floorf(py), z1 = (int)floorf(pz);
    if (x1 < 0 || y1 < 0 || z1 < 0 || x1 + 1 >= M.rx || y1 + 1 >= M.ry || z1 + 1 >= M.rz) return 0.0f;
#if PG_VOL_CHECK
    if (!VCHK((size_t)x1 + 1 < (size_t)M.rx && (size_t)y1 + 1 < (size_t)M.ry && (size_t)z1 + 1 < (size_t)M.rz, 6, x1))
        return 0.0f;
#endif
    const float fx = px - x1, fy = py - y1, fz = pz - z1, _fx = 1.0f - fx, _fy = 1.0f - fy, _fz = 1.0f - fz;
#if PG_DENSITY_BRICKS
    // per-axis (brick, in-brick) offsets of the two corner coordinates
    const int x2 = x1 + 1, y2 = y1 + 1, z2 = z1 + 1;
    const uint32_t ax1 = (uint32_t)((x1 >> 2) * 64 + (x1 & 3)), ax2 = (uint32_t)((x2 >> 2) * 64 + (x2 & 3));
    const uint32_t ay1 = (uint32_t)((y1 >> 2) * M.bx * 64 + (y1 & 3) * 4), ay2 = (uint32_t)((y2 >> 2) * M.bx * 64 + (y2 & 3) * 4);
    const uint32_t zs = (uint32_t)(M.bx * M.by * 64);
    const uint32_t az1 = (uint32_t)(z1 >> 2) * zs + (uint32_t)(z1 & 3) * 16, az2 = (uint32_t)(z2 >> 2) * zs + (uint32_t)(z2 & 3) * 16;
    const float *D = M.density;
    const float d000 = D[az1 + ay1 + ax1], d001 = D[az1 + ay1 + ax2], d010 = D[az1 + ay2 + ax1], d011 = D[az1 + ay2 + ax2];
    const float d100 = D[az2 + ay1 + ax1], d101 = D[az2 + ay1 + ax2], d110 = D[az2 + ay2 + ax1], d111 = D[az2 + ay2 + ax2];
#elif PG_DENSITY_CORNERS
    const size_t cell = ((size_t)z1 * (size_t)(M.ry - 1) + (size_t)y1) * (size_t)(M.rx - 1) + (size_t)x1;
    const float4 *cp = reinterpret_cast<const float4 *>(M.density) + 2 * cell;
    const float4 lo = cp[0], hi = cp[1];
    const float d000 = lo.x, d001 = lo.y, d010 = lo.z, d011 = lo.w;
    const float d100 = hi.x, d101 = hi.y, d110 = hi.z, d111 = hi.w;
#else
    const size_t sy = (size_t)M.rx, sz = (size_t)M.rx * M.ry;
    const float *b = M.density + (size_t)z1 * sz + (size_t)y1 * sy + x1;
    const float d000 = b[0], d001 = b[1], d010 = b[sy], d011 = b[sy + 1];
    const float d100 = b[sz], d101 = b[sz + 1], d110 = b[sz + sy], d111 = b[sz + sy + 1];
#endif
    return ((d000 * _fx + d001 * fx) * _fy + (d010 * _fx + d011 * fx) * fy) * _fz +
           ((d100 * _fx + d101 * fx) * _fy + (d110 * _fx + d111 * fx) * fy) * fz;
}
// AABB::rayIntersect of the density box, clipped to [mint, maxt]
__device__ __forceinline__ bool medClip(const MedView &M, f3 o, f3 d, float mint, float maxt, float &t0, float &t1) {
    float nearT = -__int_as_float(0x7f800000), farT = __int_as_float(0x7f800000);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float oi = i == 0 ? o.x : (i == 1 ? o.y : o.z), di = i == 0 ? d.x : (i == 1 ? d.y : d.z);
        const float mn = i == 0 ? M.lo.x : (i == 1 ? M.lo.y : M.lo.z), mx = i == 0 ? M.hi.x : (i == 1 ? M.hi.y : M.hi.z);
        if (di == 0) {
            if (oi < mn || oi > mx) return false;
        } else {
            float a = (mn - oi) / di, b = (mx - oi) / di;
            if (a > b) {
                const float tmp = a;
                a = b;
                b = tmp;
            }
            nearT = fmaxf(a, nearT);
            farT = fminf(b, farT);
            if (!(nearT <= farT)) return false;
        }
    }
    t0 = fmaxf(nearT, mint);
    t1 = fminf(farT, maxt);
    return true;
}
// Tentative-collision rules: accept(p, density, mu, u).  The reference's (heterogeneous.cpp:640)
// for the global majorant and its majorant-grid equivalent; AcceptGuided (below) is the weighted
// rule of guided free flight.
struct AcceptGlobal {
    float invMax;
    __device__ __forceinline__ bool operator()(f3, float density, float, float u) const { return density * invMax > u; }
};
struct AcceptGrid {
    __device__ __forceinline__ bool operator()(f3, float density, float mu, float u) const { return density > mu * u; }
};

// Woodcock tracking: true with the collision point (sampleDistance, 'woodcock' branch)
template <class Accept>
__device__ __forceinline__ bool sampleDistance(const MedView &M, f3 o, f3 d, float maxt, VRng &rng, f3 &pOut, Accept &acc) {
    float t0, t1;
    if (!medClip(M, o, d, 0.0f, maxt, t0, t1)) return false;
    float t = t0;
    for (;;) {
        t -= trackLog(1 - rng.next1()) * M.invMax;
        if (!(t < t1)) return false;
        const f3 p = o + d * t;
        const float density = lookupDensity(M, p) * M.scale;
        rng.lookups++;
        if (acc(p, density, M.scale, rng.next1())) {
            pOut = p;
            return true;
        }
    }
}
// Delta tracking through the majorant grid over [t0, t1] (oracle/orc_medium.h trackGrid): a 3D DDA
// over PG_MAJORANT_CELL^3-voxel cells; exponential steps at the cell majorant, restarted at each
// cell exit (memoryless); empty cells cost no draw and no lookup.
template <class Accept>
__device__ __forceinline__ bool trackGrid(const MedView &M, f3 o, f3 d, float t0, float t1, VRng &rng, float &tHit,
                                          Accept &acc) {
    const float B = (float)PG_MAJORANT_CELL, inf = __int_as_float(0x7f800000);
    const f3 og = mk(o.x * M.gs.x + M.go.x, o.y * M.gs.y + M.go.y, o.z * M.gs.z + M.go.z);
    const f3 dg = mk(d.x * M.gs.x, d.y * M.gs.y, d.z * M.gs.z);
    int c[3], stp[3];
    float tNext[3], tDelta[3];
    const int n[3] = {M.mx, M.my, M.mz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float oa = a == 0 ? og.x : (a == 1 ? og.y : og.z), da = a == 0 ? dg.x : (a == 1 ? dg.y : dg.z);
        c[a] = min(max((int)floorf((oa + da * t0) / B), 0), n[a] - 1);
        if (da > 0) {
            stp[a] = 1;
            tNext[a] = ((float)(c[a] + 1) * B - oa) / da;
            tDelta[a] = B / da;
        } else if (da < 0) {
            stp[a] = -1;
            tNext[a] = ((float)c[a] * B - oa) / da;
            tDelta[a] = -B / da;
        } else {
            stp[a] = 0;
            tNext[a] = inf;
            tDelta[a] = inf;
        }
    }
    float t = t0;
    for (;;) {
        const float tExit = fminf(fminf(tNext[0], tNext[1]), fminf(tNext[2], t1));
#if PG_VOL_CHECK
        if (!VCHK(c[0] >= 0 && c[1] >= 0 && c[2] >= 0 && c[0] < n[0] && c[1] < n[1] && c[2] < n[2], 5, c[0])) return false;
#endif
        const float mu = M.maj[((size_t)c[2] * M.my + c[1]) * M.mx + c[0]];
        if (mu > 0) {
            for (;;) {
                const float ts = t - trackLog(1 - rng.next1()) / mu;
                if (!(ts < tExit)) break;
                t = ts;
                const f3 p = o + d * t;
                const float density = lookupDensity(M, p) * M.scale;
                rng.lookups++;
                if (acc(p, density, mu, rng.next1())) {
                    tHit = t;
                    return true;
                }
            }
        }
        t = fmaxf(t, tExit);
        if (!(t < t1)) return false;
        const int a = tNext[0] <= tNext[1] ? (tNext[0] <= tNext[2] ? 0 : 2) : (tNext[1] <= tNext[2] ? 1 : 2);
        // register-resident indexing: select instead of dynamic array access
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k == a) {
                c[k] += stp[k];
                tNext[k] += tDelta[k];
            }
        if (c[0] < 0 || c[1] < 0 || c[2] < 0 || c[0] >= n[0] || c[1] >= n[1] || c[2] >= n[2]) return false;
    }
}
__device__ __forceinline__ bool trackGrid(const MedView &M, f3 o, f3 d, float t0, float t1, VRng &rng, float &tHit) {
    AcceptGrid acc;
    return trackGrid(M, o, d, t0, t1, rng, tHit, acc);
}
template <class Accept>
__device__ __forceinline__ bool sampleDistanceGrid(const MedView &M, f3 o, f3 d, float maxt, VRng &rng, f3 &pOut, Accept &acc) {
    float t0, t1, t;
    if (!medClip(M, o, d, 0.0f, maxt, t0, t1) || !(t0 < t1)) return false;
    if (!trackGrid(M, o, d, t0, t1, rng, t, acc)) return false;
    pOut = o + d * t;
    return true;
}
__device__ __forceinline__ float evalTransmittanceGrid(const MedView &M, f3 o, f3 d, float maxt, VRng &rng) {
    float t0, t1, t;
    if (!medClip(M, o, d, 0.0f, maxt, t0, t1) || !(t0 < t1)) return 1.0f;
    float result = 0;
    for (int i = 0; i < 2; ++i)
        if (!trackGrid(M, o, d, t0, t1, rng, t)) result += 1;
    return result * 0.5f;
}

// evalTransmittance with a sampler: mean of 2 delta-tracking survival indicators
__device__ __forceinline__ float evalTransmittance(const MedView &M, f3 o, f3 d, float maxt, VRng &rng) {
    float t0, t1;
    if (!medClip(M, o, d, 0.0f, maxt, t0, t1)) return 1.0f;
    float result = 0;
    for (int i = 0; i < 2; ++i) {
        float t = t0;
        for (;;) {
            t -= trackLog(1 - rng.next1()) * M.invMax;
            if (!(t < t1)) {
                result += 1;
                break;
            }
            const f3 p = o + d * t;
            const float density = lookupDensity(M, p) * M.scale;
            rng.lookups++;
            if (density * M.invMax > rng.next1()) break;
        }
    }
    return result * 0.5f;
}

__device__ __forceinline__ bool mediumSample(const VolDev &v, int m, f3 o, f3 d, float maxt, VRng &rng, f3 &p) {
    const MedView M = medView(v.media, m);
    if (v.grid) {
        AcceptGrid acc;
        return sampleDistanceGrid(M, o, d, maxt, rng, p, acc);
    }
    AcceptGlobal acc{M.invMax};
    return sampleDistance(M, o, d, maxt, rng, p, acc);
}

// Guided free flight (pg_config.distance_guiding = beta; oracle/orc_volpath.h GuidedAccept):
// weighted delta tracking toward P_g = sigma_s s / (sigma_s s + sigma_n x), x = 4 pi p_guide(x, d),
// s = |g| x + (1 - |g|): the zero-variance collision probability with the SD-tree's incident
// radiance for the unknowns; the path weight takes P_std / P (collision) or (1 - P_std) / (1 - P)
// (null collision).  The D-tree pdf of the (fixed) flight direction is re-walked only when the
// S-tree leaf changes.
struct AcceptGuided {
    SDView sv;
    const uint4 *meta;
    float beta, albedo, invMax;  // invMax > 0: global majorant
    float gAbs;
    float cu, cv;
    float w;
    uint32_t lastDt;
    float lastPg;
    __device__ __forceinline__ bool operator()(f3 p, float density, float mu, float u) {
        float pStd = invMax > 0 ? density * invMax : density / mu;
        pStd = fminf(fmaxf(pStd, 0.0f), 1.0f);
        const uint32_t dt = sdLookup(sv, p);
        if (dt != lastDt) {
            lastDt = dt;
            lastPg = sdPdfCanon(sv, meta[dt], cu, cv);
        }
        const float x = 12.566370614359172f * lastPg;
        const float sS = albedo * density * (gAbs * x + (1 - gAbs)), sN = fmaxf(mu - density, 0.0f);
        const float den = sS + sN * x;
        const float pG = den > 0 ? sS / den : pStd;
        const float P = (1 - beta) * pStd + beta * pG;
        if (u < P) {
            w *= pStd / P;
            return true;
        }
        w *= (1 - pStd) / (1 - P);
        return false;
    }
};
__device__ __forceinline__ bool mediumSampleGuided(const VolDev &v, const SDDev &sd, int m, f3 o, f3 d, float maxt,
                                                   VRng &rng, f3 &p, float &w) {
    const MedView M = medView(v.media, m);
    const GMedium &GM = v.media[m];
    AcceptGuided acc{sdv(sd), sd.meta, v.dist_beta, (GM.albedo[0] + GM.albedo[1] + GM.albedo[2]) * (1.0f / 3.0f),
                     v.grid ? 0.0f : M.invMax, fabsf(GM.g), 0.0f, 0.0f, 1.0f, 0xFFFFFFFFu, 0.0f};
    dirToCanonical(d, acc.cu, acc.cv);
    const bool hit = v.grid ? sampleDistanceGrid(M, o, d, maxt, rng, p, acc) : sampleDistance(M, o, d, maxt, rng, p, acc);
    w = acc.w;
    return hit;
}
__device__ __forceinline__ float mediumTransmittance(const VolDev &v, int m, f3 o, f3 d, float maxt, VRng &rng) {
    const MedView M = medView(v.media, m);
    return v.grid ? evalTransmittanceGrid(M, o, d, maxt, rng) : evalTransmittance(M, o, d, maxt, rng);
}

// ---- scene queries ----------------------------------------------------------------------------
// o + d t, the multiply and the add rounded separately as in the oracle (orc_volpath.h, built with
// -ffp-contract=off): the emitter walk's second pass must reproduce its first pass's origins bit for bit,
// and both must equal the oracle's (scalar expressions under the pragma: the f3 operators' bodies lie
// outside its scope; the Makefile builds this file without contraction anyway)
__device__ __forceinline__ f3 advance(f3 o, f3 d, float t) {
#pragma clang fp contract(off)
    return mk(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
}
__device__ __forceinline__ float max3abs(f3 o) { return fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)); }
// ShapeKDTree::rayIntersect(ray, its) epsilon rule for mint == Epsilon (skdtree.cpp:125-128)
__device__ __forceinline__ float itsMinT(f3 o) { return kEpsilon * fmaxf(max3abs(o), kEpsilon); }

__device__ __forceinline__ bool closestHit(const SceneDev &sc, f3 o, f3 d, float tmin, float tmax, float &t,
                                           uint32_t &tri, float &u, float &v, const TStack &stk) {
    t = tmax;
    tri = 0xFFFFFFFFu;
    u = v = 0;
    if (!(tmax > tmin)) return false;
    return traverse<false>(sc.nodes, sc.tris, o, d, tmin, t, tri, u, v, stk);
}
__device__ __forceinline__ uint32_t triBits(const SceneDev &sc, uint32_t tri) {
    return __float_as_uint(sc.tshade[(size_t)PG_TRI_SHADE_STRIDE * tri].w);
}
__device__ __forceinline__ bool isNullMat(const SceneDev &sc, uint32_t bits) {
    return (sc.mats[bits & 0xFFFFu].type & ENull) != 0;
}
// Intersection::getTargetMedium(d) from the packed (interior + 1) | (exterior + 1) << 16
__device__ __forceinline__ int targetMedium(uint32_t tm, f3 d, f3 n) {
    return dot(d, n) > 0 ? (int)(tm >> 16) - 1 : (int)(tm & 0xFFFFu) - 1;
}
__device__ __forceinline__ f3 rawFaceNormal(const SceneDev &sc, uint32_t tri) {
    const float4 *r = sc.tshade + (size_t)PG_TRI_SHADE_STRIDE * tri;
    const f3 p0 = xyz(r[0]), p1 = xyz(r[1]), p2 = xyz(r[2]);
    return normalize(cross(p1 - p0, p2 - p0));
}

// Scene::evalTransmittance (scene.cpp:662-720) from p1 to a point p2 on an emitter
__device__ __forceinline__ float sceneTransmittance(const SceneDev &sc, const VolDev &v, f3 p1, bool p1OnSurface, f3 p2, int medium,
                                    int maxInteractions, VRng &rng, const TStack &stk, uint32_t &segs) {
    f3 d = p2 - p1;
    float remaining = len(d);
    d = d / remaining;
    const float lengthFactor = 1 - kShadowEpsilon;
    f3 o = p1;
    float mint = p1OnSurface ? kEpsilon * max3abs(o) : 0.0f;  // rayIntersect(ray, t, shape, n, uv) rule
    float maxt = remaining * lengthFactor;
    float T = 1.0f;
    int interactions = 0;
    while (remaining > 0) {
        float t, u, w;
        uint32_t tri;
        const bool surface = closestHit(sc, o, d, mint, maxt, t, tri, u, w, stk);
        segs++;
        if (!surface) t = __int_as_float(0x7f800000);
        if (surface && (interactions == maxInteractions || !isNullMat(sc, triBits(sc, tri)))) return 0.0f;
        if (medium >= 0) T *= mediumTransmittance(v, medium, o, d, fminf(t, remaining), rng);
        if (!surface || T == 0) break;
        if (!VCHK(tri != 0xFFFFFFFFu, 2, interactions)) break;
        const uint32_t tm = v.tmed[tri];
        if (tm) {
            const f3 n = rawFaceNormal(sc, tri);
            if (medium != targetMedium(tm, -d, n)) return 0.0f;
            medium = targetMedium(tm, d, n);
        }
        if (++interactions > 100) break;
        o = o + d * t;
        remaining -= t;
        maxt = remaining * lengthFactor;
        mint = kEpsilon * max3abs(o);
    }
    return T;
}

struct ItsRef {  // the caller's intersection record: closest hit of the current ray
    bool valid;
    float t, u, v;
    uint32_t tri;
};

// rayIntersectAndLookForEmitter (progressive_volpath.cpp:401-460).  `its` gets the FIRST hit.  The
// walk through null surfaces is done once without the medium; `value` is the emitted radiance of the lit
// emitter it ends on (unattenuated), and when it crossed a medium the segments' transmittance is left to
// emitterWalkT (walk: its first ray and crossings), on the walk's own sub-stream (oracle/orc_volpath.h:
// the reference estimates the transmittance on every walk and discards it unless it ends on an emitter,
// the same estimator).
// exact: qdist = the whole walk's length (pg_config.volpath_exact_mis) instead of the last segment's
struct EmWalk {
    int medium, interactions;
    bool anyMedium;
};
__device__ __forceinline__ void lookForEmitter(const SceneDev &sc, const VolDev &v, int medium, int maxInteractions, f3 o0, f3 d,
                               float mint0, ItsRef &its, f3 &value, f3 &qn, float &qdist, int &qem, EmWalk &walk,
                               const TStack &stk, uint32_t &segs, bool exact) {
    value = mk1(0.f);
    qem = -1;
    f3 o = o0;
    float mint = mint0;
    int m = medium, interactions = 0;
    bool anyMedium = false;
    float t = 0, u = 0, w = 0, walked = 0;
    uint32_t tri = 0;
    uint32_t bits = 0;
    for (;;) {
        const bool surface = closestHit(sc, o, d, mint, __int_as_float(0x7f800000), t, tri, u, w, stk);
        segs++;
        if (interactions == 0) its = ItsRef{surface, surface ? t : __int_as_float(0x7f800000), u, w, tri};
        anyMedium |= m >= 0;
        if (!surface) return;  // no environment emitter
        bits = triBits(sc, tri);
        if (interactions == maxInteractions || !isNullMat(sc, bits) || (bits >> 16) != 0) break;
        const uint32_t tm = v.tmed[tri];
        if (tm) {
            Hit h;
            fetchHit(sc, tri, u, w, d, h);
            m = targetMedium(tm, d, h.geoN);
        }
        o = advance(o, d, t);
        walked += t;
        mint = itsMinT(o);
        if (++interactions > 100) return;
    }
    const int em = (int)(bits >> 16) - 1;
    if (em < 0) return;
    Hit h;
    fetchHit(sc, tri, u, w, d, h);
    if (!(dot(h.shN, -d) > 0)) return;  // AreaLight::eval: back side emits nothing
    const GEmitter &E = sc.ems[em];
    walk = EmWalk{medium, interactions, anyMedium};
    value = mk(E.radiance[0], E.radiance[1], E.radiance[2]);
    qn = h.shN;
    qdist = exact ? walked + t : t;  // setQuery: the LAST segment's length (records.inl:170-178)
    qem = em;
}
// the transmittance of an emitter walk's segments in media: the walk's rays again (origins advanced the
// same way, so the same surfaces), tracking every segment in a medium on the walk's sub-stream
__device__ __forceinline__ float emitterWalkT(const SceneDev &sc, const VolDev &v, int medium, int interactions, f3 o0,
                                              f3 d, float mint0, VRng &rng, const TStack &stk, uint32_t &segs) {
    float T = 1.0f;
    f3 oo = o0;
    float mt = mint0;
    int mm = medium;
    for (int k = 0; k <= interactions; ++k) {
        float tt, uu, ww;
        uint32_t tr;
        const bool hitR = closestHit(sc, oo, d, mt, __int_as_float(0x7f800000), tt, tr, uu, ww, stk);
        segs++;
        // the re-walk repeats the first walk's rays, so it hits the same surfaces; were a rounding
        // difference to make it miss, tr would be ~0 and v.tmed[tr] / fetchHit would read 16 GB
        // past their arrays (the round-3 C5 faults): end the estimate instead
        if (!VCHK(hitR, 1, k)) return 0.0f;
        if (mm >= 0) {
            T *= mediumTransmittance(v, mm, oo, d, tt, rng);
            if (T == 0) break;
        }
        const uint32_t tm = v.tmed[tr];
        if (tm) {
            Hit hh;
            fetchHit(sc, tr, uu, ww, d, hh);
            mm = targetMedium(tm, d, hh.geoN);
        }
        oo = advance(oo, d, tt);
        mt = itsMinT(oo);
    }
    return T;
}

// Scene::pdfEmitterDirect for a found emitter (area.cpp pdfDirect + shape.cpp:117-126)
__device__ __forceinline__ float pdfEmitter(const GParams &g, const SceneDev &sc, int em, f3 refN, f3 d, f3 n,
                                            float dist) {
    if (!(dot(d, refN) >= 0 && dot(d, n) < 0)) return 0.0f;
    return sc.ems[em].inv_area * (dist * dist) / absDot(d, n) * (1.0f / (float)g.num_emitters);
}

struct VPath {
    f3 o, d;
    ItsRef its;
    f3 T, L;
    float eta;
    int medium, depth;
    bool scattered, emission;
    uint32_t nv;  // training vertices written (GUIDED with g.record)
};

// training vertex nv of this item: (x, woPdf), (T after the bounce, packed canonical wo), (L snapshot),
// (-, -1: no learned-fraction statistics from the volumetric path)
__device__ __forceinline__ void writeVertex(const VolDev &v, uint32_t item, uint32_t k, f3 x, f3 wo, float woPdf, f3 Tn,
                                            f3 L) {
    float cu, cv;
    dirToCanonical(wo, cu, cv);
#if PG_VOL_CHECK
    if (!VCHK(item < v.vtx_P, 4, item)) return;
#endif
    float4 *vb = v.vtx + ((size_t)k * v.vtx_P + item) * PG_VTX_F4;
    vb[0] = f4(x, woPdf);
    vb[1] = f4(Tn, __uint_as_float(packCanonical(cu, cv)));
    vb[2] = f4(L, 0.0f);
    vb[3] = make_float4(0.0f, 0.0f, 0.0f, -1.0f);
}

// Deferred walks go to registers (VDefer; SINK false: k_vtail / k_volpath resolve them after the step) or
// straight to the slot's VolWave record (SINK true: k_vvertex, for k_vnee), so they hold no registers across
// the rest of the interaction.  Record: n0 (shadow walk origin, dim), n1 (emitter point, max crossings), n2
// (NEE contribution, (medium + 1) | onSurface << 16), h0 (emitter walk origin, mint), h1 (its direction,
// dim), h2 (its contribution, (medium + 1) | crossings << 16); the flags word (nflags, written by k_vvertex
// after the interaction) says which are valid, whether the path ended, and the vertex.
template <bool SINK>
__device__ __forceinline__ void deferNeeWalk(VDefer &df, const VolWave &w, uint32_t slot, f3 p1, f3 p2, bool onSurface,
                                             int medium, int maxInter, uint32_t dim) {
    df.nOnSurface = onSurface;
    df.nMedium = medium;
    if (SINK) {
        w.n0[slot] = f4(p1, __uint_as_float(dim));
        w.n1[slot] = f4(p2, __int_as_float(maxInter));
    } else {
        df.n1 = p1;
        df.n2 = p2;
        df.nMaxInter = maxInter;
        df.nDim = dim;
    }
}
template <bool SINK>
__device__ __forceinline__ void deferNeeC(VDefer &df, const VolWave &w, uint32_t slot, f3 C) {
    df.nee = true;
    if (SINK)
        w.n2[slot] = f4(C, __uint_as_float(((uint32_t)(df.nMedium + 1) & 0xFFFFu) | (df.nOnSurface ? 1u << 16 : 0u)));
    else
        df.nC = C;
}
// the emitter hit of a sampled ray: with a medium on its walk, its transmittance is deferred (the walk's
// first ray and crossings); without, the walk's transmittance is 1 and C * 1 joins L now
template <bool SINK>
__device__ __forceinline__ void deferHit(VDefer &df, const VolWave &w, uint32_t slot, f3 &L, f3 C, const EmWalk &walk,
                                         f3 o, f3 d, float mint, uint32_t dim) {
    if (!walk.anyMedium) {
        L = L + C * 1.0f;
        return;
    }
    df.hit = true;
    if (SINK) {
        w.h0[slot] = f4(o, mint);
        w.h1[slot] = f4(d, __uint_as_float(dim));
        w.h2[slot] = f4(C, __uint_as_float(((uint32_t)(walk.medium + 1) & 0xFFFFu) | ((uint32_t)walk.interactions << 16)));
        return;
    }
    df.hC = C;
    df.hO = o;
    df.hD = d;
    df.hMint = mint;
    df.hMedium = walk.medium;
    df.hInter = walk.interactions;
    df.hDim = dim;
}

// One iteration of the Li loop, in three parts that the megakernel (volStep) and the wavefront
// kernels (k_vflight, k_vvertex) share, so both run the same arithmetic on the same random streams:
//   volDepthOk   the loop condition (progressive_volpath.cpp:107) and the device bounce cap;
//   volFlight    the free flight of a path in a medium (Medium::sampleDistance, :109-115): true with
//                the medium interaction point mp, false when the flight reaches the surface its.t;
//   volMedium /  the medium (:117-196) and surface (:197-352) interactions including Russian roulette
//   volSurface   (:354-370); false when the path ends.
// GUIDED: SD-tree guiding at medium and smooth surface vertices (one-sample MIS with the phase function
// / BSDF, oracle/orc_volpath.h), guided free flight and training vertices; with an unbuilt tree it
// only writes the vertices.
__device__ __forceinline__ bool volDepthOk(const GParams &g, const VPath &P) {
    return (P.depth <= g.max_depth || g.max_depth < 0) && P.depth <= g.depth_cap;
}
template <bool GUIDED>
__device__ __forceinline__ bool volFlight(const VolDev &v, const SDDev &sd, VPath &P, VRng &rng, f3 &mp) {
    const bool guiding = GUIDED && sd.built;
    const float maxt = P.its.valid ? P.its.t : __int_as_float(0x7f800000);
    if (guiding && v.dist_beta > 0) {
        float w;
        const bool inMedium = mediumSampleGuided(v, sd, P.medium, P.o, P.d, maxt, rng, mp, w);
        P.T = P.T * w;
        return inMedium;
    }
    return mediumSample(v, P.medium, P.o, P.d, maxt, rng, mp);
}
// Russian roulette at the end of an interaction (progressive_volpath.cpp:354-370)
__device__ __forceinline__ bool volRoulette(const GParams &g, VPath &P, VRng &rng) {
    if (P.depth++ >= g.rr_depth) {
        const float q = fminf(maxc(P.T) * P.eta * P.eta, 0.95f);
        if (rng.next1() >= q) return false;
        P.T = P.T / q;
    }
    P.scattered = true;
    return true;
}
template <bool GUIDED, bool SINK>
__device__ __forceinline__ bool volMedium(const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                                          VPath &P, VRng &rng, const TStack &stk, uint32_t item, uint32_t &segs,
                                          uint32_t &shadows, f3 mp, VDefer &df, const VolWave &wk) {
    const int maxDepth = g.max_depth;
    const int maxInter = maxDepth - P.depth - 1;
    const bool guiding = GUIDED && sd.built;
    const bool record = GUIDED && g.record;
    const float alpha = g.bsdf_fraction;
    {
        // ---- medium interaction (progressive_volpath.cpp:117-196)
        if (P.depth >= maxDepth && maxDepth != -1) return false;
        const GMedium &GM = v.media[P.medium];
        P.T = P.T * mk(GM.albedo[0], GM.albedo[1], GM.albedo[2]);
        const float hg = GM.g;
        const f3 wi = -P.d;
        const SDView sv = sdv(sd);
        uint4 meta = make_uint4(0, 0, 0, 0);
        if (guiding) meta = sd.meta[sdLookup(sv, mp)];
        const float alphaM = alpha + (1 - alpha) * fabsf(hg);  // anisotropy-raised phase fraction (oracle)
        // NEE: the light sample now, its shadow walk deferred (VDefer); with guiding its MIS weight waits
        // for the D-tree pdf of the light direction, resolved in one lockstep walk with the direction (sdDual)
        f3 neeV = mk1(0.f), dD = mk1(0.f);
        float neePdf = 0, neePhase = 0;
        bool neePending = false;
        if (g.use_nee) {
            const uint32_t ndim = rng.dim;  // the shadow walk's sub-stream
            float s0, s1;
            rng.next2(s0, s1);
            f3 ep;
            float dist, pdf;
            const f3 value = sampleEmitter(g, sc, mp, mk1(0.f), s0, s1, dD, dist, pdf, &ep);
            if (pdf != 0) {
                shadows++;
                const float phaseVal = hgEval(hg, wi, dD);
                if (phaseVal != 0 && !isZero(value)) {
                    deferNeeWalk<SINK>(df, wk, item, mp, ep, false, P.medium, maxInter, ndim);
                    if (guiding) {
                        neeV = P.T * value;
                        neePdf = pdf;
                        neePhase = phaseVal;
                        neePending = true;
                    } else {
                        deferNeeC<SINK>(df, wk, item, (P.T * value) * (phaseVal * miWeight(pdf, phaseVal)));
                    }
                }
            }
        }
        float u0, u1, phasePdf;
        rng.next2(u0, u1);
        f3 wo;
        float woPdf, pw = 1.0f;
        if (!guiding) {
            wo = hgSample(hg, wi, u0, u1, phasePdf);
            woPdf = phasePdf;
        } else {
            int mode;  // 1: phase sample (D-tree pdf query), 2: D-tree sample
            float bu, bw;
            if (rng.next1() < alphaM) {
                mode = 1;
                wo = hgSample(hg, wi, u0, u1, phasePdf);
                dirToCanonical(wo, bu, bw);
            } else {
                mode = 2;
                rng.next2(bu, bw);
            }
            float au = 0, aw = 0, aPdf, dPdf, cu, cv;
            if (neePending) dirToCanonical(dD, au, aw);
            sdDual(sv, meta, neePending, au, aw, aPdf, true, mode == 2, bu, bw, cu, cv, dPdf);
            if (neePending)
                deferNeeC<SINK>(df, wk, item, neeV * (neePhase * miWeight(neePdf, alphaM * neePhase + (1 - alphaM) * aPdf)));
            if (mode == 2) {
                wo = canonicalToDir(cu, cv);
                phasePdf = hgEval(hg, wi, wo);
            }
            woPdf = alphaM * phasePdf + (1 - alphaM) * dPdf;
            if (!(woPdf > 0)) return false;
            pw = phasePdf / woPdf;
        }
        if (record && P.nv < (uint32_t)g.max_vertices) {
            df.k = (int)P.nv;
            writeVertex(v, item, P.nv++, mp, wo, woPdf, P.T * pw, P.L);
        }
        P.T = P.T * pw;
        P.o = mp;
        P.d = wo;
        f3 value, qn;
        float qdist;
        int qem;
        EmWalk walk;
        const uint32_t hdim = rng.dim;  // the emitter walk's sub-stream
        lookForEmitter(sc, v, P.medium, maxInter, mp, wo, 0.0f, P.its, value, qn, qdist, qem, walk, stk, segs, g.exact_mis != 0);
        if (!isZero(value) && fminf(value.x, fminf(value.y, value.z)) > 0.f) {
            const float emitterPdf = g.use_nee ? pdfEmitter(g, sc, qem, mk1(0.f), wo, qn, qdist) : 0.0f;
            const f3 C = (P.T * value) * (g.use_nee ? miWeight(woPdf, emitterPdf) : 1.0f);
            deferHit<SINK>(df, wk, item, P.L, C, walk, mp, wo, 0.0f, hdim);
        }
        P.emission = false;
    }
    return volRoulette(g, P, rng);
}
// MODELS: pg_device.h modelSel (-1 any material; PG_MODELS_DIFFUSE_NULL when the scene has only those)
template <bool GUIDED, bool SINK, int MODELS = -1>
__device__ __forceinline__ bool volSurface(const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                                           VPath &P, VRng &rng, const TStack &stk, uint32_t item, uint32_t &segs,
                                           uint32_t &shadows, VDefer &df, const VolWave &wk) {
    const int maxDepth = g.max_depth;
    const int maxInter = maxDepth - P.depth - 1;
    const bool guiding = GUIDED && sd.built;
    const bool record = GUIDED && g.record;
    const float alpha = g.bsdf_fraction;
    {
        // ---- surface interaction (progressive_volpath.cpp:197-352)
        if (!P.its.valid) return false;  // no environment emitter
        Hit h;
        fetchHit(sc, P.its.tri, P.its.u, P.its.v, P.d, h);
        if (h.emitter >= 0 && P.emission && (!g.hide_emitters || P.scattered) && dot(h.shN, -P.d) > 0) {
            const GEmitter &E = sc.ems[h.emitter];
            P.L = P.L + P.T * mk(E.radiance[0], E.radiance[1], E.radiance[2]);
        }
        if (P.depth >= maxDepth && maxDepth != -1) return false;
        if (g.strict_normals && -dot(h.geoN, P.d) * h.wi.z < 0) return false;
        const GMat &M = sc.mats[h.mat];
        const f3 refN = (M.type & (ETransmission | EBackSide)) == 0 ? h.shN : mk1(0.f);
        const uint32_t tm = v.tmed[P.its.tri];
        const bool guide = guiding && (M.type & ESmooth) && !(M.type & EDelta);
        const SDView sv = sdv(sd);
        uint4 meta = make_uint4(0, 0, 0, 0);
        if (guide) meta = sd.meta[sdLookup(sv, h.p)];
        f3 neeV = mk1(0.f), dD = mk1(0.f);
        float neePdf = 0, neeBp = 0;
        bool neePending = false;
        if (g.use_nee && (M.type & ESmooth)) {
            const uint32_t ndim = rng.dim;  // the shadow walk's sub-stream
            float s0, s1;
            rng.next2(s0, s1);
            f3 ep;
            float dist, pdf;
            const f3 value = sampleEmitter(g, sc, h.p, refN, s0, s1, dD, dist, pdf, &ep);
            if (pdf != 0) {
                const int m2 = tm ? targetMedium(tm, dD, h.geoN) : P.medium;
                shadows++;
                if (!isZero(value)) {
                    const f3 woL = h.sh.toLocal(dD);
                    const f3 f = bsdfEval<MODELS>(M, h.wi, woL);
                    if (!isZero(f) && (!g.strict_normals || dot(h.geoN, dD) * woL.z > 0)) {
                        const float bp = bsdfPdf<MODELS>(M, h.wi, woL);
                        deferNeeWalk<SINK>(df, wk, item, h.p, ep, true, m2, maxInter, ndim);
                        if (guide) {
                            neeV = (P.T * value) * f;
                            neePdf = pdf;
                            neeBp = bp;
                            neePending = true;
                        } else {
                            deferNeeC<SINK>(df, wk, item, ((P.T * value) * f) * miWeight(pdf, bp));
                        }
                    }
                }
            }
        }
        float b0, b1;
        rng.next2(b0, b1);
        const float b2 = rng.next1();
        BS bs;
        f3 weight;
        float woPdf;
        if (!guide) {
            weight = bsdfSample<MODELS>(M, h.wi, b0, b1, b2, bs);
            woPdf = bs.pdf;
        } else {
            int mode = 0;  // 0: BSDF sample failed, 1: BSDF sample (D-tree pdf query), 2: D-tree sample
            float bu = 0, bw = 0;
            if (rng.next1() < alpha) {
                weight = bsdfSample<MODELS>(M, h.wi, b0, b1, b2, bs);
                if (!isZero(weight)) {
                    mode = 1;
                    dirToCanonical(h.sh.toWorld(bs.wo), bu, bw);
                }
            } else {
                mode = 2;
                rng.next2(bu, bw);
            }
            float au = 0, aw = 0, aPdf, dPdf, cu, cv;
            if (neePending) dirToCanonical(dD, au, aw);
            sdDual(sv, meta, neePending, au, aw, aPdf, mode != 0, mode == 2, bu, bw, cu, cv, dPdf);
            if (neePending) deferNeeC<SINK>(df, wk, item, neeV * miWeight(neePdf, alpha * neeBp + (1 - alpha) * aPdf));
            if (mode == 0) return false;
            if (mode == 1) {
                woPdf = alpha * bs.pdf + (1 - alpha) * dPdf;
                weight = weight * (bs.pdf / woPdf);
            } else {
                const f3 woL = h.sh.toLocal(canonicalToDir(cu, cv));
                const f3 f = bsdfEval<MODELS>(M, h.wi, woL);
                const float bp = bsdfPdf<MODELS>(M, h.wi, woL);
                woPdf = alpha * bp + (1 - alpha) * dPdf;
                if (!(woPdf > 0) || isZero(f)) return false;
                weight = f / woPdf;
                bs.wo = woL;
                bs.pdf = bp;
                const bool refl = h.wi.z * woL.z > 0;
                bs.type = refl ? ((M.type & EDiffuseReflection) ? EDiffuseReflection : EGlossyReflection)
                               : EGlossyTransmission;
                bs.eta = refl ? 1.0f : (h.wi.z > 0 ? M.eta : M.invEta);
            }
        }
        if (isZero(weight)) return false;
        const f3 wo = h.sh.toWorld(bs.wo);
        if (g.strict_normals && dot(h.geoN, wo) * bs.wo.z <= 0) return false;
        if (record && !(bs.type & EDelta) && bs.type != ENull && P.nv < (uint32_t)g.max_vertices) {
            df.k = (int)P.nv;
            writeVertex(v, item, P.nv++, h.p, wo, woPdf, P.T * weight, P.L);
        }
        P.o = h.p;
        P.d = wo;
        P.T = P.T * weight;
        P.eta *= bs.eta;
        if (tm) P.medium = targetMedium(tm, wo, h.geoN);
        if (bs.type == ENull) {  // index-matched boundary: straight through, counted as a bounce
            P.emission = !P.scattered;
            float t, u, w;
            uint32_t tri;
            const bool hit = closestHit(sc, h.p, wo, itsMinT(h.p), __int_as_float(0x7f800000), t, tri, u, w, stk);
            segs++;
            P.its = ItsRef{hit, hit ? t : __int_as_float(0x7f800000), u, w, tri};
            P.depth++;
            return true;
        }
        f3 value, qn;
        float qdist;
        int qem;
        EmWalk walk;
        const uint32_t hdim = rng.dim;  // the emitter walk's sub-stream
        const float mint0 = itsMinT(h.p);
        lookForEmitter(sc, v, P.medium, maxInter, h.p, wo, mint0, P.its, value, qn, qdist, qem, walk, stk, segs,
                       g.exact_mis != 0);
        if (!isZero(value)) {
            const float emitterPdf =
                (g.use_nee && !(bs.type & EDelta)) ? pdfEmitter(g, sc, qem, refN, wo, qn, qdist) : 0.0f;
            const f3 C = (P.T * value) * (g.use_nee ? miWeight(woPdf, emitterPdf) : 1.0f);
            deferHit<SINK>(df, wk, item, P.L, C, walk, h.p, wo, mint0, hdim);
        }
        P.emission = false;
    }
    return volRoulette(g, P, rng);
}
// an interaction's deferred walks, in the oracle's order: the emitter hit, then the NEE (into L and into
// the snapshot of the interaction's training vertex); each on its own sub-stream of the path's key
// the walks' transmittances, each on its sub-stream (no radiance touched yet)
__device__ __forceinline__ void walkDeferred(const SceneDev &sc, const VolDev &v, const VDefer &df, uint32_t key,
                                             uint32_t sample, const TStack &stk, uint32_t &segs, uint32_t &lookups,
                                             float &Th, float &Tn) {
    Th = Tn = 0.0f;
    if (df.hit) {
        VRng sub = subStream(key, sample, df.hDim, 1);
        Th = emitterWalkT(sc, v, df.hMedium, df.hInter, df.hO, df.hD, df.hMint, sub, stk, segs);
        lookups += sub.lookups;
    }
    if (df.nee) {
        VRng sub = subStream(key, sample, df.nDim, 0);
        Tn = sceneTransmittance(sc, v, df.n1, df.nOnSurface, df.n2, df.nMedium, df.nMaxInter, sub, stk, segs);
        lookups += sub.lookups;
    }
}
// their contributions, in the fixed order: the emitter hit, then the NEE (also into the vertex's snapshot)
__device__ __forceinline__ void addDeferred(const VolDev &v, const VDefer &df, float Th, float Tn, uint32_t item, f3 &L) {
    if (df.hit && Th != 0) L = L + df.hC * Th;
    if (df.nee && Tn != 0) {
        const f3 add = df.nC * Tn;
        L = L + add;
        if (df.k >= 0) {
            float4 *vb = v.vtx + ((size_t)df.k * v.vtx_P + item) * PG_VTX_F4;
            vb[2] = f4(xyz(vb[2]) + add, 0.0f);
        }
    }
}
__device__ __forceinline__ void resolveDeferred(const SceneDev &sc, const VolDev &v, const VDefer &df, uint32_t key,
                                                uint32_t sample, uint32_t item, f3 &L, const TStack &stk,
                                                uint32_t &segs, uint32_t &lookups) {
    float Th, Tn;
    walkDeferred(sc, v, df, key, sample, stk, segs, lookups, Th, Tn);
    addDeferred(v, df, Th, Tn, item, L);
}
__device__ __forceinline__ void clearDefer(VDefer &df) {
    df.nee = df.hit = false;
    df.k = -1;
}

template <bool GUIDED, int MODELS = -1>
__device__ __forceinline__ bool volStep(const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                                        VPath &P, VRng &rng, const TStack &stk, uint32_t item, uint32_t &segs,
                                        uint32_t &shadows, VDefer &df) {
    if (!volDepthOk(g, P)) return false;
    f3 mp = mk1(0.f);
    const VolWave none{};
    if (P.medium >= 0 && volFlight<GUIDED>(v, sd, P, rng, mp))
        return volMedium<GUIDED, false>(g, sc, v, sd, P, rng, stk, item, segs, shadows, mp, df, none);
    return volSurface<GUIDED, false, MODELS>(g, sc, v, sd, P, rng, stk, item, segs, shadows, df, none);
}
// one step with its walks resolved right away (k_vtail, k_volpath): the same arithmetic as the wavefront's
// k_vvertex + k_vnee
template <bool GUIDED, int MODELS = -1>
__device__ __forceinline__ bool volStepResolved(const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                                                VPath &P, VRng &rng, const TStack &stk, uint32_t item, uint32_t &segs,
                                                uint32_t &shadows) {
    VDefer df;
    clearDefer(df);
    const bool alive = volStep<GUIDED, MODELS>(g, sc, v, sd, P, rng, stk, item, segs, shadows, df);
    if (df.hit || df.nee) resolveDeferred(sc, v, df, rng.key, rng.sample, item, P.L, stk, segs, rng.lookups);
    return alive;
}

// the camera ray of work item `item` (PerspectiveCamera::sampleRay, perspective.cpp:271-298) and its
// first hit: a new path state
__device__ __forceinline__ void volCamera(const GParams &g, const SceneDev &sc, const VolDev &v,
                                          const uint32_t *__restrict__ local_pixels, uint32_t pix_begin, uint32_t npix,
                                          uint32_t sample_base, uint32_t item, VPath &P, VRng &rng, const TStack &stk,
                                          uint32_t &segs) {
    const uint32_t layer = item / npix, lp = item - layer * npix;
    const uint32_t pix = local_pixels[pix_begin + lp];
    rng = VRng{rngKey(pix, g.seed), sample_base + layer, 1, 0};
    float jx, jy;
    rng2(rng.key, rng.sample, 0, jx, jy);
    const float px = (float)(pix % g.width) + jx, py = (float)(pix / g.width) + jy;
    const float sx = px / (float)g.width, sy = py / (float)g.height;
    const f3 nearP = mk((1.0f - 2.0f * sx) * g.tan_half, (1.0f - 2.0f * sy) / g.aspect * g.tan_half, 1.0f);
    const f3 dl = normalize(nearP);
    const float invZ = 1.0f / dl.z;
    P.o = mk(g.cam_o[0], g.cam_o[1], g.cam_o[2]);
    P.d = mk(g.cam_left[0], g.cam_left[1], g.cam_left[2]) * dl.x +
          mk(g.cam_up[0], g.cam_up[1], g.cam_up[2]) * dl.y + mk(g.cam_dir[0], g.cam_dir[1], g.cam_dir[2]) * dl.z;
    float t, u, w;
    uint32_t tri;
    const bool hit = closestHit(sc, P.o, P.d, g.near_clip * invZ, g.far_clip * invZ, t, tri, u, w, stk);
    segs++;
    P.its = ItsRef{hit, hit ? t : __int_as_float(0x7f800000), u, w, tri};
    P.T = mk1(1.f);
    P.L = mk1(0.f);
    P.eta = 1.0f;
    P.medium = v.cam_medium;
    P.depth = 1;
    P.scattered = false;
    P.emission = true;
    P.nv = 0;
}

// ---- wavefront state (VolWave, pg_kernels.h) ---------------------------------------------------
__device__ __forceinline__ void loadPath(const VolWave &w, uint32_t slot, VPath &P, VRng &rng) {
    const float4 o = w.o[slot], d = w.d[slot], T = w.T[slot], L = w.L[slot];
    const uint4 s = w.s[slot], r = w.r[slot];
    P.o = xyz(o);
    P.d = xyz(d);
    P.its = ItsRef{((s.z >> 16) & 1u) != 0, o.w, d.w, __uint_as_float(s.x), s.y};
    P.medium = (int)(s.z & 0xFFFFu) - 1;
    P.scattered = ((s.z >> 17) & 1u) != 0;
    P.emission = ((s.z >> 18) & 1u) != 0;
    P.depth = (int)s.w;
    P.T = xyz(T);
    P.eta = T.w;
    P.L = xyz(L);
    P.nv = __float_as_uint(L.w);
    rng = VRng{r.x, r.y, r.z, r.w};
}
__device__ __forceinline__ void storePath(const VolWave &w, uint32_t slot, const VPath &P, const VRng &rng) {
    w.o[slot] = f4(P.o, P.its.t);
    w.d[slot] = f4(P.d, P.its.u);
    w.s[slot] = make_uint4(__float_as_uint(P.its.v), P.its.tri,
                           (uint32_t)(P.medium + 1) | (P.its.valid ? 1u << 16 : 0u) | (P.scattered ? 1u << 17 : 0u) |
                               (P.emission ? 1u << 18 : 0u),
                           (uint32_t)P.depth);
    w.T[slot] = f4(P.T, P.eta);
    w.L[slot] = f4(P.L, __uint_as_float(P.nv));
    w.r[slot] = make_uint4(rng.key, rng.sample, rng.dim, rng.lookups);
}
// the flags word of a slot's deferred record (VolWave nflags): nee | hit << 1 | ended << 2 | (vertex + 1) << 8
__device__ __forceinline__ uint32_t deferFlags(const VDefer &df, bool ended) {
    return (df.nee ? 1u : 0u) | (df.hit ? 2u : 0u) | (ended ? 4u : 0u) | ((uint32_t)(df.k + 1) << 8);
}
__device__ __forceinline__ void loadDefer(const VolWave &w, uint32_t slot, VDefer &df, bool &ended, uint32_t &key,
                                          uint32_t &sample) {
    const uint4 rec = w.nflags[slot];
    const uint32_t flags = rec.x;
    key = rec.y;
    sample = rec.z;
    df.nee = flags & 1u;
    df.hit = (flags >> 1) & 1u;
    ended = (flags >> 2) & 1u;
    df.k = (int)(flags >> 8) - 1;
    if (df.nee) {
        const float4 a = w.n0[slot], b = w.n1[slot], c = w.n2[slot];
        df.n1 = xyz(a);
        df.nDim = __float_as_uint(a.w);
        df.n2 = xyz(b);
        df.nMaxInter = __float_as_int(b.w);
        df.nC = xyz(c);
        const uint32_t m = __float_as_uint(c.w);
        df.nMedium = (int)(m & 0xFFFFu) - 1;
        df.nOnSurface = (m >> 16) & 1u;
    }
    if (df.hit) {
        const float4 a = w.h0[slot], b = w.h1[slot], e = w.h2[slot];
        df.hO = xyz(a);
        df.hMint = a.w;
        df.hD = xyz(b);
        df.hDim = __float_as_uint(b.w);
        df.hC = xyz(e);
        const uint32_t m = __float_as_uint(e.w);
        df.hMedium = (int)(m & 0xFFFFu) - 1;
        df.hInter = (int)(m >> 16);
    }
}

// wave sums of the per-thread counters, one atomic each per wave
__device__ __forceinline__ void volStats(const VolDev &v, uint32_t segs, uint32_t shadows, uint32_t lookups) {
    unsigned long long s0 = segs, s1 = shadows, s2 = lookups;
    for (int off = 32; off > 0; off >>= 1) {
        s0 += __shfl_xor(s0, off);
        s1 += __shfl_xor(s1, off);
        s2 += __shfl_xor(s2, off);
    }
    if ((threadIdx.x & 63) == 0 && (s0 | s1 | s2)) {
        atomicAdd(v.stats, s0);
        atomicAdd(v.stats + 1, s1);
        atomicAdd(v.stats + 2, s2);
    }
}
// wavefront stage counters (VolDev.stats[k], [k + 1]): items processed, density lookups made
__device__ __forceinline__ void volStageStats(const VolDev &v, int k, uint32_t items, uint32_t lookups) {
    unsigned long long a = items, b = lookups;
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
    }
    if ((threadIdx.x & 63) == 0 && (a | b)) {
        atomicAdd(v.stats + k, a);
        atomicAdd(v.stats + k + 1, b);
    }
}
// a path that ended: its radiance and training-vertex count (k_film / k_commit), its lookups counted
__device__ __forceinline__ void volEnd(const VolDev &v, uint32_t slot, const VPath &P, const VRng &rng,
                                       uint32_t &lookups) {
    v.rad[slot] = f4(P.L, __uint_as_float(P.nv));
    lookups += rng.lookups;
}
__device__ __forceinline__ uint32_t slotShard(uint32_t slot) { return (slot >> 6) & (PG_QSHARDS - 1); }

// flight order key (PG_VOL_SORT; pg_layout.h PG_VOL_SORT_KEY): the Morton code of the cell of the medium's
// box that holds o -- 8^3 cells (9 bits, 512 bins) or 16^3 (12 bits), or the direction octant and an
// 8^3 cell -- so a sorted flight queue walks the density grid region by region
__device__ __forceinline__ uint16_t flightKey(const VolDev &v, int m, f3 o, f3 d) {
    const GMedium &M = v.media[m];
    constexpr int bits = PG_VOL_SORT_KEY == 0 ? 4 : 3;
    constexpr float res = (float)(1 << bits);
    const float fx = (o.x - M.lo[0]) / (M.hi[0] - M.lo[0]), fy = (o.y - M.lo[1]) / (M.hi[1] - M.lo[1]),
                fz = (o.z - M.lo[2]) / (M.hi[2] - M.lo[2]);
    const uint32_t cx = (uint32_t)fminf(fmaxf(fx * res, 0.0f), res - 1.0f), cy = (uint32_t)fminf(fmaxf(fy * res, 0.0f), res - 1.0f),
                   cz = (uint32_t)fminf(fmaxf(fz * res, 0.0f), res - 1.0f);
    uint32_t k = 0;
    for (int b = 0; b < bits; ++b)
        k |= (((cx >> b) & 1u) << (3 * b)) | (((cy >> b) & 1u) << (3 * b + 1)) | (((cz >> b) & 1u) << (3 * b + 2));
    if (PG_VOL_SORT_KEY == 1) k |= ((d.x < 0 ? 1u : 0u) | (d.y < 0 ? 2u : 0u) | (d.z < 0 ? 4u : 0u)) << 9;
    return (uint16_t)k;
}
// surface vertices split by the hit triangle (PG_VOL_SPLIT_SURF): delta surfaces (the null boundaries of
// media, smooth conductors and dielectrics: no emitter sample, no shadow walk), emitters (PG_VOL_SPLIT_EMIT:
// black in the scenes here, so the path ends there) and escaped rays go to their own queue, so the waves
// of the other surfaces' shadow walks carry no idle lanes
#ifndef PG_VOL_SPLIT_SURF
#define PG_VOL_SPLIT_SURF 1
#endif
#ifndef PG_VOL_SPLIT_EMIT
#define PG_VOL_SPLIT_EMIT 1
#endif
__device__ __forceinline__ bool cheapSurface(const SceneDev &sc, const VolDev &v, bool valid, uint32_t tri) {
    return PG_VOL_SPLIT_SURF &&
           (!valid || (PG_VOL_SPLIT_EMIT ? v.tcheap[tri] != 0 : sc.tclass[tri] == PG_CLASS_DELTA));
}
__device__ __forceinline__ void surfAppend(bool pred, bool cheap, uint32_t slot, const Queue &qs, const Queue &qd,
                                           uint32_t sh) {
    waveAppend(pred && !cheap, slot, qs.items + (size_t)sh * qs.stride, qs.counts + sh);
    if (PG_VOL_SPLIT_SURF) waveAppend(pred && cheap, slot, qd.items + (size_t)sh * qd.stride, qd.counts + sh);
}
// append to a flight queue, with the order key when the queue carries keys
__device__ __forceinline__ void flightAppend(bool pred, uint32_t slot, uint16_t key, const Queue &q, uint32_t sh) {
    if (q.keys)
        waveAppendKey(pred, slot, key, q.items + (size_t)sh * q.stride, q.keys + (size_t)sh * q.stride, q.counts + sh);
    else
        waveAppend(pred, slot, q.items + (size_t)sh * q.stride, q.counts + sh);
}

}  // namespace

// ---- volumetric wavefront (the volpath loop as a wavefront of path states) -----
// Stages per iteration of progressive_volpath.cpp:98-374: the free flight of every path in a medium
// (k_vflight), then the medium and surface interactions in one launch whose blocks take one kind each
// (k_vvertex: no wave runs both branches), each path in its slot with its random stream carried in
// VolWave, so films and trees are bit-identical to k_volpath's (which runs the same volFlight /
// volMedium / volSurface per lane).  The last few paths finish one thread each (k_vtail).
template <bool GUIDED>
__global__ __launch_bounds__(TRACE_BLOCK) void k_vcam(GParams g, SceneDev sc, VolDev v, VolWave w,
                                                      const uint32_t *__restrict__ local_pixels, uint32_t pix_begin,
                                                      uint32_t npix, uint32_t nlayers, uint32_t sample_base, Queue qf,
                                                      Queue qs, Queue qd) {
    __shared__ uint32_t stack[LDS_STACK * TRACE_BLOCK];
    const TStack stk = threadStack(stack, v.stack_ovf);
    const uint32_t n = npix * nlayers;
    uint32_t segs = 0, lookups = 0;
    for (uint32_t base = blockIdx.x * TRACE_BLOCK; base < n; base += gridDim.x * TRACE_BLOCK) {
        const uint32_t slot = base + threadIdx.x;
        bool toF = false, toS = false, cheap = false;
        uint16_t key = 0;
        if (slot < n) {
            VPath P;
            VRng rng;
            volCamera(g, sc, v, local_pixels, pix_begin, npix, sample_base, slot, P, rng, stk, segs);
            if (!volDepthOk(g, P)) {
                volEnd(v, slot, P, rng, lookups);
            } else {
                storePath(w, slot, P, rng);
                toF = P.medium >= 0;
                toS = !toF;
                if (toF && qf.keys) key = flightKey(v, P.medium, P.o, P.d);
                if (toS) cheap = cheapSurface(sc, v, P.its.valid, P.its.tri);
            }
        }
        const uint32_t sh = slotShard(base + (threadIdx.x & ~63u));
        flightAppend(toF, slot, key, qf, sh);
        surfAppend(toS, cheap, slot, qs, qd, sh);
    }
    volStats(v, segs, 0, lookups);
}

// free flights: medium interaction -> med, the flight reached its surface (or left the medium) -> surf
// waves per SIMD the stage kernels are built for (A/B knobs; 0 = the compiler's choice).  k_vflight at 4:
// 128 VGPRs without scratch (the compiler's 132 gave 3 waves); C5 363.6 / 363.4 against 351.9 / 350.5
// Mpaths/s (profiles/r04t_vol_ab/)
#ifndef PG_VFLIGHT_WAVES
#define PG_VFLIGHT_WAVES 4
#endif
#ifndef PG_VVERTEX_WAVES
#define PG_VVERTEX_WAVES PG_VOL_WAVES
#endif
template <bool GUIDED>
__global__ __launch_bounds__(TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(PG_VFLIGHT_WAVES > 0 ? PG_VFLIGHT_WAVES : 1)))
void k_vflight(GParams g, SceneDev sc, VolDev v, SDDev sd, VolWave w, Queue qf, Queue qm, Queue qs, Queue qd) {
    const uint32_t sh = blockIdx.x & (PG_QSHARDS - 1), rows = gridDim.x / PG_QSHARDS;
    const uint32_t n = qf.counts[sh];
    uint32_t flights = 0, lookups = 0;
    for (uint32_t base = (blockIdx.x / PG_QSHARDS) * TRACE_BLOCK; base < n; base += rows * TRACE_BLOCK) {
        const uint32_t i = base + threadIdx.x;
        bool toM = false, toS = false, cheap = false;
        uint32_t slot = 0;
        if (i < n) {
            slot = qf.items[(size_t)sh * qf.stride + i];
            const float4 o = w.o[slot], d = w.d[slot];
            const uint4 s = w.s[slot], r = w.r[slot];
            VPath P;
            P.o = xyz(o);
            P.d = xyz(d);
            P.its.valid = ((s.z >> 16) & 1u) != 0;
            P.its.t = o.w;
            P.medium = (int)(s.z & 0xFFFFu) - 1;
            const bool wT = GUIDED && sd.built && v.dist_beta > 0;  // guided free flight reweights T
            if (wT) P.T = xyz(w.T[slot]);
            VRng rng{r.x, r.y, r.z, r.w};
            f3 mp = mk1(0.f);
            toM = volFlight<GUIDED>(v, sd, P, rng, mp);
            toS = !toM;
            if (toS) cheap = cheapSurface(sc, v, P.its.valid, s.y);
            flights++;
            lookups += rng.lookups - r.w;
            w.r[slot] = make_uint4(rng.key, rng.sample, rng.dim, rng.lookups);
            if (wT) w.T[slot] = f4(P.T, w.T[slot].w);
            if (toM) w.mp[slot] = f4(mp, 0.0f);
        }
        waveAppend(toM, slot, qm.items + (size_t)sh * qm.stride, qm.counts + sh);
        surfAppend(toS, cheap, slot, qs, qd, sh);
    }
    volStageStats(v, 3, flights, lookups);
}

// interactions: blocks [0, mblocks) take the medium vertices, the rest the surface vertices.  KIND 2: both
// in one launch (PG_VOL_SPLIT_VERTEX=0); KIND 0 / 1 (default): the medium / surface blocks only, as launches of
// their own; KIND 3: the surface launch of a scene whose materials are all diffuse or null (VolDev::models),
// compiled without the other BSDF models.  KIND 0 / 1 / 3 are launches of
// their own, so each gets its own register budget: the medium kernel runs at 3 waves per SIMD (with the
// walks deferred to k_vnee without scratch, PG_VMEDIUM_WAVES; with them inline 44 B/lane of scratch,
// PG_VMEDIUM_INLINE_WAVES), the surface kernel's BSDFs need more
#ifndef PG_VMEDIUM_WAVES
#define PG_VMEDIUM_WAVES 3
#endif
#ifndef PG_VSURFACE_WAVES
#define PG_VSURFACE_WAVES 3
#endif
// the medium launch with its walks inline: 3 waves/SIMD (192 VGPRs uncapped; 168 with 44 B/lane of scratch,
// the path state stored before the walks): C5 405.2 / 404.6 against 393.0 / 392.6 Mpaths/s at 2 waves and
// 392.3 / 393.2 as one launch (profiles/r05o_vol_vertex_split/)
#ifndef PG_VMEDIUM_INLINE_WAVES
#define PG_VMEDIUM_INLINE_WAVES 3
#endif
// ... and the surface launch at 3 waves too (228 VGPRs uncapped; 168 with 156 B/lane of scratch): C5
// 439.2 / 439.6 against 405.8 / 405.5 at 2 waves; 4 waves 434.0 / 433.8, the medium launch at 4 with the
// surface at 3 432.9 / 431.5 (profiles/r05p_vol_waves/, r05q_vol_waves/).  With three lanes in flight the
// interactions' occupancy pays more than their spills cost
#ifndef PG_VSURFACE_INLINE_WAVES
#define PG_VSURFACE_INLINE_WAVES 3
#endif
template <bool NEE_STAGE, int KIND>
struct VVertexWaves {
    static constexpr int value = KIND == 0 ? (NEE_STAGE ? PG_VMEDIUM_WAVES : PG_VMEDIUM_INLINE_WAVES)
                                           : (KIND == 1 || KIND == 3 ? (NEE_STAGE ? PG_VSURFACE_WAVES : PG_VSURFACE_INLINE_WAVES)
                                                        : PG_VVERTEX_WAVES);
};
template <bool GUIDED, bool NEE_STAGE, int KIND>
__global__ __launch_bounds__(TRACE_BLOCK, (VVertexWaves<NEE_STAGE, KIND>::value)) void k_vvertex(GParams g, SceneDev sc, VolDev v, SDDev sd,
                                                                       VolWave w, Queue qm, Queue qs, Queue qd,
                                                                       uint32_t mblocks, uint32_t dblocks, Queue nf,
                                                                       Queue ns, Queue nd, Queue qn) {
    __shared__ uint32_t stack[LDS_STACK * TRACE_BLOCK];
    const TStack stk = threadStack(stack, v.stack_ovf);
    // blocks [0, mblocks): medium vertices; [mblocks, mblocks + dblocks): delta surfaces; the rest: surfaces
    const bool medium = KIND == 0 || (KIND == 2 && blockIdx.x < mblocks);
    const bool delta = !medium && blockIdx.x < mblocks + dblocks;
    const uint32_t b = medium ? blockIdx.x : (delta ? blockIdx.x - mblocks : blockIdx.x - mblocks - dblocks);
    const uint32_t nb = medium ? mblocks : (delta ? dblocks : gridDim.x - mblocks - dblocks);
    const Queue &q = medium ? qm : (delta ? qd : qs);
    const uint32_t sh = b & (PG_QSHARDS - 1), rows = nb / PG_QSHARDS;
    const uint32_t n = q.counts[sh];
    uint32_t segs = 0, shadows = 0, lookups = 0, vertices = 0, vlookups = 0;
    for (uint32_t base = (b / PG_QSHARDS) * TRACE_BLOCK; base < n; base += rows * TRACE_BLOCK) {
        const uint32_t i = base + threadIdx.x;
        bool toF = false, toS = false, cheap = false, toN = false;
        uint32_t slot = 0;
        uint16_t key = 0;
        if (i < n) {
            slot = q.items[(size_t)sh * q.stride + i];
            VPath P;
            VRng rng;
            loadPath(w, slot, P, rng);
            const uint32_t l0 = rng.lookups;
            VDefer df;
            clearDefer(df);
            bool alive;
            if (KIND == 0 || (KIND == 2 && medium))
                alive = volMedium<GUIDED, NEE_STAGE>(g, sc, v, sd, P, rng, stk, slot, segs, shadows, xyz(w.mp[slot]), df, w);
            else
                alive = volSurface<GUIDED, NEE_STAGE, KIND == 3 ? PG_MODELS_DIFFUSE_NULL : -1>(g, sc, v, sd, P, rng, stk,
                                                                                          slot, segs, shadows, df, w);
            vertices++;
            const bool ended = !(alive && volDepthOk(g, P));
            const uint32_t key0 = rng.key, sample0 = rng.sample;
            vlookups += rng.lookups - l0;
            // the path's state goes out first, so it holds no registers across the walks (inline below)
            if (!ended) {
                storePath(w, slot, P, rng);
                toF = P.medium >= 0;
                toS = !toF;
                if (toF && nf.keys) key = flightKey(v, P.medium, P.o, P.d);
                if (toS) cheap = cheapSurface(sc, v, P.its.valid, P.its.tri);
            } else {
                volEnd(v, slot, P, rng, lookups);
            }
            if (df.hit || df.nee) {
                if (NEE_STAGE) {  // the record is in the slot's VolWave entries; k_vnee walks it after this launch
                    w.nflags[slot] = make_uint4(deferFlags(df, ended), key0, sample0, 0u);
                    toN = true;
                } else {  // inline: the walks, then their adds into the stored radiance (the same order and sums)
                    float Th, Tn;
                    uint32_t wl = 0;
                    walkDeferred(sc, v, df, key0, sample0, stk, segs, wl, Th, Tn);
                    lookups += wl;
                    vlookups += wl;
                    float4 *dst = ended ? v.rad + slot : w.L + slot;
                    const float4 l4 = *dst;
                    f3 L = xyz(l4);
                    addDeferred(v, df, Th, Tn, slot, L);
                    *dst = f4(L, l4.w);
                }
            }
        }
        flightAppend(toF, slot, key, nf, sh);
        surfAppend(toS, cheap, slot, ns, nd, sh);
        if (NEE_STAGE) waveAppend(toN, slot, qn.items + (size_t)sh * qn.stride, qn.counts + sh);
    }
    volStats(v, segs, shadows, lookups);
    volStageStats(v, 5, vertices, vlookups);
}

// the interactions' deferred transmittance walks (VDefer, stored per slot by k_vvertex): the emitter hit's
// walk, then the NEE's shadow walk, each on its sub-stream, their contributions into the path's L (or, for
// a path that ended at that interaction, its output radiance) and the NEE into its vertex's snapshot
#ifndef PG_VNEE_WAVES
#define PG_VNEE_WAVES 3
#endif
template <bool GUIDED>
__global__ __launch_bounds__(TRACE_BLOCK, PG_VNEE_WAVES) void k_vnee(GParams g, SceneDev sc, VolDev v, VolWave w, Queue qn) {
    __shared__ uint32_t stack[LDS_STACK * TRACE_BLOCK];
    const TStack stk = threadStack(stack, v.stack_ovf);
    const uint32_t sh = blockIdx.x & (PG_QSHARDS - 1), rows = gridDim.x / PG_QSHARDS;
    const uint32_t n = qn.counts[sh];
    uint32_t segs = 0, walks = 0, lookups = 0;
    for (uint32_t i = (blockIdx.x / PG_QSHARDS) * TRACE_BLOCK + threadIdx.x; i < n; i += rows * TRACE_BLOCK) {
        const uint32_t slot = qn.items[(size_t)sh * qn.stride + i];
        bool ended;
        VDefer df;
        uint32_t key, sample;
        loadDefer(w, slot, df, ended, key, sample);
        float4 *dst = ended ? v.rad + slot : w.L + slot;
        const float4 l4 = *dst;
        f3 L = xyz(l4);
        resolveDeferred(sc, v, df, key, sample, slot, L, stk, segs, lookups);
        *dst = f4(L, l4.w);
        walks++;
    }
    volStats(v, segs, 0, lookups);
    volStageStats(v, 7, walks, lookups);
}

// the chunk's last paths: each thread runs one to its end (paths of `qf` start with their flight, those
// of `qs` with their surface interaction)
#ifndef PG_VTAIL_WAVES
#define PG_VTAIL_WAVES 3  // C5 442.3 / 441.9 against 439.2 / 439.6 at 2 (profiles/r05q_vol_waves/)
#endif
template <bool GUIDED, int MODELS>
__global__ __launch_bounds__(TRACE_BLOCK, PG_VTAIL_WAVES) void k_vtail(GParams g, SceneDev sc, VolDev v, SDDev sd,
                                                                     VolWave w, Queue qf, Queue qs, Queue qd,
                                                                     uint32_t fblocks, uint32_t dblocks) {
    __shared__ uint32_t stack[LDS_STACK * TRACE_BLOCK];
    const TStack stk = threadStack(stack, v.stack_ovf);
    // blocks [0, fblocks): flights; [fblocks, fblocks + dblocks): delta surfaces; the rest: surfaces
    const bool flight = blockIdx.x < fblocks, delta = !flight && blockIdx.x < fblocks + dblocks;
    const uint32_t b = flight ? blockIdx.x : (delta ? blockIdx.x - fblocks : blockIdx.x - fblocks - dblocks);
    const uint32_t nb = flight ? fblocks : (delta ? dblocks : gridDim.x - fblocks - dblocks);
    const Queue &q = flight ? qf : (delta ? qd : qs);
    const uint32_t sh = b & (PG_QSHARDS - 1), rows = nb / PG_QSHARDS;
    const uint32_t n = q.counts[sh];
    uint32_t segs = 0, shadows = 0, lookups = 0;
    for (uint32_t i = (b / PG_QSHARDS) * TRACE_BLOCK + threadIdx.x; i < n; i += rows * TRACE_BLOCK) {
        const uint32_t slot = q.items[(size_t)sh * q.stride + i];
        VPath P;
        VRng rng;
        loadPath(w, slot, P, rng);
        bool alive = flight;
        if (!flight) {
            VDefer df;
            clearDefer(df);
            alive = volSurface<GUIDED, false, MODELS>(g, sc, v, sd, P, rng, stk, slot, segs, shadows, df, w);
            if (df.hit || df.nee) resolveDeferred(sc, v, df, rng.key, rng.sample, slot, P.L, stk, segs, rng.lookups);
        }
        while (alive) alive = volStepResolved<GUIDED, MODELS>(g, sc, v, sd, P, rng, stk, slot, segs, shadows);
        volEnd(v, slot, P, rng, lookups);
    }
    volStats(v, segs, shadows, lookups);
}

namespace {
static inline uint32_t vrows(uint32_t max_shard, uint32_t cap) {
    const uint32_t r = (max_shard + TRACE_BLOCK - 1) / TRACE_BLOCK;
    return r < cap ? r : cap;
}
}  // namespace

void pg_launch_vol_camera(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const VolWave &w,
                          const uint32_t *local_pixels, uint32_t pix_begin, uint32_t npix, uint32_t nlayers,
                          uint32_t sample_base, Queue flight, Queue surf, Queue dsurf) {
    const uint64_t n = (uint64_t)npix * nlayers;
    if (!n) return;
    const uint64_t want = (n + TRACE_BLOCK - 1) / TRACE_BLOCK;
    const dim3 grid((uint32_t)(want < TRACE_MAX_BLOCKS ? want : TRACE_MAX_BLOCKS));  // the overflow ring's size
    if (g.guiding)
        hipLaunchKernelGGL(k_vcam<true>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, w, local_pixels, pix_begin, npix,
                           nlayers, sample_base, flight, surf, dsurf);
    else
        hipLaunchKernelGGL(k_vcam<false>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, w, local_pixels, pix_begin, npix,
                           nlayers, sample_base, flight, surf, dsurf);
}
void pg_launch_vol_flight(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                          const VolWave &w, Queue flight, uint32_t max_flight, Queue med, Queue surf, Queue dsurf) {
    if (!max_flight) return;
    const dim3 grid(PG_QSHARDS * vrows(max_flight, TRACE_MAX_BLOCKS / PG_QSHARDS));
    if (g.guiding)
        hipLaunchKernelGGL(k_vflight<true>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, sd, w, flight, med, surf, dsurf);
    else
        hipLaunchKernelGGL(k_vflight<false>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, sd, w, flight, med, surf, dsurf);
}
int pg_launch_vol_vertex(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                         const VolWave &w, Queue med, uint32_t max_med, Queue surf, uint32_t max_surf, Queue dsurf,
                         uint32_t max_dsurf, Queue next_flight, Queue next_surf, Queue next_dsurf, const Queue *nee) {
    // the three block ranges within TRACE_MAX_BLOCKS (the traversal stacks' overflow ring)
    const uint32_t cap = TRACE_MAX_BLOCKS / PG_QSHARDS / 4;
    const uint32_t mr = max_med ? vrows(max_med, cap) : 0;
    const uint32_t sr = max_surf ? vrows(max_surf, cap) : 0;
    const uint32_t dr = max_dsurf ? vrows(max_dsurf, cap) : 0;
    if (mr + sr + dr == 0) return 0;
    const Queue qn = nee ? *nee : Queue{};
    // medium and surface interactions as two launches (each its own register budget: the medium launch at
    // 3 waves/SIMD, PG_VMEDIUM_INLINE_WAVES / PG_VMEDIUM_WAVES), or one (PG_VOL_SPLIT_VERTEX=0; read per
    // launch: tests switch it within a process).  With the walks inline and the path state stored before
    // them: C5 405.2 / 404.6 split against 392.3 / 393.2 one launch (profiles/r05o_vol_vertex_split/)
    const char *se = std::getenv("PG_VOL_SPLIT_VERTEX");
    const bool split = se && *se ? std::atoi(se) != 0 : true;
#define PG_VV(GU, NS, KIND, ROWS, MB)                                                                                \
    hipLaunchKernelGGL((k_vvertex<GU, NS, KIND>), dim3(PG_QSHARDS * (ROWS)), dim3(TRACE_BLOCK), 0, s, g, sc, v, sd, w, \
                       med, surf, dsurf, MB, PG_QSHARDS * dr, next_flight, next_surf, next_dsurf, qn)
#define PG_VV_ALL(GU, NS)                                                                                            \
    if (!split) {                                                                                                    \
        PG_VV(GU, NS, 2, mr + dr + sr, PG_QSHARDS * mr);                                                             \
    } else {                                                                                                         \
        if (mr) PG_VV(GU, NS, 0, mr, PG_QSHARDS * mr);                                                               \
        if (dr + sr && v.models) PG_VV(GU, NS, 3, dr + sr, 0u);                                                      \
        else if (dr + sr) PG_VV(GU, NS, 1, dr + sr, 0u);                                                             \
    }
    if (g.guiding) {
        if (nee) { PG_VV_ALL(true, true) } else { PG_VV_ALL(true, false) }
    } else {
        if (nee) { PG_VV_ALL(false, true) } else { PG_VV_ALL(false, false) }
    }
#undef PG_VV_ALL
#undef PG_VV
    return split ? (mr ? 1 : 0) + (dr + sr ? 1 : 0) : 1;  // kernels launched (bench.py's per-launch averages)
}
void pg_launch_vol_nee(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const VolWave &w, Queue nee,
                       uint32_t max_nee) {
    if (!max_nee) return;
    const dim3 grid(PG_QSHARDS * vrows(max_nee, TRACE_MAX_BLOCKS / PG_QSHARDS));
    if (g.guiding)
        hipLaunchKernelGGL(k_vnee<true>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, w, nee);
    else
        hipLaunchKernelGGL(k_vnee<false>, grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, w, nee);
}
void pg_launch_vol_tail(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                        const VolWave &w, Queue flight, uint32_t max_flight, Queue surf, uint32_t max_surf, Queue dsurf,
                        uint32_t max_dsurf) {
    const uint32_t cap = TRACE_MAX_BLOCKS / PG_QSHARDS / 4;
    const uint32_t fr = max_flight ? vrows(max_flight, cap) : 0;
    const uint32_t sr = max_surf ? vrows(max_surf, cap) : 0;
    const uint32_t dr = max_dsurf ? vrows(max_dsurf, cap) : 0;
    if (fr + sr + dr == 0) return;
    const dim3 grid(PG_QSHARDS * (fr + dr + sr));
#define PG_VT(GU, MO)                                                                                                \
    hipLaunchKernelGGL((k_vtail<GU, MO>), grid, dim3(TRACE_BLOCK), 0, s, g, sc, v, sd, w, flight, surf, dsurf,      \
                       PG_QSHARDS * fr, PG_QSHARDS * dr)
    if (g.guiding) {
        if (v.models) PG_VT(true, PG_MODELS_DIFFUSE_NULL); else PG_VT(true, -1);
    } else {
        if (v.models) PG_VT(false, PG_MODELS_DIFFUSE_NULL); else PG_VT(false, -1);
    }
#undef PG_VT
}

namespace {
}  // namespace

template <bool GUIDED>
__global__ __launch_bounds__(VOL_BLOCK, PG_VOL_WAVES) void k_volpath(GParams g, SceneDev sc, VolDev v, SDDev sd,
                                                       const uint32_t *__restrict__ local_pixels, uint32_t pix_begin,
                                                       uint32_t npix, uint32_t nlayers, uint32_t sample_base) {
    __shared__ uint32_t stack[LDS_STACK * TRACE_BLOCK];
    const TStack stk = threadStack(stack, v.stack_ovf);
    const uint32_t nitems = npix * nlayers;
    const int lane = threadIdx.x & 63;
    uint32_t segs = 0, shadows = 0, lookups = 0;
    bool alive = false, done = false;
    uint32_t item = 0;
    VPath P;
    VRng rng{0, 0, 0, 0};
    for (;;) {
        // refill finished lanes from the work counter (one atomic per wave); with refill_min > 1 a wave
        // waits until that many lanes are idle (or none is alive), so the lanes it restarts together
        // run their camera rays and first hits in one pass instead of one refill per finished path
        const unsigned long long need = __ballot(!alive && !done);
        if (need && (__popcll(need) >= v.refill_min || !__any(alive))) {
            const int leader = __ffsll((long long)need) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(v.next, (uint32_t)__popcll(need));
            base = __shfl(base, leader);
            if (!alive && !done) {
                item = base + (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
                if (item >= nitems) {
                    done = true;
                } else {
                    volCamera(g, sc, v, local_pixels, pix_begin, npix, sample_base, item, P, rng, stk, segs);
                    alive = true;
                }
            }
        }
        if (!__any(alive)) break;
        if (alive && !volStepResolved<GUIDED>(g, sc, v, sd, P, rng, stk, item, segs, shadows)) {
#if PG_VOL_CHECK
            if (VCHK(item < nitems, 3, item))
#endif
            v.rad[item] = f4(P.L, __uint_as_float(P.nv));  // .w: training vertices (k_commit)
            lookups += rng.lookups;
            alive = false;
        }
    }
    // statistics: wave sums, one atomic per wave
    unsigned long long s0 = segs, s1 = shadows, s2 = lookups;
    for (int off = 32; off > 0; off >>= 1) {
        s0 += __shfl_xor(s0, off);
        s1 += __shfl_xor(s1, off);
        s2 += __shfl_xor(s2, off);
    }
    if (lane == 0) {
        atomicAdd(v.stats, s0);
        atomicAdd(v.stats + 1, s1);
        atomicAdd(v.stats + 2, s2);
    }
}

// corner-packed density (pg_layout.h): one thread per cell, 8 gathers -> two 16-B stores
__global__ __launch_bounds__(256) void k_density_corners(const float *__restrict__ lin, uint32_t rx, uint32_t ry,
                                                        uint32_t rz, float4 *__restrict__ out) {
    const size_t cx = rx - 1, cy = ry - 1, n = cx * cy * (size_t)(rz - 1);
    const size_t cell = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= n) return;
    const size_t x = cell % cx, y = (cell / cx) % cy, z = cell / (cx * cy);
    const size_t sy = rx, sz = (size_t)rx * ry;
    const float *b = lin + z * sz + y * sy + x;
    out[2 * cell] = make_float4(b[0], b[1], b[sy], b[sy + 1]);
    out[2 * cell + 1] = make_float4(b[sz], b[sz + 1], b[sz + sy], b[sz + sy + 1]);
}
void pg_launch_density_corners(hipStream_t s, const float *lin, uint32_t rx, uint32_t ry, uint32_t rz, float *out) {
    const size_t n = (size_t)(rx - 1) * (ry - 1) * (rz - 1);
    if (!n) return;
    hipLaunchKernelGGL(k_density_corners, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, lin, rx, ry, rz,
                       reinterpret_cast<float4 *>(out));
}

// ---- unit-level queries (pg_phase_query / pg_medium_query) --------------------------------------
__global__ __launch_bounds__(256) void k_phase_query(const GMedium *medium, const float *in, const float *wog,
                                                     uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float *a = in + 5 * (size_t)i;
    const f3 wi = mk(a[0], a[1], a[2]);
    const float g = medium->g;
    float pdf;
    const f3 wo = hgSample(g, wi, a[3], a[4], pdf);
    float *o = out + 5 * (size_t)i;
    o[0] = wo.x;
    o[1] = wo.y;
    o[2] = wo.z;
    o[3] = pdf;
    o[4] = wog ? hgEval(g, wi, mk(wog[3 * i], wog[3 * i + 1], wog[3 * i + 2])) : 0.0f;
}
__global__ __launch_bounds__(256) void k_medium_query(const GMedium *medium, int op, const float *in,
                                                      const uint32_t *keys, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const MedView M = medView(medium, 0);
    if (op == 0) {
        out[i] = lookupDensity(M, mk(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
        return;
    }
    const float *r = in + 8 * (size_t)i;
    VRng rng{keys[2 * i], keys[2 * i + 1], 1, 0};
    const f3 o = mk(r[0], r[1], r[2]), d = mk(r[4], r[5], r[6]);
    float *q = out + 4 * (size_t)i;
    const bool grid = op >= 3, trans = op == 2 || op == 4;
    float t0, t1;
    const bool overlap = medClip(M, o, d, r[3], r[7], t0, t1);
    // one tracking run over [t0, t1] with the explicit mint (the integrator always passes 0)
    auto run = [&](float &tHit) -> bool {
        if (grid) return t0 < t1 && trackGrid(M, o, d, t0, t1, rng, tHit);
        float t = t0;
        for (;;) {
            t -= trackLog(1 - rng.next1()) * M.invMax;
            if (!(t < t1)) return false;
            const float density = lookupDensity(M, o + d * t) * M.scale;
            if (density * M.invMax > rng.next1()) {
                tHit = t;
                return true;
            }
        }
    };
    float t = 0;
    if (!trans) {
        const bool ok = overlap && run(t);
        q[0] = ok ? 1.0f : 0.0f;
        q[1] = ok ? t : 0.0f;
        q[2] = (float)(rng.dim - 1);
        q[3] = 0;
    } else {
        float tr = 1.0f;
        if (overlap && !(grid && !(t0 < t1))) {
            float result = 0;
            for (int k = 0; k < 2; ++k)
                if (!run(t)) result += 1;
            tr = result * 0.5f;
        }
        q[0] = tr;
        q[1] = (float)(rng.dim - 1);
        q[2] = q[3] = 0;
    }
}

void pg_launch_phase_query(hipStream_t s, const GMedium *medium, const float *in, const float *wog, uint32_t n,
                           float *out) {
    if (!n) return;
    hipLaunchKernelGGL(k_phase_query, dim3((n + 255) / 256), dim3(256), 0, s, medium, in, wog, n, out);
}
void pg_launch_medium_query(hipStream_t s, const GMedium *medium, int op, const float *in, const uint32_t *keys,
                            uint32_t n, float *out) {
    if (!n) return;
    hipLaunchKernelGGL(k_medium_query, dim3((n + 255) / 256), dim3(256), 0, s, medium, op, in, keys, n, out);
}

void pg_launch_volpath(hipStream_t s, const GParams &g, const SceneDev &sc, const VolDev &v, const SDDev &sd,
                       const uint32_t *local_pixels, uint32_t pix_begin, uint32_t npix, uint32_t nlayers,
                       uint32_t sample_base) {
    const uint64_t n = (uint64_t)npix * nlayers;
    if (!n) return;
    (void)hipMemsetAsync(v.next, 0, sizeof(uint32_t), s);
    const uint64_t want = (n + VOL_BLOCK - 1) / VOL_BLOCK;
    const uint32_t grid = (uint32_t)(want < TRACE_MAX_BLOCKS ? want : TRACE_MAX_BLOCKS);
    if (g.guiding)
        hipLaunchKernelGGL(k_volpath<true>, dim3(grid), dim3(VOL_BLOCK), 0, s, g, sc, v, sd, local_pixels, pix_begin,
                           npix, nlayers, sample_base);
    else
        hipLaunchKernelGGL(k_volpath<false>, dim3(grid), dim3(VOL_BLOCK), 0, s, g, sc, v, sd, local_pixels, pix_begin,
                           npix, nlayers, sample_base);
}
