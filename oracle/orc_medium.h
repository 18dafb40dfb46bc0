// ORACLE — test infrastructure only.  CPU restatement of the reference's participating medium:
//   GridDataSource::lookupFloat (trilinear, data AABB -> [0, res-1]^3)  src/volume/gridvolume.cpp:186-198,337-380
//   GridDataSource::getMaximumFloatValue (= 1)                          src/volume/gridvolume.cpp:583-585
//   HeterogeneousMedium::configure (maxDensity = scale * 1)              src/medium/heterogeneous.cpp:227-242
//   HeterogeneousMedium::sampleDistance, Woodcock tracking               src/medium/heterogeneous.cpp:589-660
//   HeterogeneousMedium::evalTransmittance, 2 delta-tracking runs        src/medium/heterogeneous.cpp:546-587
//   HGPhaseFunction::sample / eval                                       src/phase/hg.cpp:74-110
//   Frame(n) via coordinateSystem                                        include/mitsuba/core/frame.h:55, src/libcore/util.cpp:594-603
// Random numbers: one sequential counter stream per path (SeqRng below) in place of the
// reference's per-pixel sampler; the i-th next1D/next2D of a path reads dimension i.
#pragma once
#include <limits>
#include <vector>

#include "orc_math.h"

namespace orc {

// Sampler::next1D / next2D over the shared counter RNG (dimension 0 is the pixel jitter)
struct SeqRng {
    Rng r;
    uint32_t dim = 1;
    float next1() { return r.next1(dim++); }
    void next2(float &a, float &b) { r.next2(dim++, a, b); }
};

// Frame(n): s = cross(c, n), t = c with c from coordinateSystem (util.cpp:594-603)
inline Frame frameFromN(V3 a) {
    Frame f;
    f.n = a;
    V3 c;
    if (std::fabs(a.x) > std::fabs(a.y)) {
        float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = V3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = V3(0.0f, a.z * invLen, -a.y * invLen);
    }
    f.t = c;
    f.s = cross(c, a);
    return f;
}

// HGPhaseFunction::eval (hg.cpp:103-106); wi points back along the incident ray
inline float hgEval(float g, V3 wi, V3 wo) {
    float temp = 1.0f + g * g + 2.0f * g * dot(wi, wo);
    return kInvFourPi * (1 - g * g) / (temp * std::sqrt(temp));
}

// HGPhaseFunction::sample (hg.cpp:74-95): wo around -wi; returns the pdf (= eval), weight 1
inline V3 hgSample(float g, V3 wi, float sx, float sy, float &pdf) {
    float cosTheta;
    if (std::fabs(g) < kEpsilon) {
        cosTheta = 1 - 2 * sx;
    } else {
        float sqrTerm = (1 - g * g) / (1 - g + 2 * g * sx);
        cosTheta = (1 + g * g - sqrTerm * sqrTerm) / (2 * g);
    }
    float sinTheta = safe_sqrt(1.0f - cosTheta * cosTheta);
    float phi = 2 * kPi * sy;
    V3 wo = frameFromN(-wi).toWorld(V3(sinTheta * std::cos(phi), sinTheta * std::sin(phi), cosTheta));
    pdf = hgEval(g, wi, wo);
    return wo;
}

struct Medium {
    uint32_t res[3] = {0, 0, 0};
    std::vector<float> data;  // x fastest
    V3 lo, hi;                // data AABB = the medium's density AABB
    float gs[3] = {0, 0, 0};  // world -> grid: g = p * gs + go  (Transform::scale * translate)
    float go[3] = {0, 0, 0};
    float scale = 1, invMax = 1;
    V3 albedo;
    float g = 0.8f;
    // majorant grid (pg_config.volume_majorant = PG_MAJORANT_GRID): cell (cx, cy, cz) covers grid
    // coordinates [c * kCell, (c + 1) * kCell) per axis; its majorant is scale * the maximum voxel
    // over [c * kCell - 1, (c + 1) * kCell + 1] (every trilinear lookup whose base voxel lies in the
    // cell, with one voxel of margin for the rounding of the traversal's cell boundaries)
#ifndef ORC_MAJORANT_CELL
#define ORC_MAJORANT_CELL 16  // = the kernels' PG_MAJORANT_CELL (ASan runs build other sizes, tools/oracle_asan.sh)
#endif
    static constexpr int kCell = ORC_MAJORANT_CELL;
    int mres[3] = {1, 1, 1};
    std::vector<float> maj;

    void init(const pg_medium &m) {
        for (int a = 0; a < 3; ++a) res[a] = m.res[a];
        data.assign(m.density, m.density + (size_t)res[0] * res[1] * res[2]);
        lo = V3(m.aabb_min[0], m.aabb_min[1], m.aabb_min[2]);
        hi = V3(m.aabb_max[0], m.aabb_max[1], m.aabb_max[2]);
        for (int a = 0; a < 3; ++a) {
            gs[a] = (float)(res[a] - 1) / (hi[a] - lo[a]);
            go[a] = gs[a] * -lo[a];
        }
        scale = m.scale;
        invMax = 1.0f / (m.scale * 1.0f);
        albedo = V3(m.albedo[0], m.albedo[1], m.albedo[2]);
        g = m.g;
        for (int a = 0; a < 3; ++a) mres[a] = std::max(1, ((int)res[a] - 1 + kCell - 1) / kCell);
        maj.assign((size_t)mres[0] * mres[1] * mres[2], 0.0f);
        for (int cz = 0; cz < mres[2]; ++cz)
            for (int cy = 0; cy < mres[1]; ++cy)
                for (int cx = 0; cx < mres[0]; ++cx) {
                    const int c[3] = {cx, cy, cz};
                    int lo3[3], hi3[3];
                    for (int a = 0; a < 3; ++a) {
                        lo3[a] = std::max(0, c[a] * kCell - 1);
                        hi3[a] = std::min((int)res[a] - 1, (c[a] + 1) * kCell + 1);
                    }
                    float mx = 0;
                    for (int z = lo3[2]; z <= hi3[2]; ++z)
                        for (int y = lo3[1]; y <= hi3[1]; ++y)
                            for (int x = lo3[0]; x <= hi3[0]; ++x)
                                mx = std::max(mx, data[((size_t)z * res[1] + y) * res[0] + x]);
                    maj[((size_t)cz * mres[1] + cy) * mres[0] + cx] = mx * scale;
                }
    }

    // lookupFloat: zero unless all 8 corners lie inside the grid
    float lookup(V3 p) const {
        float px = p.x * gs[0] + go[0], py = p.y * gs[1] + go[1], pz = p.z * gs[2] + go[2];
        int x1 = (int)std::floor(px), y1 = (int)std::floor(py), z1 = (int)std::floor(pz);
        int x2 = x1 + 1, y2 = y1 + 1, z2 = z1 + 1;
        if (x1 < 0 || y1 < 0 || z1 < 0 || x2 >= (int)res[0] || y2 >= (int)res[1] || z2 >= (int)res[2]) return 0;
        float fx = px - x1, fy = py - y1, fz = pz - z1, _fx = 1.0f - fx, _fy = 1.0f - fy, _fz = 1.0f - fz;
        auto at = [&](int x, int y, int z) { return data[((size_t)z * res[1] + y) * res[0] + x]; };
        float d000 = at(x1, y1, z1), d001 = at(x2, y1, z1), d010 = at(x1, y2, z1), d011 = at(x2, y2, z1);
        float d100 = at(x1, y1, z2), d101 = at(x2, y1, z2), d110 = at(x1, y2, z2), d111 = at(x2, y2, z2);
        return ((d000 * _fx + d001 * fx) * _fy + (d010 * _fx + d011 * fx) * fy) * _fz +
               ((d100 * _fx + d101 * fx) * _fy + (d110 * _fx + d111 * fx) * fy) * fz;
    }

    // AABB::rayIntersect of the density box, clipped to [mint, maxt]
    bool clip(V3 o, V3 d, float mint, float maxt, float &t0, float &t1) const {
        float nearT = -std::numeric_limits<float>::infinity(), farT = std::numeric_limits<float>::infinity();
        for (int i = 0; i < 3; i++) {
            float oi = o[i], di = d[i], mn = lo[i], mx = hi[i];
            if (di == 0) {
                if (oi < mn || oi > mx) return false;
            } else {
                float a = (mn - oi) / di, b = (mx - oi) / di;
                if (a > b) std::swap(a, b);
                nearT = std::max(a, nearT);
                farT = std::min(b, farT);
                if (!(nearT <= farT)) return false;
            }
        }
        t0 = std::max(nearT, mint);
        t1 = std::min(farT, maxt);
        return true;
    }

    // Woodcock tracking (sampleDistance, method 'woodcock'): true with the interaction point.
    // A sample that reaches maxt fails; a NaN distance also ends the loop (no reference analogue:
    // it can only arise from 1 - u == 0, which the reference's sampler never returns).
    // `accept(p, density, mu, u)` decides a tentative collision at p; the reference's rule is
    // StdAccept (density / mu > u); orc_volpath.h's guided free flight passes a weighted rule.
    template <class Accept>
    bool sampleDistanceA(V3 o, V3 d, float mint, float maxt, SeqRng &rng, float &tOut, V3 &pOut, Accept &&accept) const {
        float t0, t1;
        if (!clip(o, d, mint, maxt, t0, t1)) return false;
        float t = t0;
        for (;;) {
            t -= fastlog(1 - rng.next1()) * invMax;
            if (!(t < t1)) return false;
            V3 p = o + d * t;
            float density = lookup(p) * scale;
            if (accept(p, density, scale, rng.next1())) {
                tOut = t;
                pOut = p;
                return true;
            }
        }
    }
    struct StdAcceptGlobal {  // heterogeneous.cpp:640: density * m_invMaxDensity > sampler->next1D()
        float invMax;
        bool operator()(V3, float density, float, float u) const { return density * invMax > u; }
    };
    struct StdAcceptGrid {
        bool operator()(V3, float density, float mu, float u) const { return density > mu * u; }
    };
    bool sampleDistance(V3 o, V3 d, float mint, float maxt, SeqRng &rng, float &tOut, V3 &pOut) const {
        return sampleDistanceA(o, d, mint, maxt, rng, tOut, pOut, StdAcceptGlobal{invMax});
    }

    // Delta tracking through the majorant grid over [t0, t1] (3D DDA over the cells; in each cell
    // exponential steps at the cell's majorant mu, tentative collisions accepted with probability
    // density / mu; an empty cell is crossed without a draw; a step past the cell's exit restarts at
    // the exit, which the exponential's memorylessness makes exact).  Samples the same collision
    // distribution as the single-majorant loop above with fewer lookups.
    template <class Accept>
    bool trackGridA(V3 o, V3 d, float t0, float t1, SeqRng &rng, float &tHit, Accept &&accept) const {
        const float B = (float)kCell, inf = std::numeric_limits<float>::infinity();
        int c[3], step[3];
        float tNext[3], tDelta[3];
        for (int a = 0; a < 3; ++a) {
            const float og = o[a] * gs[a] + go[a], dg = d[a] * gs[a];
            c[a] = std::min(std::max((int)std::floor((og + dg * t0) / B), 0), mres[a] - 1);
            if (dg > 0) {
                step[a] = 1;
                tNext[a] = ((float)(c[a] + 1) * B - og) / dg;
                tDelta[a] = B / dg;
            } else if (dg < 0) {
                step[a] = -1;
                tNext[a] = ((float)c[a] * B - og) / dg;
                tDelta[a] = -B / dg;
            } else {
                step[a] = 0;
                tNext[a] = inf;
                tDelta[a] = inf;
            }
        }
        float t = t0;
        for (;;) {
            const float tExit = std::min(std::min(tNext[0], tNext[1]), std::min(tNext[2], t1));
            const float mu = maj[((size_t)c[2] * mres[1] + c[1]) * mres[0] + c[0]];
            if (mu > 0) {
                for (;;) {
                    const float ts = t - fastlog(1 - rng.next1()) / mu;
                    if (!(ts < tExit)) break;
                    t = ts;
                    const V3 p = o + d * t;
                    const float density = lookup(p) * scale;
                    if (accept(p, density, mu, rng.next1())) {
                        tHit = t;
                        return true;
                    }
                }
            }
            t = std::max(t, tExit);
            if (!(t < t1)) return false;
            const int a = tNext[0] <= tNext[1] ? (tNext[0] <= tNext[2] ? 0 : 2) : (tNext[1] <= tNext[2] ? 1 : 2);
            c[a] += step[a];
            if (c[a] < 0 || c[a] >= mres[a]) return false;
            tNext[a] += tDelta[a];
        }
    }

    bool trackGrid(V3 o, V3 d, float t0, float t1, SeqRng &rng, float &tHit) const {
        return trackGridA(o, d, t0, t1, rng, tHit, StdAcceptGrid{});
    }
    template <class Accept>
    bool sampleDistanceGridA(V3 o, V3 d, float mint, float maxt, SeqRng &rng, float &tOut, V3 &pOut, Accept &&accept) const {
        float t0, t1;
        if (!clip(o, d, mint, maxt, t0, t1) || !(t0 < t1)) return false;
        if (!trackGridA(o, d, t0, t1, rng, tOut, accept)) return false;
        pOut = o + d * tOut;
        return true;
    }
    bool sampleDistanceGrid(V3 o, V3 d, float mint, float maxt, SeqRng &rng, float &tOut, V3 &pOut) const {
        return sampleDistanceGridA(o, d, mint, maxt, rng, tOut, pOut, StdAcceptGrid{});
    }

    float evalTransmittanceGrid(V3 o, V3 d, float mint, float maxt, SeqRng &rng) const {
        float t0, t1;
        if (!clip(o, d, mint, maxt, t0, t1) || !(t0 < t1)) return 1.0f;
        float result = 0, th;
        for (int i = 0; i < 2; ++i)
            if (!trackGrid(o, d, t0, t1, rng, th)) result += 1;
        return result / 2;
    }

    // dispatch on pg_config.volume_majorant
    bool sample(bool grid, V3 o, V3 d, float mint, float maxt, SeqRng &rng, float &tOut, V3 &pOut) const {
        return grid ? sampleDistanceGrid(o, d, mint, maxt, rng, tOut, pOut) : sampleDistance(o, d, mint, maxt, rng, tOut, pOut);
    }
    float transmittance(bool grid, V3 o, V3 d, float mint, float maxt, SeqRng &rng) const {
        return grid ? evalTransmittanceGrid(o, d, mint, maxt, rng) : evalTransmittance(o, d, mint, maxt, rng);
    }

    // evalTransmittance with a sampler: the mean of 2 delta-tracking survival indicators
    float evalTransmittance(V3 o, V3 d, float mint, float maxt, SeqRng &rng) const {
        float t0, t1;
        if (!clip(o, d, mint, maxt, t0, t1)) return 1.0f;
        const int nSamples = 2;
        float result = 0;
        for (int i = 0; i < nSamples; ++i) {
            float t = t0;
            for (;;) {
                t -= fastlog(1 - rng.next1()) * invMax;
                if (!(t < t1)) {
                    result += 1;
                    break;
                }
                V3 p = o + d * t;
                float density = lookup(p) * scale;
                if (density * invMax > rng.next1()) break;
            }
        }
        return result / nSamples;
    }
};

}  // namespace orc
