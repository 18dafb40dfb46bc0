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
    bool sampleDistance(V3 o, V3 d, float mint, float maxt, SeqRng &rng, float &tOut, V3 &pOut) const {
        float t0, t1;
        if (!clip(o, d, mint, maxt, t0, t1)) return false;
        float t = t0;
        for (;;) {
            t -= std::log(1 - rng.next1()) * invMax;
            if (!(t < t1)) return false;
            V3 p = o + d * t;
            float density = lookup(p) * scale;
            if (density * invMax > rng.next1()) {
                tOut = t;
                pOut = p;
                return true;
            }
        }
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
                t -= std::log(1 - rng.next1()) * invMax;
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
