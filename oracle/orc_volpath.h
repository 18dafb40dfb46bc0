// ORACLE — test infrastructure only.  CPU restatement of the reference's volumetric path tracer:
//   ProgressiveVolumetricPathTracer::Li             src/integrators/path/progressive_volpath.cpp:98-374
//   ...::rayIntersectAndLookForEmitter              progressive_volpath.cpp:401-460
//   Scene::evalTransmittance                        src/librender/scene.cpp:662-720
//   Scene::sampleAttenuatedEmitterDirect (medium / surface)   scene.cpp:897-940
//   Shape::getTargetMedium / isMediumTransition     include/mitsuba/render/shape.h, records.inl
//   DirectSamplingRecord(its / mRec), setQuery      include/mitsuba/render/records.inl:159-178
// with MTS_IGNORE_NULLBSDF_INTERSECTIONS on (a null crossing counts as a bounce), no environment
// emitter, and the HG phase function (orc_medium.h).
//
// `lazy` (default, and what the GPU kernel does): rayIntersectAndLookForEmitter estimates the
// transmittance of the segments it walks only when the walk ends on an emitter.  The reference
// estimates it on every walk and discards it otherwise; both give the same estimator (each
// segment's estimate is independent of where the walk ends), lazy just skips the discarded work.
// tests/test_volume.py compares the two renders.
#pragma once
#include <vector>

#include "orc_scene.h"

namespace orc {

inline float miWeightV(float a, float b) {
    a *= a;
    b *= b;
    return a / (a + b);
}

inline bool isMediumTransition(const pg_shape &sh) { return sh.interior_medium >= 0 || sh.exterior_medium >= 0; }
// Intersection::getTargetMedium(d): exterior when d leaves through the normal's side
inline int targetMedium(const pg_shape &sh, V3 d, V3 n) { return dot(d, n) > 0 ? sh.exterior_medium : sh.interior_medium; }

inline V3 rawFaceNormal(const Scene &S, uint32_t prim) {
    V3 p0 = S.pos[S.idx[3 * prim]], p1 = S.pos[S.idx[3 * prim + 1]], p2 = S.pos[S.idx[3 * prim + 2]];
    return normalize(cross(p1 - p0, p2 - p0));
}

struct VolCounters {
    uint64_t segments = 0, shadow = 0;
};

// Scene::evalTransmittance: transmittance from p1 to p2 through null surfaces and media; any
// other surface, more than maxInteractions crossings, or a medium inconsistency gives zero
inline float sceneTransmittance(const Scene &S, V3 p1, bool p1OnSurface, V3 p2, bool p2OnSurface, int medium,
                                int maxInteractions, SeqRng &rng, bool grid) {
    V3 d = p2 - p1;
    float remaining = length(d);
    d = d / remaining;
    const float lengthFactor = p2OnSurface ? (1 - kShadowEpsilon) : 1;
    Ray ray{p1, d, p1OnSurface ? kEpsilon : 0.0f, remaining * lengthFactor};
    float T = 1.0f;
    int interactions = 0;
    while (remaining > 0) {
        float t;
        uint32_t prim = 0;
        const bool surface = S.intersectRaw(ray, t, prim);
        const pg_shape *sh = surface ? &S.shapes[S.triShape[prim]] : nullptr;
        if (surface && (interactions == maxInteractions || !(S.mats[sh->material].type & ENull))) return 0.0f;
        if (medium >= 0) T *= S.media[medium].transmittance(grid, ray.o, ray.d, 0.0f, std::min(t, remaining), rng);
        if (!surface || T == 0) break;
        // null BSDF in the discrete measure: 1
        if (isMediumTransition(*sh)) {
            const V3 n = rawFaceNormal(S, prim);
            if (medium != targetMedium(*sh, -d, n)) return 0.0f;
            medium = targetMedium(*sh, d, n);
        }
        if (++interactions > 100) break;
        ray.o = ray.o + ray.d * t;
        remaining -= t;
        ray.maxt = remaining * lengthFactor;
        ray.mint = kEpsilon;
    }
    return T;
}

struct EmitterQuery {
    V3 value;         // attenuated emitted radiance (0: none)
    V3 n, d;          // setQuery: emitter shading normal, last segment direction
    float dist = 0;   // setQuery: length of the LAST segment (the reference's dRec.dist)
    int emitter = -1;
};

// rayIntersectAndLookForEmitter: `its` receives the FIRST intersection; the walk continues through
// null surfaces (updating the medium) to find an emitter behind them
inline void lookForEmitter(const Scene &S, SeqRng &rng, int medium, int maxInteractions, Ray ray, Its &its,
                           EmitterQuery &q, bool lazy, bool grid, VolCounters &cnt) {
    q.value = V3(0.f);
    q.emitter = -1;
    Its its2;
    Its *cur = &its;
    float T = 1.0f;
    bool surface = false;
    int interactions = 0;
    struct Seg {
        V3 o;
        float maxt;
        int medium;
    };
    std::vector<Seg> segs;
    for (;;) {
        surface = S.intersect(ray, *cur);
        cnt.segments++;
        const float segT = surface ? cur->t : kInf;
        if (medium >= 0) {
            if (lazy) segs.push_back({ray.o, segT, medium});
            else T *= S.media[medium].transmittance(grid, ray.o, ray.d, 0.0f, segT, rng);
        }
        if (!surface) break;
        const pg_shape &sh = S.shapes[cur->shape];
        if (interactions == maxInteractions || !(S.mats[sh.material].type & ENull) || sh.emitter >= 0) break;
        if (!lazy && T == 0) return;
        if (isMediumTransition(sh)) medium = targetMedium(sh, ray.d, cur->geoN);
        ray.o = ray.o + ray.d * cur->t;
        ray.mint = kEpsilon;
        cur = &its2;
        if (++interactions > 100) return;
    }
    if (!surface) return;  // no environment emitter
    const pg_shape &sh = S.shapes[cur->shape];
    if (sh.emitter < 0) return;
    V3 Le = emitterLe(S, *cur, -ray.d);
    if (lazy && !isZero(Le)) {
        for (const Seg &s : segs) {
            T *= S.media[s.medium].transmittance(grid, s.o, ray.d, 0.0f, s.maxt, rng);
            if (T == 0) break;
        }
    }
    q.value = Le * T;
    q.n = cur->sh.n;
    q.d = ray.d;
    q.dist = cur->t;
    q.emitter = sh.emitter;
}

inline V3 VolLi(const Scene &S, const pg_config &cfg, SeqRng &rng, Ray ray, VolCounters &cnt, bool lazy) {
    const int maxDepth = cfg.max_depth;
    const bool grid = cfg.volume_majorant == PG_MAJORANT_GRID;
    Its its;
    if (!S.intersect(ray, its)) its.t = kInf;
    cnt.segments++;
    int medium = S.camMedium;
    V3 L(0.f), T(1.f);
    float eta = 1.0f;
    bool scattered = false;
    bool emission = true;  // RadianceQueryRecord::ERadiance; ERadianceNoEmission after a scattering event
    int depth = 1;
    auto maxInter = [&](int dep) { return maxDepth - dep - 1; };

    while (depth <= maxDepth || maxDepth < 0) {
        float mt = 0;
        V3 mp;
        const bool inMedium =
            medium >= 0 && S.media[medium].sample(grid, ray.o, ray.d, 0.0f, its.valid ? its.t : kInf, rng, mt, mp);
        if (inMedium) {
            // ---- medium interaction (progressive_volpath.cpp:117-196)
            const Medium &M = S.media[medium];
            if (depth >= maxDepth && maxDepth != -1) break;
            T *= M.albedo;  // sigmaS * transmittance / pdfSuccess = albedo * density / density
            const V3 wi = -ray.d;
            if (cfg.use_nee) {
                float s0, s1;
                rng.next2(s0, s1);
                DirectRec dr;
                dr.ref = mp;
                dr.refN = V3(0.f);
                V3 value = sampleEmitterNoVis(S, dr, s0, s1);
                if (dr.pdf != 0) {
                    cnt.shadow++;
                    value = value * sceneTransmittance(S, mp, false, dr.p, true, medium, maxInter(depth), rng, grid);
                    if (!isZero(value)) {
                        const float phaseVal = hgEval(M.g, wi, dr.d);
                        if (phaseVal != 0) L += T * value * (phaseVal * miWeightV(dr.pdf, phaseVal));
                    }
                }
            }
            float u0, u1, phasePdf;
            rng.next2(u0, u1);
            const V3 wo = hgSample(M.g, wi, u0, u1, phasePdf);
            ray = Ray{mp, wo, 0.0f, kInf};
            EmitterQuery q;
            lookForEmitter(S, rng, medium, maxInter(depth), ray, its, q, lazy, grid, cnt);
            if (!its.valid) its.t = kInf;
            if (!isZero(q.value) && std::min(q.value.x, std::min(q.value.y, q.value.z)) > 0.f) {
                const float emitterPdf = cfg.use_nee ? pdfEmitterDirect(S, q.emitter, V3(0.f), q.d, q.n, q.dist) : 0.0f;
                const float w = cfg.use_nee ? miWeightV(phasePdf, emitterPdf) : 1.0f;
                L += T * q.value * w;
            }
            emission = false;
        } else {
            // ---- surface interaction (progressive_volpath.cpp:197-352)
            if (!its.valid) break;  // no environment emitter
            const pg_shape &sh = S.shapes[its.shape];
            const Material &Mt = S.mats[sh.material];
            if (sh.emitter >= 0 && emission && (!cfg.hide_emitters || scattered)) L += T * emitterLe(S, its, -ray.d);
            if (depth >= maxDepth && maxDepth != -1) break;
            if (cfg.strict_normals && -dot(its.geoN, ray.d) * its.wi.z < 0) break;
            const V3 refN = (Mt.type & (ETransmission | EBackSide)) == 0 ? its.sh.n : V3(0.f);
            if (cfg.use_nee && (Mt.type & ESmooth)) {
                float s0, s1;
                rng.next2(s0, s1);
                DirectRec dr;
                dr.ref = its.p;
                dr.refN = refN;
                V3 value = sampleEmitterNoVis(S, dr, s0, s1);
                if (dr.pdf != 0) {
                    const int med = isMediumTransition(sh) ? targetMedium(sh, dr.d, its.geoN) : medium;
                    cnt.shadow++;
                    value = value * sceneTransmittance(S, its.p, true, dr.p, true, med, maxInter(depth), rng, grid);
                    if (!isZero(value)) {
                        const V3 woL = its.toLocal(dr.d);
                        const V3 bsdfVal = bsdfEval(Mt, its.wi, woL);
                        if (!isZero(bsdfVal) && (!cfg.strict_normals || dot(its.geoN, dr.d) * woL.z > 0)) {
                            const float bp = bsdfPdf(Mt, its.wi, woL);
                            L += T * value * bsdfVal * miWeightV(dr.pdf, bp);
                        }
                    }
                }
            }
            float b0, b1;
            rng.next2(b0, b1);
            const float b2 = rng.next1();
            BSample bs;
            const V3 weight = bsdfSample(Mt, its.wi, b0, b1, b2, bs);
            if (isZero(weight)) break;
            const V3 wo = its.toWorld(bs.wo);
            if (cfg.strict_normals && dot(its.geoN, wo) * bs.wo.z <= 0) break;
            const V3 itsP = its.p, itsGeoN = its.geoN;
            ray = Ray{itsP, wo, kEpsilon, kInf};
            T *= weight;
            eta *= bs.eta;
            if (isMediumTransition(sh)) medium = targetMedium(sh, wo, itsGeoN);
            if (bs.sampledType == ENull) {  // index-matched boundary: continue straight through
                emission = !scattered;
                if (!S.intersect(ray, its)) its.t = kInf;
                cnt.segments++;
                depth++;
                continue;
            }
            EmitterQuery q;
            lookForEmitter(S, rng, medium, maxInter(depth), ray, its, q, lazy, grid, cnt);
            if (!its.valid) its.t = kInf;
            if (!isZero(q.value)) {
                const float emitterPdf = (cfg.use_nee && !(bs.sampledType & EDelta))
                                             ? pdfEmitterDirect(S, q.emitter, refN, q.d, q.n, q.dist)
                                             : 0.0f;
                const float w = cfg.use_nee ? miWeightV(bs.pdf, emitterPdf) : 1.0f;
                L += T * q.value * w;
            }
            emission = false;
        }
        if (depth++ >= cfg.rr_depth) {
            const float qq = std::min(maxc(T) * eta * eta, 0.95f);
            if (rng.next1() >= qq) break;
            T /= qq;
        }
        scattered = true;
    }
    return L;
}

}  // namespace orc
