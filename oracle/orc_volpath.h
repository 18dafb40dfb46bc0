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
#include "orc_sdtree.h"

namespace orc {

inline float miWeightV(float a, float b) {
    a *= a;
    b *= b;
    return a / (a + b);
}

// Transmittance sub-streams (round 5).  Every transmittance estimate an interaction
// makes -- the NEE shadow walk (Scene::evalTransmittance) and the re-walk of a phase/BSDF-sampled ray that
// found a lit emitter through media (rayIntersectAndLookForEmitter) -- draws from a counter sub-stream of
// its own instead of the path's sequential stream: the Philox key key ^ 0x9E3779B9 (2 dim + kind + 1) at
// dimensions 0x80000000 + j, where dim is the main-stream dimension at which the interaction drew its light
// sample (kind 0, NEE) or started its emitter walk (kind 1), and j counts the walk's draws.  Odd-constant
// multiplication is a bijection mod 2^32, so two walks of one path never share a stream (round 6: until
// then dim and kind were bit-packed into the dimension, which aliased from dim = 2^15 or j = 2^15 on), and
// main-stream dimensions stay below 2^31, so no walk draws a main-stream number.  The main stream then does
// not depend on how many numbers a walk used, so the GPU runs the walks as a stage of its own after the
// interactions (pg_volpath.hip k_vnee).  Per interaction the contributions enter L in a fixed order: the
// emitter hit (its product T Le w, then times the walk's transmittance), then the NEE (its product
// T value (f mis), then times the shadow walk's transmittance); the NEE joins the vertex's training
// snapshot, the emitter hit does not (it is radiance along the sampled direction).
inline SeqRng subStream(const SeqRng &rng, uint32_t dim, uint32_t kind) {
    SeqRng s;
    s.r = rng.r;
    s.r.key = rng.r.key ^ (0x9E3779B9u * (2u * dim + kind + 1u));
    s.dim = 0x80000000u;
    return s;
}
// a pending NEE of one interaction: its contribution before the shadow walk's transmittance
struct PendingNee {
    bool valid = false;
    V3 C, p1, p2;
    bool p1OnSurface = false;
    int medium = -1, maxInter = 0;
    uint32_t dim = 0;
};

inline bool isMediumTransition(const pg_shape &sh) { return sh.interior_medium >= 0 || sh.exterior_medium >= 0; }
// Intersection::getTargetMedium(d): exterior when d leaves through the normal's side
inline int targetMedium(const pg_shape &sh, V3 d, V3 n) { return dot(d, n) > 0 ? sh.exterior_medium : sh.interior_medium; }

inline V3 rawFaceNormal(const Scene &S, uint32_t prim) {
    V3 p0 = S.pos[S.idx[3 * prim]], p1 = S.pos[S.idx[3 * prim + 1]], p2 = S.pos[S.idx[3 * prim + 2]];
    return normalize(cross(p1 - p0, p2 - p0));
}

struct VolCounters {
    uint64_t segments = 0, shadow = 0, records = 0;
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
    V3 value;         // emitted radiance of the emitter the walk ended on (0: none), NOT attenuated
    float T = 1.0f;   // the walk's transmittance (its own sub-stream, kind 1)
    V3 n, d;          // setQuery: emitter shading normal, last segment direction
    float dist = 0;   // setQuery: length of the LAST segment (the reference's dRec.dist)
    int emitter = -1;
};

// rayIntersectAndLookForEmitter: `its` receives the FIRST intersection; the walk continues through
// null surfaces (updating the medium) to find an emitter behind them
// exact: q.dist = the whole walk's length (pg_config.volpath_exact_mis; unbiased MIS) instead of the
// reference's last segment
inline void lookForEmitter(const Scene &S, const SeqRng &main, int medium, int maxInteractions, Ray ray, Its &its,
                           EmitterQuery &q, bool lazy, bool grid, VolCounters &cnt, bool exact = false) {
    q.value = V3(0.f);
    q.T = 1.0f;
    q.emitter = -1;
    SeqRng rng = subStream(main, main.dim, 1);
    Its its2;
    Its *cur = &its;
    float T = 1.0f, walked = 0.0f;
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
            else if (T != 0) T *= S.media[medium].transmittance(grid, ray.o, ray.d, 0.0f, segT, rng);  // lazy's draws
        }
        if (!surface) break;
        const pg_shape &sh = S.shapes[cur->shape];
        if (interactions == maxInteractions || !(S.mats[sh.material].type & ENull) || sh.emitter >= 0) break;
        if (isMediumTransition(sh)) medium = targetMedium(sh, ray.d, cur->geoN);
        walked += cur->t;
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
    q.value = Le;
    q.T = T;
    q.n = cur->sh.n;
    q.d = ray.d;
    q.dist = exact ? walked + cur->t : cur->t;
    q.emitter = sh.emitter;
}

// Guided free flight (pg_config.distance_guiding = beta > 0, only with a built SD-tree): weighted
// delta tracking.  At a tentative collision with the reference's real-collision probability
// P_std = sigma_t / mu, the walk takes the collision with P = (1 - beta) P_std + beta P_g and
// multiplies the path weight by P_std / P (collision) or (1 - P_std) / (1 - P) (null collision),
// so every free-flight outcome keeps the reference's expectation.  P_g is the zero-variance ratio
// (Herholz et al. 2019) with the SD-tree's incident radiance standing in for the unknowns.  With
// Lbar the leaf's mean radiance and x = 4 pi p_guide(x, d), continuing gathers sigma_n * x * Lbar;
// scattering gathers sigma_s * Lbar * integral(f_p * 4 pi p_guide), approximated for an HG lobe
// of asymmetry g by the mixture |g| * x + (1 - |g|) (a forward spike plus an isotropic part), so
//   P_g = sigma_s s / (sigma_s s + sigma_n x),  s = |g| x + (1 - |g|).
// Per-step weights lie in [0, 1 / (1 - beta)].  PARITY UNPINNED (absent from the reference).
constexpr float kFourPi = 12.566370614359172f;
struct GuidedAccept {
    const SDTree *tree;
    float beta, albedo, invMax;  // invMax > 0: the global majorant (P_std = density * invMax)
    float gAbs;                  // |g| of the medium's HG phase function
    float cu, cv;                // canonical coordinates of the flight direction
    float w = 1.0f;              // accumulated tracking weight
    bool operator()(V3 p, float density, float mu, float u) {
        float pStd = invMax > 0 ? density * invMax : density / mu;
        pStd = std::min(std::max(pStd, 0.0f), 1.0f);
        const DTreeW &dt = tree->dtrees[tree->lookup(p)];
        const float pg = SDTree::pdfCanon(dt, cu, cv);
        const float x = kFourPi * pg;
        const float sS = albedo * density * (gAbs * x + (1 - gAbs)), sN = std::max(mu - density, 0.0f);
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

// training-record vertex of the guided volpath (medium or non-delta surface vertex)
struct VVtx {
    V3 p, dir, T, Lat;
    float woPdf;
};

inline V3 VolLi(const Scene &S, const pg_config &cfg, SeqRng &rng, Ray ray, VolCounters &cnt, bool lazy,
                const SDTree *tree = nullptr, std::vector<pg_record> *recs = nullptr) {
    const int maxDepth = cfg.max_depth;
    const bool grid = cfg.volume_majorant == PG_MAJORANT_GRID;
    const bool guiding = cfg.guiding && tree && tree->built;
    const float alpha = cfg.bsdf_sampling_fraction;
    const float beta = guiding ? cfg.distance_guiding : 0.0f;
    const int maxV = std::min(cfg.record_max_vertices, 64);
    VVtx vtx[64];
    int nv = 0;
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
    // an interaction's NEE, once its emitter hit is in L: the shadow walk's transmittance on the NEE's
    // sub-stream, the contribution into L and into the training snapshot of the interaction's vertex k
    auto resolveNee = [&](const PendingNee &n, int k) {
        if (!n.valid) return;
        SeqRng sub = subStream(rng, n.dim, 0);
        const float tr = sceneTransmittance(S, n.p1, n.p1OnSurface, n.p2, true, n.medium, n.maxInter, sub, grid);
        if (tr == 0) return;
        const V3 add = n.C * tr;
        L += add;
        if (k >= 0) vtx[k].Lat += add;
    };

    while (depth <= maxDepth || maxDepth < 0) {
        float mt = 0;
        V3 mp;
        bool inMedium = false;
        if (medium >= 0) {
            const Medium &Md = S.media[medium];
            const float maxt = its.valid ? its.t : kInf;
            if (beta > 0) {
                GuidedAccept acc{tree, beta, avg(Md.albedo), grid ? 0.0f : Md.invMax, std::fabs(Md.g), 0, 0};
                dirToCanonical(ray.d, acc.cu, acc.cv);
                inMedium = grid ? Md.sampleDistanceGridA(ray.o, ray.d, 0.0f, maxt, rng, mt, mp, acc)
                                : Md.sampleDistanceA(ray.o, ray.d, 0.0f, maxt, rng, mt, mp, acc);
                T *= acc.w;
            } else {
                inMedium = Md.sample(grid, ray.o, ray.d, 0.0f, maxt, rng, mt, mp);
            }
        }
        if (inMedium) {
            // ---- medium interaction (progressive_volpath.cpp:117-196)
            const Medium &M = S.media[medium];
            if (depth >= maxDepth && maxDepth != -1) break;
            T *= M.albedo;  // sigmaS * transmittance / pdfSuccess = albedo * density / density
            const V3 wi = -ray.d;
            const DTreeW *dt = guiding ? &tree->dtrees[tree->lookup(mp)] : nullptr;
            // phase-sampling fraction: alpha raised toward 1 by the lobe's anisotropy.  The one-sample
            // MIS weight f / (a f + (1 - a) p_guide) reaches 1 / a where the guide misses the lobe,
            // and compounds over the many vertices of a dense forward-scattering walk (a = 0.5 at
            // g = 0.8: 2x the unguided RMSE on C5 from a few paths with weights near 2^k)
            const float alphaM = alpha + (1 - alpha) * std::fabs(M.g);
            PendingNee nee;
            if (cfg.use_nee) {
                const uint32_t ndim = rng.dim;  // the NEE's transmittance sub-stream (kind 0)
                float s0, s1;
                rng.next2(s0, s1);
                DirectRec dr;
                dr.ref = mp;
                dr.refN = V3(0.f);
                V3 value = sampleEmitterNoVis(S, dr, s0, s1);
                if (dr.pdf != 0) {
                    cnt.shadow++;
                    const float phaseVal = hgEval(M.g, wi, dr.d);
                    if (phaseVal != 0 && !isZero(value)) {
                        const float mixPdf = dt ? alphaM * phaseVal + (1 - alphaM) * SDTree::pdfDir(*dt, dr.d) : phaseVal;
                        nee = PendingNee{true, (T * value) * (phaseVal * miWeightV(dr.pdf, mixPdf)), mp, dr.p, false,
                                         medium, maxInter(depth), ndim};
                    }
                }
            }
            float u0, u1, phasePdf;
            rng.next2(u0, u1);
            V3 wo;
            float woPdf, pw = 1.0f;  // pw: phase weight f / woPdf (1 for plain HG sampling)
            if (!dt) {
                wo = hgSample(M.g, wi, u0, u1, phasePdf);
                woPdf = phasePdf;
            } else if (rng.next1() < alphaM) {
                wo = hgSample(M.g, wi, u0, u1, phasePdf);
                woPdf = alphaM * phasePdf + (1 - alphaM) * SDTree::pdfDir(*dt, wo);
                pw = phasePdf / woPdf;
            } else {
                float g0, g1, dPdf;
                rng.next2(g0, g1);
                wo = SDTree::sampleDir(*dt, g0, g1, dPdf);
                phasePdf = hgEval(M.g, wi, wo);
                woPdf = alphaM * phasePdf + (1 - alphaM) * dPdf;
                if (!(woPdf > 0)) {
                    resolveNee(nee, -1);
                    break;
                }
                pw = phasePdf / woPdf;
            }
            int k = -1;
            if (recs && nv < maxV) {
                k = nv;
                vtx[nv++] = VVtx{mp, wo, T * pw, L, woPdf};
            }
            T *= pw;
            ray = Ray{mp, wo, 0.0f, kInf};
            EmitterQuery q;
            lookForEmitter(S, rng, medium, maxInter(depth), ray, its, q, lazy, grid, cnt, cfg.volpath_exact_mis != 0);
            if (!its.valid) its.t = kInf;
            if (!isZero(q.value) && std::min(q.value.x, std::min(q.value.y, q.value.z)) > 0.f) {
                const float emitterPdf = cfg.use_nee ? pdfEmitterDirect(S, q.emitter, V3(0.f), q.d, q.n, q.dist) : 0.0f;
                const float w = cfg.use_nee ? miWeightV(woPdf, emitterPdf) : 1.0f;
                if (q.T != 0) L += ((T * q.value) * w) * q.T;
            }
            resolveNee(nee, k);
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
            const bool guidable = guiding && (Mt.type & ESmooth) && !(Mt.type & EDelta);
            const DTreeW *dt = guidable ? &tree->dtrees[tree->lookup(its.p)] : nullptr;
            PendingNee nee;
            if (cfg.use_nee && (Mt.type & ESmooth)) {
                const uint32_t ndim = rng.dim;  // the NEE's transmittance sub-stream (kind 0)
                float s0, s1;
                rng.next2(s0, s1);
                DirectRec dr;
                dr.ref = its.p;
                dr.refN = refN;
                V3 value = sampleEmitterNoVis(S, dr, s0, s1);
                if (dr.pdf != 0) {
                    const int med = isMediumTransition(sh) ? targetMedium(sh, dr.d, its.geoN) : medium;
                    cnt.shadow++;
                    if (!isZero(value)) {
                        const V3 woL = its.toLocal(dr.d);
                        const V3 bsdfVal = bsdfEval(Mt, its.wi, woL);
                        if (!isZero(bsdfVal) && (!cfg.strict_normals || dot(its.geoN, dr.d) * woL.z > 0)) {
                            float bp = bsdfPdf(Mt, its.wi, woL);
                            if (dt) bp = alpha * bp + (1 - alpha) * SDTree::pdfDir(*dt, dr.d);
                            nee = PendingNee{true, ((T * value) * bsdfVal) * miWeightV(dr.pdf, bp), its.p, dr.p, true, med,
                                             maxInter(depth), ndim};
                        }
                    }
                }
            }
            float b0, b1;
            rng.next2(b0, b1);
            const float b2 = rng.next1();
            BSample bs;
            V3 weight;
            float woPdf;
            if (!dt) {
                weight = bsdfSample(Mt, its.wi, b0, b1, b2, bs);
                woPdf = bs.pdf;
            } else if (rng.next1() < alpha) {
                weight = bsdfSample(Mt, its.wi, b0, b1, b2, bs);
                if (isZero(weight)) {
                    resolveNee(nee, -1);
                    break;
                }
                woPdf = alpha * bs.pdf + (1 - alpha) * SDTree::pdfDir(*dt, its.toWorld(bs.wo));
                weight = weight * (bs.pdf / woPdf);
            } else {
                float g0, g1, dPdf;
                rng.next2(g0, g1);
                const V3 dW = SDTree::sampleDir(*dt, g0, g1, dPdf);
                const V3 woL = its.toLocal(dW);
                const V3 f = bsdfEval(Mt, its.wi, woL);
                const float bp = bsdfPdf(Mt, its.wi, woL);
                woPdf = alpha * bp + (1 - alpha) * dPdf;
                if (!(woPdf > 0) || isZero(f)) {
                    resolveNee(nee, -1);
                    break;
                }
                weight = f / woPdf;
                bs.wo = woL;
                bs.pdf = bp;
                const bool refl = its.wi.z * woL.z > 0;
                bs.sampledType = refl ? ((Mt.type & EDiffuseReflection) ? EDiffuseReflection : EGlossyReflection)
                                      : EGlossyTransmission;
                bs.eta = refl ? 1.0f : (its.wi.z > 0 ? Mt.eta : Mt.invEta);
            }
            if (isZero(weight)) {
                resolveNee(nee, -1);
                break;
            }
            const V3 wo = its.toWorld(bs.wo);
            if (cfg.strict_normals && dot(its.geoN, wo) * bs.wo.z <= 0) {
                resolveNee(nee, -1);
                break;
            }
            int k = -1;
            if (recs && !(bs.sampledType & EDelta) && bs.sampledType != ENull && nv < maxV) {
                k = nv;
                vtx[nv++] = VVtx{its.p, wo, T * weight, L, woPdf};
            }
            const V3 itsP = its.p, itsGeoN = its.geoN;
            ray = Ray{itsP, wo, kEpsilon, kInf};
            T *= weight;
            eta *= bs.eta;
            if (isMediumTransition(sh)) medium = targetMedium(sh, wo, itsGeoN);
            if (bs.sampledType == ENull) {  // index-matched boundary: continue straight through
                resolveNee(nee, k);  // (a null BSDF has no smooth lobe: never an NEE here)
                emission = !scattered;
                if (!S.intersect(ray, its)) its.t = kInf;
                cnt.segments++;
                depth++;
                continue;
            }
            EmitterQuery q;
            lookForEmitter(S, rng, medium, maxInter(depth), ray, its, q, lazy, grid, cnt, cfg.volpath_exact_mis != 0);
            if (!its.valid) its.t = kInf;
            if (!isZero(q.value)) {
                const float emitterPdf = (cfg.use_nee && !(bs.sampledType & EDelta))
                                             ? pdfEmitterDirect(S, q.emitter, refN, q.d, q.n, q.dist)
                                             : 0.0f;
                const float w = cfg.use_nee ? miWeightV(woPdf, emitterPdf) : 1.0f;
                if (q.T != 0) L += ((T * q.value) * w) * q.T;
            }
            resolveNee(nee, k);
            emission = false;
        }
        if (depth++ >= cfg.rr_depth) {
            const float qq = std::min(maxc(T) * eta * eta, 0.95f);
            if (rng.next1() >= qq) break;
            T /= qq;
        }
        scattered = true;
    }
    // training records: incident radiance along each vertex's sampled direction (as oracle.cpp Li)
    if (recs) {
        for (int i = 0; i < nv; ++i) {
            const VVtx &v = vtx[i];
            V3 loc;
            for (int c = 0; c < 3; ++c) loc[c] = (v.T[c] * v.woPdf > 1e-4f) ? (L[c] - v.Lat[c]) / v.T[c] : 0.0f;
            pg_record r;
            r.pos[0] = v.p.x;
            r.pos[1] = v.p.y;
            r.pos[2] = v.p.z;
            float cu, cv;
            dirToCanonical(v.dir, cu, cv);
            r.dir = packCanonical(cu, cv);
            r.radiance = avg(loc);
            r.wo_pdf = v.woPdf;
            r.product = 0.0f;
            r.weight = -1.0f;  // no learned-fraction statistics from the volumetric path
            recs->push_back(r);
        }
        cnt.records += (uint64_t)nv;
    }
    return L;
}

}  // namespace orc
