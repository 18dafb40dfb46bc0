// ORACLE — test infrastructure only.  CPU restatement of the reference BSDF plugins used by the
// guided path-tracing configs, in local shading coordinates, solid-angle measure for eval/pdf:
//   diffuse        src/bsdfs/diffuse.cpp:116-153
//   conductor      src/bsdfs/conductor.cpp (smooth mirror, fresnelConductorExact)
//   roughconductor src/bsdfs/roughconductor.cpp:268-430
//   dielectric     src/bsdfs/dielectric.cpp:235-340
//   roughdielectric src/bsdfs/roughdielectric.cpp:277-620
//   plastic        src/bsdfs/plastic.cpp:271-460
//   roughplastic   src/bsdfs/roughplastic.cpp:258-510 (rough transmittance: orc_rtrans.h)
//   twosided       src/bsdfs/twosided.cpp:116-190 (flag PG_MAT_TWOSIDED)
// Type bits are EBSDFType (include/mitsuba/render/bsdf.h:224-262).
#pragma once
#include "../include/pg_capi.h"
#include "orc_math.h"
#include "orc_rtrans.h"

#include <memory>

namespace orc {

enum : uint32_t {
    ENull = 0x1, EDiffuseReflection = 0x2, EDiffuseTransmission = 0x4, EGlossyReflection = 0x8,
    EGlossyTransmission = 0x10, EDeltaReflection = 0x20, EDeltaTransmission = 0x40,
    EFrontSide = 0x8000, EBackSide = 0x10000,
    EDiffuse = EDiffuseReflection | EDiffuseTransmission,
    EGlossy = EGlossyReflection | EGlossyTransmission,
    ESmooth = EDiffuse | EGlossy,
    EDelta = ENull | EDeltaReflection | EDeltaTransmission,                            // bsdf.h:280
    ETransmission = EDiffuseTransmission | EGlossyTransmission | EDeltaTransmission | ENull,  // bsdf.h:270-272
};

struct Material {
    pg_material m;
    // derived constants (configure())
    float eta = 1, invEta = 1;        // dielectric / plastic: int/ext
    float fdrInt = 0, fdrExt = 0;     // plastic
    float specSamplingWeight = 0;     // plastic, roughplastic
    float invEta2 = 1;
    std::shared_ptr<std::vector<float>> rtrans;  // roughplastic: external rough transmittance
    uint32_t type = 0;                // combined EBSDFType
    V3 diff() const { return {m.diffuse_reflectance[0], m.diffuse_reflectance[1], m.diffuse_reflectance[2]}; }
    V3 spec() const { return {m.specular_reflectance[0], m.specular_reflectance[1], m.specular_reflectance[2]}; }
    V3 trans() const { return {m.specular_transmittance[0], m.specular_transmittance[1], m.specular_transmittance[2]}; }
    V3 ceta() const { return {m.eta[0], m.eta[1], m.eta[2]}; }
    V3 ck() const { return {m.k[0], m.k[1], m.k[2]}; }
    bool twosided() const { return (m.flags & PG_MAT_TWOSIDED) != 0; }
    // BSDF::getAlbedo (diffuse.cpp:112, conductor.cpp:225, roughconductor.cpp:264, dielectric.cpp:230,
    // roughdielectric.cpp:272, plastic.cpp:266, roughplastic.cpp:354; null: bsdf.h:361)
    V3 albedoOf() const {
        switch (m.type) {
            case PG_BSDF_DIFFUSE: return diff();
            case PG_BSDF_CONDUCTOR:
            case PG_BSDF_ROUGHCONDUCTOR: return spec();
            case PG_BSDF_DIELECTRIC: return trans() * 0.5f + spec() * (1 - 0.5f);
            case PG_BSDF_ROUGHDIELECTRIC: return spec() * 0.5f + trans() * (1 - 0.5f);
            case PG_BSDF_PLASTIC: return diff() * 0.5f + spec() * (1 - 0.5f);
            case PG_BSDF_ROUGHPLASTIC: return spec() * 0.5f + diff() * (1 - 0.5f);
            default: return V3(0.f);
        }
    }
    Microfacet distr() const {
        return Microfacet((int)m.distribution, m.alpha_u, m.alpha_v, (m.flags & PG_MAT_SAMPLE_ALL) == 0);
    }
};

inline float luminance(V3 c) { return c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f; }

inline Material makeMaterial(const pg_material &pm) {
    Material M;
    M.m = pm;
    M.eta = pm.int_ior / pm.ext_ior;
    M.invEta = 1.0f / M.eta;
    M.invEta2 = 1.0f / (M.eta * M.eta);
    uint32_t sides = EFrontSide;
    switch (pm.type) {
        case PG_BSDF_DIFFUSE: M.type = EDiffuseReflection; break;
        case PG_BSDF_CONDUCTOR: M.type = EDeltaReflection; break;
        case PG_BSDF_ROUGHCONDUCTOR: M.type = EGlossyReflection; break;
        case PG_BSDF_DIELECTRIC: M.type = EDeltaReflection | EDeltaTransmission; sides |= EBackSide; break;
        case PG_BSDF_ROUGHDIELECTRIC: M.type = EGlossyReflection | EGlossyTransmission; sides |= EBackSide; break;
        case PG_BSDF_PLASTIC: {
            M.type = EDeltaReflection | EDiffuseReflection;
            M.fdrInt = fresnelDiffuseReflectance(1 / M.eta);
            M.fdrExt = fresnelDiffuseReflectance(M.eta);
            float dAvg = luminance(M.diff()), sAvg = luminance(M.spec());
            M.specSamplingWeight = sAvg / (dAvg + sAvg);
            break;
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:258-307
            M.type = EGlossyReflection | EDiffuseReflection;
            float dAvg = luminance(M.diff()), sAvg = luminance(M.spec());
            M.specSamplingWeight = sAvg / (dAvg + sAvg);
            M.rtrans = std::make_shared<std::vector<float>>();
            roughPlasticTables((int)pm.distribution, std::max(pm.alpha_u, 1e-4f), M.eta, *M.rtrans, M.fdrInt);
            break;
        }
        case PG_BSDF_NULL: M.type = ENull; sides |= EBackSide; break;  // null.cpp:40
        default: M.type = 0;
    }
    if (M.twosided()) sides |= EBackSide;
    M.type |= sides;
    return M;
}

struct BSample {
    V3 wo;
    float pdf = 0;
    float eta = 1;
    uint32_t sampledType = 0;
};

// ---- the one-sided nested models (called with wi.z possibly flipped by twosided) ----------
namespace detail {

inline V3 plasticDiff(const Material &M) {
    V3 d = M.diff();
    if (M.m.flags & PG_MAT_NONLINEAR) return d / (V3(1.0f) - d * M.fdrInt);
    return d / (1 - M.fdrInt);
}

inline float roughPlasticProbSpec(const Material &M, float cosThetaI) {  // roughplastic.cpp:405-414
    float p = 1 - rtransEval(M.rtrans->data(), cosThetaI);
    return (p * M.specSamplingWeight) / (p * M.specSamplingWeight + (1 - p) * (1 - M.specSamplingWeight));
}

inline V3 eval1(const Material &M, V3 wi, V3 wo) {
    switch (M.m.type) {
        case PG_BSDF_DIFFUSE:
            if (wi.z <= 0 || wo.z <= 0) return V3(0.f);
            return M.diff() * (kInvPi * wo.z);
        case PG_BSDF_ROUGHCONDUCTOR: {
            if (wi.z <= 0 || wo.z <= 0) return V3(0.f);
            V3 H = normalize(wo + wi);
            Microfacet d = M.distr();
            float D = d.eval(H);
            if (D == 0) return V3(0.f);
            V3 F = fresnelConductorExact(dot(wi, H), M.ceta(), M.ck()) * M.spec();
            float G = d.G(wi, wo, H);
            return F * (D * G / (4.0f * wi.z));
        }
        case PG_BSDF_ROUGHDIELECTRIC: {
            if (wi.z == 0) return V3(0.f);
            bool refl = wi.z * wo.z > 0;
            V3 H;
            if (refl) {
                H = normalize(wo + wi);
            } else {
                float eta = wi.z > 0 ? M.eta : M.invEta;
                H = normalize(wi + wo * eta);
            }
            H = H * signum(H.z);
            Microfacet d = M.distr();
            float D = d.eval(H);
            if (D == 0) return V3(0.f);
            float F = fresnelDielectricExt(dot(wi, H), M.eta);
            float G = d.G(wi, wo, H);
            if (refl) {
                float value = F * D * G / (4.0f * std::fabs(wi.z));
                return M.spec() * value;
            } else {
                float eta = wi.z > 0.0f ? M.eta : M.invEta;
                float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
                float value = ((1 - F) * D * G * eta * eta * dot(wi, H) * dot(wo, H)) /
                              (wi.z * sqrtDenom * sqrtDenom);
                float factor = wi.z > 0 ? M.invEta : M.eta;
                return M.trans() * std::fabs(value * factor * factor);
            }
        }
        case PG_BSDF_PLASTIC: {
            if (wo.z <= 0 || wi.z <= 0) return V3(0.f);
            float Fi = fresnelDielectricExt(wi.z, M.eta);
            float Fo = fresnelDielectricExt(wo.z, M.eta);
            return plasticDiff(M) * (cosineHemispherePdf(wo) * M.invEta2 * (1 - Fi) * (1 - Fo));
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:344-397
            if (wi.z <= 0 || wo.z <= 0) return V3(0.f);
            Microfacet d = M.distr();
            V3 H = normalize(wo + wi);
            float D = d.eval(H);
            float F = fresnelDielectricExt(dot(wi, H), M.eta);
            float G = d.G(wi, wo, H);
            float value = F * D * G / (4.0f * wi.z);
            float T12 = rtransEval(M.rtrans->data(), wi.z), T21 = rtransEval(M.rtrans->data(), wo.z);
            return M.spec() * value + plasticDiff(M) * (kInvPi * wo.z * T12 * T21 * M.invEta2);
        }
        default: return V3(0.f);  // delta-only models have no solid-angle density
    }
}

inline float pdf1(const Material &M, V3 wi, V3 wo) {
    switch (M.m.type) {
        case PG_BSDF_DIFFUSE:
            if (wi.z <= 0 || wo.z <= 0) return 0.0f;
            return cosineHemispherePdf(wo);
        case PG_BSDF_ROUGHCONDUCTOR: {
            if (wi.z <= 0 || wo.z <= 0) return 0.0f;
            V3 H = normalize(wo + wi);
            Microfacet d = M.distr();
            if (d.visible) return d.eval(H) * d.smithG1(wi, H) / (4.0f * wi.z);
            return d.pdf(wi, H) / (4 * absDot(wo, H));
        }
        case PG_BSDF_ROUGHDIELECTRIC: {
            bool refl = wi.z * wo.z > 0;
            V3 H;
            float dwh_dwo;
            if (refl) {
                H = normalize(wo + wi);
                dwh_dwo = 1.0f / (4.0f * dot(wo, H));
            } else {
                float eta = wi.z > 0 ? M.eta : M.invEta;
                H = normalize(wi + wo * eta);
                float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
                dwh_dwo = (eta * eta * dot(wo, H)) / (sqrtDenom * sqrtDenom);
            }
            H = H * signum(H.z);
            Microfacet sd = M.distr();
            if (!sd.visible) sd.scaleAlpha(1.2f - 0.2f * std::sqrt(std::fabs(wi.z)));
            float prob = sd.pdf(wi * signum(wi.z), H);
            float F = fresnelDielectricExt(dot(wi, H), M.eta);
            prob *= refl ? F : (1 - F);
            return std::fabs(prob * dwh_dwo);
        }
        case PG_BSDF_PLASTIC: {
            if (wo.z <= 0 || wi.z <= 0) return 0.0f;
            float Fi = fresnelDielectricExt(wi.z, M.eta);
            float ps = (Fi * M.specSamplingWeight) /
                       (Fi * M.specSamplingWeight + (1 - Fi) * (1 - M.specSamplingWeight));
            return cosineHemispherePdf(wo) * (1 - ps);
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:398-447
            if (wi.z <= 0 || wo.z <= 0) return 0.0f;
            Microfacet d = M.distr();
            V3 H = normalize(wo + wi);
            float probSpecular = roughPlasticProbSpec(M, wi.z), probDiffuse = 1 - probSpecular;
            float dwh_dwo = 1.0f / (4.0f * dot(wo, H));
            float prob = d.pdf(wi, H);
            return prob * dwh_dwo * probSpecular + probDiffuse * cosineHemispherePdf(wo);
        }
        default: return 0.0f;
    }
}

// returns weight = f*cos/pdf (zero on failure); u = (u0,u1) 2D sample, u2 = extra 1D sample
inline V3 sample1(const Material &M, V3 wi, float u0, float u1, float u2, BSample &bs) {
    switch (M.m.type) {
        case PG_BSDF_NULL: {  // null.cpp:64-75: pass straight through (eval/pdf of continuous measures are 0)
            bs.wo = -wi;
            bs.eta = 1.0f;
            bs.sampledType = ENull;
            bs.pdf = 1.0f;
            return V3(1.0f);
        }
        case PG_BSDF_DIFFUSE: {
            if (wi.z <= 0) return V3(0.f);
            bs.wo = squareToCosineHemisphere(u0, u1);
            bs.eta = 1.0f;
            bs.sampledType = EDiffuseReflection;
            bs.pdf = cosineHemispherePdf(bs.wo);
            return M.diff();
        }
        case PG_BSDF_CONDUCTOR: {
            if (wi.z <= 0) return V3(0.f);
            bs.wo = V3(-wi.x, -wi.y, wi.z);
            bs.eta = 1.0f;
            bs.sampledType = EDeltaReflection;
            bs.pdf = 1;
            return M.spec() * fresnelConductorExact(wi.z, M.ceta(), M.ck());
        }
        case PG_BSDF_ROUGHCONDUCTOR: {
            if (wi.z < 0) return V3(0.f);
            Microfacet d = M.distr();
            float pdf;
            V3 m = d.sample(wi, u0, u1, pdf);
            if (pdf == 0) return V3(0.f);
            bs.wo = reflectV(wi, m);
            bs.eta = 1.0f;
            bs.sampledType = EGlossyReflection;
            if (bs.wo.z <= 0) return V3(0.f);
            V3 F = fresnelConductorExact(dot(wi, m), M.ceta(), M.ck()) * M.spec();
            float weight;
            if (d.visible) weight = d.smithG1(bs.wo, m);
            else weight = d.eval(m) * d.G(wi, bs.wo, m) * dot(wi, m) / (pdf * wi.z);
            bs.pdf = pdf / (4.0f * dot(bs.wo, m));
            return F * weight;
        }
        case PG_BSDF_DIELECTRIC: {
            float cosThetaT;
            float F = fresnelDielectricExt(wi.z, cosThetaT, M.eta);
            if (u0 <= F) {
                bs.sampledType = EDeltaReflection;
                bs.wo = V3(-wi.x, -wi.y, wi.z);
                bs.eta = 1.0f;
                bs.pdf = F;
                return M.spec();
            } else {
                float scale = -(cosThetaT < 0 ? M.invEta : M.eta);
                bs.sampledType = EDeltaTransmission;
                bs.wo = V3(scale * wi.x, scale * wi.y, cosThetaT);
                bs.eta = cosThetaT < 0 ? M.eta : M.invEta;
                bs.pdf = 1 - F;
                float factor = cosThetaT < 0 ? M.invEta : M.eta;
                return M.trans() * (factor * factor);
            }
        }
        case PG_BSDF_ROUGHDIELECTRIC: {
            Microfacet d = M.distr();
            Microfacet sd = d;
            if (!sd.visible) sd.scaleAlpha(1.2f - 0.2f * std::sqrt(std::fabs(wi.z)));
            float mpdf;
            V3 m = sd.sample(wi * signum(wi.z), u0, u1, mpdf);
            if (mpdf == 0) return V3(0.f);
            float pdf = mpdf;
            float cosThetaT;
            float F = fresnelDielectricExt(dot(wi, m), cosThetaT, M.eta);
            V3 weight(1.0f);
            bool sampleReflection = true;
            if (u2 > F) {
                sampleReflection = false;
                pdf *= 1 - F;
            } else {
                pdf *= F;
            }
            float dwh_dwo;
            if (sampleReflection) {
                bs.wo = reflectV(wi, m);
                bs.eta = 1.0f;
                bs.sampledType = EGlossyReflection;
                if (wi.z * bs.wo.z <= 0) return V3(0.f);
                weight *= M.spec();
                dwh_dwo = 1.0f / (4.0f * dot(bs.wo, m));
            } else {
                if (cosThetaT == 0) return V3(0.f);
                bs.wo = refractV(wi, m, M.eta, cosThetaT);
                bs.eta = cosThetaT < 0 ? M.eta : M.invEta;
                bs.sampledType = EGlossyTransmission;
                if (wi.z * bs.wo.z >= 0) return V3(0.f);
                float factor = cosThetaT < 0 ? M.invEta : M.eta;
                weight *= M.trans() * (factor * factor);
                float sqrtDenom = dot(wi, m) + bs.eta * dot(bs.wo, m);
                dwh_dwo = (bs.eta * bs.eta * dot(bs.wo, m)) / (sqrtDenom * sqrtDenom);
            }
            if (d.visible) weight *= d.smithG1(bs.wo, m);
            else weight *= std::fabs(d.eval(m) * d.G(wi, bs.wo, m) * dot(wi, m) / (mpdf * wi.z));
            bs.pdf = pdf * std::fabs(dwh_dwo);
            return weight;
        }
        case PG_BSDF_PLASTIC: {
            if (wi.z <= 0) return V3(0.f);
            float Fi = fresnelDielectricExt(wi.z, M.eta);
            bs.eta = 1.0f;
            float ps = (Fi * M.specSamplingWeight) /
                       (Fi * M.specSamplingWeight + (1 - Fi) * (1 - M.specSamplingWeight));
            if (u0 < ps) {
                bs.sampledType = EDeltaReflection;
                bs.wo = V3(-wi.x, -wi.y, wi.z);
                bs.pdf = ps;
                return M.spec() * (Fi / ps);
            } else {
                bs.sampledType = EDiffuseReflection;
                bs.wo = squareToCosineHemisphere((u0 - ps) / (1 - ps), u1);
                float Fo = fresnelDielectricExt(bs.wo.z, M.eta);
                bs.pdf = (1 - ps) * cosineHemispherePdf(bs.wo);
                return plasticDiff(M) * (M.invEta2 * (1 - Fi) * (1 - Fo) / (1 - ps));
            }
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:449-510
            if (wi.z <= 0) return V3(0.f);
            float ps = roughPlasticProbSpec(M, wi.z);
            float sy = u1;
            bool spec = true;
            if (sy < ps) {
                sy /= ps;
            } else {
                sy = (sy - ps) / (1 - ps);
                spec = false;
            }
            if (spec) {
                Microfacet d = M.distr();
                float mpdf;
                V3 m = d.sample(wi, u0, sy, mpdf);
                bs.wo = reflectV(wi, m);
                bs.sampledType = EGlossyReflection;
                if (bs.wo.z <= 0) return V3(0.f);
            } else {
                bs.sampledType = EDiffuseReflection;
                bs.wo = squareToCosineHemisphere(u0, sy);
            }
            bs.eta = 1.0f;
            bs.pdf = pdf1(M, wi, bs.wo);
            if (bs.pdf == 0) return V3(0.f);
            return eval1(M, wi, bs.wo) / bs.pdf;
        }
        default: return V3(0.f);
    }
}

}  // namespace detail

// BSDF::getGlossySamplingRate (bsdf.h:365-381; roughplastic.cpp:323-345; twosided.cpp:221-235): 1 for
// all-glossy models, the glossy lobe's probability for roughplastic, else 0 (kernels: glossyRate)
inline float glossyRate(const Material &M, float cosThetaI) {
    switch (M.m.type) {
        case PG_BSDF_ROUGHCONDUCTOR:
        case PG_BSDF_ROUGHDIELECTRIC: return 1.0f;
        case PG_BSDF_ROUGHPLASTIC: return detail::roughPlasticProbSpec(M, M.twosided() ? std::fabs(cosThetaI) : cosThetaI);
        default: return 0.0f;
    }
}

// ---- public interface with the twosided adapter -------------------------------------------
inline V3 bsdfEval(const Material &M, V3 wi, V3 wo) {
    if (M.twosided() && !(wi.z > 0)) {
        wi.z = -wi.z;
        wo.z = -wo.z;
    }
    return detail::eval1(M, wi, wo);
}
inline float bsdfPdf(const Material &M, V3 wi, V3 wo) {
    if (M.twosided() && !(wi.z > 0)) {
        wi.z = -wi.z;
        wo.z = -wo.z;
    }
    return detail::pdf1(M, wi, wo);
}
inline V3 bsdfSample(const Material &M, V3 wi, float u0, float u1, float u2, BSample &bs) {
    bool flipped = false;
    if (M.twosided() && wi.z < 0) {
        wi.z = -wi.z;
        flipped = true;
    }
    V3 r = detail::sample1(M, wi, u0, u1, u2, bs);
    if (flipped && !isZero(r) && bs.pdf != 0) bs.wo.z = -bs.wo.z;
    return r;
}

}  // namespace orc
