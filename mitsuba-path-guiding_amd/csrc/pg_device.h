// Device-side building blocks of the gfx950 path: vector math, the counter RNG, warps, Fresnel,
// microfacet models, the BSDF set, and SD-tree queries.  Semantics follow the reference plugins
// (cited per function); layouts are the GPU records described in DESIGN.md §"Data layout in HBM".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pg_layout.h"
#include "pg_fastmath.h"  // fastlog / fastexp: the reference's math::fastlog / fastexp call sites only

#define PGD __device__ __forceinline__

namespace pgd {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kInvFourPi = 0.07957747154594766788f;
constexpr float kEpsilon = 1e-4f;        // include/mitsuba/core/constants.h:28
constexpr float kShadowEpsilon = 1e-3f;  // constants.h:29

struct f3 {
    float x, y, z;
};
PGD f3 mk(float a, float b, float c) { return f3{a, b, c}; }
PGD f3 mk1(float a) { return f3{a, a, a}; }
PGD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PGD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PGD f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
PGD f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
PGD f3 operator*(float s, f3 a) { return mk(a.x * s, a.y * s, a.z * s); }
PGD f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
PGD f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
PGD f3 operator/(f3 a, f3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
PGD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PGD float absDot(f3 a, f3 b) { return fabsf(dot(a, b)); }
PGD f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
PGD float len(f3 a) { return sqrtf(dot(a, a)); }
PGD f3 normalize(f3 a) { return a / len(a); }
PGD float maxc(f3 a) { return fmaxf(a.x, fmaxf(a.y, a.z)); }
PGD float avg3(f3 a) { return (a.x + a.y + a.z) * (1.0f / 3.0f); }
PGD bool isZero(f3 a) { return a.x == 0.f && a.y == 0.f && a.z == 0.f; }
PGD float safe_sqrt(float v) { return sqrtf(fmaxf(0.0f, v)); }
PGD float signum(float v) { return copysignf(1.0f, v); }
PGD f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }
PGD float4 f4(f3 a, float w) { return make_float4(a.x, a.y, a.z, w); }

struct Frame {
    f3 s, t, n;
    PGD f3 toLocal(f3 v) const { return mk(dot(v, s), dot(v, t), dot(v, n)); }
    PGD f3 toWorld(f3 v) const { return s * v.x + t * v.y + n * v.z; }
};
// computeShadingFrame (include/mitsuba/render/skdtree.h:428 via shape.h)
PGD Frame shadingFrame(f3 n, f3 dpdu) {
    Frame f;
    f.n = n;
    f.s = normalize(dpdu - n * dot(n, dpdu));
    f.t = cross(f.n, f.s);
    return f;
}

// ---- counter RNG: Philox-2x32-10 (DESIGN.md "RNG"); key = global pixel, counter = (sample, dim)
PGD void philox(uint32_t c0, uint32_t c1, uint32_t key, uint32_t &o0, uint32_t &o1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint32_t hi = __umulhi(0xD256D193u, c0);
        uint32_t lo = 0xD256D193u * c0;
        c0 = hi ^ key ^ c1;
        c1 = lo;
        key += 0x9E3779B9u;
    }
    o0 = c0;
    o1 = c1;
}
PGD float u2f(uint32_t v) { return (float)(v >> 8) * 0x1p-24f; }
PGD uint32_t rngKey(uint32_t pixel, uint32_t seed) { return pixel ^ (seed * 0x85EBCA6Bu); }
enum { SLOT_NEE = 0, SLOT_BSDF = 1, SLOT_COMP = 2, SLOT_GUIDE_CHOICE = 3, SLOT_RR = 4, SLOT_GUIDE = 5 };
PGD uint32_t dimOf(uint32_t depth, uint32_t slot) { return depth * 8u + slot; }
PGD void rng2(uint32_t key, uint32_t sample, uint32_t dim, float &a, float &b) {
    uint32_t o0, o1;
    philox(sample, dim, key, o0, o1);
    a = u2f(o0);
    b = u2f(o1);
}
PGD float rng1(uint32_t key, uint32_t sample, uint32_t dim) {
    float a, b;
    rng2(key, sample, dim, a, b);
    return a;
}

// ---- warps (src/libcore/warp.cpp:25-180)
PGD f3 squareToCosineHemisphere(float sx, float sy) {
    float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f, phi, r;
    if (r1 == 0 && r2 == 0) {
        r = phi = 0;
    } else if (r1 * r1 > r2 * r2) {
        r = r1;
        phi = (kPi / 4.0f) * (r2 / r1);
    } else {
        r = r2;
        phi = (kPi / 2.0f) - (r1 / r2) * (kPi / 4.0f);
    }
    float sp, cp;
    sincosf(phi, &sp, &cp);
    float px = r * cp, py = r * sp;
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return mk(px, py, z);
}
PGD float cosineHemispherePdf(f3 d) { return kInvPi * d.z; }

// ---- Fresnel (src/libcore/util.cpp:653-683, 741-763)
PGD float fresnelDielectricExt(float cosThetaI_, float &cosThetaT_, float eta) {
    if (eta == 1) {
        cosThetaT_ = -cosThetaI_;
        return 0.0f;
    }
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta;
    float cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) {
        cosThetaT_ = 0.0f;
        return 1.0f;
    }
    float cosThetaI = fabsf(cosThetaI_);
    float cosThetaT = sqrtf(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}
PGD float fresnelDielectricExt(float cosThetaI, float eta) {
    float ct;
    return fresnelDielectricExt(cosThetaI, ct, eta);
}
PGD float fresnelConductor1(float cosThetaI, float eta, float k) {
    float c2 = cosThetaI * cosThetaI, s2 = 1 - c2, s4 = s2 * s2;
    float temp1 = eta * eta - k * k - s2;
    float a2pb2 = safe_sqrt(temp1 * temp1 + k * k * eta * eta * 4);
    float a = safe_sqrt((a2pb2 + temp1) * 0.5f);
    float term1 = a2pb2 + c2, term2 = a * (2 * cosThetaI);
    float Rs2 = (term1 - term2) / (term1 + term2);
    float term3 = a2pb2 * c2 + s4, term4 = term2 * s2;
    float Rp2 = Rs2 * (term3 - term4) / (term3 + term4);
    return 0.5f * (Rp2 + Rs2);
}
PGD f3 fresnelConductorExact(float c, f3 eta, f3 k) {
    return mk(fresnelConductor1(c, eta.x, k.x), fresnelConductor1(c, eta.y, k.y), fresnelConductor1(c, eta.z, k.z));
}
PGD f3 reflectV(f3 wi, f3 m) { return m * (2 * dot(wi, m)) - wi; }
PGD f3 refractV(f3 wi, f3 m, float eta, float cosThetaT) {
    if (cosThetaT < 0) eta = 1 / eta;
    return m * (dot(wi, m) * eta + cosThetaT) - wi * eta;
}

PGD float erfinvf_(float x) {  // Giles 2010 single-precision fit (math.cpp:25-53)
    float w = -fastlog((1.0f - x) * (1.0f + x)), p;
    if (w < 5.0f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = 3.43273939e-07f + p * w;
        p = -3.5233877e-06f + p * w;
        p = -4.39150654e-06f + p * w;
        p = 0.00021858087f + p * w;
        p = -0.00125372503f + p * w;
        p = -0.00417768164f + p * w;
        p = 0.246640727f + p * w;
        p = 1.50140941f + p * w;
    } else {
        w = sqrtf(w) - 3.0f;
        p = -0.000200214257f;
        p = 0.000100950558f + p * w;
        p = 0.00134934322f + p * w;
        p = -0.00367342844f + p * w;
        p = 0.00573950773f + p * w;
        p = -0.0076224613f + p * w;
        p = 0.00943887047f + p * w;
        p = 1.00167406f + p * w;
        p = 2.83297682f + p * w;
    }
    return p * x;
}
PGD float erfAS(float x) {  // math.cpp:55-72 (A&S 7.1.26, not the device library's erff)
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f,
                a5 = 1.061405429f, p = 0.3275911f;
    const float sign = copysignf(1.0f, x);
    x = fabsf(x);
    const float t = 1.0f / (1.0f + p * x);
    const float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * fastexp(-x * x);
    return sign * y;
}

// ---- microfacet distribution (src/bsdfs/microfacet.h:191-600)
struct Mf {
    int type;  // 0 beckmann, 1 ggx
    float au, av;
    bool visible;
    PGD bool iso() const { return au == av; }
    PGD float eval(f3 m) const {
        if (m.z <= 0) return 0.0f;
        float c2 = m.z * m.z;
        float be = ((m.x * m.x) / (au * au) + (m.y * m.y) / (av * av)) / c2;
        float r;
        if (type == 0) {
            r = fastexp(-be) / (kPi * au * av * c2 * c2);
        } else {
            float root = (1.0f + be) * c2;
            r = 1.0f / (kPi * au * av * root * root);
        }
        if (r * m.z < 1e-20f) r = 0;
        return r;
    }
    PGD float projectRoughness(f3 v) const {
        float sin2 = 1.0f - v.z * v.z;
        float inv = 1 / sin2;
        if (iso() || inv <= 0) return au;
        float cp2 = v.x * v.x * inv, sp2 = v.y * v.y * inv;
        return sqrtf(cp2 * au * au + sp2 * av * av);
    }
    PGD float smithG1(f3 v, f3 m) const {
        if (dot(v, m) * v.z <= 0) return 0.0f;
        float sin2 = 1.0f - v.z * v.z;
        if (sin2 <= 0) return 1.0f;
        float tanTheta = fabsf(sqrtf(sin2) / v.z);
        if (tanTheta == 0.0f) return 1.0f;
        float alpha = projectRoughness(v);
        if (type == 0) {
            float a = 1.0f / (alpha * tanTheta);
            if (a >= 1.6f) return 1.0f;
            float a2 = a * a;
            return (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
        }
        float root = alpha * tanTheta;
        return 2.0f / (1.0f + sqrtf(1.0f + root * root));
    }
    PGD float G(f3 wi, f3 wo, f3 m) const { return smithG1(wi, m) * smithG1(wo, m); }
    PGD float pdfVisible(f3 wi, f3 m) const {
        if (wi.z == 0) return 0.0f;
        return smithG1(wi, m) * absDot(wi, m) * eval(m) / fabsf(wi.z);
    }
    PGD float pdf(f3 wi, f3 m) const { return visible ? pdfVisible(wi, m) : eval(m) * m.z; }
    PGD f3 sampleAll(float sx, float sy, float &pdf) const {
        float cosThetaM, sinPhiM, cosPhiM, alphaSqr;
        if (iso()) {
            sincosf(2.0f * kPi * sy, &sinPhiM, &cosPhiM);
            alphaSqr = au * au;
        } else {
            float phiM = atanf(av / au * tanf(kPi + 2 * kPi * sy)) + kPi * floorf(2 * sy + 0.5f);
            sincosf(phiM, &sinPhiM, &cosPhiM);
            float cs = cosPhiM / au, ss = sinPhiM / av;
            alphaSqr = 1.0f / (cs * cs + ss * ss);
        }
        if (type == 0) {
            float t2 = alphaSqr * -fastlog(1.0f - sx);
            cosThetaM = 1.0f / sqrtf(1.0f + t2);
            pdf = (1.0f - sx) / (kPi * au * av * cosThetaM * cosThetaM * cosThetaM);
        } else {
            float t2 = alphaSqr * sx / (1.0f - sx);
            cosThetaM = 1.0f / sqrtf(1.0f + t2);
            float temp = 1 + t2 / alphaSqr;
            pdf = kInvPi / (au * av * cosThetaM * cosThetaM * cosThetaM * temp * temp);
        }
        if (pdf < 1e-20f) pdf = 0;
        float sinThetaM = sqrtf(fmaxf(0.0f, 1 - cosThetaM * cosThetaM));
        return mk(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
    }
    PGD void sampleVisible11(float thetaI, float sx, float sy, float &slx, float &sly) const {
        if (type == 0) {
            if (thetaI < 1e-4f) {
                float r = sqrtf(-fastlog(1.0f - sx)), s, c;
                sincosf(2 * kPi * sy, &s, &c);
                slx = r * c;
                sly = r * s;
                return;
            }
            const float SQRT_PI_INV = 0.56418955f;  // microfacet.h:574, 1 / std::sqrt(M_PI) in float (M_PI is float)
            float tanThetaI = tanf(thetaI), cotThetaI = 1 / tanThetaI;
            float a = -1, c = erfAS(cotThetaI);
            float sample_x = fmaxf(sx, 1e-6f);
            float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
            float b = c - (1 + c) * powf(1 - sample_x, fit);
            float norm = 1 / (1 + c + SQRT_PI_INV * tanThetaI * expf(-cotThetaI * cotThetaI));
            int it = 0;
            while (++it < 10) {
                if (!(b >= a && b <= c)) b = 0.5f * (a + c);
                float ie = erfinvf_(b);
                float value = norm * (1 + b + SQRT_PI_INV * tanThetaI * expf(-ie * ie)) - sample_x;
                float deriv = norm * (1 - ie * tanThetaI);
                if (fabsf(value) < 1e-5f) break;
                if (value > 0) c = b; else a = b;
                b -= value / deriv;
            }
            slx = erfinvf_(b);
            sly = erfinvf_(2.0f * fmaxf(sy, 1e-6f) - 1.0f);
        } else {
            if (thetaI < 1e-4f) {
                float r = safe_sqrt(sx / (1 - sx)), s, c;
                sincosf(2 * kPi * sy, &s, &c);
                slx = r * c;
                sly = r * s;
                return;
            }
            float tanThetaI = tanf(thetaI);
            float a = 1 / tanThetaI;
            float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
            float A = 2.0f * sx / G1 - 1.0f;
            if (fabsf(A) == 1) A -= signum(A) * kEpsilon;
            float tmp = 1.0f / (A * A - 1.0f);
            float B = tanThetaI;
            float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
            float s1 = B * tmp - D, s2 = B * tmp + D;
            slx = (A < 0.0f || s2 > 1.0f / tanThetaI) ? s1 : s2;
            float S, y = sy;
            if (y > 0.5f) { S = 1.0f; y = 2.0f * (y - 0.5f); }
            else { S = -1.0f; y = 2.0f * (0.5f - y); }
            float z = (y * (y * (y * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) +
                       0.000152998850436920f) /
                      (y * (y * (y * (y * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) + 1.0f) -
                       0.539825872510702f);
            sly = S * z * sqrtf(1.0f + slx * slx);
        }
    }
    PGD f3 sampleVisible(f3 wi_, float sx, float sy) const {
        f3 wi = normalize(mk(au * wi_.x, av * wi_.y, wi_.z));
        float theta = 0, phi = 0;
        if (wi.z < 0.99999f) {
            theta = acosf(wi.z);
            phi = atan2f(wi.y, wi.x);
        }
        float sinPhi, cosPhi;
        sincosf(phi, &sinPhi, &cosPhi);
        float slx, sly;
        sampleVisible11(theta, sx, sy, slx, sly);
        float tx = cosPhi * slx - sinPhi * sly, ty = sinPhi * slx + cosPhi * sly;
        tx *= au;
        ty *= av;
        float nrm = 1.0f / sqrtf(tx * tx + ty * ty + 1.0f);
        return mk(-tx * nrm, -ty * nrm, nrm);
    }
    PGD f3 sample(f3 wi, float sx, float sy, float &pdf) const {
        if (visible) {
            f3 m = sampleVisible(wi, sx, sy);
            pdf = pdfVisible(wi, m);
            return m;
        }
        return sampleAll(sx, sy, pdf);
    }
};

// ---- BSDFs on the GPU material record (pg_layout.h GMat) -----------------------------------
enum : uint32_t {
    ENull = 0x1, EDiffuseReflection = 0x2, EDiffuseTransmission = 0x4, EGlossyReflection = 0x8,
    EGlossyTransmission = 0x10, EDeltaReflection = 0x20, EDeltaTransmission = 0x40,
    EFrontSide = 0x8000, EBackSide = 0x10000,
    ESmooth = EDiffuseReflection | EDiffuseTransmission | EGlossyReflection | EGlossyTransmission,
    EDelta = ENull | EDeltaReflection | EDeltaTransmission,                            // bsdf.h:280
    ETransmission = EDiffuseTransmission | EGlossyTransmission | EDeltaTransmission | ENull,  // bsdf.h:270-272
};

struct BS {
    f3 wo;
    float pdf;
    float eta;
    uint32_t type;
};

PGD Mf mfOf(const GMat &M) { return Mf{(int)M.dist, M.alpha_u, M.alpha_v, (M.flags & PG_MAT_SAMPLE_ALL) == 0}; }
PGD f3 diffOf(const GMat &M) { return mk(M.diff[0], M.diff[1], M.diff[2]); }
PGD f3 specOf(const GMat &M) { return mk(M.spec[0], M.spec[1], M.spec[2]); }
PGD f3 transOf(const GMat &M) { return mk(M.trans[0], M.trans[1], M.trans[2]); }
PGD f3 cetaOf(const GMat &M) { return mk(M.ceta[0], M.ceta[1], M.ceta[2]); }
PGD f3 ckOf(const GMat &M) { return mk(M.ck[0], M.ck[1], M.ck[2]); }
// plastic diffuse term with the internal-scattering normalization (plastic.cpp:288-296)
PGD f3 plasticDiff(const GMat &M) {
    f3 d = diffOf(M);
    if (M.flags & PG_MAT_NONLINEAR) return d / (mk1(1.0f) - d * M.fdrInt);
    return d / (1 - M.fdrInt);
}
PGD float plasticProbSpec(const GMat &M, float Fi) {
    return (Fi * M.specWeight) / (Fi * M.specWeight + (1 - Fi) * (1 - M.specWeight));
}
// Rough transmittance of a roughplastic material at cos(theta) (RoughTransmittance::eval with eta
// and alpha fixed, rtrans.h): Catmull-Rom in cos^(1/4) over the 100-entry table
// (spline.cpp:23-60), clamped to [0, 1].  cos^(1/4) is sqrt(sqrt(.)) so that the oracle agrees
// bit for bit (the reference uses std::pow).
PGD float rtransEval(const float *tab, float cosTheta) {
    if (!(cosTheta >= 0)) return 0.0f;
    const float x = sqrtf(sqrtf(fabsf(cosTheta)));
    if (!(x >= 0.0f && x <= 1.0f)) return 0.0f;
    const int n = 100;
    float t = x * (float)(n - 1);
    const int k = max(0, min((int)t, n - 2));
    const float f0 = tab[k], f1 = tab[k + 1];
    const float d0 = k > 0 ? 0.5f * (tab[k + 1] - tab[k - 1]) : tab[k + 1] - tab[k];
    const float d1 = k + 2 < n ? 0.5f * (tab[k + 2] - tab[k]) : tab[k + 1] - tab[k];
    t = t - (float)k;
    const float t2 = t * t, t3 = t2 * t;
    const float r = (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
    return fminf(1.0f, fmaxf(0.0f, r));
}
// probability of sampling the glossy lobe (roughplastic.cpp:405-414)
PGD float roughPlasticProbSpec(const GMat &M, float cosThetaI) {
    const float p = 1 - rtransEval(M.rtrans, cosThetaI);
    return (p * M.specWeight) / (p * M.specWeight + (1 - p) * (1 - M.specWeight));
}

// Compile-time BSDF model selection: MODEL >= 0 compiles that model only (the surface path's material-class
// queues); PG_MODELS_DIFFUSE_NULL compiles the diffuse and null models only (a volumetric scene whose every
// material is one of them: the surface launches drop the microfacet, dielectric and plastic code and its
// registers, pg_volpath.hip k_vvertex KIND 3); -1 dispatches on M.model at run time
constexpr int PG_MODELS_DIFFUSE_NULL = -2;
template <int MODEL>
PGD int modelSel(const GMat &M) {
    if constexpr (MODEL >= 0) return MODEL;
    else if constexpr (MODEL == PG_MODELS_DIFFUSE_NULL) return M.model == PG_BSDF_NULL ? PG_BSDF_NULL : PG_BSDF_DIFFUSE;
    else return (int)M.model;
}

// f * cos(theta_o), solid-angle measure (BSDF::eval with ESolidAngle)
template <int MODEL = -1>
PGD f3 bsdfEval1(const GMat &M, f3 wi, f3 wo) {
    switch (modelSel<MODEL>(M)) {
        case PG_BSDF_DIFFUSE:  // diffuse.cpp:116-124
            if (wi.z <= 0 || wo.z <= 0) return mk1(0.f);
            return diffOf(M) * (kInvPi * wo.z);
        case PG_BSDF_ROUGHCONDUCTOR: {  // roughconductor.cpp:268-306
            if (wi.z <= 0 || wo.z <= 0) return mk1(0.f);
            f3 H = normalize(wo + wi);
            Mf d = mfOf(M);
            float D = d.eval(H);
            if (D == 0) return mk1(0.f);
            f3 F = fresnelConductorExact(dot(wi, H), cetaOf(M), ckOf(M)) * specOf(M);
            return F * (D * d.G(wi, wo, H) / (4.0f * wi.z));
        }
        case PG_BSDF_ROUGHDIELECTRIC: {  // roughdielectric.cpp:277-356
            if (wi.z == 0) return mk1(0.f);
            bool refl = wi.z * wo.z > 0;
            f3 H;
            if (refl) H = normalize(wo + wi);
            else H = normalize(wi + wo * (wi.z > 0 ? M.eta : M.invEta));
            H = H * signum(H.z);
            Mf d = mfOf(M);
            float D = d.eval(H);
            if (D == 0) return mk1(0.f);
            float F = fresnelDielectricExt(dot(wi, H), M.eta);
            float G = d.G(wi, wo, H);
            if (refl) return specOf(M) * (F * D * G / (4.0f * fabsf(wi.z)));
            float eta = wi.z > 0.0f ? M.eta : M.invEta;
            float sqrtDenom = dot(wi, H) + eta * dot(wo, H);
            float value = ((1 - F) * D * G * eta * eta * dot(wi, H) * dot(wo, H)) / (wi.z * sqrtDenom * sqrtDenom);
            float factor = wi.z > 0 ? M.invEta : M.eta;
            return transOf(M) * fabsf(value * factor * factor);
        }
        case PG_BSDF_PLASTIC: {  // plastic.cpp:271-304 (diffuse lobe)
            if (wo.z <= 0 || wi.z <= 0) return mk1(0.f);
            float Fi = fresnelDielectricExt(wi.z, M.eta), Fo = fresnelDielectricExt(wo.z, M.eta);
            return plasticDiff(M) * (cosineHemispherePdf(wo) * M.invEta2 * (1 - Fi) * (1 - Fo));
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:344-397
            if (wi.z <= 0 || wo.z <= 0) return mk1(0.f);
            Mf d = mfOf(M);
            const f3 H = normalize(wo + wi);
            const float D = d.eval(H);
            const float F = fresnelDielectricExt(dot(wi, H), M.eta);
            const float G = d.G(wi, wo, H);
            const float value = F * D * G / (4.0f * wi.z);
            const float T12 = rtransEval(M.rtrans, wi.z), T21 = rtransEval(M.rtrans, wo.z);
            return specOf(M) * value + plasticDiff(M) * (kInvPi * wo.z * T12 * T21 * M.invEta2);
        }
        default: return mk1(0.f);
    }
}

template <int MODEL = -1>
PGD float bsdfPdf1(const GMat &M, f3 wi, f3 wo) {
    switch (modelSel<MODEL>(M)) {
        case PG_BSDF_DIFFUSE:
            if (wi.z <= 0 || wo.z <= 0) return 0.0f;
            return cosineHemispherePdf(wo);
        case PG_BSDF_ROUGHCONDUCTOR: {  // roughconductor.cpp:308-334
            if (wi.z <= 0 || wo.z <= 0) return 0.0f;
            f3 H = normalize(wo + wi);
            Mf d = mfOf(M);
            if (d.visible) return d.eval(H) * d.smithG1(wi, H) / (4.0f * wi.z);
            return d.pdf(wi, H) / (4 * absDot(wo, H));
        }
        case PG_BSDF_ROUGHDIELECTRIC: {  // roughdielectric.cpp:358-418
            bool refl = wi.z * wo.z > 0;
            f3 H;
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
            Mf sd = mfOf(M);
            if (!sd.visible) {
                float s = 1.2f - 0.2f * sqrtf(fabsf(wi.z));
                sd.au *= s;
                sd.av *= s;
            }
            float prob = sd.pdf(wi * signum(wi.z), H);
            float F = fresnelDielectricExt(dot(wi, H), M.eta);
            prob *= refl ? F : (1 - F);
            return fabsf(prob * dwh_dwo);
        }
        case PG_BSDF_PLASTIC: {
            if (wo.z <= 0 || wi.z <= 0) return 0.0f;
            float Fi = fresnelDielectricExt(wi.z, M.eta);
            return cosineHemispherePdf(wo) * (1 - plasticProbSpec(M, Fi));
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:398-447
            if (wi.z <= 0 || wo.z <= 0) return 0.0f;
            Mf d = mfOf(M);
            const f3 H = normalize(wo + wi);
            const float probSpecular = roughPlasticProbSpec(M, wi.z), probDiffuse = 1 - probSpecular;
            const float dwh_dwo = 1.0f / (4.0f * dot(wo, H));
            const float prob = d.pdf(wi, H);
            return prob * dwh_dwo * probSpecular + probDiffuse * cosineHemispherePdf(wo);
        }
        default: return 0.0f;
    }
}

// BSDF::sample(bRec, pdf, sample) -> weight = f*cos/pdf; u2 = component sample (roughdielectric)
template <int MODEL = -1>
PGD f3 bsdfSample1(const GMat &M, f3 wi, float u0, float u1, float u2, BS &bs) {
    switch (modelSel<MODEL>(M)) {
        case PG_BSDF_NULL: {  // null.cpp:64-75 (eval/pdf of the continuous measures are 0)
            bs.wo = -wi;
            bs.eta = 1.0f;
            bs.type = ENull;
            bs.pdf = 1.0f;
            return mk1(1.0f);
        }
        case PG_BSDF_DIFFUSE: {  // diffuse.cpp:139-153
            if (wi.z <= 0) return mk1(0.f);
            bs.wo = squareToCosineHemisphere(u0, u1);
            bs.eta = 1.0f;
            bs.type = EDiffuseReflection;
            bs.pdf = cosineHemispherePdf(bs.wo);
            return diffOf(M);
        }
        case PG_BSDF_CONDUCTOR: {  // conductor.cpp sample (smooth mirror)
            if (wi.z <= 0) return mk1(0.f);
            bs.wo = mk(-wi.x, -wi.y, wi.z);
            bs.eta = 1.0f;
            bs.type = EDeltaReflection;
            bs.pdf = 1;
            return specOf(M) * fresnelConductorExact(wi.z, cetaOf(M), ckOf(M));
        }
        case PG_BSDF_ROUGHCONDUCTOR: {  // roughconductor.cpp:383-430
            if (wi.z < 0) return mk1(0.f);
            Mf d = mfOf(M);
            float pdf;
            f3 m = d.sample(wi, u0, u1, pdf);
            if (pdf == 0) return mk1(0.f);
            bs.wo = reflectV(wi, m);
            bs.eta = 1.0f;
            bs.type = EGlossyReflection;
            if (bs.wo.z <= 0) return mk1(0.f);
            f3 F = fresnelConductorExact(dot(wi, m), cetaOf(M), ckOf(M)) * specOf(M);
            float weight = d.visible ? d.smithG1(bs.wo, m) : d.eval(m) * d.G(wi, bs.wo, m) * dot(wi, m) / (pdf * wi.z);
            bs.pdf = pdf / (4.0f * dot(bs.wo, m));
            return F * weight;
        }
        case PG_BSDF_DIELECTRIC: {  // dielectric.cpp:285-340
            float cosThetaT;
            float F = fresnelDielectricExt(wi.z, cosThetaT, M.eta);
            if (u0 <= F) {
                bs.type = EDeltaReflection;
                bs.wo = mk(-wi.x, -wi.y, wi.z);
                bs.eta = 1.0f;
                bs.pdf = F;
                return specOf(M);
            }
            float scale = -(cosThetaT < 0 ? M.invEta : M.eta);
            bs.type = EDeltaTransmission;
            bs.wo = mk(scale * wi.x, scale * wi.y, cosThetaT);
            bs.eta = cosThetaT < 0 ? M.eta : M.invEta;
            bs.pdf = 1 - F;
            float factor = cosThetaT < 0 ? M.invEta : M.eta;
            return transOf(M) * (factor * factor);
        }
        case PG_BSDF_ROUGHDIELECTRIC: {  // roughdielectric.cpp:522-620
            Mf d = mfOf(M);
            Mf sd = d;
            if (!sd.visible) {
                float s = 1.2f - 0.2f * sqrtf(fabsf(wi.z));
                sd.au *= s;
                sd.av *= s;
            }
            float mpdf;
            f3 m = sd.sample(wi * signum(wi.z), u0, u1, mpdf);
            if (mpdf == 0) return mk1(0.f);
            float pdf = mpdf;
            float cosThetaT;
            float F = fresnelDielectricExt(dot(wi, m), cosThetaT, M.eta);
            f3 weight = mk1(1.0f);
            bool refl = true;
            if (u2 > F) {
                refl = false;
                pdf *= 1 - F;
            } else {
                pdf *= F;
            }
            float dwh_dwo;
            if (refl) {
                bs.wo = reflectV(wi, m);
                bs.eta = 1.0f;
                bs.type = EGlossyReflection;
                if (wi.z * bs.wo.z <= 0) return mk1(0.f);
                weight = weight * specOf(M);
                dwh_dwo = 1.0f / (4.0f * dot(bs.wo, m));
            } else {
                if (cosThetaT == 0) return mk1(0.f);
                bs.wo = refractV(wi, m, M.eta, cosThetaT);
                bs.eta = cosThetaT < 0 ? M.eta : M.invEta;
                bs.type = EGlossyTransmission;
                if (wi.z * bs.wo.z >= 0) return mk1(0.f);
                float factor = cosThetaT < 0 ? M.invEta : M.eta;
                weight = weight * transOf(M) * (factor * factor);
                float sqrtDenom = dot(wi, m) + bs.eta * dot(bs.wo, m);
                dwh_dwo = (bs.eta * bs.eta * dot(bs.wo, m)) / (sqrtDenom * sqrtDenom);
            }
            if (d.visible) weight = weight * d.smithG1(bs.wo, m);
            else weight = weight * fabsf(d.eval(m) * d.G(wi, bs.wo, m) * dot(wi, m) / (mpdf * wi.z));
            bs.pdf = pdf * fabsf(dwh_dwo);
            return weight;
        }
        case PG_BSDF_PLASTIC: {  // plastic.cpp:398-460
            if (wi.z <= 0) return mk1(0.f);
            float Fi = fresnelDielectricExt(wi.z, M.eta);
            bs.eta = 1.0f;
            float ps = plasticProbSpec(M, Fi);
            if (u0 < ps) {
                bs.type = EDeltaReflection;
                bs.wo = mk(-wi.x, -wi.y, wi.z);
                bs.pdf = ps;
                return specOf(M) * (Fi / ps);
            }
            bs.type = EDiffuseReflection;
            bs.wo = squareToCosineHemisphere((u0 - ps) / (1 - ps), u1);
            float Fo = fresnelDielectricExt(bs.wo.z, M.eta);
            bs.pdf = (1 - ps) * cosineHemispherePdf(bs.wo);
            return plasticDiff(M) * (M.invEta2 * (1 - Fi) * (1 - Fo) / (1 - ps));
        }
        case PG_BSDF_ROUGHPLASTIC: {  // roughplastic.cpp:449-510
            if (wi.z <= 0) return mk1(0.f);
            const float ps = roughPlasticProbSpec(M, wi.z);
            float sy = u1;
            bool spec = true;
            if (sy < ps) {
                sy /= ps;
            } else {
                sy = (sy - ps) / (1 - ps);
                spec = false;
            }
            if (spec) {
                Mf d = mfOf(M);
                float mpdf;
                const f3 m = d.sample(wi, u0, sy, mpdf);
                bs.wo = reflectV(wi, m);
                bs.type = EGlossyReflection;
                if (bs.wo.z <= 0) return mk1(0.f);
            } else {
                bs.type = EDiffuseReflection;
                bs.wo = squareToCosineHemisphere(u0, sy);
            }
            bs.eta = 1.0f;
            bs.pdf = bsdfPdf1<PG_BSDF_ROUGHPLASTIC>(M, wi, bs.wo);
            if (bs.pdf == 0) return mk1(0.f);
            return bsdfEval1<PG_BSDF_ROUGHPLASTIC>(M, wi, bs.wo) / bs.pdf;
        }
        default: return mk1(0.f);
    }
}

// BSDF::getGlossySamplingRate (bsdf.h:365-381; roughplastic.cpp:323-345; twosided.cpp:221-235): 1 for
// the all-glossy models, the glossy lobe's sampling probability for roughplastic, 0 for the rest (the
// delta models are never guided).  pg_config.glossy_prior; oracle glossyRate (orc_bsdf.h).
template <int MODEL = -1>
PGD float glossyRate(const GMat &M, float cosThetaI) {
    switch (modelSel<MODEL>(M)) {
        case PG_BSDF_ROUGHCONDUCTOR:
        case PG_BSDF_ROUGHDIELECTRIC: return 1.0f;
        case PG_BSDF_ROUGHPLASTIC:
            return roughPlasticProbSpec(M, (M.flags & PG_MAT_TWOSIDED) ? fabsf(cosThetaI) : cosThetaI);
        default: return 0.0f;
    }
}

// twosided adapter (twosided.cpp:116-190)
template <int MODEL = -1>
PGD f3 bsdfEval(const GMat &M, f3 wi, f3 wo) {
    if ((M.flags & PG_MAT_TWOSIDED) && !(wi.z > 0)) {
        wi.z = -wi.z;
        wo.z = -wo.z;
    }
    return bsdfEval1<MODEL>(M, wi, wo);
}
template <int MODEL = -1>
PGD float bsdfPdf(const GMat &M, f3 wi, f3 wo) {
    if ((M.flags & PG_MAT_TWOSIDED) && !(wi.z > 0)) {
        wi.z = -wi.z;
        wo.z = -wo.z;
    }
    return bsdfPdf1<MODEL>(M, wi, wo);
}
template <int MODEL = -1>
PGD f3 bsdfSample(const GMat &M, f3 wi, float u0, float u1, float u2, BS &bs) {
    bool flipped = false;
    if ((M.flags & PG_MAT_TWOSIDED) && wi.z < 0) {
        wi.z = -wi.z;
        flipped = true;
    }
    bs.pdf = 0;
    bs.type = 0;
    bs.eta = 1;
    f3 r = bsdfSample1<MODEL>(M, wi, u0, u1, u2, bs);
    if (flipped && !isZero(r) && bs.pdf != 0) bs.wo.z = -bs.wo.z;
    return r;
}

// ---- SD-tree queries on the sampling tree (DESIGN.md "SD-tree"; Mueller et al. 2017) ---------
// fp contraction is disabled here so pdfs are bit-identical with the host-side restatement.
#pragma clang fp contract(off)
PGD void dirToCanonical(f3 d, float &u, float &v) {
    float cosTheta = fminf(fmaxf(d.z, -1.0f), 1.0f);
    float phi = atan2f(d.y, d.x);
    if (phi < 0) phi += 2 * kPi;
    u = (cosTheta + 1) * 0.5f;
    v = phi * (1.0f / (2 * kPi));
    if (!(u >= 0)) u = 0;
    if (!(u < 1)) u = 0.99999994f;
    if (!(v >= 0)) v = 0;
    if (!(v < 1)) v = 0.99999994f;
}
PGD f3 canonicalToDir(float u, float v) {
    float cosTheta = 2 * u - 1;
    float phi = 2 * kPi * v;
    float sinTheta = safe_sqrt(1 - cosTheta * cosTheta);
    float sp, cp;
    sincosf(phi, &sp, &cp);
    return mk(sinTheta * cp, sinTheta * sp, cosTheta);
}
PGD uint32_t packCanonical(float u, float v) {
    uint32_t a = min(65535u, (uint32_t)(u * 65536.0f));
    uint32_t b = min(65535u, (uint32_t)(v * 65536.0f));
    return a | (b << 16);
}
PGD int childIndex(float &u, float &v) {
    int q = 0;
    if (u >= 0.5f) { q |= 1; u = u * 2 - 1; } else { u = u * 2; }
    if (v >= 0.5f) { q |= 2; v = v * 2 - 1; } else { v = v * 2; }
    return q;
}
PGD float quadTotal(float4 s) { return ((s.x + s.y) + s.z) + s.w; }
PGD float q4(float4 s, int q) { return q == 0 ? s.x : (q == 1 ? s.y : (q == 2 ? s.z : s.w)); }
PGD uint32_t c4(uint4 c, int q) { return q == 0 ? c.x : (q == 1 ? c.y : (q == 2 ? c.z : c.w)); }

struct SDView {
    const uint2 *snodes;
    const uint4 *meta;      // per D-tree: sampling root, building root, count, bits(samplingTotal)
    const float4 *qsum;     // sampling nodes, interleaved: node n = {qsum[2n] energies, qchild[2n] children}
    const uint4 *qchild;    // = (const uint4 *)(qsum + 1)
    const uint32_t *jump;   // S-tree jump grid: (2^jumpBits)^3 cells -> node at depth <= 3*jumpBits, or
                            // 0x80000000 | D-tree id where the cell lies inside one leaf (k_sd_jump)
    float3 lo;
    float extent;           // cube edge; lookups divide by it (bit-identical with the host spec)
    int jumpBits;
    int built;
};

// the jump-grid cell of position p (sdLookup's first step)
PGD uint32_t sdJumpCell(const SDView &v, f3 p) {
    const float qx = fminf(fmaxf((p.x - v.lo.x) / v.extent, 0.0f), 1.0f);
    const float qy = fminf(fmaxf((p.y - v.lo.y) / v.extent, 0.0f), 1.0f);
    const float qz = fminf(fmaxf((p.z - v.lo.z) / v.extent, 0.0f), 1.0f);
    const int R = 1 << v.jumpBits;
    const float fR = (float)R;
    const int ix = min((int)(qx * fR), R - 1), iy = min((int)(qy * fR), R - 1), iz = min((int)(qz * fR), R - 1);
    return ((uint32_t)iz * R + iy) * R + ix;
}
PGD uint32_t sdLookup(const SDView &v, f3 p) {
    float q[3];
    q[0] = fminf(fmaxf((p.x - v.lo.x) / v.extent, 0.0f), 1.0f);
    q[1] = fminf(fmaxf((p.y - v.lo.y) / v.extent, 0.0f), 1.0f);
    q[2] = fminf(fmaxf((p.z - v.lo.z) / v.extent, 0.0f), 1.0f);
    // Jump grid: the first 3*jumpBits axis-cycling midpoint decisions are the bits of
    // floor(q * 2^jumpBits) per axis, and the residual q*2^k - i is exactly what k sequential
    // (2q | 2q - 1) steps produce, so this is bit-identical with the plain descent.
    const int R = 1 << v.jumpBits;
    const float fR = (float)R;
    int ix = min((int)(q[0] * fR), R - 1), iy = min((int)(q[1] * fR), R - 1), iz = min((int)(q[2] * fR), R - 1);
    uint32_t n = v.jump[((size_t)iz * R + iy) * R + ix];
    if (n & 0x80000000u) return n & 0x7FFFFFFFu;  // the cell lies inside one leaf: its D-tree id
    uint2 nd = v.snodes[n];
    if (nd.x == 0xFFFFFFFFu) return nd.y;
    q[0] = q[0] * fR - (float)ix;
    q[1] = q[1] * fR - (float)iy;
    q[2] = q[2] * fR - (float)iz;
    int axis = 0;
    while (nd.x != 0xFFFFFFFFu) {
        float x = axis == 0 ? q[0] : (axis == 1 ? q[1] : q[2]);
        if (x < 0.5f) {
            x = x * 2;
            n = nd.x;
        } else {
            x = x * 2 - 1;
            n = nd.y;
        }
        if (axis == 0) q[0] = x; else if (axis == 1) q[1] = x; else q[2] = x;
        axis = axis == 2 ? 0 : axis + 1;
        nd = v.snodes[n];
    }
    return nd.y;
}

// pdf = prod_l 4 E_q(l) / E_node(l) / 4pi telescoped to 4^d E_leafquadrant / E_root / 4pi: the
// descent reads only child links; the energies are read once, at the leaf quadrant.
PGD float telescopedPdf(float leafEnergy, float rootTotal, int depth) {
    if (!(leafEnergy > 0)) return 0.0f;
    return ldexpf(leafEnergy / rootTotal, 2 * depth) * kInvFourPi;
}
PGD float sdPdfCanon(const SDView &v, uint4 meta, float u, float w) {
    float total = __uint_as_float(meta.w);
    if (!(total > 0)) return kInvFourPi;
    uint32_t n = meta.x;
    int depth = 1;
    for (int guard = 0; guard < 64; ++guard, ++depth) {
        int q = childIndex(u, w);
        uint32_t c = c4(v.qchild[2 * (n)], q);
        if (c == 0) return telescopedPdf(q4(v.qsum[2 * (n)], q), total, depth);
        n = c;
    }
    return 0.0f;
}
PGD float sdPdf(const SDView &v, uint4 meta, f3 d) {
    if (!(__uint_as_float(meta.w) > 0)) return kInvFourPi;
    float u, w;
    dirToCanonical(d, u, w);
    return sdPdfCanon(v, meta, u, w);
}
PGD void sdSampleCanon(const SDView &v, uint4 meta, float px, float py, float &cu, float &cv, float &pdf) {
    float total0 = __uint_as_float(meta.w);
    if (!(total0 > 0)) {
        cu = px;
        cv = py;
        pdf = kInvFourPi;
        return;
    }
    uint32_t n = meta.x;
    float ox = 0, oy = 0, scale = 1;
    int depth = 0;
    float parentEnergy = total0;
    for (int guard = 0; guard < 64; ++guard) {
        float4 s = v.qsum[2 * (n)];
        float total = quadTotal(s);
        if (!(total > 0)) {
            cu = ox + scale * px;
            cv = oy + scale * py;
            pdf = telescopedPdf(parentEnergy, total0, depth);
            return;
        }
        float partial = s.x + s.z;
        float boundary = partial / total;
        int q = 0;
        float qx = 0, qy = 0;
        if (px < boundary) {
            px = px / boundary;
            boundary = s.x / partial;
        } else {
            partial = total - partial;
            qx = 0.5f;
            px = (px - boundary) / (1.0f - boundary);
            boundary = s.y / partial;
            q |= 1;
        }
        if (py < boundary) {
            py = py / boundary;
        } else {
            qy = 0.5f;
            py = (py - boundary) / (1.0f - boundary);
            q |= 2;
        }
        px = fminf(fmaxf(px, 0.0f), 0.99999994f);
        py = fminf(fmaxf(py, 0.0f), 0.99999994f);
        ox = ox + scale * qx;
        oy = oy + scale * qy;
        scale = scale * 0.5f;
        ++depth;
        uint32_t c = c4(v.qchild[2 * (n)], q);
        if (c == 0) {
            cu = ox + scale * px;
            cv = oy + scale * py;
            pdf = telescopedPdf(q4(s, q), total0, depth);
            return;
        }
        parentEnergy = q4(s, q);
        n = c;
    }
    cu = ox + scale * px;
    cv = oy + scale * py;
    pdf = 0.0f;
}

// Two D-tree walks of one lane in lockstep, so their dependent load chains overlap (the shading
// kernel's two sequential descents were its longest latency chains).  Cursor A is a pdf query at
// canonical (au, aw) (NEE direction); cursor B is a pdf query at (bu, bw) or, with bSample, a
// sample draw with random numbers (bu, bw) (one-sample MIS direction).  Per cursor the arithmetic
// is exactly that of sdPdfCanon / sdSampleCanon, so the results are bit-identical with them.
PGD void sdDual(const SDView &v, uint4 meta, bool aOn, float au, float aw, float &aPdf, bool bOn, bool bSample,
                float bu, float bw, float &cu, float &cv, float &bPdf) {
    const float total0 = __uint_as_float(meta.w);
    aPdf = kInvFourPi;
    bPdf = kInvFourPi;
    cu = bu;
    cv = bw;
    if (!(total0 > 0)) return;
    uint32_t an = meta.x, bn = meta.x;
    int ad = 1, bd = bSample ? 0 : 1;
    int aq = 0, bq = 0;
    bool aAct = aOn, bAct = bOn, aLeaf = false, bLeaf = false;
    float ox = 0, oy = 0, scale = 1, parentEnergy = total0;
    float bEnd = 0.0f;  // sample mode: energy the pdf telescopes to (0: guard exhausted)
    bool bEmpty = false;
    for (int guard = 0; guard < 64 && (aAct || bAct); ++guard) {
        // issue every load of this level before using any of them
        const uint4 ach = v.qchild[2 * (an)];
        const uint4 bch = v.qchild[2 * (bn)];
        const float4 s = v.qsum[2 * (bn)];
        if (aAct) {
            aq = childIndex(au, aw);
            const uint32_t c = c4(ach, aq);
            if (c == 0) {
                aAct = false;
                aLeaf = true;
            } else {
                an = c;
                ++ad;
            }
        }
        if (bAct) {
            if (!bSample) {
                bq = childIndex(bu, bw);
                const uint32_t c = c4(bch, bq);
                if (c == 0) {
                    bAct = false;
                    bLeaf = true;
                } else {
                    bn = c;
                    ++bd;
                }
            } else {
                const float total = quadTotal(s);
                if (!(total > 0)) {
                    bAct = false;
                    bEmpty = true;
                    bEnd = parentEnergy;
                } else {
                    float partial = s.x + s.z;
                    float boundary = partial / total;
                    int q = 0;
                    float qx = 0, qy = 0;
                    if (bu < boundary) {
                        bu = bu / boundary;
                        boundary = s.x / partial;
                    } else {
                        partial = total - partial;
                        qx = 0.5f;
                        bu = (bu - boundary) / (1.0f - boundary);
                        boundary = s.y / partial;
                        q |= 1;
                    }
                    if (bw < boundary) {
                        bw = bw / boundary;
                    } else {
                        qy = 0.5f;
                        bw = (bw - boundary) / (1.0f - boundary);
                        q |= 2;
                    }
                    bu = fminf(fmaxf(bu, 0.0f), 0.99999994f);
                    bw = fminf(fmaxf(bw, 0.0f), 0.99999994f);
                    ox = ox + scale * qx;
                    oy = oy + scale * qy;
                    scale = scale * 0.5f;
                    ++bd;
                    const uint32_t c = c4(bch, q);
                    if (c == 0) {
                        bAct = false;
                        bEmpty = true;
                        bEnd = q4(s, q);
                    } else {
                        parentEnergy = q4(s, q);
                        bn = c;
                    }
                }
            }
        }
    }
    if (aOn) aPdf = aLeaf ? telescopedPdf(q4(v.qsum[2 * (an)], aq), total0, ad) : 0.0f;
    if (bOn) {
        if (!bSample) {
            bPdf = bLeaf ? telescopedPdf(q4(v.qsum[2 * (bn)], bq), total0, bd) : 0.0f;
        } else {
            cu = ox + scale * bu;
            cv = oy + scale * bw;
            bPdf = bEmpty ? telescopedPdf(bEnd, total0, bd) : 0.0f;
        }
    }
}

// ---- learned BSDF-sampling fraction per S-tree leaf (pg_config.bsdf_fraction_bound =
// PG_FRACTION_LEARNED; after Mueller 2019, "Practical Path Guiding in Production", which optimizes the
// selection probability per spatial cell against the KL divergence from the product f * L_i).
// Instead of Mueller's per-sample Adam steps (sequential, not reproducible across devices), each
// training iteration estimates the cross-entropy E_{p*}[log2 q_k] of a fixed set of candidate
// mixtures q_k = a_k p_bsdf + (1 - a_k) p_guide from the iteration's guided records, by importance
// weights w = f L_i / q0 (q0: the mixture that drew the record):  sum_j w_j log2(q_k(wj) / q0(wj)).
// The sums are 2^-16 fixed point (exact, order-independent, like the splat) and the refit picks the
// candidate with the largest (oracle: orc_sdtree.h SDTree::learnedFractions).  Arithmetic shared
// bit for bit with the oracle (fp contraction off, no libm).
constexpr int kFracCandidates = 10;
PGD float fracCandidate(int k) { return 0.05f + 0.1f * (float)k; }  // 0.05 .. 0.95
constexpr float kFracFixedScale = 65536.0f;                         // 2^16
constexpr float kFracCap = 70368744177664.0f;                       // 2^46: |w log2 ratio| <= 2^30
// log2 without libm: exponent bits + 2 atanh((m - 1) / (m + 1)) / ln 2 as a 5-term series, m in [1, 2)
PGD float pgLog2(float x) {
    if (!(x > 1.17549435e-38f)) return -126.0f;
    const uint32_t b = __float_as_uint(x);
    const float e = (float)((int)((b >> 23) & 0xFFu) - 127);
    const float m = __uint_as_float((b & 0x7FFFFFu) | 0x3F800000u);
    const float t = (m - 1.0f) / (m + 1.0f), t2 = t * t;
    const float s = t * (1.0f + t2 * (0.333333343f + t2 * (0.2f + t2 * (0.142857149f + t2 * 0.111111112f))));
    return e + s * 2.88539004f;  // 2 / ln 2
}
// 2^-16 fixed-point value of w * log2(q_k / q0) for candidate k (two's complement in a u64)
PGD unsigned long long fracStat(float w, float pb, float pg, float q0, int k) {
    const float a = fracCandidate(k);
    const float qk = a * pb + (1.0f - a) * pg;
    float v = w * pgLog2(qk / q0) * kFracFixedScale;
    if (v > kFracCap) v = kFracCap;
    if (v < -kFracCap) v = -kFracCap;
    return (unsigned long long)(long long)v;
}
// back to the translation unit's own contraction (Makefile FPC: -DPG_FPC_ON / -DPG_FPC_FAST), not a fixed
// setting: until round 5's last commits a bare contract(on) here re-enabled contraction for every kernel
// after this header in the off build
#if defined(PG_FPC_FAST)
#pragma clang fp contract(fast)
#elif defined(PG_FPC_ON)
#pragma clang fp contract(on)
#else
#pragma clang fp contract(off)
#endif

}  // namespace pgd
