// ORACLE — test infrastructure only (see oracle/README.md).  CPU restatement of the reference's
// fp32 math used on the guided path-tracing hot path.  Never linked into the product library.
//
// Follows:  include/mitsuba/core/frame.h (Frame, coordinateSystem), src/libcore/warp.cpp:25-180
// (cosine hemisphere via concentric disk, uniform triangle), src/libcore/util.cpp:653-683,741-763
// (fresnelDielectricExt, fresnelConductorExact), src/bsdfs/microfacet.h:191-600 (GGX/Beckmann),
// src/libcore/math.cpp erfinv (Giles single-precision fit), and the shared counter RNG spec
// (DESIGN.md "RNG"), which replaces the per-pixel SFMT streams of src/samplers/deterministic.cpp.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace orc {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kInvFourPi = 0.07957747154594766788f;
constexpr float kEpsilon = 1e-4f;        // include/mitsuba/core/constants.h:28
constexpr float kShadowEpsilon = 1e-3f;  // constants.h:29
constexpr float kDeltaEpsilon = 1e-3f;   // constants.h:31

struct V3 {
    float x = 0, y = 0, z = 0;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(float a) : x(a), y(a), z(a) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(float s, V3 a) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
inline V3 &operator+=(V3 &a, V3 b) { a = a + b; return a; }
inline V3 &operator*=(V3 &a, V3 b) { a = a * b; return a; }
inline V3 &operator*=(V3 &a, float s) { a = a * s; return a; }
inline V3 &operator/=(V3 &a, float s) { a = a / s; return a; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float absDot(V3 a, V3 b) { return std::fabs(dot(a, b)); }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float lengthSq(V3 a) { return dot(a, a); }
inline float length(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 normalize(V3 a) { return a / length(a); }
inline float maxc(V3 a) { return std::max(a.x, std::max(a.y, a.z)); }
inline float avg(V3 a) { return (a.x + a.y + a.z) * (1.0f / 3.0f); }
inline bool isZero(V3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }
inline float safe_sqrt(float v) { return std::sqrt(std::max(0.0f, v)); }
inline float signum(float v) { return std::copysign(1.0f, v); }

// Frame (frame.h); shading frame from (n, dpdu) as computeShadingFrame (skdtree.h:428)
struct Frame {
    V3 s, t, n;
    V3 toLocal(V3 v) const { return {dot(v, s), dot(v, t), dot(v, n)}; }
    V3 toWorld(V3 v) const { return s * v.x + t * v.y + n * v.z; }
};
inline Frame shadingFrame(V3 n, V3 dpdu) {
    Frame f;
    f.n = n;
    f.s = normalize(dpdu - n * dot(n, dpdu));
    f.t = cross(f.n, f.s);
    return f;
}

// ---- counter-based RNG (DESIGN.md "RNG"): Philox-2x32-10 keyed by the global pixel id,
// counter = (sample index, dimension).  The GPU kernels implement the same spec bit-for-bit.
inline void philox2x32(uint32_t c0, uint32_t c1, uint32_t key, uint32_t &o0, uint32_t &o1) {
    for (int i = 0; i < 10; ++i) {
        uint64_t p = (uint64_t)0xD256D193u * (uint64_t)c0;
        uint32_t hi = (uint32_t)(p >> 32), lo = (uint32_t)p;
        c0 = hi ^ key ^ c1;
        c1 = lo;
        key += 0x9E3779B9u;
    }
    o0 = c0;
    o1 = c1;
}
inline float u32ToFloat(uint32_t v) { return (float)(v >> 8) * 0x1p-24f; }
inline uint32_t rngKey(uint32_t pixel, uint32_t seed) { return pixel ^ (seed * 0x85EBCA6Bu); }
// dimension slots per bounce
enum { SLOT_NEE = 0, SLOT_BSDF = 1, SLOT_COMP = 2, SLOT_GUIDE_CHOICE = 3, SLOT_RR = 4, SLOT_GUIDE = 5 };
inline uint32_t dimOf(uint32_t depth, uint32_t slot) { return depth * 8u + slot; }
struct Rng {
    uint32_t key, sample;
    void next2(uint32_t dim, float &a, float &b) const {
        uint32_t o0, o1;
        philox2x32(sample, dim, key, o0, o1);
        a = u32ToFloat(o0);
        b = u32ToFloat(o1);
    }
    float next1(uint32_t dim) const {
        float a, b;
        next2(dim, a, b);
        return a;
    }
};

// ---- warp (src/libcore/warp.cpp)
inline void squareToDiskConcentric(float sx, float sy, float &px, float &py) {
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
    px = r * std::cos(phi);
    py = r * std::sin(phi);
}
inline V3 squareToCosineHemisphere(float sx, float sy) {
    float px, py;
    squareToDiskConcentric(sx, sy, px, py);
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0) z = 1e-10f;
    return {px, py, z};
}
inline float cosineHemispherePdf(V3 d) { return kInvPi * d.z; }

// ---- Fresnel (util.cpp)
inline float fresnelDielectricExt(float cosThetaI_, float &cosThetaT_, float eta) {
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
    float cosThetaI = std::fabs(cosThetaI_);
    float cosThetaT = std::sqrt(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5f * (Rs * Rs + Rp * Rp);
}
inline float fresnelDielectricExt(float cosThetaI, float eta) {
    float ct;
    return fresnelDielectricExt(cosThetaI, ct, eta);
}
inline float fresnelConductor1(float cosThetaI, float eta, float k) {
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
inline V3 fresnelConductorExact(float cosThetaI, V3 eta, V3 k) {
    return {fresnelConductor1(cosThetaI, eta.x, k.x), fresnelConductor1(cosThetaI, eta.y, k.y),
            fresnelConductor1(cosThetaI, eta.z, k.z)};
}
// Diffuse Fresnel reflectance by numerical integration (util.cpp fresnelDiffuseReflectance,
// fast=false): 2 * int_0^1 F(sqrt(xi)) dxi, Simpson's rule in double.
inline float fresnelDiffuseReflectance(float eta) {
    const int N = 2000;  // even
    double h = 1.0 / N, acc = 0;
    for (int i = 0; i <= N; ++i) {
        double xi = i * h;
        double w = (i == 0 || i == N) ? 1 : ((i & 1) ? 4 : 2);
        acc += w * fresnelDielectricExt((float)std::sqrt(xi), eta);
    }
    return (float)(acc * h / 3.0);
}

inline V3 reflectV(V3 wi, V3 m) { return m * (2 * dot(wi, m)) - wi; }
inline V3 refractV(V3 wi, V3 m, float eta, float cosThetaT) {
    if (cosThetaT < 0) eta = 1 / eta;
    return m * (dot(wi, m) * eta + cosThetaT) - wi * eta;
}

// ---- math::fastlog / math::fastexp as the reference builds them on Linux x86_64
// (include/mitsuba/core/math.h:175-199): the double-precision libm call, rounded to float.  Every call
// site the reference writes as math::fastlog / fastexp uses these; its plain std::exp / std::log stay float.
inline float fastlog(float x) { return (float)std::log((double)x); }
inline float fastexp(float x) { return (float)std::exp((double)x); }

// ---- erf / erfinv (math.cpp:25-72): Giles 2010 single-precision fit; erf is A&S 7.1.26, not libm's
inline float erfinvf_(float x) {
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
        w = std::sqrt(w) - 3.0f;
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
inline float erfAS(float x) {  // math.cpp:55-72
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f,
                a5 = 1.061405429f, p = 0.3275911f;
    const float sign = signum(x);
    x = std::fabs(x);
    const float t = 1.0f / (1.0f + p * x);
    const float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * fastexp(-x * x);
    return sign * y;
}

// ---- microfacet distribution (microfacet.h)
struct Microfacet {
    int type;  // 0 beckmann, 1 ggx
    float au, av;
    bool visible;
    Microfacet(int t, float a_u, float a_v, bool vis)
        : type(t), au(std::max(a_u, 1e-4f)), av(std::max(a_v, 1e-4f)), visible(vis) {}
    bool iso() const { return au == av; }
    float eval(V3 m) const {
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
    float projectRoughness(V3 v) const {
        float sin2 = std::max(0.0f, 1.0f - v.z * v.z);
        float inv = 1 / sin2;
        if (iso() || inv <= 0) return au;
        float cp2 = v.x * v.x * inv, sp2 = v.y * v.y * inv;
        return std::sqrt(cp2 * au * au + sp2 * av * av);
    }
    float smithG1(V3 v, V3 m) const {
        if (dot(v, m) * v.z <= 0) return 0.0f;
        float sin2 = 1.0f - v.z * v.z;
        if (sin2 <= 0) return 1.0f;
        float tanTheta = std::fabs(std::sqrt(sin2) / v.z);
        if (tanTheta == 0.0f) return 1.0f;
        float alpha = projectRoughness(v);
        if (type == 0) {
            float a = 1.0f / (alpha * tanTheta);
            if (a >= 1.6f) return 1.0f;
            float a2 = a * a;
            return (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
        } else {
            float root = alpha * tanTheta;
            return 2.0f / (1.0f + std::sqrt(1.0f + root * root));
        }
    }
    float G(V3 wi, V3 wo, V3 m) const { return smithG1(wi, m) * smithG1(wo, m); }
    float pdfVisible(V3 wi, V3 m) const {
        if (wi.z == 0) return 0.0f;
        return smithG1(wi, m) * absDot(wi, m) * eval(m) / std::fabs(wi.z);
    }
    float pdfAll(V3 m) const { return eval(m) * m.z; }
    float pdf(V3 wi, V3 m) const { return visible ? pdfVisible(wi, m) : pdfAll(m); }
    V3 sampleAll(float sx, float sy, float &pdf) const {
        float cosThetaM, sinPhiM, cosPhiM, alphaSqr;
        if (iso()) {
            sinPhiM = std::sin(2.0f * kPi * sy);
            cosPhiM = std::cos(2.0f * kPi * sy);
            alphaSqr = au * au;
        } else {
            float phiM = std::atan(av / au * std::tan(kPi + 2 * kPi * sy)) + kPi * std::floor(2 * sy + 0.5f);
            sinPhiM = std::sin(phiM);
            cosPhiM = std::cos(phiM);
            float cs = cosPhiM / au, ss = sinPhiM / av;
            alphaSqr = 1.0f / (cs * cs + ss * ss);
        }
        if (type == 0) {
            float t2 = alphaSqr * -fastlog(1.0f - sx);
            cosThetaM = 1.0f / std::sqrt(1.0f + t2);
            pdf = (1.0f - sx) / (kPi * au * av * cosThetaM * cosThetaM * cosThetaM);
        } else {
            float t2 = alphaSqr * sx / (1.0f - sx);
            cosThetaM = 1.0f / std::sqrt(1.0f + t2);
            float temp = 1 + t2 / alphaSqr;
            pdf = kInvPi / (au * av * cosThetaM * cosThetaM * cosThetaM * temp * temp);
        }
        if (pdf < 1e-20f) pdf = 0;
        float sinThetaM = std::sqrt(std::max(0.0f, 1 - cosThetaM * cosThetaM));
        return {sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM};
    }
    void sampleVisible11(float thetaI, float sx, float sy, float &slx, float &sly) const {
        if (type == 0) {
            if (thetaI < 1e-4f) {
                float r = std::sqrt(-fastlog(1.0f - sx));
                slx = r * std::cos(2 * kPi * sy);
                sly = r * std::sin(2 * kPi * sy);
                return;
            }
            const float SQRT_PI_INV = 1 / std::sqrt(kPi);
            float tanThetaI = std::tan(thetaI), cotThetaI = 1 / tanThetaI;
            float a = -1, c = erfAS(cotThetaI);
            float sample_x = std::max(sx, 1e-6f);
            float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
            float b = c - (1 + c) * std::pow(1 - sample_x, fit);
            float norm = 1 / (1 + c + SQRT_PI_INV * tanThetaI * std::exp(-cotThetaI * cotThetaI));
            int it = 0;
            while (++it < 10) {
                if (!(b >= a && b <= c)) b = 0.5f * (a + c);
                float ie = erfinvf_(b);
                float value = norm * (1 + b + SQRT_PI_INV * tanThetaI * std::exp(-ie * ie)) - sample_x;
                float deriv = norm * (1 - ie * tanThetaI);
                if (std::fabs(value) < 1e-5f) break;
                if (value > 0) c = b; else a = b;
                b -= value / deriv;
            }
            slx = erfinvf_(b);
            sly = erfinvf_(2.0f * std::max(sy, 1e-6f) - 1.0f);
        } else {
            if (thetaI < 1e-4f) {
                float r = safe_sqrt(sx / (1 - sx));
                slx = r * std::cos(2 * kPi * sy);
                sly = r * std::sin(2 * kPi * sy);
                return;
            }
            float tanThetaI = std::tan(thetaI);
            float a = 1 / tanThetaI;
            float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
            float A = 2.0f * sx / G1 - 1.0f;
            if (std::fabs(A) == 1) A -= signum(A) * kEpsilon;
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
            sly = S * z * std::sqrt(1.0f + slx * slx);
        }
    }
    V3 sampleVisible(V3 wi_, float sx, float sy) const {
        V3 wi = normalize(V3(au * wi_.x, av * wi_.y, wi_.z));
        float theta = 0, phi = 0;
        if (wi.z < 0.99999f) {
            theta = std::acos(wi.z);
            phi = std::atan2(wi.y, wi.x);
        }
        float sinPhi = std::sin(phi), cosPhi = std::cos(phi);
        float slx, sly;
        sampleVisible11(theta, sx, sy, slx, sly);
        float tx = cosPhi * slx - sinPhi * sly, ty = sinPhi * slx + cosPhi * sly;
        tx *= au;
        ty *= av;
        float nrm = 1.0f / std::sqrt(tx * tx + ty * ty + 1.0f);
        return {-tx * nrm, -ty * nrm, nrm};
    }
    V3 sample(V3 wi, float sx, float sy, float &pdf) const {
        if (visible) {
            V3 m = sampleVisible(wi, sx, sy);
            pdf = pdfVisible(wi, m);
            return m;
        }
        return sampleAll(sx, sy, pdf);
    }
    void scaleAlpha(float v) { au *= v; av *= v; }
};

}  // namespace orc
