// ORACLE — test infrastructure only.  Rough dielectric transmittance slices for roughplastic,
// restating how the reference produces them:
//   src/utils/rdielprec.cpp:40-110  T(wi) = integral over the sample square of roughdielectric's
//       transmission-only sample weight (importance mode); the diffuse transmittance is
//       int_0^1 2 x T(x) dx over the cubic-interpolated table; theta grid cos = t^4, t_0 = step/10
//   src/bsdfs/rtrans.h              eval = Catmull-Rom in cos^(1/4) over the table, clamped
//   src/bsdfs/roughplastic.cpp:283-299  external table at eta, Fdr = 1 - internal diffuse at 1/eta
// The sample square is integrated on a midpoint grid of roughdielectric's sampleVisible=false
// path (Walter et al.: m drawn from D cos with alpha scaled by 1.2 - 0.2 sqrt|cos theta_i|, weight
// |D G <wi, m> / (pdf cos theta_i)| (1 - F)).  That estimator reproduces the shipped .dat tables
// to ~1e-4; the visible-normal path differs by ~3e-3 for Beckmann, whose G1 is Walter's rational
// approximation while visible-normal sampling is normalised with the exact one.  The library
// integrates the same quantity over normals (csrc/pg_rtrans.cpp); tests/test_rtrans.py compares
// both with the reference's .dat slices.
#pragma once
#include <cmath>
#include <thread>
#include <vector>

#include "orc_math.h"

namespace orc {

constexpr int kRtransSamples = 100;

inline float rtransCubic1D(float x, const float *v, int n) {  // spline.cpp:23-60 on [0, 1]
    if (!(x >= 0.0f && x <= 1.0f)) return 0.0f;
    float t = (x * (float)(n - 1)) / 1.0f;
    int k = std::max(0, std::min((int)t, n - 2));
    float f0 = v[k], f1 = v[k + 1];
    float d0 = k > 0 ? 0.5f * (v[k + 1] - v[k - 1]) : v[k + 1] - v[k];
    float d1 = k + 2 < n ? 0.5f * (v[k + 2] - v[k]) : v[k + 1] - v[k];
    t = t - (float)k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}

// RoughTransmittance::eval with eta and alpha fixed; cos^(1/4) as sqrt(sqrt(.)) (as the kernels)
inline float rtransEval(const float *tab, float cosTheta) {
    if (!(cosTheta >= 0)) return 0.0f;
    float r = rtransCubic1D(std::sqrt(std::sqrt(std::fabs(cosTheta))), tab, kRtransSamples);
    return std::min(1.0f, std::max(0.0f, r));
}

// roughdielectric transmission-only sample weight, importance mode, sampleVisible=false
// (roughdielectric.cpp:431-518)
inline double transmissionWeight(const Microfacet &d, float eta, V3 wi, float u0, float u1) {
    Microfacet sd = d;
    const float s = 1.2f - 0.2f * std::sqrt(std::fabs(wi.z));
    sd.au *= s;
    sd.av *= s;
    float mpdf;
    V3 m = sd.sample(wi, u0, u1, mpdf);
    if (mpdf == 0) return 0.0;
    float cosThetaT;
    float F = fresnelDielectricExt(dot(wi, m), cosThetaT, eta);
    if (cosThetaT == 0) return 0.0;
    V3 wo = refractV(wi, m, eta, cosThetaT);
    if (wi.z * wo.z >= 0) return 0.0;
    return (double)(1 - F) * std::fabs(d.eval(m) * d.G(wi, wo, m) * dot(wi, m) / (mpdf * wi.z));
}

inline void rtransTable(int dist, float alpha, float eta, std::vector<float> &out) {
    out.assign(kRtransSamples, 0.0f);
    const Microfacet d(dist, alpha, alpha, false);
    const int N = 200;
    const double step = 1.0 / (kRtransSamples - 1);
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (int i = (int)t; i < kRtransSamples; i += (int)nt) {
                double x = i == 0 ? step / 10 : i * step;
                float c = (float)std::pow(x, 4.0);
                V3 wi(std::sqrt(std::max(0.0f, 1 - c * c)), 0.0f, c);
                // u0 = 1 - (1 - v)^2 (Jacobian 2 (1 - v)) resolves GGX's heavy tail near u0 = 1
                double acc = 0;
                for (int a = 0; a < N; ++a) {
                    const double v = (a + 0.5) / N;
                    const float u0 = (float)(1.0 - (1.0 - v) * (1.0 - v));
                    double row = 0;
                    for (int b = 0; b < N; ++b) row += transmissionWeight(d, eta, wi, u0, (b + 0.5f) / N);
                    acc += row * 2.0 * (1.0 - v);
                }
                out[i] = (float)(acc / ((double)N * N));
            }
        });
    for (auto &th : pool) th.join();
}

// external table at eta and the internal diffuse Fresnel reflectance at 1/eta
inline void roughPlasticTables(int dist, float alpha, float eta, std::vector<float> &ext, float &fdrInt) {
    std::vector<float> in;
    rtransTable(dist, alpha, eta, ext);
    rtransTable(dist, alpha, 1.0f / eta, in);
    const int M = 1 << 14;
    double acc = 0;
    for (int i = 0; i < M; ++i) {
        double x = (i + 0.5) / M;
        acc += 2 * x * rtransCubic1D((float)std::pow(x, 0.25), in.data(), kRtransSamples);
    }
    fdrInt = (float)(1.0 - std::min(1.0, std::max(0.0, acc / M)));
}

}  // namespace orc
