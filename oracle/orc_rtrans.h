// ORACLE — test infrastructure only.  Rough dielectric transmittance slices for roughplastic,
// restating how the reference produces them:
//   src/utils/rdielprec.cpp:40-110  T(wi) = integral over the sample square of roughdielectric's
//       transmission-only sample weight (importance mode); the diffuse transmittance is
//       int_0^1 2 x T(x) dx over the cubic-interpolated table; theta grid cos = t^4, t_0 = step/10
//   src/bsdfs/rtrans.h              eval = Catmull-Rom in cos^(1/4) over the table, clamped
//   src/bsdfs/roughplastic.cpp:283-299  external table at eta, Fdr = 1 - internal diffuse at 1/eta
// T(wi) is the transmission albedo of the rough interface, integrated over the microfacet normals in
// double (rtAlbedo below, the same quadrature as csrc/pg_rtrans.cpp since round 5, so oracle and library
// hold the same tables).  Round 4's estimator integrated the sample square of roughdielectric's
// sampleVisible=false path (Walter et al.: alpha scaled by 1.2 - 0.2 sqrt|cos theta_i|); it reproduced the
// shipped .dat tables to ~1e-4 as this one does (tests/test_rtrans.py compares both sides with them); the
// visible-normal path differs by ~3e-3 for Beckmann, whose G1 is Walter's rational approximation while
// visible-normal sampling is normalised with the exact one.
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

// T(wi), the transmission albedo of the rough interface (rdielprec.cpp:40-110 estimates it by sampling
// roughdielectric's transmission-only weight over the sample square).  Round 5: the same integral over the
// microfacet normals as the library (csrc/pg_rtrans.cpp), in double with the same operation order and
// quadrature, so the oracle's and the kernels' roughplastic tables are the same floats and the BSDF unit
// parity of roughplastic is as tight as the other models'.  The integrand: normals drawn with density
// D(m) cos(theta_m) (sampleAll's mapping, microfacet.h:354-420) on an N x N midpoint grid, u -> 1 - (1 - u)^2
// for GGX's tail, reweighted to the visible-normal density G1(wi, m) <wi, m> D(m) / cos(theta_i) and times
// (1 - F) G1(wo, m) for the refracted wo.  Both sides stay pinned to the shipped .dat slices
// (tests/test_rtrans.py); round 4's sample-square estimator agreed with this one to < 1e-3.
inline double rtG1(int dist, double alpha, const double v[3], const double m[3]) {  // microfacet.h:556-600
    const double vm = v[0] * m[0] + v[1] * m[1] + v[2] * m[2];
    if (vm * v[2] <= 0) return 0.0;
    const double sin2 = 1.0 - v[2] * v[2];
    if (sin2 <= 0) return 1.0;
    const double tanTheta = std::fabs(std::sqrt(sin2) / v[2]);
    if (tanTheta == 0) return 1.0;
    if (dist == 0) {  // Beckmann: Walter's rational approximation
        const double a = 1.0 / (alpha * tanTheta);
        if (a >= 1.6) return 1.0;
        return (3.535 * a + 2.181 * a * a) / (1.0 + 2.276 * a + 2.577 * a * a);
    }
    const double root = alpha * tanTheta;
    return 2.0 / (1.0 + std::sqrt(1.0 + root * root));
}
inline double rtFresnel(double cosI, double eta, double &cosT) {  // fresnelDielectricExt in double
    if (eta == 1) {
        cosT = -cosI;
        return 0.0;
    }
    const double scale = cosI > 0 ? 1.0 / eta : eta;
    const double cosT2 = 1 - (1 - cosI * cosI) * (scale * scale);
    if (cosT2 <= 0) {
        cosT = 0;
        return 1.0;
    }
    const double ci = std::fabs(cosI), ct = std::sqrt(cosT2);
    const double Rs = (ci - eta * ct) / (ci + eta * ct), Rp = (eta * ci - ct) / (eta * ci + ct);
    cosT = cosI > 0 ? -ct : ct;
    return 0.5 * (Rs * Rs + Rp * Rp);
}
inline double rtAlbedo(int dist, double alpha, double eta, double cosThetaI, int N) {
    const double kPiD = 3.14159265358979323846;
    const double wi[3] = {std::sqrt(std::max(0.0, 1 - cosThetaI * cosThetaI)), 0.0, cosThetaI};
    double sum = 0;
    for (int a = 0; a < N; ++a) {
        const double u = (a + 0.5) / N, sx = 1.0 - (1.0 - u) * (1.0 - u), jac = 2.0 * (1.0 - u);
        const double tan2 = dist == 0 ? alpha * alpha * -std::log(1.0 - sx) : alpha * alpha * sx / (1.0 - sx);
        const double cosM = 1.0 / std::sqrt(1.0 + tan2), sinM = std::sqrt(std::max(0.0, 1 - cosM * cosM));
        double row = 0;
        for (int b = 0; b < N; ++b) {
            const double phi = 2 * kPiD * (b + 0.5) / N;
            const double m[3] = {sinM * std::cos(phi), sinM * std::sin(phi), cosM};
            const double wim = wi[0] * m[0] + wi[1] * m[1] + wi[2] * m[2];
            if (wim <= 0) continue;
            const double w = rtG1(dist, alpha, wi, m) * wim / (cosThetaI * cosM);
            if (w == 0) continue;
            double cosT;
            const double F = rtFresnel(wim, eta, cosT);
            if (cosT == 0) continue;
            const double sc = cosT < 0 ? 1.0 / eta : eta;  // refract (roughdielectric.cpp)
            const double wo[3] = {m[0] * (wim * sc + cosT) - wi[0] * sc, m[1] * (wim * sc + cosT) - wi[1] * sc,
                                  m[2] * (wim * sc + cosT) - wi[2] * sc};
            if (wi[2] * wo[2] >= 0) continue;
            row += w * (1 - F) * rtG1(dist, alpha, wo, m);
        }
        sum += row * jac;
    }
    return sum / ((double)N * N);
}

inline void rtransTable(int dist, double alpha, double eta, std::vector<float> &out) {
    out.assign(kRtransSamples, 0.0f);
    const double step = 1.0 / (kRtransSamples - 1);
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (int i = (int)t; i < kRtransSamples; i += (int)nt) {
                const double x = i == 0 ? step / 10 : i * step;  // rdielprec.cpp:87-90: cos = t^4
                out[i] = (float)rtAlbedo(dist, alpha, eta, std::pow(x, 4.0), 128);
            }
        });
    for (auto &th : pool) th.join();
}

// external table at eta and the internal diffuse Fresnel reflectance at 1/eta
inline void roughPlasticTables(int dist, float alpha, float eta, std::vector<float> &ext, float &fdrInt) {
    std::vector<float> in;
    rtransTable(dist, alpha, eta, ext);
    rtransTable(dist, alpha, 1.0 / (double)eta, in);
    const int M = 1 << 14;
    double acc = 0;
    for (int i = 0; i < M; ++i) {
        double x = (i + 0.5) / M;
        acc += 2 * x * rtransCubic1D((float)std::pow(x, 0.25), in.data(), kRtransSamples);
    }
    fdrInt = (float)(1.0 - std::min(1.0, std::max(0.0, acc / M)));
}

}  // namespace orc
