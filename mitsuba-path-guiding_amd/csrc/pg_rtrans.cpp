// Rough dielectric transmittance tables (see pg_rtrans.h).
#include "pg_rtrans.h"

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "../../include/pg_capi.h"

namespace pgh {
namespace {

constexpr double kPi = 3.14159265358979323846;

// Smith G1 of the reference's isotropic distributions (microfacet.h:556-600): Beckmann uses
// Walter's rational approximation, GGX the exact form.
double smithG1(int dist, double alpha, const double v[3], const double m[3]) {
    const double vm = v[0] * m[0] + v[1] * m[1] + v[2] * m[2];
    if (vm * v[2] <= 0) return 0.0;
    const double sin2 = 1.0 - v[2] * v[2];
    if (sin2 <= 0) return 1.0;
    const double tanTheta = std::fabs(std::sqrt(sin2) / v[2]);
    if (tanTheta == 0) return 1.0;
    if (dist == PG_DIST_BECKMANN) {
        const double a = 1.0 / (alpha * tanTheta);
        if (a >= 1.6) return 1.0;
        return (3.535 * a + 2.181 * a * a) / (1.0 + 2.276 * a + 2.577 * a * a);
    }
    const double root = alpha * tanTheta;
    return 2.0 / (1.0 + std::sqrt(1.0 + root * root));
}

// Fresnel for a dielectric with relative IOR eta (fresnelDielectricExt, util.cpp); cosT signed
double fresnel(double cosI, double eta, double &cosT) {
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

// T(wi): microfacet normals m drawn with density D(m) cos(theta_m) on an N x N midpoint grid
// (the distribution's sampleAll mapping, microfacet.h:354-420), weighted to the visible-normal
// density G1(wi, m) <wi, m> D(m) / cos(theta_i) that roughdielectric samples, times the
// transmission weight (1 - F) G1(wo, m) for the refracted wo.
double transmittance(int dist, double alpha, double eta, double cosThetaI, int N) {
    const double wi[3] = {std::sqrt(std::max(0.0, 1 - cosThetaI * cosThetaI)), 0.0, cosThetaI};
    double sum = 0;
    for (int a = 0; a < N; ++a) {
        // sx = 1 - (1 - u)^2 (Jacobian 2 (1 - u)): cancels the 1 / cos(theta_m) growth of the
        // weight towards grazing normals, which left plain midpoints converging as N^-1/2 for GGX
        const double u = (a + 0.5) / N, sx = 1.0 - (1.0 - u) * (1.0 - u), jac = 2.0 * (1.0 - u);
        const double tan2 = dist == PG_DIST_BECKMANN ? alpha * alpha * -std::log(1.0 - sx) : alpha * alpha * sx / (1.0 - sx);
        const double cosM = 1.0 / std::sqrt(1.0 + tan2), sinM = std::sqrt(std::max(0.0, 1 - cosM * cosM));
        double row = 0;
        for (int b = 0; b < N; ++b) {
            const double phi = 2 * kPi * (b + 0.5) / N;
            const double m[3] = {sinM * std::cos(phi), sinM * std::sin(phi), cosM};
            const double wim = wi[0] * m[0] + wi[1] * m[1] + wi[2] * m[2];
            if (wim <= 0) continue;
            double w = smithG1(dist, alpha, wi, m) * wim / (cosThetaI * cosM);
            if (w == 0) continue;
            double cosT;
            const double F = fresnel(wim, eta, cosT);
            if (cosT == 0) continue;
            // refract (roughdielectric.cpp:refract): wo = m (wim * scale + cosT) - wi * scale
            const double scale = cosT < 0 ? 1.0 / eta : eta;
            const double wo[3] = {m[0] * (wim * scale + cosT) - wi[0] * scale, m[1] * (wim * scale + cosT) - wi[1] * scale,
                                  m[2] * (wim * scale + cosT) - wi[2] * scale};
            if (wi[2] * wo[2] >= 0) continue;
            row += w * (1 - F) * smithG1(dist, alpha, wo, m);
        }
        sum += row * jac;
    }
    return sum / ((double)N * N);
}

void table(int dist, double alpha, double eta, std::vector<double> &out) {
    const int n = kRoughTransSamples;
    out.assign(n, 0.0);
    const double step = 1.0 / (n - 1);
    const int quad = 128;  // converged to ~3e-5 (substituted midpoint rule)
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (int i = (int)t; i < n; i += (int)nt) {
                double x = i == 0 ? step / 10 : i * step;  // rdielprec.cpp:87-90
                out[i] = transmittance(dist, alpha, eta, std::pow(x, 4.0), quad);
            }
        });
    for (auto &th : pool) th.join();
}

}  // namespace

float cubicInterp1D(float x, const float *v, int size) {
    if (!(x >= 0.0f && x <= 1.0f)) return 0.0f;
    float t = (x * (float)(size - 1)) / 1.0f;
    int k = std::max(0, std::min((int)t, size - 2));
    float f0 = v[k], f1 = v[k + 1];
    float d0 = k > 0 ? 0.5f * (v[k + 1] - v[k - 1]) : v[k + 1] - v[k];
    float d1 = k + 2 < size ? 0.5f * (v[k + 2] - v[k]) : v[k + 1] - v[k];
    t = t - (float)k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}

void roughTransmittance(int dist, float alpha, float eta, float *out, float *fdrInt) {
    std::vector<double> ext, in;
    table(dist, alpha, eta, ext);
    table(dist, alpha, 1.0 / eta, in);
    for (int i = 0; i < kRoughTransSamples; ++i) out[i] = (float)ext[i];
    // internal diffuse transmittance: int_0^1 2 x T_int(x) dx over the interpolated table
    std::vector<float> inf(in.begin(), in.end());
    const int M = 1 << 14;
    double acc = 0;
    for (int i = 0; i < M; ++i) {
        const double x = (i + 0.5) / M;
        acc += 2 * x * cubicInterp1D((float)std::pow(x, 0.25), inf.data(), kRoughTransSamples);
    }
    const double diffTrans = std::min(1.0, std::max(0.0, acc / M));
    *fdrInt = (float)(1.0 - diffTrans);
}

}  // namespace pgh
