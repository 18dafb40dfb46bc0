// How often do the device's logf and (float)log((double)x) round differently from the reference's
// math::fastlog ((float)::log((double)x), include/mitsuba/core/math.h:193-195) and from glibc's logf?
// Also the kernels' own fastlog (csrc/pg_fastmath.h).  Inputs: every value 1 - u of the counter RNG (u = k 2^-24), i.e. every argument of the tracking
// loops' log (heterogeneous.cpp:568,634).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/log_rounding.hip -o tools/log_rounding
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mitsuba-path-guiding_amd/csrc/pg_fastmath.h"

__global__ void k_logs(uint32_t n, float *a, float *b, float *c) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x + 1;
    if (k > n) return;
    const float x = (float)k * 0x1p-24f;
    a[k - 1] = logf(x);
    b[k - 1] = (float)log((double)x);
    c[k - 1] = fastlog(x);
}
// every 97th positive normal float through the kernels' fastlog
__global__ void k_span(uint32_t n, float *c) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    c[i] = fastlog(__uint_as_float(0x00800000u + i * 97u));
}

int main() {
    const uint32_t n = 1u << 24;
    const uint32_t ns = (0x7F800000u - 0x00800000u) / 97u;
    float *a, *b, *c, *sp;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess || hipMalloc(&c, n * 4) != hipSuccess ||
        hipMalloc(&sp, (size_t)ns * 4) != hipSuccess)
        return 1;
    k_logs<<<n / 256, 256>>>(n, a, b, c);
    k_span<<<(ns + 255) / 256, 256>>>(ns, sp);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<float> ha(n), hb(n), hc(n), hs(ns);
    if (hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hc.data(), c, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hs.data(), sp, (size_t)ns * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    uint64_t dLogfCr = 0, dLogfGlibc = 0, dDblCr = 0, glibcCr = 0, dFastCr = 0, dSpan = 0;
    for (uint32_t i = 0; i < ns; ++i) {
        uint32_t bits = 0x00800000u + i * 97u;
        float x;
        std::memcpy(&x, &bits, 4);
        dSpan += hs[i] != (float)std::log((double)x);
    }
    for (uint32_t k = 1; k <= n; ++k) {
        const float x = (float)k * 0x1p-24f;
        const float cr = (float)std::log((double)x), gl = logf(x);
        dLogfCr += ha[k - 1] != cr;
        dLogfGlibc += ha[k - 1] != gl;
        dDblCr += hb[k - 1] != cr;
        dFastCr += hc[k - 1] != cr;
        glibcCr += gl != cr;
    }
    std::printf("{\"inputs\": %u, \"device_logf_vs_fastlog\": %llu, \"device_logf_vs_glibc_logf\": %llu, "
                "\"device_double_log_vs_fastlog\": %llu, \"glibc_logf_vs_fastlog\": %llu, "
                "\"kernels_fastlog_vs_fastlog\": %llu, \"span_inputs\": %u, \"kernels_fastlog_vs_fastlog_span\": %llu}\n",
                n, (unsigned long long)dLogfCr, (unsigned long long)dLogfGlibc, (unsigned long long)dDblCr,
                (unsigned long long)glibcCr, (unsigned long long)dFastCr, ns, (unsigned long long)dSpan);
    return 0;
}
