// Which XCDs / CUs a CU-masked stream's blocks land on (hipExtStreamCreateWithCUMask): each block records its
// HW_REG_XCC_ID and HW_REG_HW_ID; the host prints per-mask XCD histograms and distinct CU counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <set>
#include <vector>

__global__ void k_where(uint32_t *out, int spin) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    float acc = (float)threadIdx.x;
    for (int i = 0; i < spin; ++i) acc = acc * 1.0000001f + 0.5f;
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw + (acc == -1.0f ? 1u : 0u);
    }
}

static void run(const char *name, const std::vector<uint32_t> &mask) {
    hipStream_t s;
    if (mask.empty()) {
        if (hipStreamCreate(&s) != hipSuccess) { printf("%s: stream failed\n", name); return; }
    } else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
        printf("%s: masked stream failed\n", name);
        return;
    }
    const int nb = 4096;
    uint32_t *d;
    (void)hipMalloc(&d, nb * 8);
    hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d, 20000);
    std::vector<uint32_t> h(2 * nb);
    (void)hipMemcpyAsync(h.data(), d, nb * 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    int hist[16] = {0};
    std::set<uint64_t> cus;
    for (int b = 0; b < nb; ++b) {
        hist[h[2 * b] & 15]++;
        const uint32_t hw = h[2 * b + 1];
        const uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        cus.insert(((uint64_t)(h[2 * b] & 15) << 16) | (se << 8) | (sh << 4) | cu);
    }
    printf("%-22s xcd blocks:", name);
    for (int x = 0; x < 8; ++x) printf(" %4d", hist[x]);
    printf("   distinct CUs %zu\n", cus.size());
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", ncu);
    const int words = (ncu + 31) / 32;
    run("default", {});
    std::vector<uint32_t> m(words, 0);
    for (int i = 0; i < ncu / 2; ++i) m[i / 32] |= 1u << (i % 32);
    run("first half", m);
    std::fill(m.begin(), m.end(), 0);
    for (int i = ncu / 2; i < ncu; ++i) m[i / 32] |= 1u << (i % 32);
    run("second half", m);
    std::fill(m.begin(), m.end(), 0);
    for (int i = 0; i < ncu; i += 2) m[i / 32] |= 1u << (i % 32);
    run("even bits", m);
    std::fill(m.begin(), m.end(), 0);
    for (int i = 0; i < ncu; ++i) if ((i % 8) < 4) m[i / 32] |= 1u << (i % 32);
    run("bits i%8<4", m);
    std::fill(m.begin(), m.end(), 0);
    for (int i = 0; i < 32; ++i) m[i / 32] |= 1u << (i % 32);
    run("first 32", m);
    return 0;
}
