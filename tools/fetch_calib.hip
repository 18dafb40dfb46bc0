// FETCH_SIZE calibration for the gather widths of the path kernels.
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for wide coalesced streaming reads (it reports half
// their bytes); every other access width is "uncalibrated".  Each launch below moves a KNOWN number of
// bytes in one access pattern; run under rocprofv3 --pmc FETCH_SIZE (and the TCC request / hit counters
// in their own passes) it gives FETCH_SIZE per true byte for that pattern:
//   k_cal_stream    16 B/lane coalesced read of a 1 GiB buffer (the guide's reference case)
//   k_cal_gather    one row of W = 16 / 32 / 48 / 64 / 128 B per lane, every row in its own 256-B slot of
//                   the table (a bijective slot hash: no two lanes share a cache line), at a byte offset
//                   inside the slot (0, or 96 so a 48-B row straddles two 128-B lines as unaligned TriAccel
//                   records do); tables of 2 GiB (beyond the 256 MiB Infinity Cache: HBM), 64 MiB
//                   (Infinity-Cache resident, beyond the XCD's 4 MiB L2) and 4 MiB (the C3 closest-hit
//                   working set: BVH + TriAccel records)
//   k_cal_scatter16 16 B/lane at slots permuted within each 64-lane group's 1 KiB (the SoA path state
//                   read through a queue whose slots are a permutation of a contiguous range)
// Every launch is timed with a HIP event pair (printed as JSON lines) and the rocprofv3 kernel names carry
// the case id, so tools/fetch_calib_summary.py joins the counter passes to the cases.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

// bijection on [0, 2^bits): odd multiply + xorshift, masked
__device__ __forceinline__ uint32_t permute(uint32_t x, uint32_t bits) {
    const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
    x = (x * 0x9E3779B1u) & m;
    x ^= x >> (bits / 2 + 1);
    x = (x * 0x85EBCA77u) & m;
    x ^= x >> (bits / 2 + 1);
    return x & m;
}

template <int CASE>
__global__ void __launch_bounds__(256) k_cal_stream(const float4 *__restrict__ src, uint32_t n, float *sink) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 v = src[i];
    const float a = v.x + v.y + v.z + v.w;
    if (a == 1234.5f) sink[i & 1023] = a;  // never true (the table is zero): keeps the load
}

// W16: row size in 16-B units (48-B rows: 3); OFF: byte offset of the row in its 256-B slot
template <int CASE, int W16, int OFF>
__global__ void __launch_bounds__(256) k_cal_gather(const uint8_t *__restrict__ table, uint32_t slotBits, uint32_t n,
                                                    float *sink) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = permute(i, slotBits);  // n <= 2^slotBits: distinct slots
    const float4 *p = reinterpret_cast<const float4 *>(table + (size_t)slot * 256 + OFF);
    float a = 0;
#pragma unroll
    for (int k = 0; k < W16; ++k) {
        const float4 v = p[k];
        a += v.x + v.y + v.z + v.w;
    }
    if (a == 1234.5f) sink[i & 1023] = a;
}

// gathers with reuse: n lanes draw rows uniformly from a table of 2^slotBits slots (n >> slots)
template <int CASE, int W16, int OFF>
__global__ void __launch_bounds__(256) k_cal_reuse(const uint8_t *__restrict__ table, uint32_t slotBits, uint32_t n,
                                                   float *sink) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = permute(i, 32) & ((1u << slotBits) - 1u);
    const float4 *p = reinterpret_cast<const float4 *>(table + (size_t)slot * 256 + OFF);
    float a = 0;
#pragma unroll
    for (int k = 0; k < W16; ++k) {
        const float4 v = p[k];
        a += v.x + v.y + v.z + v.w;
    }
    if (a == 1234.5f) sink[i & 1023] = a;
}

template <int CASE>
__global__ void __launch_bounds__(256) k_cal_scatter16(const float4 *__restrict__ src, uint32_t n, float *sink) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = (i & ~63u) | permute(i & 63u, 6);  // a permutation inside each 64-entry group
    const float4 v = src[j];
    const float a = v.x + v.y + v.z + v.w;
    if (a == 1234.5f) sink[i & 1023] = a;
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
    }
};

static void report(const char *name, const char *pattern, uint64_t n, uint64_t bytes, uint64_t lines, float ms) {
    std::printf("{\"case\": \"%s\", \"pattern\": \"%s\", \"lanes\": %llu, \"true_bytes\": %llu, \"lines_128\": %llu, "
                "\"ms\": %.4f, \"gbs\": %.1f}\n",
                name, pattern, (unsigned long long)n, (unsigned long long)bytes, (unsigned long long)lines, ms,
                bytes / (ms * 1e-3) / 1e9);
    std::fflush(stdout);
}

template <typename F>
static float timed(F launch) {
    static Timer t;
    launch();  // warm (TLB, code); the counters see both launches, the summary takes the second
    CHECK(hipEventRecord(t.a));
    launch();
    CHECK(hipEventRecord(t.b));
    CHECK(hipEventSynchronize(t.b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, t.a, t.b));
    return ms;
}

// flush the L2s and the Infinity Cache between cases: stream 1 GiB of writes
__global__ void k_cal_flush(float4 *p, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = make_float4(0, 0, 0, 0);
}

int main() {
    const size_t big = (size_t)2 << 30;  // 2 GiB table
    uint8_t *table;
    float4 *flushBuf;
    float *sink;
    CHECK(hipMalloc(&table, big + 4096));
    CHECK(hipMemset(table, 0, big + 4096));
    CHECK(hipMalloc(&flushBuf, (size_t)1 << 30));
    CHECK(hipMalloc(&sink, 4096));
    const uint32_t nflush = (1u << 30) / 16;
    auto flush = [&] {
        k_cal_flush<<<nflush / 256, 256>>>(flushBuf, nflush);
        CHECK(hipDeviceSynchronize());
    };
    const uint32_t blocks = 1u << 14;  // 2^22 lanes per gather case
    const uint32_t n = blocks * 256;

    {  // 1 GiB coalesced stream, 16 B per lane
        const uint32_t ns = (1u << 30) / 16;
        flush();
        const float ms = timed([&] { k_cal_stream<0><<<ns / 256, 256>>>((const float4 *)table, ns, sink); });
        report("stream16", "coalesced 16 B/lane, 1 GiB", ns, (uint64_t)ns * 16, (uint64_t)ns * 16 / 128, ms);
    }
    {  // permuted 16-B reads inside 1-KiB groups (queue-ordered SoA state), 1 GiB
        const uint32_t ns = (1u << 30) / 16;
        flush();
        const float ms = timed([&] { k_cal_scatter16<1><<<ns / 256, 256>>>((const float4 *)table, ns, sink); });
        report("scatter16", "16 B/lane permuted within 1 KiB groups, 1 GiB", ns, (uint64_t)ns * 16, (uint64_t)ns * 16 / 128, ms);
    }
    // distinct-slot gathers from the 2 GiB table (2^23 slots of 256 B; 2^22 lanes)
#define GATHER(ID, W16, OFF, LINES)                                                                              \
    {                                                                                                            \
        flush();                                                                                                 \
        const float ms = timed([&] { k_cal_gather<ID, W16, OFF><<<blocks, 256>>>(table, 23, n, sink); });       \
        report("gather" #W16 "x16_off" #OFF "_2GiB", "distinct 256-B slots of a 2 GiB table", n,                  \
               (uint64_t)n * 16 * W16, (uint64_t)n * (LINES), ms);                                               \
    }
    GATHER(10, 1, 0, 1)
    GATHER(11, 2, 0, 1)
    GATHER(12, 3, 0, 1)
    GATHER(13, 3, 96, 2)
    GATHER(14, 4, 0, 1)
    GATHER(15, 8, 0, 1)
#undef GATHER
    // gathers with reuse from a 64 MiB table (2^18 slots) and a 4 MiB table (2^14 slots): 2^22 lanes each
#define REUSE(ID, W16, OFF, BITS, TAG)                                                                           \
    {                                                                                                            \
        flush();                                                                                                 \
        const float ms = timed([&] { k_cal_reuse<ID, W16, OFF><<<blocks, 256>>>(table, BITS, n, sink); });      \
        report("reuse" #W16 "x16_off" #OFF "_" TAG, "uniform rows of a " TAG " table (slots of 256 B)", n,      \
               (uint64_t)n * 16 * W16, (uint64_t)1 << (BITS), ms);                                               \
    }
    REUSE(20, 3, 96, 18, "64MiB")
    REUSE(21, 4, 0, 18, "64MiB")
    REUSE(22, 3, 96, 14, "4MiB")
    REUSE(23, 4, 0, 14, "4MiB")
#undef REUSE
    CHECK(hipFree(table));
    CHECK(hipFree(flushBuf));
    CHECK(hipFree(sink));
    std::printf("{\"done\": true}\n");
    return 0;
}
