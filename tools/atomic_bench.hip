// Microbenchmark: throughput of same-address device-scope atomics (queue-append pattern).
// hipcc --offload-arch=gfx950 -O3 tools/atomic_bench.hip -o /tmp/atomic_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

// one returning atomic per wave onto one of `naddr` counters (cache-line separated)
__global__ void k_wave(unsigned *c, unsigned *out, int naddr, int bymod) {
    unsigned lane = threadIdx.x & 63;
    unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned slot = bymod ? (blockIdx.x % naddr) : 0;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(&c[slot * 32], 64u);
    base = __shfl(base, 0);
    out[w * 64 + lane] = base + lane;
}
// one returning atomic per block
__global__ void k_block(unsigned *c, unsigned *out) {
    __shared__ unsigned b;
    if (threadIdx.x == 0) b = atomicAdd(&c[0], blockDim.x);
    __syncthreads();
    out[blockIdx.x * blockDim.x + threadIdx.x] = b + threadIdx.x;
}
// no atomics (store only) for the floor
__global__ void k_none(unsigned *out) { out[blockIdx.x * blockDim.x + threadIdx.x] = threadIdx.x; }

int main() {
    const unsigned n = 3700000u / 256 * 256;
    unsigned *c, *out;
    hipMalloc(&c, 4096 * 4);
    hipMalloc(&out, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char *name, auto f) {
        for (int it = 0; it < 3; ++it) f();
        hipMemset(c, 0, 4096 * 4);
        hipEventRecord(a);
        for (int it = 0; it < 20; ++it) f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("%-28s %8.3f us/launch\n", name, ms * 1000 / 20);
    };
    run("store only", [&] { hipLaunchKernelGGL(k_none, dim3(n / 256), dim3(256), 0, 0, out); });
    run("wave atomic, 1 addr", [&] { hipLaunchKernelGGL(k_wave, dim3(n / 256), dim3(256), 0, 0, c, out, 1, 0); });
    run("wave atomic, 8 addr (blk%8)", [&] { hipLaunchKernelGGL(k_wave, dim3(n / 256), dim3(256), 0, 0, c, out, 8, 1); });
    run("wave atomic, 64 addr", [&] { hipLaunchKernelGGL(k_wave, dim3(n / 256), dim3(256), 0, 0, c, out, 64, 1); });
    run("block(256) atomic", [&] { hipLaunchKernelGGL(k_block, dim3(n / 256), dim3(256), 0, 0, c, out); });
    run("block(1024) atomic", [&] { hipLaunchKernelGGL(k_block, dim3(n / 1024), dim3(1024), 0, 0, c, out); });
    return 0;
}
