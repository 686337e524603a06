// Random 32-B record scatter on MI355X: the write pattern of the direct path's partition (k_ev_scatter_rec) without
// its compute.  n records of 32 B, two lanes per record (16-B stores), three destination patterns:
//   seq     record i -> slot i (coalesced: the HBM write roofline of the same bytes)
//   binned  record i -> bin b = hash(i) mod B, slot = b * (n / B) + i / B (each bin's slots fill in order, as the
//           partition's per-bin cursors do; consecutive records of a wave land in ~64 different bins), for
//           B = 8192 (the partition's bins) down to 64
//   random  record i -> slot (i * odd) mod n (no locality at all)
// Build: hipcc --offload-arch=gfx950 -O3 -o scatter_bw scatter_bw.hip      Run: ./scatter_bw [n]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__device__ __forceinline__ uint64_t mixh(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}
template <int MODE>
__global__ __launch_bounds__(512) void k_scatter(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n, int bins) {
    const int64_t nb = n / bins;
    for (int64_t base = (int64_t)blockIdx.x * 512; base < 2 * n; base += (int64_t)gridDim.x * 512) {
        const int64_t j = base + threadIdx.x;   // 16-B part j of record j / 2
        if (j >= 2 * n) continue;
        const int64_t i = j >> 1;
        int64_t p;
        if (MODE == 0) p = i;
        else if (MODE == 1) p = (int64_t)(mixh((uint64_t)i) & (uint64_t)(bins - 1)) * nb + (i / bins) % nb;
        else p = (int64_t)(((uint64_t)i * 0x9e3779b97f4a7c15ULL) % (uint64_t)n);
        dst[p * 2 + (j & 1)] = src[j];
    }
}
int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    uint4 *src, *dst;
    if (hipMalloc(&src, n * 32) != hipSuccess || hipMalloc(&dst, n * 32) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(src, 1, n * 32);
    hipMemset(dst, 0, n * 32);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](int m, int bins) {
        hipEventRecord(a);
        if (m == 0) hipLaunchKernelGGL(k_scatter<0>, dim3(8192), dim3(512), 0, 0, src, dst, n, bins);
        if (m == 1) hipLaunchKernelGGL(k_scatter<1>, dim3(8192), dim3(512), 0, 0, src, dst, n, bins);
        if (m == 2) hipLaunchKernelGGL(k_scatter<2>, dim3(8192), dim3(512), 0, 0, src, dst, n, bins);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        return ms;
    };
    for (int rep = 0; rep < 2; rep++) {
        printf("rep %d seq     %.3f ms\n", rep, run(0, 8192));
        for (int bins = 8192; bins >= 64; bins /= 2) {
            const float ms = run(1, bins);
            printf("rep %d binned %5d bins %.3f ms  %.2f GB/s written\n", rep, bins, ms, n * 32 / (ms * 1e-3) / 1e9);
        }
        printf("rep %d random  %.3f ms\n", rep, run(2, 8192));
    }
    return 0;
}
