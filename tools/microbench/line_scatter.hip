// Round 5: what bounds k_merge_owned's state-line stores -- 1e8 whole 64-B lines written to random slots of a table
// (the bench's new keys: each a line at its hash slot), against the same lines confined to a window of the table per
// workgroup at a time (what a merge that took a bin's records in slot order would write), and in order.
//   rand      line i -> a random slot of the whole table (8.6 GB)
//   win W     workgroup g's lines -> random slots inside a W-line window (W x 64 B), one window per 512 lines
//   seq       line i -> slot i
// Each 16-B store instruction writes 16 whole lines (lane L writes part L & 3 of line L / 4, as the merge does).
// Build: hipcc --offload-arch=gfx950 -O3 -o line_scatter line_scatter.hip      Run: ./line_scatter [lines]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mixh(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}

// mode 0 rand, 1 window, 2 seq; tab_lines a power of two; win a power of two (mode 1)
__global__ __launch_bounds__(512) void k_lines(uint4 *__restrict__ tab, uint64_t tab_lines, int64_t n, int mode, uint64_t win) {
    const int ln = threadIdx.x & 63;
    for (int64_t base = (int64_t)blockIdx.x * 512; base < n; base += (int64_t)gridDim.x * 512) {
        // the 512 lines of this round: line j = base + w * 64 + k (wave w, 16 lines per instruction, 4 instructions)
        const int64_t chunk = base / 512;
        const uint64_t wbase = mode == 1 ? (mixh((uint64_t)chunk * 7919) & (tab_lines - 1)) & ~(win - 1) : 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t j = base + (threadIdx.x >> 6) * 64 + k * 16 + (ln >> 2);
            if (j >= n) continue;
            uint64_t slot;
            if (mode == 0) slot = mixh((uint64_t)j) & (tab_lines - 1);
            else if (mode == 1) slot = wbase + (mixh((uint64_t)j) & (win - 1));
            else slot = (uint64_t)j & (tab_lines - 1);
            tab[slot * 4 + (ln & 3)] = make_uint4((unsigned)j, (unsigned)slot, 1u, 2u);
        }
    }
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    const uint64_t tab_lines = uint64_t(1) << 27;   // 8.6 GB
    uint4 *tab;
    CHK(hipMalloc(&tab, tab_lines * 64));
    CHK(hipMemset(tab, 0, tab_lines * 64));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](int mode, uint64_t win) {
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(k_lines, dim3(4096), dim3(512), 0, 0, tab, tab_lines, n, mode, win);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    for (int rep = 0; rep < 2; rep++) {
        printf("rep %d rand          %.3f ms\n", rep, run(0, 0));
        for (uint64_t w : {uint64_t(1) << 10, uint64_t(1) << 12, uint64_t(1) << 13, uint64_t(1) << 14, uint64_t(1) << 16})
            printf("rep %d win %6llu    %.3f ms  (%llu KB)\n", rep, (unsigned long long)w, run(1, w), (unsigned long long)(w * 64 / 1024));
        printf("rep %d seq           %.3f ms\n", rep, run(2, 0));
    }
    return 0;
}
