// Ablation timing of the device latLngToCell (profiling tool, not product code).
// Built once per variant of csrc/h3_device.h (make_variants.py); prints one JSON line per run:
// {"variant": V, "res": R, "n": N, "ms": best-of-reps kernel time, "checksum": xor of cells}
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include "h3_device.h"
#include "kernels.h"
#define H3T_CONST static const
#include "h3_tables.inc"
#include "h3_tables_host.h"
using namespace hm;

#ifndef VARIANT
#define VARIANT "base"
#endif
#ifndef H3B_WAVES
#define H3B_WAVES 3
#endif

__constant__ H3Tables c_tab;

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(H3B_WAVES))) void k_cells(const double *lat, const double *lon,
                                                                                       long n, int res, uint64_t *out) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        out[i] = latLngToCellDeg(lat[i], lon[i], res, c_tab);
}

// uniform points on the sphere from a counter hash (same on every run)
__global__ void k_points(double *lat, double *lon, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        uint64_t a = mix64((uint64_t)i * 2 + 1), b = mix64((uint64_t)i * 2 + 2);
        double u = (double)(a >> 11) * 0x1p-53, v = (double)(b >> 11) * 0x1p-53;
        lat[i] = asin(2.0 * u - 1.0) * (180.0 / M_PI);
        lon[i] = v * 360.0 - 180.0;
    }
}

__global__ void k_xor(const uint64_t *c, long n, unsigned long long *acc) {
    uint64_t x = 0;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) x ^= c[i] * (uint64_t)(i | 1);
    atomicXor(acc, (unsigned long long)x);
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 100000000L;
    int res = argc > 2 ? atoi(argv[2]) : 8;
    int reps = argc > 3 ? atoi(argv[3]) : 5;
    H3Tables T = hm_make_tables();
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &T, sizeof(T)) != hipSuccess) return 2;
    double *lat, *lon;
    uint64_t *out;
    unsigned long long *acc;
    if (hipMalloc(&lat, n * 8) || hipMalloc(&lon, n * 8) || hipMalloc(&out, n * 8) || hipMalloc(&acc, 8)) return 3;
    hipLaunchKernelGGL(k_points, dim3(4096), dim3(256), 0, 0, lat, lon, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_cells, dim3(256 * H3B_WAVES * 8), dim3(256), 0, 0, lat, lon, n, res, out);
        hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 4;
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    hipMemset(acc, 0, 8);
    hipLaunchKernelGGL(k_xor, dim3(1024), dim3(256), 0, 0, out, n, acc);
    unsigned long long h = 0;
    hipMemcpy(&h, acc, 8, hipMemcpyDeviceToHost);
    printf("{\"variant\": \"%s\", \"res\": %d, \"n\": %ld, \"ms\": %.4f, \"checksum\": \"%016llx\"}\n", VARIANT, res, n, best, h);
    return 0;
}
