// Round 5: calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on the access patterns of k_ingest<true> (VERDICT r4:
// its counted traffic was 1.92x its algorithmic bytes, partly counter artefacts).  Each kernel moves a known number of
// bytes in one of those patterns; tools/pmc_calib.py divides the counters by the known bytes:
//   nt8     k_ingest's column loads: 8-B non-temporal loads, one per lane, consecutive lanes consecutive rows (5 columns
//           of 1e8 doubles) + two 1-B columns; known: 42 B per row read
//   st9     k_ingest's per-row outputs: a 1-B flag and an 8-B key per row, one per lane; known: 9 B per row written
//   atom    k_ingest<true>'s bin cursors: one returned 32-bit atomicAdd per row on 8192 counters (nothing else);
//           known: 0 bytes of data (the counters themselves: 32 KB)
//   scat32  the binned records: 32 B per row as two 16-B stores per lane at a scattered slot (a bijection of the row,
//           no atomic); known: 32 B per row written
// Build: hipcc --offload-arch=gfx950 -O3 -o pmc_calib pmc_calib.hip      Run: ./pmc_calib [rows]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mixh(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}

__global__ __launch_bounds__(256) void k_nt8(const double *__restrict__ a, const double *__restrict__ b,
                                             const int64_t *__restrict__ c, const double *__restrict__ d,
                                             const uint64_t *__restrict__ e, const uint8_t *__restrict__ f,
                                             const uint8_t *__restrict__ g, int64_t n, unsigned long long *sink) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double x = __builtin_nontemporal_load(&a[i]) + __builtin_nontemporal_load(&b[i]) + __builtin_nontemporal_load(&d[i]);
        acc += (unsigned long long)__builtin_nontemporal_load(&c[i]) ^ __builtin_nontemporal_load(&e[i]) ^
               __builtin_bit_cast(unsigned long long, x) ^ __builtin_nontemporal_load(&f[i]) ^ __builtin_nontemporal_load(&g[i]);
    }
    if (acc == 0x123456789ull) atomicAdd(sink, 1ull);   // (never: keeps the loads)
}

__global__ __launch_bounds__(256) void k_st9(uint8_t *__restrict__ flags, uint64_t *__restrict__ keys, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        flags[i] = (uint8_t)i;
        keys[i] = mixh((uint64_t)i);
    }
}

__global__ __launch_bounds__(256) void k_atom(unsigned *cur, int64_t n, unsigned long long *sink) {
    unsigned acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        acc += atomicAdd(&cur[(unsigned)(mixh((uint64_t)i) >> 51)], 1u);
    if (acc == 0x12345u) atomicAdd(sink, 1ull);
}

// a bijection of [0, n) for n a multiple of 8192: row i -> bin (i mod 8192), slot (i / 8192): consecutive rows land in
// different bins (the scattered pattern), every slot written once
__global__ __launch_bounds__(256) void k_scat32(uint4 *__restrict__ dst, int64_t n) {
    const int64_t per = n / 8192;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t b = (int64_t)(mixh((uint64_t)(i & 8191)) & 8191), s = i >> 13;
        const int64_t r = b * per + s;
        dst[2 * r] = make_uint4((unsigned)i, 1u, 2u, 3u);
        dst[2 * r + 1] = make_uint4(4u, 5u, 6u, 7u);
    }
}

int main(int argc, char **argv) {
    int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    n = n / 8192 * 8192;
    double *a, *b, *d;
    int64_t *c;
    uint64_t *e, *keys;
    uint8_t *f, *g, *flags;
    unsigned *cur;
    uint4 *dst;
    unsigned long long *sink;
    CHK(hipMalloc(&a, n * 8)); CHK(hipMalloc(&b, n * 8)); CHK(hipMalloc(&c, n * 8)); CHK(hipMalloc(&d, n * 8));
    CHK(hipMalloc(&e, n * 8)); CHK(hipMalloc(&f, n)); CHK(hipMalloc(&g, n)); CHK(hipMalloc(&flags, n));
    CHK(hipMalloc(&keys, n * 8)); CHK(hipMalloc(&cur, 8192 * 4)); CHK(hipMalloc(&dst, n * 32)); CHK(hipMalloc(&sink, 8));
    CHK(hipMemset(a, 1, n * 8)); CHK(hipMemset(b, 2, n * 8)); CHK(hipMemset(c, 3, n * 8)); CHK(hipMemset(d, 4, n * 8));
    CHK(hipMemset(e, 5, n * 8)); CHK(hipMemset(f, 6, n)); CHK(hipMemset(g, 7, n)); CHK(hipMemset(cur, 0, 8192 * 4));
    CHK(hipDeviceSynchronize());
    const int grid = 256 * 6;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_nt8, dim3(grid), dim3(256), 0, 0, a, b, c, d, e, f, g, n, sink);
        hipLaunchKernelGGL(k_st9, dim3(grid), dim3(256), 0, 0, flags, keys, n);
        hipLaunchKernelGGL(k_atom, dim3(grid), dim3(256), 0, 0, cur, n, sink);
        hipLaunchKernelGGL(k_scat32, dim3(grid), dim3(256), 0, 0, dst, n);
    }
    CHK(hipDeviceSynchronize());
    printf("rows %lld: known bytes per dispatch -- k_nt8 read %lld, k_st9 write %lld, k_atom 0 (+%d counter bytes), "
           "k_scat32 write %lld\n", (long long)n, (long long)(42 * n), (long long)(9 * n), 8192 * 4, (long long)(32 * n));
    return 0;
}
