// VALU issue ceiling on MI355X, to read k_ingest's PMC numbers against (VERDICT r3 "What's weak" 4): streams of
// independent VALU instructions of one kind at 1..8 waves per SIMD.  Run under
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -- ./valu_rate
// and compare, per dispatch, SQ_INSTS_VALU / (1024 SIMDs x cycles) (wave-instructions per SIMD-cycle) and
// SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES at saturation with k_ingest's.  The kernel also times itself (hipEvents).
// build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int CHAINS = 8;

// op 0: int32 add/xor; 1: fp64 fma; 2: int64 shift/xor; 3: fp32 fma
template <int OP>
__global__ __launch_bounds__(256) void k_valu(int iters, uint64_t *out) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (OP == 0) {
        unsigned a[CHAINS];
        for (int j = 0; j < CHAINS; j++) a[j] = t * (j + 3);
        for (int i = 0; i < iters; i++)
#pragma unroll
            for (int j = 0; j < CHAINS; j++) a[j] = (a[j] ^ (unsigned)i) + 0x9e3779b9u;
        unsigned r = 0;
        for (int j = 0; j < CHAINS; j++) r ^= a[j];
        if (r == 0x12345678u) out[t] = r;
    } else if constexpr (OP == 1) {
        double a[CHAINS];
        for (int j = 0; j < CHAINS; j++) a[j] = t * 1e-9 + j;
        for (int i = 0; i < iters; i++)
#pragma unroll
            for (int j = 0; j < CHAINS; j++) a[j] = __builtin_fma(a[j], 0.999999, 1e-7);
        double r = 0;
        for (int j = 0; j < CHAINS; j++) r += a[j];
        if (r == 1.2345) out[t] = 1;
    } else if constexpr (OP == 2) {
        uint64_t a[CHAINS];
        for (int j = 0; j < CHAINS; j++) a[j] = (uint64_t)t * (j + 7);
        for (int i = 0; i < iters; i++)
#pragma unroll
            for (int j = 0; j < CHAINS; j++) a[j] = (a[j] << (i & 7)) ^ (a[j] >> 3);
        uint64_t r = 0;
        for (int j = 0; j < CHAINS; j++) r ^= a[j];
        if (r == 0x12345678ull) out[t] = r;
    } else {
        float a[CHAINS];
        for (int j = 0; j < CHAINS; j++) a[j] = t * 1e-6f + j;
        for (int i = 0; i < iters; i++)
#pragma unroll
            for (int j = 0; j < CHAINS; j++) a[j] = __builtin_fmaf(a[j], 0.9999f, 1e-3f);
        float r = 0;
        for (int j = 0; j < CHAINS; j++) r += a[j];
        if (r == 1.2345f) out[t] = 1;
    }
}

template <int OP>
static int run(const char *name, int iters, uint64_t *out, int n_cu) {
    for (int w = 1; w <= 8; w *= 2) {
        const int blocks = n_cu * w;   // 256 threads = 4 waves per block: one per SIMD, w per SIMD
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0));
        CHK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, iters, out);   // warm
        CHK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, iters, out);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-12s waves/SIMD %d: %.3f ms\n", name, w, ms);
        CHK(hipEventDestroy(e0));
        CHK(hipEventDestroy(e1));
    }
    return 0;
}

int main() {
    int dev = 0, n_cu = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    uint64_t *out;
    CHK(hipMalloc(&out, (size_t)n_cu * 8 * 256 * 8));
    const int iters = 20000;
    if (run<0>("int32", iters, out, n_cu) || run<1>("fp64-fma", iters / 4, out, n_cu) ||
        run<2>("int64-shift", iters / 2, out, n_cu) || run<3>("fp32-fma", iters, out, n_cu))
        return 1;
    CHK(hipFree(out));
    return 0;
}
