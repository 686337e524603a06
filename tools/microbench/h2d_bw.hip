// Host->device bandwidth on one MI355X, for the host-input boundary:
//   (1) one hipMemcpyAsync of B bytes from pinned memory, (2) the same split over S streams, (3) pageable source,
//   (4) a kernel reading pinned host memory directly (zero-copy, 16-B loads) and writing it to HBM.
// Build: hipcc --offload-arch=gfx950 -O2 -o h2d_bw h2d_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_pull(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

static double time_ms(hipEvent_t a, hipEvent_t b) { float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }

int main(int argc, char **argv) {
    const size_t B = (argc > 1 ? strtoull(argv[1], 0, 10) : 1ull << 30);
    void *h_pin, *d;
    CK(hipHostMalloc(&h_pin, B, hipHostMallocDefault));
    void *h_page = malloc(B);
    memset(h_pin, 1, B);
    memset(h_page, 1, B);
    CK(hipMalloc(&d, B));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<hipStream_t> st(8);
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int rep = 0; rep < 3; rep++) {
        for (int S : {1, 2, 4, 8}) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st[0]));
            for (int s = 1; s < S; s++) CK(hipStreamWaitEvent(st[s], e0, 0));
            const size_t part = B / S;
            for (int s = 0; s < S; s++)
                CK(hipMemcpyAsync((char *)d + s * part, (char *)h_pin + s * part, part, hipMemcpyHostToDevice, st[s]));
            std::vector<hipEvent_t> done(S);
            for (int s = 1; s < S; s++) { CK(hipEventCreate(&done[s])); CK(hipEventRecord(done[s], st[s])); CK(hipStreamWaitEvent(st[0], done[s], 0)); }
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            const double ms = time_ms(e0, e1);
            printf("rep %d pinned memcpy, %d stream(s): %.2f ms  %.1f GB/s\n", rep, S, ms, B / ms / 1e6);
            for (int s = 1; s < S; s++) CK(hipEventDestroy(done[s]));
        }
        CK(hipEventRecord(e0, st[0]));
        CK(hipMemcpyAsync(d, h_page, B, hipMemcpyHostToDevice, st[0]));
        CK(hipEventRecord(e1, st[0]));
        CK(hipEventSynchronize(e1));
        printf("rep %d pageable memcpy: %.2f ms  %.1f GB/s\n", rep, time_ms(e0, e1), B / time_ms(e0, e1) / 1e6);
        for (int grid : {256, 1024, 4096}) {
            CK(hipEventRecord(e0, st[0]));
            hipLaunchKernelGGL(k_pull, dim3(grid), dim3(256), 0, st[0], (const uint4 *)h_pin, (uint4 *)d, B / 16);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            printf("rep %d zero-copy kernel pull, grid %d: %.2f ms  %.1f GB/s\n", rep, grid, time_ms(e0, e1), B / time_ms(e0, e1) / 1e6);
        }
    }
    CK(hipDeviceSynchronize());
    for (auto &s : st) CK(hipStreamDestroy(s));
    CK(hipFree(d));
    CK(hipHostFree(h_pin));
    free(h_page);
    return 0;
}
