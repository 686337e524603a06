// Round 5: where the cost of k_ingest<true>'s binned record writes comes from, and whether per-workgroup slot chunks
// remove it.  1e8 32-B records (read sequentially from a source array, bin = a hash of the index) into 8192 bins:
//   seq        record i -> slot i (the HBM write roofline of the same bytes)
//   direct     a returned atomic on the bin's cursor per record, the record stored there (k_ingest<true> today)
//   atomics    the same atomics, the records stored in order (the atomics' cost alone)
//   pre        the direct pattern's scattered stores into slots reserved by an untimed pass (the stores' cost alone)
//   xcdpre     slots reserved beforehand per (bin, XCD): each sub-slab written from one XCD, so a line's four records
//              meet in that XCD's L2 (whether scattered stores that combine in L2 are cheap)
//   chunk C    persistent 768-lane workgroups (2 per CU) keep, per bin, a chunk of C slots reserved with ONE atomic; a
//              record takes the next slot of its workgroup's chunk with an LDS atomic (chunk full: the lane that finds it
//              full reserves the next chunk, the others retry); unused slots of the last chunks written as holes
//   chunkx C   chunk, with the chunks of a bin reserved per (bin, XCD) (sub-slabs per XCD: a chunk's lines meet in L2)
//   xcddir     direct with a cursor and a sub-slab per (bin, XCD of the executing workgroup): agent-scope atomics
//   xcdl2      xcddir with the cursor atomics at workgroup scope (executed in the XCD's L2, no sc1; each XCD's cursors on
//              lines of their own, cur[x * BINS + bin], touched only by that XCD's workgroups); checked: every slot below
//              each cursor written once, the record ids' sum
// Build: hipcc --offload-arch=gfx950 -O3 -o bin_chunk bin_chunk.hip      Run: ./bin_chunk [n]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#ifndef BINS_N
#define BINS_N 8192
#endif
constexpr int BINS = BINS_N;

__device__ __forceinline__ uint64_t mixh(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}
__device__ __forceinline__ unsigned bin_of(int64_t i) { return (unsigned)(mixh((uint64_t)i) >> (64 - __builtin_ctz(BINS))); }   // log2(BINS) bits
__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 7u; }

__global__ __launch_bounds__(512) void k_seq(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n) {
    for (int64_t j = (int64_t)blockIdx.x * 512 + threadIdx.x; j < 2 * n; j += (int64_t)gridDim.x * 512) dst[j] = src[j];
}

__global__ __launch_bounds__(256) void k_direct(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n,
                                                unsigned *cur, unsigned cap) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        const unsigned s = bin_of(i);
        const unsigned p = atomicAdd(&cur[s], 1u);
        if (p < cap) {
            dst[2 * ((int64_t)s * cap + p)] = a;
            dst[2 * ((int64_t)s * cap + p) + 1] = b;
        }
    }
}

template <bool L2>
__global__ __launch_bounds__(256) void k_xcddir(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n,
                                                unsigned *cur, unsigned cap) {
    const unsigned x = xcc_id();
    unsigned *cx = cur + x * BINS;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        const unsigned s = bin_of(i);
        const unsigned p = L2 ? __hip_atomic_fetch_add(&cx[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                              : atomicAdd(&cx[s], 1u);
        if (p < cap) {
            const int64_t d = ((int64_t)s * 8 + x) * cap + p;
            dst[2 * d] = make_uint4((unsigned)i + 1u, a.y, a.z, a.w);
            dst[2 * d + 1] = b;
        }
    }
}
// check of xcddir/xcdl2: per sub-slab (bin, x), slots [0, min(cur, cap)) hold ids (nonzero), the rest 0; sums of ids
__global__ __launch_bounds__(256) void k_xcdcheck(const uint4 *__restrict__ dst, const unsigned *cur, unsigned cap,
                                                  unsigned long long *out) {
    unsigned long long sum = 0, bad = 0, cnt = 0;
    for (int sb = blockIdx.x; sb < BINS * 8; sb += gridDim.x) {
        const int bin = sb >> 3, x = sb & 7;
        const unsigned c = cur[x * BINS + bin] < cap ? cur[x * BINS + bin] : cap;
        for (unsigned k = threadIdx.x; k < cap; k += 256) {
            const unsigned id = dst[2 * ((int64_t)sb * cap + k)].x;
            if (k < c) { sum += id; cnt++; bad += id == 0; } else bad += id != 0;
        }
    }
    atomicAdd(&out[0], sum);
    atomicAdd(&out[1], bad);
    atomicAdd(&out[2], cnt);
}

__global__ __launch_bounds__(256) void k_atomics(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n,
                                                 unsigned *cur) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        const unsigned p = atomicAdd(&cur[bin_of(i)], 1u);
        dst[2 * i] = make_uint4(a.x, a.y, a.z, p);
        dst[2 * i + 1] = b;
    }
}

// the same patterns with each record stored by two lanes together (lane 2k + h writes half h of record k of the
// round): one 16-B store instruction writes 32 whole 32-B records instead of one 16-B half of 64 records
__device__ __forceinline__ void store_coop(uint4 *__restrict__ dst, int64_t d, uint4 a, uint4 b, bool ok) {
    const int ln = __lane_id();
    const unsigned long long dd = ok ? (unsigned long long)d : ~0ull;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int src = r * 32 + (ln >> 1), h = ln & 1;
        const unsigned long long t = __shfl(dd, src, 64);
        uint4 va, vb;   // (both halves shuffled: the lane keeps the one it stores)
        va.x = __shfl(a.x, src, 64); va.y = __shfl(a.y, src, 64); va.z = __shfl(a.z, src, 64); va.w = __shfl(a.w, src, 64);
        vb.x = __shfl(b.x, src, 64); vb.y = __shfl(b.y, src, 64); vb.z = __shfl(b.z, src, 64); vb.w = __shfl(b.w, src, 64);
        const uint4 v = h ? vb : va;
        if (t != ~0ull) dst[2 * t + h] = v;
    }
}
template <bool PRE>
__global__ __launch_bounds__(256) void k_coop(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n,
                                              unsigned *cur, const unsigned *__restrict__ slot, unsigned cap) {
    for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
        const int64_t i = base + threadIdx.x;
        const bool in = i < n;
        const int64_t j = in ? i : n - 1;
        const uint4 a = src[2 * j], b = src[2 * j + 1];
        unsigned s, p;
        if (PRE) { s = slot[n + j]; p = slot[j]; }
        else { s = bin_of(j); p = in ? atomicAdd(&cur[s], 1u) : cap; }
        store_coop(dst, (int64_t)s * cap + p, a, b, in && p < cap);
    }
}

// slots for the pre-reserved patterns (untimed): sub = 1 -> per bin; 8 -> per (bin, XCD of the executing workgroup)
__global__ __launch_bounds__(256) void k_slots(int64_t n, unsigned *cur, unsigned *slot, int sub) {
    const unsigned x = sub > 1 ? xcc_id() : 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const unsigned s = bin_of(i) * sub + x;
        slot[i] = atomicAdd(&cur[s], 1u);
        slot[n + i] = s;
    }
}
__global__ __launch_bounds__(256) void k_pre(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n,
                                             const unsigned *__restrict__ slot, unsigned cap) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        const unsigned s = slot[n + i], p = slot[i];
        if (p < cap) {
            dst[2 * ((int64_t)s * cap + p)] = a;
            dst[2 * ((int64_t)s * cap + p) + 1] = b;
        }
    }
}

// per-workgroup chunks: LDS word per (sub-)bin = chunk index << 16 | fill; fill == C: full (first finder reserves)
constexpr int CW = 768;
template <int C, bool XCD>
__global__ __launch_bounds__(CW) void k_chunk(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n,
                                              unsigned *chunks, unsigned cap_chunks, unsigned long long *holes) {
    __shared__ unsigned st[BINS];
    for (int b = threadIdx.x; b < BINS; b += CW) st[b] = (0xffffu << 16) | C;   // no chunk yet: "full"
    __syncthreads();
    const unsigned x = XCD ? xcc_id() : 0;
    const int64_t stride = (int64_t)gridDim.x * CW;
    for (int64_t base = (int64_t)blockIdx.x * CW; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        if (i >= n) continue;
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        const unsigned bin = bin_of(i);
        const unsigned sb = XCD ? bin * 8 + x : bin;
        // a wave-uniform loop: each round a lane still without a slot either takes the next slot of its bin's chunk
        // (LDS atomic), or -- the one lane that finds the chunk exactly full -- reserves the next chunk and publishes it,
        // or waits (one LDS read per round) until the chunk index changes; nobody spins inside a divergent branch
        unsigned slot = 0xffffffffu;
        bool done = false, waiting = false;
        unsigned seen = 0;
        while (__ballot(!done)) {
            if (!done) {
                if (waiting) {
                    waiting = (__hip_atomic_load(&st[bin], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >> 16) == seen;
                } else {
                    const unsigned old = atomicAdd(&st[bin], 1u);
                    const unsigned f = old & 0xffffu;
                    if (f < C) {
                        slot = (old >> 16) * C + f;
                        done = true;
                    } else if (f == C) {
                        const unsigned c = atomicAdd(&chunks[sb], 1u);
                        __hip_atomic_store(&st[bin], (c << 16) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        slot = c * C;
                        done = true;
                    } else {
                        waiting = true;
                        seen = old >> 16;
                    }
                }
            }
        }
        if (slot / C < cap_chunks) {
            const int64_t d = (int64_t)sb * cap_chunks * C + slot;
            dst[2 * d] = a;
            dst[2 * d + 1] = b;
        }
    }
    __syncthreads();
    // the unused slots of the last chunks: holes (key word 0)
    unsigned long long h = 0;
    for (int bin = threadIdx.x; bin < BINS; bin += CW) {
        const unsigned s = st[bin], f = s & 0xffffu, c = s >> 16;
        if (f < C && c < cap_chunks) {
            const unsigned sb = XCD ? bin * 8 + x : bin;
            for (unsigned k = f; k < C; k++) {
                dst[2 * ((int64_t)sb * cap_chunks * C + c * C + k)] = make_uint4(0, 0, 0, 0);
                h++;
            }
        }
    }
    atomicAdd(holes, h);
}

__global__ void k_fill(uint4 *p, int64_t n2) {
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n2; j += (int64_t)gridDim.x * 256)
        p[j] = make_uint4((unsigned)(mixh(j) & 0xffffffff) | 1u, 1u, 2u, 3u);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    const char *only = argc > 2 ? argv[2] : "";   // run only the patterns whose name starts with this
    const unsigned cap = (unsigned)(n / BINS + n / BINS / 4 + 256);
    uint4 *src, *dst;
    unsigned *cur, *slot;
    unsigned long long *holes;
    // >= every pattern's slabs (chunk 16: cap + 1024 * 16 slots per bin; per-XCD sub-slabs: 8 x (cap / 8 x 2 + 512))
    const size_t dst_bytes = (size_t)BINS * std::max<size_t>(48000, 2 * (size_t)cap + 8 * 512 + 1024 * 16) * 32;
    CHK(hipMalloc(&src, n * 32));
    CHK(hipMalloc(&dst, dst_bytes));
    CHK(hipMalloc(&cur, BINS * 8 * 4));
    CHK(hipMalloc(&slot, n * 8));
    CHK(hipMalloc(&holes, 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, src, 2 * n);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto timed = [&](auto launch) {
        CHK(hipMemset(cur, 0, BINS * 8 * 4));
        CHK(hipMemset(holes, 0, 8));
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a));
        launch();
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    const int grid = 256 * 16;
    auto want = [&](const char *name) { return strncmp(name, only, strlen(only)) == 0; };
    for (int rep = 0; rep < 2; rep++) {
        if (want("seq")) printf("rep %d seq          %.3f ms\n", rep, timed([&] { hipLaunchKernelGGL(k_seq, dim3(8192), dim3(512), 0, 0, src, dst, n); }));
        if (want("direct")) printf("rep %d direct       %.3f ms\n", rep,
               timed([&] { hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, src, dst, n, cur, cap); }));
        if (want("gridscan"))   // the direct pattern with fewer resident workgroups (k_ingest<true> runs 2 per CU)
            for (int g : {256, 512, 1024, 2048, 4096})
                printf("rep %d gridscan %-5d %.3f ms\n", rep, g,
                       timed([&] { hipLaunchKernelGGL(k_direct, dim3(g), dim3(256), 0, 0, src, dst, n, cur, cap); }));
        if (want("capscan"))   // the direct pattern at slab capacities around the default: alignment of the bins' append points
            for (unsigned d : {0u, 2u, 4u, 6u, 8u, 16u, 32u, 64u, 128u, 256u, 512u, 1000u, 1024u})
                printf("rep %d capscan +%-4u %.3f ms (cap %u)\n", rep, d,
                       timed([&] { hipLaunchKernelGGL(k_direct, dim3(grid), dim3(256), 0, 0, src, dst, n, cur, cap + d); }), cap + d);
        if (want("atomics")) printf("rep %d atomics      %.3f ms\n", rep,
               timed([&] { hipLaunchKernelGGL(k_atomics, dim3(grid), dim3(256), 0, 0, src, dst, n, cur); }));
        for (int l2 = 0; l2 < 2; l2++) {
            if (!want(l2 ? "xcdl2" : "xcddir")) continue;
            const unsigned c = cap / 8 * 2 + 512;
            CHK(hipMemset(dst, 0, (size_t)BINS * 8 * c * 32));
            const float t = timed([&] {
                if (l2) hipLaunchKernelGGL(k_xcddir<true>, dim3(grid), dim3(256), 0, 0, src, dst, n, cur, c);
                else hipLaunchKernelGGL(k_xcddir<false>, dim3(grid), dim3(256), 0, 0, src, dst, n, cur, c);
            });
            unsigned long long *chk;
            CHK(hipMalloc(&chk, 24));
            CHK(hipMemset(chk, 0, 24));
            hipLaunchKernelGGL(k_xcdcheck, dim3(4096), dim3(256), 0, 0, dst, cur, c, chk);
            unsigned long long h[3];
            CHK(hipMemcpy(h, chk, 24, hipMemcpyDeviceToHost));
            CHK(hipFree(chk));
            const unsigned long long want_sum = (unsigned long long)n * (n + 1) / 2;
            printf("rep %d %s       %.3f ms  (records %llu of %lld, bad slots %llu, id sum %s)\n", rep, l2 ? "xcdl2 " : "xcddir", t,
                   h[2], (long long)n, h[1], h[0] == want_sum ? "ok" : "WRONG");
        }
        for (int sub : {1, 8}) {
            if (!want(sub == 1 ? "pre" : "xcdpre")) continue;
            CHK(hipMemset(cur, 0, BINS * 8 * 4));
            hipLaunchKernelGGL(k_slots, dim3(grid), dim3(256), 0, 0, n, cur, slot, sub);
            CHK(hipDeviceSynchronize());
            const unsigned c = sub == 1 ? cap : cap / 8 * 2 + 512;
            const float t = timed([&] { hipLaunchKernelGGL(k_pre, dim3(grid), dim3(256), 0, 0, src, dst, n, slot, c); });
            printf("rep %d %s       %.3f ms\n", rep, sub == 1 ? "pre   " : "xcdpre", t);
        }
        if (want("coop")) {
            printf("rep %d coopdirect   %.3f ms\n", rep,
                   timed([&] { hipLaunchKernelGGL(k_coop<false>, dim3(grid), dim3(256), 0, 0, src, dst, n, cur, slot, cap); }));
            CHK(hipMemset(cur, 0, BINS * 8 * 4));
            hipLaunchKernelGGL(k_slots, dim3(grid), dim3(256), 0, 0, n, cur, slot, 1);
            CHK(hipDeviceSynchronize());
            printf("rep %d cooppre      %.3f ms\n", rep,
                   timed([&] { hipLaunchKernelGGL(k_coop<true>, dim3(grid), dim3(256), 0, 0, src, dst, n, cur, slot, cap); }));
        }
        auto chunk = [&](auto kern, const char *name, int C, bool xcd) {
            if (!want(name)) return;
            const unsigned capc = xcd ? (cap / 8 * 2 + 512) / C : (cap + 2 * 512 * C) / C;
            const float t = timed([&] { hipLaunchKernelGGL(kern, dim3(512), dim3(CW), 0, 0, src, dst, n, cur, capc, holes); });
            unsigned long long h = 0;
            CHK(hipMemcpy(&h, holes, 8, hipMemcpyDeviceToHost));
            unsigned hc[BINS * 8];
            CHK(hipMemcpy(hc, cur, sizeof(hc), hipMemcpyDeviceToHost));
            unsigned long long chunks = 0, mx = 0;
            for (int k = 0; k < BINS * (xcd ? 8 : 1); k++) { chunks += hc[k]; mx = hc[k] > mx ? hc[k] : mx; }
            printf("rep %d %s %2d     %.3f ms  (%llu chunk atomics, %llu holes = %.1f%%, max chunks/bin %llu of %u)\n", rep,
                   name, C, t, chunks, h, 100.0 * h / n, mx, capc);
        };
        chunk(k_chunk<4, false>, "chunk ", 4, false);
        chunk(k_chunk<8, false>, "chunk ", 8, false);
        chunk(k_chunk<16, false>, "chunk ", 16, false);
        chunk(k_chunk<4, true>, "chunkx", 4, true);
        chunk(k_chunk<8, true>, "chunkx", 8, true);
    }
    return 0;
}
