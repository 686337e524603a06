// mobheat: MI355X-native per-micro-batch hot path of the reference's streaming job.
//
// Pipeline per batch (one HIP stream per context; every arithmetic step runs on the GPU):
//   k_ingest      one pass over the events: filter (heatmap_stream.py:96-104) + H3 latLngToCell UDF
//                 (:65-75,105) + tumbling window (:115) + late-row test against the watermark (:107) + batch
//                 max event time; per-vkey max ts for the dedup (:200-203); LDS hash pre-aggregation of
//                 (cell, windowStart) -> count, n_speed, sum speed/lat/lon into 64-B partial records
//                 (Spark's partial HashAggregate, :112-123)
//   [multi-GPU: partials partitioned by owner rank, exchanged by the caller with RCCL all-to-all]
//   k_census      partials per window -> sizes each window's state table (kernels.h: GenDesc); on one GPU
//                 k_ingest counts its own partials and this pass is skipped
//   k_rp_*        radix partition of the partials into one bin per (window, table region)
//   k_merge_owned one workgroup per bin merges its partials into the persistent per-window state tables
//                 (update mode, :243; Spark's StateStoreRestore/Save) with the regions' slot tags in LDS, and
//                 writes each touched key's cumulative output row (:124-132) into the bin's row segment
//   k_fill_gaps     the per-bin row segments -> dense update-mode rows (in place: gap rows filled from the tail)
//   eviction      (watermark, :107) releases a window's whole table; k_dump_gen + a rehash merge grow one
//   k_dedup_flag  latest position per (provider, vehicleId): rows whose ts equals the max (:204-207)
//
// Semantics follow SURVEY.md App. A (Spark 3.5.1): see DESIGN.md for the rules and their provenance.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <ctime>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/mobheat.h"
#include "kernels.h"
#include "bson_docs.h"
#include "json_decode.h"
#include "h3_boundary.h"
#include <chrono>
#include <mutex>

#define H3T_CONST static const
#include "h3_tables.inc"

using namespace hm;

__constant__ H3Tables c_tab;
// glibc's sincos/acos/atan2/tan tables for the exact path (glibc_libm.h); c_tab.glm points here
__device__ glm::Tables g_glm = {GLM_TABLE_INIT};   // (not const: a const namespace-scope symbol has internal linkage, which hipGetSymbolAddress cannot resolve)

#include "h3_tables_host.h"
static H3Tables make_tables() { return hm_make_tables(); }
// c_tab of the current device, its glibc table pointer aimed at the device copy
static hipError_t upload_tables() {
    H3Tables T = make_tables();
    void *g = nullptr;
    hipError_t e = hipGetSymbolAddress(&g, HIP_SYMBOL(g_glm));
    if (e != hipSuccess) return e;
    T.glm = (const glm::Tables *)g;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &T, sizeof(T));
}

// =====================================================================================================
// wave helpers
// =====================================================================================================
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ long long wave_max(long long v) {
    for (int o = 32; o > 0; o >>= 1) { long long w = __shfl_xor(v, o, 64); v = w > v ? w : v; }
    return v;
}
// exclusive prefix of v over a workgroup of 1024 threads (wave scans by shuffles, one LDS round for the 16 wave
// totals: two barriers instead of the 20 of a Hillis-Steele scan in LDS); *total = the sum over the workgroup
__device__ __forceinline__ unsigned long long block1024_exclusive(unsigned long long v, unsigned long long *total) {
    __shared__ unsigned long long wtot[16];
    const int ln = lane_id(), w = threadIdx.x >> 6;
    unsigned long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o, 64);
        if (ln >= o) x += y;
    }
    if (ln == 63) wtot[w] = x;
    __syncthreads();
    if (w == 0) {
        unsigned long long t = ln < 16 ? wtot[ln] : 0;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const unsigned long long y = __shfl_up(t, o, 64);
            if (ln >= o) t += y;
        }
        if (ln < 16) wtot[ln] = t;
    }
    __syncthreads();
    *total = wtot[15];
    return x - v + (w ? wtot[w - 1] : 0ull);
}
__device__ __forceinline__ long long wave_min(long long v) {
    for (int o = 32; o > 0; o >>= 1) { long long w = __shfl_xor(v, o, 64); v = w < v ? w : v; }
    return v;
}
// Wave-aggregated append: returns this lane's slot index (valid only where pred), one atomic per wave.
__device__ __forceinline__ unsigned long long wave_append(bool pred, unsigned long long *counter) {
    unsigned long long m = __ballot(pred);
    unsigned long long base = 0;
    if (m) {
        int leader = __ffsll((long long)m) - 1;
        if (lane_id() == leader) base = atomicAdd(counter, (unsigned long long)__popcll(m));
        base = __shfl(base, leader, 64);
    }
    unsigned long long below = m & ((UINT64_C(1) << lane_id()) - 1);
    return base + __popcll(below);
}

// =====================================================================================================
// K3: per-window state tables (kernels.h: GenDesc) -- lookup, census, growth dump
// =====================================================================================================
__device__ __forceinline__ int gmap_find(const GenDesc *gm, unsigned long long we) {
    unsigned h = (unsigned)(mix64(we) & (GMAP_SLOTS - 1));
    for (int probe = 0; probe < GMAP_SLOTS; probe++) {
        const unsigned long long w = gm[h].wenc;
        if (w == we) return (int)h;
        if (w == 0) return -1;
        h = (h + 1) & (GMAP_SLOTS - 1);
    }
    return -1;
}
__device__ __forceinline__ unsigned long long home_slot(const GenDesc &g, uint64_t h) {
    return ((unsigned long long)(region_field(h) >> (REGION_BITS - g.rbits)) << g.rshift) | (h & g.rmask);
}
// linear probing wraps inside the key's region
__device__ __forceinline__ unsigned long long next_slot(unsigned long long s, unsigned long long rmask) {
    return (s & ~rmask) | ((s + 1) & rmask);
}

// LDS copy of the live windows' table descriptors (a batch touches a few windows; the global map is the
// fallback when there are more than GC_MAX)
constexpr int GC_MAX = 32;
constexpr int GC_IDX = 64;   // open-addressing index over the cached descriptors
struct GenCache {
    GenDesc e[GC_MAX];
    signed char idx[GC_IDX];   // -1 = empty
    int n;   // -1: use the global map
};
__device__ __forceinline__ unsigned gc_home(unsigned long long we) {
    return (unsigned)((we * UINT64_C(0x9e3779b97f4a7c15)) >> 58);   // 6 bits
}
// (callers __syncthreads() before the first lookup)
__device__ __forceinline__ void gc_load(GenCache &C, const GenDesc *glist, int n) {
    if (threadIdx.x == 0) {
        C.n = n <= GC_MAX ? n : -1;
        for (int q = 0; q < GC_IDX; q++) C.idx[q] = -1;
        if (n <= GC_MAX)
            for (int q = 0; q < n; q++) {
                unsigned h = gc_home(glist[q].wenc);
                while (C.idx[h] >= 0) h = (h + 1) & (GC_IDX - 1);
                C.idx[h] = (signed char)q;
            }
    }
    if (n <= GC_MAX)
        for (int q = threadIdx.x; q < n; q += blockDim.x) C.e[q] = glist[q];
}
__device__ __forceinline__ const GenDesc *gen_lookup(const GenCache &C, const GenDesc *gm, unsigned long long we) {
    if (C.n >= 0) {
        unsigned h = gc_home(we);
        for (int p = 0; p < GC_IDX; p++) {
            const int i = C.idx[h];
            if (i < 0) return nullptr;
            if (C.e[i].wenc == we) return &C.e[i];
            h = (h + 1) & (GC_IDX - 1);
        }
        return nullptr;
    }
    const int g = gmap_find(gm, we);
    return g < 0 ? nullptr : &gm[g];
}
// radix bin of a key (hash h): every partial of one (window, region) lands in one bin; -1 if the window has no table
__device__ __forceinline__ int bin_of_c(const GenCache &C, const GenDesc *gm, uint64_t h, int64_t w) {
    const unsigned long long we = wenc_of(w);
    const GenDesc *g = gen_lookup(C, gm, we);
    if (!g) return -1;
    const unsigned sb = REGION_BITS - g->rbits;
    const unsigned reg = region_field(h) >> sb;
    return (int)((reg << sb) | (window_salt(we) & ((1u << sb) - 1)));
}

// census map: partial count per window (open addressing; counts added by one atomic per window per workgroup)
__device__ __forceinline__ bool wmap_add(WinCount *m, unsigned long long we, unsigned long long cnt) {
    unsigned h = (unsigned)(mix64(we) & (GMAP_SLOTS - 1));
    for (int probe = 0; probe < GMAP_SLOTS; probe++) {
        unsigned long long cur = __hip_atomic_load(&m[h].wenc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == 0) cur = atomicCAS(&m[h].wenc, 0ull, we);
        if (cur == 0 || cur == we) {
            atomicAdd(&m[h].count, cnt);
            return true;
        }
        h = (h + 1) & (GMAP_SLOTS - 1);
    }
    return false;
}
// created keys -> the window's table key count
__device__ __forceinline__ bool gmap_add(GenDesc *gm, unsigned long long we, unsigned long long cnt) {
    const int g = gmap_find(gm, we);
    if (g < 0) return false;
    atomicAdd(&gm[g].count, cnt);
    return true;
}
struct CensusSink {
    WinCount *m;
    __device__ bool add(unsigned long long we, unsigned long long c) const { return wmap_add(m, we, c); }
};
struct GenSink {
    GenDesc *m;
    __device__ bool add(unsigned long long we, unsigned long long c) const { return gmap_add(m, we, c); }
};
// Per-workgroup window counts in LDS, flushed to the global map once per workgroup: a batch touches only a
// few windows, so per-wave global adds would all hit the same few counters.
constexpr int WL_SLOTS = 32;
struct WinLds {
    unsigned long long key[WL_SLOTS];
    unsigned long long cnt[WL_SLOTS];
};
__device__ __forceinline__ void wl_init(WinLds &L) {
    for (int q = threadIdx.x; q < WL_SLOTS; q += blockDim.x) { L.key[q] = 0; L.cnt[q] = 0; }
}
template <class Sink>
__device__ __forceinline__ bool wl_add(WinLds &L, const Sink &g, unsigned long long we, unsigned long long c) {
    unsigned h = (unsigned)(mix64(we) & (WL_SLOTS - 1));
    for (int probe = 0; probe < WL_SLOTS; probe++) {
        unsigned long long o = atomicCAS(&L.key[h], 0ull, we);
        if (o == 0 || o == we) { atomicAdd(&L.cnt[h], c); return true; }
        h = (h + 1) & (WL_SLOTS - 1);
    }
    return g.add(we, c);   // more distinct windows than LDS slots: straight to the global map
}
// after a __syncthreads(): one lane per LDS slot adds its count to the global map
template <class Sink>
__device__ __forceinline__ bool wl_flush(WinLds &L, const Sink &g) {
    bool ok = true;
    for (int q = threadIdx.x; q < WL_SLOTS; q += blockDim.x)
        if (L.key[q]) ok &= g.add(L.key[q], L.cnt[q]);
    return ok;
}
// wave-cooperative: lanes with `pred` add `c` each to their window's count (one LDS add per window per wave)
template <class Sink>
__device__ __forceinline__ bool wave_count_windows(bool pred, unsigned long long we, unsigned long long c, WinLds &L,
                                                   const Sink &g) {
    bool ok = true;
    while (true) {
        unsigned long long pend = __ballot(pred);
        if (!pend) break;
        int leader = __ffsll((long long)pend) - 1;
        unsigned long long wl = __shfl(we, leader, 64);
        bool match = pred && we == wl;
        unsigned long long sum = 0;
        {
            unsigned long long v = match ? c : 0;
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            sum = v;
        }
        if (lane_id() == leader) ok = wl_add(L, g, wl, sum);
        pred = pred && !match;
    }
    return ok;
}

// =====================================================================================================
// K1: latLngToCell.  The per-event kernels run latLngToCellFast (h3_device.h: direct gnomonic projection,
// ~60 VGPRs) and append the rare events whose decision margins are below the error bound to an exception
// list; a second kernel runs upstream's exact sequence (latLngToCellDeg, ~170 VGPRs) on that list only, so
// the register footprint of the exact path never limits the occupancy of the streaming kernel.
// =====================================================================================================
// waves per SIMD for k_ingest: 6 (<= 80 VGPRs, no spills; the 512-slot LDS table allows 6 workgroups per CU)
#ifndef HM_SNAP_WAVES
#define HM_SNAP_WAVES 6
#endif
#if HM_SNAP_WAVES > 0
#define HM_SNAP_ATTR __attribute__((amdgpu_waves_per_eu(HM_SNAP_WAVES)))
#else
#define HM_SNAP_ATTR
#endif
// standalone UDF: cells only (hm_latlng_to_cell); exceptions -> slow[]
__global__ __launch_bounds__(256) void k_cells(const double *__restrict__ lat, const double *__restrict__ lon, int64_t n,
                                               int res, uint64_t *__restrict__ out, unsigned int *__restrict__ slow,
                                               unsigned long long *n_slow) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool exc = false;
        if (i < n) {
            uint64_t c;
            exc = !latLngToCellFast(lat[i], lon[i], res, c_tab, c);
            out[i] = c;
        }
        const unsigned long long pos = wave_append(exc, n_slow);
        if (exc) slow[pos] = (unsigned int)i;
    }
}
__global__ __launch_bounds__(256) void k_cells_exact(const double *__restrict__ lat, const double *__restrict__ lon,
                                                     int res, uint64_t *__restrict__ out, const unsigned int *__restrict__ slow,
                                                     const unsigned long long *n_slow) {
    const int64_t m = (int64_t)*n_slow;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
        const unsigned i = slow[q];
        out[i] = latLngToCellDeg(lat[i], lon[i], res, c_tab);
    }
}

// =====================================================================================================
// K2: the batch's window registry.  Every window a batch aggregates into gets a slot (its index widx, kept in
// the rows' event keys, kernels.h ekey); a workgroup caches the windows it has seen in LDS.
// =====================================================================================================
// registry slot of window quotient wq (enc = wenc of its start); -1 when the registry is full
__device__ __forceinline__ int wreg_find(unsigned long long *reg, int64_t wq, unsigned long long enc) {
    unsigned h = (unsigned)((uint64_t)wq % (uint64_t)WREG_SLOTS);   // consecutive windows -> consecutive slots
    for (int p = 0; p < WREG_SLOTS; p++) {
        // a stale (L2) copy can only show a slot empty: the CAS then returns its owner
        unsigned long long cur = __hip_atomic_load(&reg[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == 0) cur = atomicCAS(&reg[h], 0ull, enc);
        if (cur == 0 || cur == enc) return (int)h;
        h = h + 1 == (unsigned)WREG_SLOTS ? 0u : h + 1;
    }
    return -1;
}
// per-workgroup cache of registry slots: one word per entry, ((wq mod 2^52) << 12) | (widx + 1), 0 = empty, so that
// one CAS publishes both (hm_create requires tile_us >= 1 s: |wq| < 2^44, so wq mod 2^52 identifies the window)
constexpr int WC_SLOTS = 32;
struct WinCacheL {
    unsigned long long e[WC_SLOTS];
    unsigned cnt[WC_SLOTS];   // aggregated rows per cached window (the direct path's census)
};
__device__ __forceinline__ void wc_init(WinCacheL &C) {
    for (int q = threadIdx.x; q < WC_SLOTS; q += blockDim.x) { C.e[q] = 0; C.cnt[q] = 0; }
}
// widx of window wq (-1: registry full); slot = its cache entry (-1: the cache is full)
__device__ __forceinline__ int wc_lookup(WinCacheL &C, unsigned long long *reg, int64_t wq, unsigned long long enc, int &slot) {
    const unsigned long long tag = (uint64_t)wq & CELL_LO;
    unsigned h = (unsigned)wq & (WC_SLOTS - 1);
    int w = -2;
    for (int p = 0; p < WC_SLOTS; p++) {
        unsigned long long c = __hip_atomic_load(&C.e[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (c == 0) {
            if (w == -2) w = wreg_find(reg, wq, enc);
            if (w < 0) { slot = -1; return -1; }
            c = atomicCAS(&C.e[h], 0ull, (tag << 12) | (unsigned long long)(w + 1));
            if (c == 0) { slot = (int)h; return w; }
        }
        if ((c >> 12) == tag) { slot = (int)h; return (int)(c & 0xfff) - 1; }
        h = (h + 1) & (WC_SLOTS - 1);
    }
    slot = -1;
    return w == -2 ? wreg_find(reg, wq, enc) : w;
}

// census of a batch's partials per window (sizes the window tables before the merge)
__global__ __launch_bounds__(256) void k_census(const TilePartial *__restrict__ parts, int64_t n, WinCount *cmap, DevStats *st) {
    __shared__ WinLds WL;
    wl_init(WL);
    __syncthreads();
    const CensusSink sink{cmap};
    bool ok = true;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        const bool in = i < n;
        const unsigned long long we = in ? wenc_of(parts[i].wstart) : 0;
        ok &= wave_count_windows(in, we, 1ull, WL, sink);
    }
    __syncthreads();
    ok &= wl_flush(WL, sink);
    if (__ballot(!ok) && lane_id() == 0) atomicAdd(&st->overflow, 1ull);
}

// growth: the live keys of one window's old table as partial records (aux = the key's touched word), to be
// merged into its new table by k_merge_owned in rehash mode
// (only_seq != 0: only the keys whose touched word carries that batch sequence -- an incremental checkpoint)
__global__ __launch_bounds__(256) void k_dump_gen(GenDesc g, GrowRec *__restrict__ out, unsigned long long *n_out,
                                                  unsigned only_seq = 0) {
    const unsigned long long cap = (g.rmask + 1) << g.rbits;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < (int64_t)cap; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool live = false;
        GrowRec p;
        if (i < (int64_t)cap) {
            const TileSlot sl = g.tab[i];
            live = sl.wenc == g.wenc && (only_seq == 0 || (unsigned)(sl.touched >> 32) == only_seq);
            p.cell = sl.cell;
            p.wstart = wdec(sl.wenc);
            p.count = sl.count;
            p.nspeed = sl.nspeed;
            p.sspeed = sl.sspeed;
            p.slat = sl.slat;
            p.slon = sl.slon;
            p.touched = sl.touched;
        }
        const unsigned long long pos = wave_append(live, n_out);
        if (live) out[pos] = p;
    }
}

// =====================================================================================================
// K2b: radix partition of the partials into RP_BINS bins (kernels.h: one bin per (window, region)), so that
// one merge workgroup owns each region: tile histogram (LDS) -> digit-major exclusive scan -> LDS-cursor
// scatter.  Records are one 64-B line each, so the scattered writes are whole lines.
// =====================================================================================================
constexpr int RP_BITS = REGION_BITS;
constexpr int RP_BINS = 1 << RP_BITS;
#ifndef HM_RP_TILE
#define HM_RP_TILE 131072
#endif
constexpr int RP_TILE = HM_RP_TILE;    // partials per tile (one workgroup) at most
// records per tile for n records: RP_TILE for large partitions, smaller ones so that a small partition (table mode's
// partials, a stage merge) still spreads over the CUs (every tile writes a full histogram: at least 4096 records)
static inline int64_t rp_tile_for(int64_t n) {
    int64_t t = 4096;
    while (t < RP_TILE && t * 512 < n) t <<= 1;
    return t;
}
constexpr int RP_THREADS = 256;

// the radix digit of a key: its (window, region) bin, or with nranks > 0 its owner rank (the multi-GPU
// exchange, hm_stage_local)
__device__ __forceinline__ unsigned rp_digit(uint64_t cell, int64_t ws, const GenCache &C, const GenDesc *gm, int nranks,
                                             bool &bad) {
    const uint64_t h = tile_hash(cell, ws);
    if (nranks > 0) return (unsigned)owner_of(h, nranks);
    const int b = bin_of_c(C, gm, h, ws);
    bad |= b < 0;
    return b < 0 ? 0u : (unsigned)b;
}

template <typename Rec>
__global__ __launch_bounds__(RP_THREADS) void k_rp_hist(const Rec *__restrict__ parts, int64_t n, int64_t tile, const GenDesc *gm,
                                                       const GenDesc *glist, int n_glist, int nranks, int nbins,
                                                       unsigned *__restrict__ H, int64_t ntiles, DevStats *st) {
    __shared__ unsigned h[RP_BINS + 1];
    __shared__ GenCache C;
    gc_load(C, glist, n_glist);
    for (int d = threadIdx.x; d <= RP_BINS; d += RP_THREADS) h[d] = 0;
    __syncthreads();
    int64_t t0 = (int64_t)blockIdx.x * tile;
    int64_t t1 = t0 + tile < n ? t0 + tile : n;
    bool bad = false;
    unsigned gaps = 0;   // gaps (cell 0) count in the extra digit nbins, after every bin
    for (int64_t i = t0 + threadIdx.x; i < t1; i += RP_THREADS) {
        const uint64_t cell = parts[i].cell;
        if (cell == EMPTY_CELL) gaps++;
        else atomicAdd(&h[rp_digit(cell, parts[i].wstart, C, gm, nranks, bad)], 1u);
    }
    gaps = (unsigned)wave_sum((unsigned long long)gaps);
    if (gaps && lane_id() == 0) atomicAdd(&h[nbins], gaps);
    __syncthreads();
    for (int d = threadIdx.x; d <= nbins; d += RP_THREADS) H[(int64_t)d * ntiles + blockIdx.x] = h[d];
    if (__ballot(bad) && lane_id() == 0) atomicAdd(&st->overflow, 1ull);
}

// exclusive scan of m u32 entries into u64 offsets, 3 phases; block size 1024, 4096 entries per block
constexpr int SC_PER = 4096;
__global__ __launch_bounds__(1024) void k_scan_blocks(const unsigned *__restrict__ in, int64_t m, unsigned long long *__restrict__ out,
                                                      unsigned *__restrict__ block_tot) {
    int64_t b0 = (int64_t)blockIdx.x * SC_PER + (int64_t)threadIdx.x * 4;
    unsigned v[4];
    unsigned long long sum = 0;
    for (int q = 0; q < 4; q++) { v[q] = (b0 + q < m) ? in[b0 + q] : 0u; sum += v[q]; }
    unsigned long long tot;
    unsigned long long run = block1024_exclusive(sum, &tot);
    for (int q = 0; q < 4; q++) {
        if (b0 + q < m) out[b0 + q] = run;
        run += v[q];
    }
    if (threadIdx.x == 1023) block_tot[blockIdx.x] = (unsigned)tot;
}
// first offset of each digit (the owner partition's per-rank segment starts)
__global__ void k_digit_starts(const unsigned long long *__restrict__ O, int64_t ntiles, int nbins, unsigned long long *out) {
    for (int d = threadIdx.x; d < nbins; d += blockDim.x) out[d] = O[(int64_t)d * ntiles];
}
__global__ __launch_bounds__(256) void k_scan_add(unsigned long long *__restrict__ out, int64_t m,
                                                  const unsigned long long *__restrict__ block_off) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) out[i] += block_off[i / SC_PER];
}

// HM_NT_STORES bit 0: the partition scatter's 16-B stores non-temporal; bit 1: the merge's output rows (both written
// once, read by the next kernel from HBM)
#ifndef HM_NT_STORES
#define HM_NT_STORES 0
#endif
typedef unsigned hm_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_stream(uint4 *p, uint4 v) {
    if constexpr ((HM_NT_STORES & 1) != 0) {
        const hm_v4u w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (hm_v4u *)p);
    } else {
        *p = v;
    }
}

// bit 2: the merge's partitioned records loaded non-temporal (each is read once)
template <typename Rec>
__device__ __forceinline__ Rec ld_stream(const Rec *p) {
    if constexpr ((HM_NT_STORES & 4) != 0 && sizeof(Rec) % 16 == 0) {
        Rec r;
        const hm_v4u *s = (const hm_v4u *)p;
        hm_v4u *d = (hm_v4u *)&r;
#pragma unroll
        for (int q = 0; q < (int)(sizeof(Rec) / 16); q++) d[q] = __builtin_nontemporal_load(s + q);
        return r;
    } else {
        return *p;
    }
}

// output part q (16 B) of record `rec` of a wave's 64: In = Out is a plain copy; TilePartial (48 B) -> SortedRec
// (64 B) widens the counts and appends the key hash the digit lane computed
template <typename In, typename Out>
__device__ __forceinline__ uint4 rp_part(const uint4 *__restrict__ src, int64_t rec, int q, uint64_t h) {
    if constexpr (std::is_same<In, Out>::value) {
        return src[rec * (sizeof(In) / 16) + q];
    } else {
        static_assert(std::is_same<In, TilePartial>::value && std::is_same<Out, SortedRec>::value, "conversion");
        const uint4 *r = src + rec * 3;
        if (q == 0) return r[0];
        if (q == 1) { const uint4 a = r[1]; return make_uint4(a.x, 0u, a.y, 0u); }
        if (q == 2) { const uint4 a = r[1], b = r[2]; return make_uint4(a.z, a.w, b.x, b.y); }
        const uint4 b = r[2];
        return make_uint4(b.z, b.w, (unsigned)h, (unsigned)(h >> 32));
    }
}

// Per wave and iteration, 64 records: each lane reads its record's first 16 B (cell, window start) and takes its
// digit and position (all lanes busy with the hash); then the wave writes the 64 records as sizeof(Out)/16 rounds
// of 16-B parts, whole 64-B lines at random places -- per-lane 64-B records bounded this kernel's vector-memory
// issue (6.4 -> 3.5 ms per 1e8 records).
template <typename In, typename Out>
__global__ __launch_bounds__(RP_THREADS) void k_rp_scatter(const In *__restrict__ parts, int64_t n, int64_t tile,
                                                          const GenDesc *gm, const GenDesc *glist, int n_glist,
                                                          int nranks, int nbins, const unsigned long long *__restrict__ O,
                                                          int64_t ntiles, Out *__restrict__ dst) {
    constexpr int QI = sizeof(In) / 16, QO = sizeof(Out) / 16;
    constexpr bool widen = !std::is_same<In, Out>::value;
    __shared__ unsigned cur[RP_BINS];   // positions < 2^32 - 1 (partition() checks n)
    __shared__ GenCache C;
    __shared__ uint4 stage[widen ? (RP_THREADS / 64) * 64 * QI : 1];   // widening: each wave's 64 input records
    gc_load(C, glist, n_glist);
    for (int d = threadIdx.x; d < nbins; d += RP_THREADS) cur[d] = (unsigned)O[(int64_t)d * ntiles + blockIdx.x];
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * tile;
    const int64_t t1 = t0 + tile < n ? t0 + tile : n;
    const uint4 *__restrict__ src = (const uint4 *)parts;
    uint4 *__restrict__ d4 = (uint4 *)dst;
    const int ln = lane_id();
    for (int64_t i0 = t0 + (int64_t)(threadIdx.x >> 6) * 64; i0 < t1; i0 += RP_THREADS) {
        const int64_t i = i0 + ln;
        unsigned pos = ~0u;   // ~0u: a gap (cell 0), not moved (its digit nbins lies after every bin)
        uint64_t h = 0;
        if (i < t1) {
            const uint4 k = src[i * QI];   // part 0 = (cell, window start)
            const uint64_t cell = (uint64_t)k.x | ((uint64_t)k.y << 32);
            const int64_t ws = (int64_t)((uint64_t)k.z | ((uint64_t)k.w << 32));
            if (cell != EMPTY_CELL) {
                h = tile_hash(cell, ws);
                unsigned d;
                if (nranks > 0) {
                    d = (unsigned)owner_of(h, nranks);
                } else {
                    const int b = bin_of_c(C, gm, h, ws);
                    d = b < 0 ? 0u : (unsigned)b;   // (k_rp_hist flagged it)
                }
                pos = atomicAdd(&cur[d], 1u);
            }
        }
        const int64_t nrec = t1 - i0 < 64 ? t1 - i0 : 64;
        if constexpr (widen) {
            // the wave's records through LDS: QI contiguous 1-KB loads in, then each lane builds output parts
            uint4 *ws = stage + (threadIdx.x >> 6) * 64 * QI;
            for (int r = 0; r < QI; r++) {
                const int idx = r * 64 + ln;
                if (idx < nrec * QI) ws[idx] = src[i0 * QI + idx];
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            for (int r = 0; r < QO; r++) {
                const int idx = r * 64 + ln, rec = idx / QO, q = idx % QO;
                const unsigned p = __shfl(pos, rec, 64);
                const unsigned hl = __shfl((unsigned)h, rec, 64), hh = __shfl((unsigned)(h >> 32), rec, 64);
                if (rec < nrec && p != ~0u) st_stream(&d4[(int64_t)p * QO + q], rp_part<In, Out>(ws, rec, q, (uint64_t)hl | ((uint64_t)hh << 32)));
            }
            __builtin_amdgcn_wave_barrier();
        } else {
            for (int r = 0; r < QO; r++) {
                const int idx = r * 64 + ln, rec = idx / QO, q = idx % QO;
                const unsigned p = __shfl(pos, rec, 64);
                if (rec < nrec && p != ~0u) st_stream(&d4[(int64_t)p * QO + q], src[(i0 + rec) * QI + q]);
            }
        }
    }
}

// =====================================================================================================
// K2c: radix partition of the direct path: the batch's event keys (8 B per row) -> EventRecs (32 B) in
// (window, region) bins, or (multi-GPU) 48-B TilePartials grouped by owner rank.  The histogram reads only the
// keys; the scatter reads a record's speed/lat/lon only for aggregated rows.
// =====================================================================================================
// LDS copy of the host's WInfo image (kernels.h WiCacheImg), stored right after the per-slot array
struct WiCacheL {
    unsigned tag[WI_CACHE];
    WInfo e[WI_CACHE];
};
__device__ __forceinline__ void wi_load(WiCacheL &C, const WInfo *winfo) {   // (a barrier must follow)
    const WiCacheImg *img = (const WiCacheImg *)(winfo + WREG_SLOTS + 1);
    for (int q = threadIdx.x; q < WI_CACHE; q += blockDim.x) {
        C.tag[q] = img->tag[q];
        C.e[q] = img->e[q];
    }
}
// Before a software-pipelined loop (the next round's columns loaded while this round computes): wait for the first
// round's loads.  Without it the compiler's wait-count pass merges, at the loop header, the preheader's pending loads
// into the registers the loop's back edge fills by copies, and then waits inside every round until only a few loads
// are in flight -- i.e. for the next round's prefetch too (the vector memory counter retires in order).
__device__ __forceinline__ void preheader_wait() { __builtin_amdgcn_s_waitcnt(0); }

// A miss reads the registry in HBM and waits for it inside the miss branch (relaxed atomic loads: a plain load would
// be folded with the LDS read into one flat load of a selected address, whose wait -- vmcnt(0) after every row --
// also waited for the next round's prefetched columns).
__device__ __forceinline__ WInfo wi_get(const WiCacheL &C, const WInfo *winfo, unsigned slot) {
    const unsigned e = slot & (WI_CACHE - 1);
    WInfo w = C.e[e];
    if (C.tag[e] != slot) {
        static_assert(sizeof(WInfo) % 8 == 0, "WInfo: 8-B words");
        const unsigned long long *g = (const unsigned long long *)&winfo[slot];
        unsigned long long *d = (unsigned long long *)&w;
#pragma unroll
        for (int q = 0; q < (int)(sizeof(WInfo) / 8); q++) d[q] = __hip_atomic_load(&g[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0);
    }
    return w;
}

// the key's radix digit: with nranks > 0 its owner rank, else its (window, region) bin (binp: kernels.h WInfo)
__device__ __forceinline__ unsigned ev_digit(uint64_t h, unsigned binp, int nranks) {
    if (nranks > 0) return (unsigned)owner_of(h, nranks);
    const unsigned sb = binp >> 24;
    return ((region_field(h) >> sb) << sb) | (binp & 0xffffffu);
}

constexpr int EV_THREADS = 512;
__global__ __launch_bounds__(EV_THREADS) void k_ev_hist(const uint64_t *__restrict__ keys, int64_t n, int64_t tile,
                                                       const WInfo *__restrict__ winfo, uint64_t cell_hi, int nranks, int nbins,
                                                       unsigned *__restrict__ H, int64_t ntiles) {
    __shared__ unsigned h[RP_BINS + 1];
    __shared__ WiCacheL WI;
    for (int d = threadIdx.x; d <= nbins; d += EV_THREADS) h[d] = 0;
    wi_load(WI, winfo);
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * tile;
    const int64_t t1 = t0 + tile < n ? t0 + tile : n;
    unsigned gaps = 0;   // rows without a key count in the extra digit nbins, after every bin
    constexpr int U = 8;   // loads in flight per lane
    for (int64_t b = t0 + threadIdx.x; b < t1; b += (int64_t)EV_THREADS * U) {
        uint64_t k[U];
#pragma unroll
        for (int u = 0; u < U; u++) k[u] = b + u * EV_THREADS < t1 ? __builtin_nontemporal_load(&keys[b + u * EV_THREADS]) : 0;
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (b + u * EV_THREADS >= t1) continue;
            if (!k[u]) { gaps++; continue; }
            const WInfo wi = wi_get(WI, winfo, ekey_widx(k[u]));
            const uint64_t hh = mix64(((k[u] & CELL_LO) | cell_hi) ^ wi.inner);
            atomicAdd(&h[ev_digit(hh, wi.binp, nranks)], 1u);
        }
    }
    gaps = (unsigned)wave_sum((unsigned long long)gaps);
    if (gaps && lane_id() == 0) atomicAdd(&h[nbins], gaps);
    __syncthreads();
    for (int d = threadIdx.x; d <= nbins; d += EV_THREADS) H[(int64_t)d * ntiles + blockIdx.x] = h[d];
}

// the direct path's multi-GPU wire format (hm_stage_send): a key stream (8 B per row: the cell's low 52 bits | 1 + the
// batch's GLOBAL window slot << 52) and a payload stream (24 B: speed bits as in EventRec, lat, lon), both grouped by
// owner rank; the owner partitions them into EventRecs (k_ev_scatter with payload_in)
struct WireKey {
    uint64_t key;
};
constexpr int WIRE_PAYLOAD_WORDS = 3;

// Per wave and round, 64 rows: each lane takes its row's digit and position (LDS cursor) and builds its record in
// LDS; then the wave writes the 64 records as rounds of 16-B parts, consecutive lanes covering consecutive parts of
// one record (whole 32-B sectors at random places).
//   Out = EventRec: the direct path's (window, region) bins; the row's speed/lat/lon come from the batch's columns,
//         or (payload_in, the multi-GPU owner) from the received payload stream;
//   Out = WireKey:  grouped by owner rank into the caller's key and payload streams (payload_out), the key's window
//         slot rewritten from the rank's registry to the batch's global registry (WInfo.gslot).
template <typename Out>
__global__ __launch_bounds__(EV_THREADS) void k_ev_scatter(const uint64_t *__restrict__ keys, int64_t n, int64_t tile,
                                                          const double *__restrict__ speed, const uint8_t *__restrict__ speed_valid,
                                                          const double *__restrict__ lat, const double *__restrict__ lon,
                                                          const uint64_t *__restrict__ payload_in,
                                                          const WInfo *__restrict__ winfo, uint64_t cell_hi, int nranks, int nbins,
                                                          const unsigned long long *__restrict__ O, int64_t ntiles,
                                                          Out *__restrict__ dst, uint64_t *__restrict__ payload_out) {
    constexpr bool wire = std::is_same<Out, WireKey>::value;
    static_assert(wire || std::is_same<Out, EventRec>::value, "k_ev_scatter output");
    constexpr int QO = wire ? 1 : sizeof(Out) / 16;
    __shared__ unsigned cur[RP_BINS];   // positions < 2^32 - 1 (hm_process_batch checks n)
    __shared__ uint4 stage[wire ? 1 : (EV_THREADS / 64) * 64 * QO];
    __shared__ WiCacheL WI;
    for (int d = threadIdx.x; d < nbins; d += EV_THREADS) cur[d] = (unsigned)O[(int64_t)d * ntiles + blockIdx.x];
    wi_load(WI, winfo);
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * tile;
    const int64_t t1 = t0 + tile < n ? t0 + tile : n;
    uint4 *__restrict__ d4 = (uint4 *)dst;
    uint4 *ws = stage + (wire ? 0 : (threadIdx.x >> 6) * 64 * QO);
    const int ln = lane_id();
    // a row's columns, loaded one round ahead (every load of a round is issued before the first is used); sv = 2:
    // the speed word is already encoded (payload stream)
    struct Row { uint64_t k, sp; double la, lo; uint8_t sv; };
    auto load = [&](int64_t i) {
        Row r{0, 0, 0.0, 0.0, 0};
        if (i < t1) {
            r.k = __builtin_nontemporal_load(&keys[i]);
            if (payload_in) {
                r.sp = __builtin_nontemporal_load(&payload_in[i * WIRE_PAYLOAD_WORDS]);
                r.la = __builtin_bit_cast(double, __builtin_nontemporal_load(&payload_in[i * WIRE_PAYLOAD_WORDS + 1]));
                r.lo = __builtin_bit_cast(double, __builtin_nontemporal_load(&payload_in[i * WIRE_PAYLOAD_WORDS + 2]));
                r.sv = 2;
            } else {
                r.sp = speed ? __builtin_bit_cast(uint64_t, __builtin_nontemporal_load(&speed[i])) : 0;
                r.sv = speed ? (speed_valid ? __builtin_nontemporal_load(&speed_valid[i]) : (uint8_t)1) : (uint8_t)0;
                r.la = __builtin_nontemporal_load(&lat[i]);
                r.lo = __builtin_nontemporal_load(&lon[i]);
            }
        }
        return r;
    };
    int64_t i0 = t0 + (int64_t)(threadIdx.x >> 6) * 64;
    Row nx = load(i0 + ln);
    preheader_wait();
    for (; i0 < t1; i0 += EV_THREADS) {
        const Row r = nx;
        nx = load(i0 + EV_THREADS + ln);
        unsigned pos = ~0u;   // ~0u: no record
        if (r.k) {
            const uint64_t k = r.k;
            const WInfo wi = wi_get(WI, winfo, ekey_widx(k));
            const uint64_t cell = (k & CELL_LO) | cell_hi;
            const uint64_t hh = mix64(cell ^ wi.inner);
            pos = atomicAdd(&cur[ev_digit(hh, wi.binp, nranks)], 1u);
            const double sp = __builtin_bit_cast(double, r.sp);
            const uint64_t spb = r.sv == 2 ? r.sp : r.sv == 0 ? SPEED_NULL_BITS : sp != sp ? CANON_NAN_BITS : r.sp;
            const uint64_t lab = __builtin_bit_cast(uint64_t, r.la), lob = __builtin_bit_cast(uint64_t, r.lo);
            if constexpr (wire) {
                // few digits (owner ranks): a wave's rows land in a few contiguous runs, written lane by lane
                dst[pos].key = ekey_make(k, wi.gslot);
                payload_out[(int64_t)pos * WIRE_PAYLOAD_WORDS + 0] = spb;
                payload_out[(int64_t)pos * WIRE_PAYLOAD_WORDS + 1] = lab;
                payload_out[(int64_t)pos * WIRE_PAYLOAD_WORDS + 2] = lob;
            } else {
                ws[ln * 2 + 0] = make_uint4((unsigned)k, (unsigned)(k >> 32), (unsigned)spb, (unsigned)(spb >> 32));
                ws[ln * 2 + 1] = make_uint4((unsigned)lab, (unsigned)(lab >> 32), (unsigned)lob, (unsigned)(lob >> 32));
            }
        }
        if constexpr (!wire) {
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            for (int q = 0; q < QO; q++) {
                const int idx = q * 64 + ln, rec = idx / QO, part = idx % QO;
                const unsigned p = __shfl(pos, rec, 64);
                if (p != ~0u) d4[(int64_t)p * QO + part] = ws[idx];
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// Out = EventRec (the direct path's (window, region) bins; the single-GPU partition and the multi-GPU owner's): the same
// rows and records as k_ev_scatter above, with no wait for the stores or the next round's loads inside the loop.
// Rounds alternate between two register sets (no loop-carried copy: a register copy of a pending load waits for it);
// every load is unconditional (the row clamped into the tile, absent columns read from one-element device constants,
// the payload stream chosen at compile time), and every lane stores a record each round -- a row without a key goes
// to the gap digit after every bin (counted by k_ev_hist; never read by the merge), a lane past the tile to the slack
// records after the n-th (ensured by ev_partition) -- so the stores are unconditional too: the wait before a round's
// rows only waits for them, not for the previous round's stores (measured before: a vmcnt(0) at the loop latch and
// one after the prefetch, i.e. every round waited for its own stores and the next round's loads).
__device__ const double g_zero_double = 0.0;
__device__ const uint8_t g_zero_byte = 0;
__device__ const uint8_t g_one_byte = 1;   // (also k_ingest's row validity when the batch has no validity column)
typedef __attribute__((address_space(1))) const hm_v4u g_cv4u;
typedef __attribute__((address_space(1))) hm_v4u g_v4u;
__device__ __forceinline__ void st_g16(void *p, uint4 v) { *(g_v4u *)p = hm_v4u{v.x, v.y, v.z, v.w}; }   // global 16-B store
// k_ev_scatter_rec's record stores (HM_NT_STORES bit 3: non-temporal, A/B builds)
__device__ __forceinline__ void st_g16_rec(void *p, uint4 v) {
    if constexpr ((HM_NT_STORES & 8) != 0) __builtin_nontemporal_store(hm_v4u{v.x, v.y, v.z, v.w}, (g_v4u *)p);
    else st_g16(p, v);
}
// workgroup size of k_ev_scatter_rec (its LDS: the 8193 cursors + a 32-B record per lane)
#ifndef HM_SR_THREADS
#define HM_SR_THREADS 512
#endif
constexpr int SR_THREADS = HM_SR_THREADS;
template <bool kPayload>
__global__ __launch_bounds__(SR_THREADS) void k_ev_scatter_rec(const uint64_t *__restrict__ keys, int64_t n, int64_t tile,
                                                              const double *__restrict__ speed, const uint8_t *__restrict__ speed_valid,
                                                              const double *__restrict__ lat, const double *__restrict__ lon,
                                                              const uint64_t *__restrict__ payload_in,
                                                              const WInfo *__restrict__ winfo, uint64_t cell_hi, int nbins,
                                                              const unsigned long long *__restrict__ O, int64_t ntiles,
                                                              EventRec *__restrict__ dst) {
    __shared__ unsigned cur[RP_BINS + 1];   // the bins' cursors and the gap digit's (positions < 2^32 - 1)
    __shared__ uint4 stage[(SR_THREADS / 64) * 64 * 2];
    __shared__ WiCacheL WI;
    for (int d = threadIdx.x; d <= nbins; d += SR_THREADS) cur[d] = (unsigned)O[(int64_t)d * ntiles + blockIdx.x];
    wi_load(WI, winfo);
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * tile;
    const int64_t t1 = t0 + tile < n ? t0 + tile : n;
    typedef __attribute__((address_space(1))) const double gcd;
    typedef __attribute__((address_space(1))) const uint8_t gcu8;
    typedef __attribute__((address_space(1))) const uint64_t gcu64;
    uint4 *__restrict__ d4 = (uint4 *)dst;
    uint4 *ws = stage + (threadIdx.x >> 6) * 64 * 2;
    const int ln = lane_id();
    struct Row { uint64_t k, sp; double la, lo; unsigned sv; bool in; };
    auto load = [&](int64_t i) __attribute__((always_inline)) {
        Row r;
        r.in = i < t1;
        const int64_t j = r.in ? i : t1 - 1;
        r.k = __builtin_nontemporal_load((gcu64 *)&keys[j]);
        if constexpr (kPayload) {
            r.sp = __builtin_nontemporal_load((gcu64 *)&payload_in[j * WIRE_PAYLOAD_WORDS]);
            r.la = __builtin_bit_cast(double, __builtin_nontemporal_load((gcu64 *)&payload_in[j * WIRE_PAYLOAD_WORDS + 1]));
            r.lo = __builtin_bit_cast(double, __builtin_nontemporal_load((gcu64 *)&payload_in[j * WIRE_PAYLOAD_WORDS + 2]));
            r.sv = 2;
        } else {
            r.sp = __builtin_bit_cast(uint64_t, __builtin_nontemporal_load((gcd *)(speed ? &speed[j] : &g_zero_double)));
            r.sv = __builtin_nontemporal_load((gcu8 *)(speed_valid ? &speed_valid[j] : speed ? &g_one_byte : &g_zero_byte));
            r.la = __builtin_nontemporal_load((gcd *)&lat[j]);
            r.lo = __builtin_nontemporal_load((gcd *)&lon[j]);
        }
        return r;
    };
    auto put = [&](const Row &r) __attribute__((always_inline)) {
        const uint64_t k = r.in ? r.k : 0;
        unsigned pos;
        if (k) {
            const WInfo wi = wi_get(WI, winfo, ekey_widx(k));
            const uint64_t hh = mix64(((k & CELL_LO) | cell_hi) ^ wi.inner);
            pos = atomicAdd(&cur[ev_digit(hh, wi.binp, 0)], 1u);
        }
        // rows without a key: the gap digit (one LDS add per wave); lanes past the tile: the slack after record n
        const unsigned long long gm = __ballot(r.in && !k);
        if (gm) {
            const int leader = __ffsll((long long)gm) - 1;
            unsigned gb = 0;
            if (ln == leader) gb = atomicAdd(&cur[nbins], (unsigned)__popcll(gm));
            gb = __shfl(gb, leader, 64);
            if (r.in && !k) pos = gb + (unsigned)__popcll(gm & ((UINT64_C(1) << ln) - 1));
        }
        if (!r.in) pos = (unsigned)n + (unsigned)ln;
        const uint64_t spb = kPayload ? r.sp : r.sv == 0 ? SPEED_NULL_BITS
                                                        : __builtin_bit_cast(double, r.sp) != __builtin_bit_cast(double, r.sp) ? CANON_NAN_BITS : r.sp;
        const uint64_t lab = __builtin_bit_cast(uint64_t, r.la), lob = __builtin_bit_cast(uint64_t, r.lo);
        ws[ln * 2 + 0] = make_uint4((unsigned)k, (unsigned)(k >> 32), (unsigned)spb, (unsigned)(spb >> 32));
        ws[ln * 2 + 1] = make_uint4((unsigned)lab, (unsigned)(lab >> 32), (unsigned)lob, (unsigned)(lob >> 32));
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int idx = q * 64 + ln, rec = idx >> 1, part = idx & 1;
            const unsigned p = __shfl(pos, rec, 64);
            st_g16_rec(&d4[(int64_t)p * 2 + part], ws[idx]);
        }
        __builtin_amdgcn_wave_barrier();
    };
    int64_t i0 = t0 + (int64_t)(threadIdx.x >> 6) * 64;
    if (i0 >= t1) return;
    Row a = load(i0 + ln);
    preheader_wait();
    for (;;) {
        const Row b = load(i0 + SR_THREADS + ln);
        put(a);
        if (i0 + SR_THREADS >= t1) break;
        a = load(i0 + 2 * SR_THREADS + ln);
        put(b);
        i0 += 2 * SR_THREADS;
        if (i0 >= t1) break;
    }
}

// the multi-GPU owner's census: received direct-path records per global window slot (sizes the window tables)
struct SlotSink {
    unsigned long long *cnt;   // WREG_SLOTS counters
    __device__ bool add(unsigned long long id, unsigned long long c) const {
        atomicAdd(&cnt[id - 1], c);
        return true;
    }
};
__global__ __launch_bounds__(256) void k_key_census(const uint64_t *__restrict__ keys, int64_t n, unsigned long long *cnt) {
    __shared__ WinLds WL;
    wl_init(WL);
    __syncthreads();
    const SlotSink sink{cnt};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        const uint64_t k = i < n ? __builtin_nontemporal_load(&keys[i]) : 0;
        wave_count_windows(k != 0, (unsigned long long)ekey_widx(k) + 1, 1ull, WL, sink);
    }
    __syncthreads();
    wl_flush(WL, sink);
}

// =====================================================================================================
// K2d: table mode (low-cardinality batches: few distinct (cell, window) keys, heavily repeated -- city-scale data).
// Per-workgroup partial aggregation cannot get far below the keys a workgroup sees (a Zipf tail of keys that
// recur about once per workgroup), so the batch is aggregated in two LDS passes instead of per-row partials:
//  k_agg         one 1024-thread workgroup per CU streams a contiguous span of the event keys through an LDS
//                table of AG_SLOTS aggregates; when it fills, the entries with the lowest counts are evicted (the
//                hot keys stay resident until the end) into 256 buckets by key hash (x 8 sub-buckets by XCD, for
//                locality only: any placement is correct);
//  k_bin_reduce  one workgroup per bucket aggregates its evicted entries (a bucket holds 1/256 of the keys) and
//                writes one partial record per key -> the usual partition + merge.
// =====================================================================================================
// LDS-only workgroup barrier: orders the workgroup's LDS accesses without draining the waves' outstanding global
// loads and stores (__syncthreads' fence also waits for every global access of the wave).  (k_agg keeps
// __syncthreads: this barrier in its rounds and flushes measured neutral, profiles/r2/abc3c/)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
constexpr int AG_THREADS = 1024;
#ifndef HM_AG_LINEAR
// 40 B each: 150 KB of LDS, one workgroup per CU.  A prime, so that every double-hashing step visits every slot.
constexpr int AG_SLOTS = 3833;
#else
constexpr int AG_SLOTS = 3840;
#endif
constexpr int AG_PER = AG_SLOTS / AG_THREADS + (AG_SLOTS % AG_THREADS != 0);
#ifndef HM_AG_HEADROOM
#define HM_AG_HEADROOM 640
#endif
// flush when fewer than HM_AG_HEADROOM slots are free.  A round adds at most AG_THREADS keys, ~360 on C3; when one
// adds more than the headroom, probes fail and those rows go out as partial records (exact, just not pre-aggregated).
// C3 shard (profiles/r2/abh/): headroom 1024 -> k_agg + k_bin_reduce 4.01 ms, 640 -> 3.89 ms (~200 such partials
// per batch), 400 -> 4.1 ms (13k)
constexpr int AG_FLUSH_AT = AG_SLOTS - HM_AG_HEADROOM;
#ifndef HM_AG_KEEP_DIV
#define HM_AG_KEEP_DIV 8
#endif
// aggregates kept resident by a flush.  Fewer kept = more room per flush = fewer flushes, which cost more than the
// extra evicted aggregates (C3 shard, profiles/r2/abk*/: keep 1/2 -> k_agg + k_bin_reduce 6.4 ms, 1/3 -> 4.9,
// 1/5 -> 4.35, 1/8 -> 4.0, 1/12 and 1/24 -> 4.0; evicted aggregates 30.1M / 33.7M / 37.5M / 40.1M / 41.9M / 44.1M)
constexpr int AG_KEEP_MAX = AG_SLOTS / HM_AG_KEEP_DIV;
constexpr int AG_PROBES = 64;
constexpr int AG_BINS = 256, AG_SUB = 8;        // buckets x sub-buckets (XCD)
struct AgTable {
    unsigned long long key[AG_SLOTS];   // ekey, 0 = free
    unsigned long long cnt[AG_SLOTS];   // count | n_speed << 32
    double ssp[AG_SLOTS];
    double slat[AG_SLOTS];
    double slon[AG_SLOTS];
    unsigned occ;
    unsigned keep_from;
    unsigned hist[16];
    unsigned bcnt[AG_BINS];
    unsigned long long bbase[AG_BINS];
    unsigned scan[AG_THREADS / 64];
    unsigned long long obase;
};
__device__ __forceinline__ unsigned ag_home(uint64_t k) { return (unsigned)(((mix64(k) >> 32) * (uint64_t)AG_SLOTS) >> 32); }
// Probe sequence: double hashing (step in [1, AG_SLOTS - 1] from other hash bits).  Every round of k_agg ends at a
// workgroup barrier, so a round lasts as long as its longest probe chain; linear probing's clusters at the table's
// 70-80% fill before a flush made those chains run to the 64-probe bound (each probe a dependent LDS load).
__device__ __forceinline__ unsigned ag_step(uint64_t k) {
#ifndef HM_AG_LINEAR
    return 1u + (unsigned)(((mix64(k) & 0xffffffffu) * (uint64_t)(AG_SLOTS - 1)) >> 32);
#else
    (void)k;
    return 1u;
#endif
}
__device__ __forceinline__ unsigned ag_bin(uint64_t k) { return (unsigned)mix64(k ^ UINT64_C(0x94d049bb133111eb)) & (AG_BINS - 1); }
__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v & (AG_SUB - 1);
}
__device__ __forceinline__ void ag_clear(AgTable &T) {
    for (int s = threadIdx.x; s < AG_SLOTS; s += AG_THREADS) {
        T.key[s] = 0;
        T.cnt[s] = 0;
        T.ssp[s] = 0.0;
        T.slat[s] = 0.0;
        T.slon[s] = 0.0;
    }
    if (threadIdx.x == 0) T.occ = 0;
}
// add an aggregate for key k (inserted if new); false when no slot was found within AG_PROBES
__device__ __forceinline__ bool ag_add(AgTable &T, uint64_t k, unsigned long long c, double ssp, double sla, double slo,
                                       bool &fresh) {
    unsigned h = ag_home(k);
    const unsigned step = ag_step(k);
    fresh = false;
    for (int p = 0; p < AG_PROBES; p++) {
        unsigned long long cur = __hip_atomic_load(&T.key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (cur == 0) {
            cur = atomicCAS(&T.key[h], 0ull, (unsigned long long)k);
            fresh = cur == 0;
        }
        if (cur == 0 || cur == k) {
            atomicAdd(&T.cnt[h], c);
            if (c >> 32) atomicAdd(&T.ssp[h], ssp);   // (only non-null speeds: Spark's sum skips nulls)
            atomicAdd(&T.slat[h], sla);
            atomicAdd(&T.slon[h], slo);
            return true;
        }
        h += step;
        h = h >= (unsigned)AG_SLOTS ? h - (unsigned)AG_SLOTS : h;
    }
    return false;
}
// one partial record for key k (rare spill paths and k_bin_reduce's output), appended to out
__device__ __forceinline__ TilePartial ag_partial(uint64_t k, unsigned long long c, double ssp, double sla, double slo,
                                                  const unsigned long long *wreg, uint64_t cell_hi) {
    TilePartial p;
    p.cell = (k & CELL_LO) | cell_hi;
    p.wstart = wdec(wreg[ekey_widx(k)]);
    p.count = (uint32_t)c;
    p.nspeed = (uint32_t)(c >> 32);
    p.sspeed = ssp;
    p.slat = sla;
    p.slon = slo;
    return p;
}
__device__ __forceinline__ void ag_spill(uint64_t k, unsigned long long c, double ssp, double sla, double slo,
                                         const unsigned long long *wreg, uint64_t cell_hi, TilePartial *out, DevStats *st,
                                         WinLds &WL, const CensusSink &census, bool &ok) {
    const TilePartial p = ag_partial(k, c, ssp, sla, slo, wreg, cell_hi);
    out[atomicAdd(&st->n_partials, 1ull)] = p;
    atomicAdd(&st->agg_spill, 1ull);
    ok &= wl_add(WL, census, wenc_of(p.wstart), 1ull);
}
// k_agg's flush: the entries below the keep threshold go to their buckets; kept ones are re-inserted into the
// cleared table (so that probe chains stay intact).  final: every entry is evicted.
__device__ void ag_flush(AgTable &T, bool final, AggRec *__restrict__ bucket, unsigned long long *cursor, unsigned cap,
                         const unsigned long long *wreg, uint64_t cell_hi, TilePartial *out, DevStats *st, WinLds &WL,
                         const CensusSink &census, bool &ok) {
    const int t = threadIdx.x;
    if (t < 16) T.hist[t] = 0;
    for (int b = t; b < AG_BINS; b += AG_THREADS) T.bcnt[b] = 0;
    __syncthreads();
    int lg[AG_PER];
    for (int q = 0; q < AG_PER; q++) {
        const int s = t + q * AG_THREADS;
        lg[q] = -1;
        if (s < AG_SLOTS && T.key[s]) {
            const unsigned c = (unsigned)T.cnt[s];
            lg[q] = min(31 - __clz(c), 15);
        }
        // the keep threshold reads hist[1..15] only (singletons always go): no atomics for the many count-1
        // entries, and the count-2/3 class (the next most common) counted per wave -- every lane adding into one
        // LDS word serialises the wave
        const unsigned long long m1 = __ballot(lg[q] == 1);
        if (m1 && lane_id() == 0) atomicAdd(&T.hist[1], (unsigned)__popcll(m1));
        if (lg[q] >= 2) atomicAdd(&T.hist[lg[q]], 1u);
    }
    __syncthreads();
    if (t == 0) {   // keep the entries with count >= 2^kf, at most AG_KEEP_MAX of them (kf >= 1: singletons go)
        unsigned kf = 16, acc = 0;
        if (!final)
            for (int b = 15; b >= 1; b--) {
                if (acc + T.hist[b] > (unsigned)AG_KEEP_MAX) break;
                acc += T.hist[b];
                kf = (unsigned)b;
            }
        T.keep_from = kf;
    }
    __syncthreads();
    const int kf = (int)T.keep_from;
    unsigned rk[AG_PER];
    for (int q = 0; q < AG_PER; q++) {
        const int s = t + q * AG_THREADS;
        rk[q] = 0;
        if (lg[q] >= 0 && lg[q] < kf) rk[q] = atomicAdd(&T.bcnt[ag_bin(T.key[s])], 1u);
    }
    __syncthreads();
    const unsigned xs = xcc_id();
    for (int b = t; b < AG_BINS; b += AG_THREADS)
        if (T.bcnt[b]) T.bbase[b] = atomicAdd(&cursor[b * AG_SUB + xs], (unsigned long long)T.bcnt[b]);
    __syncthreads();
    uint64_t kk[AG_PER];
    unsigned long long kc[AG_PER];
    double ks[AG_PER], kla[AG_PER], klo[AG_PER];
    unsigned long long evicted = 0;
    for (int q = 0; q < AG_PER; q++) {
        const int s = t + q * AG_THREADS;
        kk[q] = 0;
        if (lg[q] < 0) continue;
        const uint64_t k = T.key[s];
        const unsigned long long c = T.cnt[s];
        const double a = T.ssp[s], b = T.slat[s], d = T.slon[s];
        if (lg[q] >= kf) {
            kk[q] = k; kc[q] = c; ks[q] = a; kla[q] = b; klo[q] = d;
            continue;
        }
        evicted++;
        const unsigned bin = ag_bin(k);
        const unsigned long long pos = T.bbase[bin] + rk[q];
        if (pos < cap) {
            AggRec r;
            r.key = k;
            r.cnt = c;
            r.ssp = a;
            r.slat = b;
            r.slon = d;
            r.pad = 0;
            bucket[(uint64_t)(bin * AG_SUB + xs) * cap + pos] = r;
        } else {
            ag_spill(k, c, a, b, d, wreg, cell_hi, out, st, WL, census, ok);
        }
    }
    evicted = wave_sum(evicted);
    if (evicted && lane_id() == 0) atomicAdd(&st->n_evicted, evicted);
    __syncthreads();
    ag_clear(T);
    __syncthreads();
    unsigned kept = 0;
    for (int q = 0; q < AG_PER; q++) {
        bool fresh;
        if (kk[q]) { ag_add(T, kk[q], kc[q], ks[q], kla[q], klo[q], fresh); kept++; }   // (<= AG_KEEP_MAX: always fits)
    }
    kept = (unsigned)wave_sum((unsigned long long)kept);
    if (kept && lane_id() == 0) atomicAdd(&T.occ, kept);
    __syncthreads();
}

// keys inserted into the LDS table so far, identical in every thread: per round each wave adds its fresh keys to
// one of three LDS counters, a barrier, every thread reads it; the counter two rounds ahead is cleared (its last
// readers passed the previous barrier, its next writers are a barrier away), so one barrier per round suffices
struct FreshCount {
    unsigned *c;
    int r3 = 0;
    unsigned occ = 0;
    __device__ explicit FreshCount(unsigned *ctr) : c(ctr) {}
    __device__ unsigned round(bool fresh) {
        const unsigned long long fb = __ballot(fresh);
        if (fb && lane_id() == 0) atomicAdd(&c[r3], (unsigned)__popcll(fb));
        __syncthreads();
        occ += c[r3];
        if (threadIdx.x == 0) c[r3 == 0 ? 2 : r3 - 1] = 0;
        r3 = r3 == 2 ? 0 : r3 + 1;
        return occ;
    }
};

__global__ __launch_bounds__(AG_THREADS) void k_agg(const uint64_t *__restrict__ keys, int64_t n, int64_t span,
                                                    const double *__restrict__ speed, const uint8_t *__restrict__ speed_valid,
                                                    const double *__restrict__ lat, const double *__restrict__ lon,
                                                    AggRec *__restrict__ bucket, unsigned long long *cursor, unsigned cap,
                                                    const unsigned long long *wreg, uint64_t cell_hi, TilePartial *out,
                                                    WinCount *cmap, DevStats *st) {
    __shared__ AgTable T;
    __shared__ WinLds WL;
    __shared__ unsigned fresh_ctr[3];
    ag_clear(T);
    wl_init(WL);
    if (threadIdx.x < 3) fresh_ctr[threadIdx.x] = 0;
    __syncthreads();
    const CensusSink census{cmap};
    bool ok = true;
    const int64_t b0 = (int64_t)blockIdx.x * span;
    const int64_t b1 = b0 + span < n ? b0 + span : n;
    FreshCount FC(fresh_ctr);
    // a row's columns, loaded one round ahead (the round's loads are in flight while the previous one aggregates).
    // (Measured on C3: keeping the validity byte raw and waiting for the first round before the loop -- so that no
    // round waits for the next round's loads -- made k_agg 0.3 ms slower, profiles/r2/ab1/: its rounds are not
    // load-bound, its flushes are.)
    struct Row { uint64_t k; double sp, la, lo; bool sv; };
    auto load = [&](int64_t i) {
        Row r{0, 0.0, 0.0, 0.0, false};
        if (i < b1) {
            r.k = __builtin_nontemporal_load(&keys[i]);
            r.sv = speed ? (speed_valid ? __builtin_nontemporal_load(&speed_valid[i]) != 0 : true) : false;
            r.sp = speed ? __builtin_nontemporal_load(&speed[i]) : 0.0;
            r.la = __builtin_nontemporal_load(&lat[i]);
            r.lo = __builtin_nontemporal_load(&lon[i]);
        }
        return r;
    };
    auto round_of = [&](const Row &r) __attribute__((always_inline)) {
        const uint64_t k = r.k;
        bool fresh = false;
        if (k) {
            const double sp = r.sv ? r.sp : 0.0, la = r.la, lo = r.lo;
            const unsigned long long c = 1ull | ((unsigned long long)r.sv << 32);
            if (!ag_add(T, k, c, sp, la, lo, fresh)) ag_spill(k, c, sp, la, lo, wreg, cell_hi, out, st, WL, census, ok);
        }
        if (FC.round(fresh) > (unsigned)AG_FLUSH_AT) {
            ag_flush(T, false, bucket, cursor, cap, wreg, cell_hi, out, st, WL, census, ok);
            FC.occ = T.occ;
        }
    };
    Row nx = load(b0 + threadIdx.x);
    for (int64_t c0 = b0; c0 < b1; c0 += AG_THREADS) {
        const Row r = nx;
        nx = load(c0 + AG_THREADS + threadIdx.x);
        round_of(r);
    }
    ag_flush(T, true, bucket, cursor, cap, wreg, cell_hi, out, st, WL, census, ok);
    __syncthreads();
    ok &= wl_flush(WL, census);
    if (__ballot(!ok) && lane_id() == 0) atomicAdd(&st->overflow, 1ull);
}

// every entry of the table as a partial record (a block-wide scan reserves one contiguous run), counted per window
__device__ void ag_emit_all(AgTable &T, const unsigned long long *wreg, uint64_t cell_hi, TilePartial *__restrict__ out,
                            DevStats *st, WinLds &WL, const CensusSink &census, bool &ok) {
    const int t = threadIdx.x;
    unsigned c = 0;
    for (int q = 0; q < AG_PER; q++) {
        const int s = t + q * AG_THREADS;
        c += s < AG_SLOTS && T.key[s] != 0;
    }
    unsigned incl = c;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(incl, o, 64);
        if (lane_id() >= o) incl += v;
    }
    const int wv = t >> 6;
    if (lane_id() == 63) T.scan[wv] = incl;
    __syncthreads();
    unsigned off = 0, total = 0;
    for (int q = 0; q < AG_THREADS / 64; q++) {
        if (q < wv) off += T.scan[q];
        total += T.scan[q];
    }
    if (t == 0) T.obase = total ? atomicAdd(&st->n_partials, (unsigned long long)total) : 0;
    __syncthreads();
    unsigned long long pos = T.obase + off + incl - c;
    for (int q = 0; q < AG_PER; q++) {
        const int s = t + q * AG_THREADS;
        const bool live = s < AG_SLOTS && T.key[s] != 0;
        unsigned long long we = 0;
        if (live) {
            const TilePartial p = ag_partial(T.key[s], T.cnt[s], T.ssp[s], T.slat[s], T.slon[s], wreg, cell_hi);
            out[pos++] = p;
            we = wenc_of(p.wstart);
        }
        ok &= wave_count_windows(live, we, 1ull, WL, census);
    }
    __syncthreads();
    ag_clear(T);
    __syncthreads();
}

// one workgroup per bucket: its sub-buckets' aggregates -> one partial record per key (more if the bucket holds
// more keys than the table: it is then emitted whenever it fills)
__global__ __launch_bounds__(AG_THREADS) void k_bin_reduce(const AggRec *__restrict__ bucket, const unsigned long long *cursor,
                                                           unsigned cap, const unsigned long long *wreg, uint64_t cell_hi,
                                                           TilePartial *__restrict__ out, WinCount *cmap, DevStats *st) {
    __shared__ AgTable T;
    __shared__ WinLds WL;
    __shared__ unsigned long long sub_end[AG_SUB + 1];
    __shared__ unsigned fresh_ctr[3];
    ag_clear(T);
    wl_init(WL);
    if (threadIdx.x < 3) fresh_ctr[threadIdx.x] = 0;
    const int bin = blockIdx.x;
    if (threadIdx.x == 0) {
        unsigned long long acc = 0;
        sub_end[0] = 0;
        for (int x = 0; x < AG_SUB; x++) {
            const unsigned long long c = cursor[bin * AG_SUB + x];
            acc += c < cap ? c : cap;
            sub_end[x + 1] = acc;
        }
    }
    __syncthreads();
    const CensusSink census{cmap};
    bool ok = true;
    const unsigned long long total = sub_end[AG_SUB];
    FreshCount FC(fresh_ctr);
    for (unsigned long long c0 = 0; c0 < total; c0 += AG_THREADS) {
        const unsigned long long j = c0 + threadIdx.x;
        bool fresh = false;
        if (j < total) {
            int x = 0;
            while (j >= sub_end[x + 1]) x++;
            const AggRec r = bucket[(uint64_t)(bin * AG_SUB + x) * cap + (j - sub_end[x])];
            if (!ag_add(T, r.key, r.cnt, r.ssp, r.slat, r.slon, fresh))
                ag_spill(r.key, r.cnt, r.ssp, r.slat, r.slon, wreg, cell_hi, out, st, WL, census, ok);
        }
        if (FC.round(fresh) > (unsigned)AG_FLUSH_AT) {
            ag_emit_all(T, wreg, cell_hi, out, st, WL, census, ok);
            FC.occ = 0;
        }
    }
    ag_emit_all(T, wreg, cell_hi, out, st, WL, census, ok);
    ok &= wl_flush(WL, census);
    if (__ballot(!ok) && lane_id() == 0) atomicAdd(&st->overflow, 1ull);
}

// =====================================================================================================
// K3': owner merge + emission. The workgroup of a bin is the only writer of the (window, region)s the partition
// sent it, so the state is updated with plain loads/stores instead of device-scope atomics. Per chunk of 256
// partials (one per lane), each lane finds its key's slot and claims it in an LDS claim set keyed by slot
// address; a lane whose slot is already claimed by the same key in this chunk adds its values into the
// claimer's LDS staging entry and is done (in-chunk de-duplication without a separate hash table):
//  * resident windows (the bin's regions of the windows this batch merges into, while their tags fit in
//    MO_TAG_BYTES of LDS): probing runs over the region's slot tags in LDS -- a new key reads nothing from HBM;
//    an occupied slot not claimed in this chunk is read only on a tag match;
//  * other windows (too many/too large regions, or growth): probing reads the slots' window words from HBM;
//    the tag byte of a created slot is stored to HBM.
// The update-mode output row of a key (cumulative count/avg, heatmap_stream.py:124-132,243) is written at its
// first touch in the batch to row b0 + k of the bin's segment (b0 = the bin's first partial, k = touch order
// in the bin; the slot's `touched` word keeps (batch seq, k)), and rewritten in place when a later chunk
// updates the key again; k_fill_gaps closes the gaps left by keys that had several partials.
// rehash != 0: growth (k_dump_gen records, unique keys, into the window's new table): created slots keep the
// record's touched word, no rows are written.
// =====================================================================================================
#ifndef HM_MO_THREADS
#define HM_MO_THREADS 512
#endif
constexpr int MO_THREADS = HM_MO_THREADS;      // partials per chunk (one per lane)
#ifndef HM_MO_COOP_LINES
#define HM_MO_COOP_LINES 1
#endif
#ifndef HM_MO_EARLY_LINES
#define HM_MO_EARLY_LINES 1
#endif
// the resident-only merge's wave-cooperative probe (needs the early-lines scratch)
#ifndef HM_MO_COOP_PROBE
#define HM_MO_COOP_PROBE HM_MO_EARLY_LINES
#endif
// claim-set entries per record of a chunk (the resident-only merge: 2x as many 32-bit entries; 2 + the early old-line
// scratch fit the same LDS as 4 without it)
#ifndef HM_MO_CLAIM_MULT
#define HM_MO_CLAIM_MULT (HM_MO_EARLY_LINES ? 2 : 4)
#endif
constexpr int MO_CLAIM = HM_MO_CLAIM_MULT * MO_THREADS;   // claim-set entries (load <= 1 / HM_MO_CLAIM_MULT)
#ifndef HM_MO_TAG_MAX
#define HM_MO_TAG_MAX 90112
#endif
// LDS for resident region tags per workgroup: dynamic, sized per launch to the regions a bin can receive (the sum
// over the batch's windows of slots per region, 1 B each) up to MO_TAG_MAX -- 24 KB on the bench (3 windows x 8 K
// slots: two workgroups per CU), 32 KB for a res-7 window of 2^28 slots, which would otherwise probe through HBM
constexpr int MO_TAG_MAX = HM_MO_TAG_MAX;
constexpr int MO_RES_MAX = 16;                   // resident (window, region)s per bin

struct MoShared {
    // this chunk's records by lane; a duplicate key's values are added into its claimer's entry
    unsigned long long sc[MO_THREADS];
    unsigned long long sh[MO_THREADS];
    unsigned long long scnt[MO_THREADS];
    unsigned long long snsp[MO_THREADS];
    double sssp[MO_THREADS];
    double sslat[MO_THREADS];
    double sslon[MO_THREADS];
    unsigned long long claim[MO_CLAIM];   // (slot address << 16) | claimer lane; 0 = free
    unsigned n_touched;                   // keys of the current bin touched for the first time this batch
    int n_res;
    unsigned res_new[MO_RES_MAX];         // keys created in the resident region this bin
    unsigned long long res_we[MO_RES_MAX];
    TileSlot *res_slots[MO_RES_MAX];      // the region's first slot
    uint8_t *res_gtags[MO_RES_MAX];       // the region's tags in HBM
    unsigned res_off[MO_RES_MAX];         // byte offset of the region's tags in `tags`
    unsigned res_mask[MO_RES_MAX];        // slots per region - 1
    unsigned res_dirty[MO_RES_MAX];
#if HM_MO_EARLY_LINES
    uint4 xline[MO_THREADS / 64][64];     // per wave: one round of the cooperative old-line loads (16 lines)
#endif
};

template <typename T>
__device__ __forceinline__ T ld_l2(const T *p) {   // bypass the CU's L1 (chunks of one workgroup re-read slots)
    // (a global-address-space access: the slot pointers come from LDS, and as generic pointers every access became a
    // flat instruction, which also counts on lgkmcnt -- so each later LDS wait waited for it to complete)
    return __hip_atomic_load((__attribute__((address_space(1))) const T *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned mo_claim_home(unsigned long long addr) {
    return (unsigned)(((addr >> 6) * UINT64_C(0x9e3779b97f4a7c15)) >> 40) & (MO_CLAIM - 1);
}
// claim slot `addr` for `lane` in claim set cl: -1 = claimed (entry index in ci), else the lane that already holds it
__device__ __forceinline__ int mo_claim(unsigned long long *cl, unsigned long long addr, int lane, int &ci) {
    const unsigned long long packed = (addr << 16) | (unsigned)lane;
    unsigned h = mo_claim_home(addr);
    for (int k = 0; k < MO_CLAIM; k++) {
        const unsigned long long o = atomicCAS(&cl[h], 0ull, packed);
        if (o == 0) { ci = (int)h; return -1; }
        if ((o >> 16) == addr) return (int)(o & 0xffff);
        h = (h + 1) & (MO_CLAIM - 1);
    }
    return -2;
}
// the lane holding slot `addr` in claim set cl, -1 if none
__device__ __forceinline__ int mo_holder(const unsigned long long *cl, unsigned long long addr) {
    unsigned h = mo_claim_home(addr);
    for (int k = 0; k < MO_CLAIM; k++) {
        const unsigned long long o = __hip_atomic_load(&cl[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (o == 0) return -1;
        if ((o >> 16) == addr) return (int)(o & 0xffff);
        h = (h + 1) & (MO_CLAIM - 1);
    }
    return -1;
}
// The resident-only merge keys its claims by the slot's tag index (< 2^17: MO_TAG_MAX) instead of its address, so an
// entry is 32 bits -- ((tag index + 1) << 9) | claimer lane -- and the same LDS holds twice the entries (load <= 1/8).
constexpr int MO_CLAIM32 = 2 * MO_CLAIM;
static_assert(MO_TAG_MAX < (1 << 17) && MO_THREADS <= 512, "32-bit claim entries");
__device__ __forceinline__ unsigned mo_claim_home32(unsigned key) { return (key * 0x9e3779b1u) >> (32 - __builtin_ctz(MO_CLAIM32)); }
__device__ __forceinline__ int mo_claim32(unsigned *cl, unsigned key, int lane, int &ci) {
    const unsigned packed = ((key + 1) << 9) | (unsigned)lane;
    unsigned h = mo_claim_home32(key);
    for (int k = 0; k < MO_CLAIM32; k++) {
        const unsigned o = atomicCAS(&cl[h], 0u, packed);
        if (o == 0) { ci = (int)h; return -1; }
        if ((o >> 9) == key + 1) return (int)(o & 511u);
        h = (h + 1) & (MO_CLAIM32 - 1);
    }
    return -2;
}
__device__ __forceinline__ int mo_holder32(const unsigned *cl, unsigned key) {
    unsigned h = mo_claim_home32(key);
    for (int k = 0; k < MO_CLAIM32; k++) {
        const unsigned o = __hip_atomic_load(&cl[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (o == 0) return -1;
        if ((o >> 9) == key + 1) return (int)(o & 511u);
        h = (h + 1) & (MO_CLAIM32 - 1);
    }
    return -1;
}
// a merge input record, normalised: SortedRec (table mode / stage merge), GrowRec (growth), EventRec (direct path)
struct MRec {
    uint64_t cell;
    unsigned long long we;   // wenc of the window start
    uint64_t hk;             // tile_hash(cell, window start)
    unsigned long long cnt, nsp;
    double ssp, slat, slon;
    unsigned long long touched;   // GrowRec only
};
__device__ __forceinline__ MRec mrec_of(const SortedRec &p, const WInfo *, uint64_t) {
    return MRec{p.cell, wenc_of(p.wstart), p.hash, p.count, p.nspeed, p.sspeed, p.slat, p.slon, 0ull};
}
__device__ __forceinline__ MRec mrec_of(const GrowRec &p, const WInfo *, uint64_t) {
    return MRec{p.cell, wenc_of(p.wstart), tile_hash(p.cell, p.wstart), p.count, p.nspeed, p.sspeed, p.slat, p.slon, p.touched};
}
__device__ __forceinline__ MRec mrec_of(const EventRec &p, const WInfo *winfo, uint64_t cell_hi) {
    const WInfo &wi = winfo[ekey_widx(p.key)];   // (an LDS copy measured no faster here: the chunk loop hides it)
    const uint64_t cell = (p.key & CELL_LO) | cell_hi;
    const bool sv = __builtin_bit_cast(uint64_t, p.speed) != SPEED_NULL_BITS;
    return MRec{cell, wi.wenc, mix64(cell ^ wi.inner), 1ull, sv ? 1ull : 0ull, sv ? p.speed : 0.0, p.lat, p.lon, 0ull};
}
// the same from the LDS image of the batch's window parameters (the partition's WiCacheL)
__device__ __forceinline__ MRec mrec_of_wi(const EventRec &p, const WiCacheL &WI, const WInfo *winfo, uint64_t cell_hi) {
    const WInfo wi = wi_get(WI, winfo, ekey_widx(p.key));
    const uint64_t cell = (p.key & CELL_LO) | cell_hi;
    const bool sv = __builtin_bit_cast(uint64_t, p.speed) != SPEED_NULL_BITS;
    return MRec{cell, wi.wenc, mix64(cell ^ wi.inner), 1ull, sv ? 1ull : 0ull, sv ? p.speed : 0.0, p.lat, p.lon, 0ull};
}
// a duplicate of lane x's key: add this record's values into x's staging entry
__device__ __forceinline__ void mo_add_into(MoShared &S, int x, const MRec &p) {
    atomicAdd(&S.scnt[x], p.cnt);
    if (p.nsp) {
        atomicAdd(&S.snsp[x], p.nsp);
        atomicAdd(&S.sssp[x], p.ssp);
    }
    atomicAdd(&S.sslat[x], p.slat);
    atomicAdd(&S.sslon[x], p.slon);
}

struct RowsOut {   // update-mode output rows (SoA), heatmap_stream.py:124-132
    uint64_t *cell;
    int64_t *ws;
    int64_t *cnt;
    double *sp;
    uint8_t *spnull;
    double *lon;
    double *lat;
};
// Spark Average: sum / count (count of non-null inputs) as double; null when that count is 0
__device__ __forceinline__ void put_row(const RowsOut &o, int64_t t, uint64_t cell, unsigned long long we,
                                        unsigned long long count, unsigned long long nspeed, double sspeed, double slat,
                                        double slon) {
    const bool null_sp = nspeed == 0;
    // x / 1.0 == x: a key's first row (count 1) skips the fp64 divisions
    double asp = null_sp ? 0.0 : sspeed, alon = slon, alat = slat;
    if (count != 1) {   // (a branch: a wave whose keys all have one row skips the three fp64 divisions)
        if (!null_sp && nspeed != 1) asp = sspeed / (double)nspeed;
        alon = slon / (double)count;
        alat = slat / (double)count;
    }
    if constexpr ((HM_NT_STORES & 2) != 0) {
        __builtin_nontemporal_store(cell, &o.cell[t]);
        __builtin_nontemporal_store(wdec(we), &o.ws[t]);
        __builtin_nontemporal_store((int64_t)count, &o.cnt[t]);
        __builtin_nontemporal_store(asp, &o.sp[t]);
        __builtin_nontemporal_store((uint8_t)null_sp, &o.spnull[t]);
        __builtin_nontemporal_store(alon, &o.lon[t]);
        __builtin_nontemporal_store(alat, &o.lat[t]);
    } else {
        o.cell[t] = cell;
        o.ws[t] = wdec(we);
        o.cnt[t] = (int64_t)count;
        o.sp[t] = asp;
        o.spnull[t] = null_sp;
        o.lon[t] = alon;
        o.lat[t] = alat;
    }
}

// a state line's new values (cell and window word are the key's)
struct MLine {
    unsigned long long count, nspeed;
    double sspeed, slat, slon;
    unsigned long long touched;
};

// Rec = SortedRec: a batch's partials (partitioned); EventRec: the direct path's rows; GrowRec: growth (rehash).
// kResident: the host found every window of the batch resident in every bin (merge_sorted), so the variant carries
// no HBM-probing fallback (less code, fewer live registers); a record outside the resident windows sets overflow.
// kCoop (resident only): the wave-cooperative probe (probe_coop) -- chosen when the last batch re-touched mostly
// existing keys (their lines then cost one cooperative round trip); a batch of mostly new keys runs the per-lane probe,
// which carries less machinery per probed slot (bench leg: 3.72-3.81 vs 4.03-4.11 ms; state-read leg: 6.86-6.89 vs
// 6.22-6.30 ms, profiles/r3/r3ab9/)
template <typename Rec, bool kResident = false, bool kCoop = false>
__global__ __launch_bounds__(MO_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_merge_owned(const Rec *__restrict__ parts, int64_t n,
                                                            const unsigned long long *__restrict__ O, int64_t ntiles, int nbins,
                                                            GenDesc *gm, const GenDesc *glist, int n_glist,
                                                            const WInfo *__restrict__ winfo, uint64_t cell_hi,
                                                            unsigned seq, RowsOut rows, unsigned *bin_cnt, DevStats *st,
                                                            unsigned tag_bytes) {
    constexpr bool rehash = std::is_same<Rec, GrowRec>::value;
    __shared__ MoShared S;
    extern __shared__ unsigned mo_tags[];   // tag_bytes of resident region tags
    __shared__ WinLds WL;
    __shared__ GenCache C;
#ifndef HM_MO_WI_LDS   // (off: the image's LDS cost the state-read leg's merge ~1 ms, profiles/r3/r3ab11)
#define HM_MO_WI_LDS 0
#endif
    constexpr bool kWi = HM_MO_WI_LDS && std::is_same<Rec, EventRec>::value;
    __shared__ std::conditional_t<kWi, WiCacheL, char> WI;   // EventRec: the window parameters' LDS image
    if constexpr (kWi) wi_load(WI, winfo);
    wl_init(WL);
    gc_load(C, glist, n_glist);
    const GenSink sink{gm};
    const int t = threadIdx.x;
    unsigned long long created_cnt = 0;
    bool overflow = false;
    for (int q = t; q < MO_CLAIM; q += MO_THREADS) S.claim[q] = 0;
    if (t == 0) S.n_touched = 0;
    __syncthreads();
    for (int bin = blockIdx.x; bin < nbins; bin += gridDim.x) {
        const int64_t b0 = (int64_t)O[(int64_t)bin * ntiles];
        const int64_t b1 = (int64_t)O[(int64_t)(bin + 1) * ntiles];   // (digit nbins: the gaps, after every bin)
        // 0. the bin's resident regions: windows merged into this batch whose region maps to this bin
        if (t == 0) {
            int nr = 0;
            unsigned off = 0;
            if (!rehash && C.n >= 0 && b1 > b0) {
                for (int q = 0; q < C.n; q++) {
                    const GenDesc &g = C.e[q];
                    if (!g.batch_parts) continue;
                    const unsigned sb = REGION_BITS - g.rbits, smask = (1u << sb) - 1;
                    if (((unsigned)bin & smask) != (window_salt(g.wenc) & smask)) continue;
                    const unsigned slots = (unsigned)g.rmask + 1;
                    if (nr == MO_RES_MAX || off + slots > tag_bytes) continue;
                    const unsigned long long first = (unsigned long long)((unsigned)bin >> sb) << g.rshift;
                    S.res_we[nr] = g.wenc;
                    S.res_slots[nr] = g.tab + first;
                    S.res_gtags[nr] = gen_tags(g) + first;
                    S.res_off[nr] = off;
                    S.res_mask[nr] = slots - 1;
                    S.res_dirty[nr] = 0;
                    S.res_new[nr] = 0;
                    off += slots;
                    nr++;
                }
            }
            S.n_res = nr;
        }
        lds_barrier();
        const int nres = S.n_res;
        // the resident regions' tags (16-B words, regions >= 256 slots): every load of a thread in flight together
        {
            unsigned tot = 0;
            for (int r = 0; r < nres; r++) tot += (S.res_mask[r] + 1) >> 4;
            typedef __attribute__((address_space(1))) const hm_v4u gv4u;   // global loads (the pointers sit in LDS)
            for (unsigned q0 = t; q0 < tot; q0 += 4 * MO_THREADS) {
                uint4 v0, v1, v2, v3;
                unsigned a0 = ~0u, a1 = ~0u, a2 = ~0u, a3 = ~0u;
                auto fetch = [&](unsigned q, uint4 &v, unsigned &a) __attribute__((always_inline)) {
                    if (q >= tot) return;
                    unsigned w = q;
                    int r = 0;
                    while (w >= ((S.res_mask[r] + 1) >> 4)) { w -= (S.res_mask[r] + 1) >> 4; r++; }
                    const hm_v4u x = ((gv4u *)S.res_gtags[r])[w];
                    v = make_uint4(x.x, x.y, x.z, x.w);
                    a = (S.res_off[r] >> 4) + w;
                };
                fetch(q0, v0, a0);
                fetch(q0 + MO_THREADS, v1, a1);
                fetch(q0 + 2 * MO_THREADS, v2, a2);
                fetch(q0 + 3 * MO_THREADS, v3, a3);
                if (a0 != ~0u) ((uint4 *)mo_tags)[a0] = v0;
                if (a1 != ~0u) ((uint4 *)mo_tags)[a1] = v1;
                if (a2 != ~0u) ((uint4 *)mo_tags)[a2] = v2;
                if (a3 != ~0u) ((uint4 *)mo_tags)[a3] = v3;
            }
        }
        lds_barrier();
        // find (and claim) the slot of lane t's key p, or join the lane of this chunk that holds it
        auto probe = [&](const MRec &p, TileSlot *&gslot, bool &created, int &r, int &ci) __attribute__((always_inline)) {
            unsigned long long *cl = S.claim;
            const unsigned long long we = p.we;
            const uint64_t hk = p.hk;
            const unsigned tg = tag8(hk);
            bool done = false;
            r = -1;
            for (int q = 0; q < nres; q++)
                if (S.res_we[q] == we) r = q;
            if (r >= 0) {
                const unsigned rmask = S.res_mask[r], off = S.res_off[r];
                TileSlot *const base = S.res_slots[r];
                unsigned s = (unsigned)hk & rmask;
                // Tags scanned 8 at a time (one 8-B LDS read): only slots whose tag is empty or this key's are visited
                // one by one, so a wave's loop runs its lanes' longest count of such slots, not of probed slots.
                // (regions are >= 256 slots and start at multiples of their size: a word never crosses a region)
                const unsigned long long tgv = (unsigned long long)tg * UINT64_C(0x0101010101010101);
                const unsigned long long *tags64 = (const unsigned long long *)mo_tags;
                for (unsigned scanned = 0; scanned <= rmask && !done;) {
                    const unsigned bw = off + s, p0 = bw & 7;
                    const unsigned long long word = __hip_atomic_load(&tags64[bw >> 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    // high bit of each byte that is 0 (exact per byte: no borrow between bytes), or equal to tg
                    constexpr unsigned long long LO7 = UINT64_C(0x7f7f7f7f7f7f7f7f);
                    const unsigned long long y = word ^ tgv;
                    unsigned long long cand = ~(((word & LO7) + LO7) | word | LO7) | ~(((y & LO7) + LO7) | y | LO7);
                    cand &= ~UINT64_C(0) << (8 * p0);
                    if (!cand) {   // no candidate in the rest of the word: the next word
                        scanned += 8 - p0;
                        s = (s + 8 - p0) & rmask;
                        continue;
                    }
                    const unsigned pos = (unsigned)__builtin_ctzll(cand) >> 3;
                    scanned += pos - p0 + 1;
                    s = (s + pos - p0) & rmask;
                    TileSlot *const sl = base + s;
                    const unsigned long long addr = (unsigned long long)sl;
                    const unsigned bi = off + s, sh = (bi & 3) * 8;
                    const unsigned b = (unsigned)(word >> (8 * pos)) & 0xffu;
                    {
                        unsigned *const cl32 = (unsigned *)cl;
                        int x = b == 0 ? -1 : kResident ? mo_holder32(cl32, bi) : mo_holder(cl, addr);
                        bool old_match = false;
                        if (b == tg && x < 0) old_match = ld_l2(&sl->cell) == p.cell && ld_l2(&sl->wenc) == we;
                        if (b == 0 || old_match) {
                            x = kResident ? mo_claim32(cl32, bi, t, ci) : mo_claim(cl, addr, t, ci);
                            if (x == -1) {
                                gslot = sl;
                                created = b == 0;
                                if (created) {
                                    atomicOr(&mo_tags[bi >> 2], tg << sh);
                                    S.res_dirty[r] = 1;
                                }
                                done = true;
                            }
                        }
                        if (!done && x >= 0 && S.sc[x] == p.cell && S.sh[x] == hk) {   // same key, this chunk
                            mo_add_into(S, x, p);
                            done = true;
                        }
                    }
                    s = (s + 1) & rmask;
                }
            } else if constexpr (!kResident) {
                const GenDesc *g = gen_lookup(C, gm, we);
                if (g) {
                    TileSlot *const tab = g->tab;
                    const unsigned long long rmask = g->rmask;
                    unsigned long long sidx = home_slot(*g, hk);
                    for (unsigned long long pr = 0; pr <= rmask && !done; pr++) {
                        TileSlot *const sl = &tab[sidx];
                        const unsigned long long addr = (unsigned long long)sl;
                        const bool free_here = ld_l2(&sl->wenc) != we;   // never used, or another window's key
                        if (free_here || ld_l2(&sl->cell) == p.cell) {
                            const int x = mo_claim(cl, addr, t, ci);
                            if (x == -1) {
                                gslot = sl;
                                created = free_here;
                                if (created) ((__attribute__((address_space(1))) uint8_t *)gen_tags(*g))[sidx] = (uint8_t)tag8(hk);
                                done = true;
                            } else if (S.sc[x] == p.cell && S.sh[x] == hk) {
                                mo_add_into(S, x, p);
                                done = true;
                            }
                        }
                        sidx = next_slot(sidx, rmask);
                    }
                }
            }
            if (!done) overflow = true;
        };
#if HM_MO_COOP_PROBE
        // The resident-only merge's probe, wave-cooperative: each round every lane still probing scans its region's
        // tags to its next candidate slot (empty or its tag); the lanes whose candidate holds an older key of the same
        // tag then load those lines TOGETHER, whole (lane L loads part L & 3 of the line of lane 16k + L / 4, 16 lines
        // per 16-B instruction, through the wave's LDS scratch), compare the key and keep the line: one round trip per
        // existing key, and no second load of the line after the barrier.
        auto probe_coop = [&](const MRec &p, bool has, TileSlot *&gslot, bool &created, int &r, int &ci, MLine &pre,
                              bool &preloaded) __attribute__((always_inline)) {
            unsigned *const cl32 = (unsigned *)S.claim;
            const unsigned long long we = p.we;
            const uint64_t hk = p.hk;
            const unsigned tg = tag8(hk);
            r = -1;
            if (has)
                for (int q = 0; q < nres; q++)
                    if (S.res_we[q] == we) r = q;
            bool done = !has || r < 0, lost = has && r < 0;
            unsigned rmask = 0, off = 0, s = 0, scanned = 0;
            TileSlot *base = nullptr;
            if (r >= 0) {
                rmask = S.res_mask[r];
                off = S.res_off[r];
                base = S.res_slots[r];
                s = (unsigned)hk & rmask;
            }
            const unsigned long long tgv = (unsigned long long)tg * UINT64_C(0x0101010101010101);
            const unsigned long long *tags64 = (const unsigned long long *)mo_tags;
            uint4 *xa = &S.xline[t >> 6][0], *xb = &S.xline[t >> 6][32];
            const int ln = lane_id();
            while (__ballot(!done)) {
                // 1. this lane's next candidate slot
                unsigned b = 0;
                bool found = false;
                if (!done) {
                    while (scanned <= rmask) {
                        const unsigned bw = off + s, p0 = bw & 7;
                        const unsigned long long word = __hip_atomic_load(&tags64[bw >> 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        constexpr unsigned long long LO7 = UINT64_C(0x7f7f7f7f7f7f7f7f);
                        const unsigned long long y = word ^ tgv;
                        unsigned long long cand = ~(((word & LO7) + LO7) | word | LO7) | ~(((y & LO7) + LO7) | y | LO7);
                        cand &= ~UINT64_C(0) << (8 * p0);
                        if (!cand) {
                            scanned += 8 - p0;
                            s = (s + 8 - p0) & rmask;
                            continue;
                        }
                        const unsigned pos = (unsigned)__builtin_ctzll(cand) >> 3;
                        scanned += pos - p0 + 1;
                        s = (s + pos - p0) & rmask;
                        b = (unsigned)(word >> (8 * pos)) & 0xffu;
                        found = true;
                        break;
                    }
                    if (!found) { done = true; lost = true; }   // the region is full
                }
                const unsigned bi = off + s;
                TileSlot *const sl = base + s;
                // 2. a tag-matching slot: claimed in this chunk (its holder), else its line from HBM, loaded together
                int x = -1;
                if (found && b != 0) x = mo_holder32(cl32, bi);
                const bool need = found && b == tg && x < 0;
                hm_v4u q0{}, q1{}, q2{}, q3{};
                const unsigned long long ga = need ? (unsigned long long)sl : 0ull;
                const unsigned long long needm = __ballot(need);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (!((needm >> (16 * k)) & 0xffffull)) continue;   // (wave-uniform)
                    const int src = k * 16 + (ln >> 2), part = ln & 3;
                    const unsigned long long sa = __shfl(ga, src, 64);
                    if (sa) {
                        const hm_v4u v = __builtin_nontemporal_load((g_cv4u *)sa + part);
                        ((part < 2) ? xa : xb)[(src & 15) * 2 + (part & 1)] = make_uint4(v.x, v.y, v.z, v.w);
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    if (need && (ln >> 4) == k) {
                        const int e = (ln & 15) * 2;
                        const uint4 a0 = xa[e], a1 = xa[e + 1], a2 = xb[e], a3 = xb[e + 1];
                        q0 = hm_v4u{a0.x, a0.y, a0.z, a0.w};
                        q1 = hm_v4u{a1.x, a1.y, a1.z, a1.w};
                        q2 = hm_v4u{a2.x, a2.y, a2.z, a2.w};
                        q3 = hm_v4u{a3.x, a3.y, a3.z, a3.w};
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                }
                const bool old_match = need && ((unsigned long long)q0.x | ((unsigned long long)q0.y << 32)) == p.cell &&
                                       ((unsigned long long)q0.z | ((unsigned long long)q0.w << 32)) == we;
                // 3. claim an empty slot or the key's own
                if (found && (b == 0 || old_match)) {
                    x = mo_claim32(cl32, bi, t, ci);
                    if (x == -1) {
                        gslot = sl;
                        created = b == 0;
                        if (created) {
                            atomicOr(&mo_tags[bi >> 2], tg << ((bi & 3) * 8));
                            S.res_dirty[r] = 1;
                        } else {
                            pre.count = (unsigned long long)q1.x | ((unsigned long long)q1.y << 32);
                            pre.nspeed = (unsigned long long)q1.z | ((unsigned long long)q1.w << 32);
                            pre.sspeed = __builtin_bit_cast(double, (unsigned long long)q2.x | ((unsigned long long)q2.y << 32));
                            pre.slat = __builtin_bit_cast(double, (unsigned long long)q2.z | ((unsigned long long)q2.w << 32));
                            pre.slon = __builtin_bit_cast(double, (unsigned long long)q3.x | ((unsigned long long)q3.y << 32));
                            pre.touched = (unsigned long long)q3.z | ((unsigned long long)q3.w << 32);
                            preloaded = true;
                        }
                        done = true;
                    }
                }
                if (found && !done && x >= 0 && S.sc[x] == p.cell && S.sh[x] == hk) {   // same key, this chunk
                    mo_add_into(S, x, p);
                    done = true;
                }
                if (found && !done) s = (s + 1) & rmask;
            }
            if (lost) overflow = true;
        };
#endif
        // the new state line of a claimed slot (old values read here: the slot's last store is visible) and its
        // update-mode row index
        // the slot's current line (all loads of a lane issued together; created slots read nothing)
        auto old_line = [&](TileSlot *gslot, bool created, const MLine &pre, bool preloaded) __attribute__((always_inline)) -> MLine {
            MLine o{};
            if (preloaded) o = pre;
            created = created || preloaded;   // (the probe loaded it: nothing to load here)
#if HM_MO_COOP_LINES
            // whole lines per load instruction (the mirror of step 4's stores): in round k, lane L loads part L & 3 of
            // the line of lane 16k + L / 4 (16-B non-temporal loads: L2-served, like ld_l2) into the wave's LDS slice,
            // and lanes 16k..16k+15 take their lines from there.  Every lane of the wave runs it (shuffles).
            const bool need = gslot && !created;
            if (__ballot(need)) {
#if HM_MO_EARLY_LINES
                // (its own scratch: the lines are loaded before the barrier, while other waves' joiners still read
                // this wave's staged keys in S.sc / S.sh)
                uint4 *xa = &S.xline[t >> 6][0], *xb = &S.xline[t >> 6][32];
#else
                uint4 *xa = (uint4 *)&S.sc[t & ~63], *xb = (uint4 *)&S.sh[t & ~63];
#endif
                const int ln = lane_id();
                const unsigned long long ga = need ? (unsigned long long)gslot : 0ull;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int src = k * 16 + (ln >> 2), part = ln & 3;
                    const unsigned long long sa = __shfl(ga, src, 64);
                    if (sa) {
                        const hm_v4u x = __builtin_nontemporal_load((g_cv4u *)sa + part);
                        ((part < 2) ? xa : xb)[(src & 15) * 2 + (part & 1)] = make_uint4(x.x, x.y, x.z, x.w);
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    if (need && (ln >> 4) == k) {
                        const int e = (ln & 15) * 2;
                        const uint4 q1 = xa[e + 1], q2 = xb[e], q3 = xb[e + 1];   // (part 0: cell, window)
                        o.count = (unsigned long long)q1.x | ((unsigned long long)q1.y << 32);
                        o.nspeed = (unsigned long long)q1.z | ((unsigned long long)q1.w << 32);
                        o.sspeed = __builtin_bit_cast(double, (unsigned long long)q2.x | ((unsigned long long)q2.y << 32));
                        o.slat = __builtin_bit_cast(double, (unsigned long long)q2.z | ((unsigned long long)q2.w << 32));
                        o.slon = __builtin_bit_cast(double, (unsigned long long)q3.x | ((unsigned long long)q3.y << 32));
                        o.touched = (unsigned long long)q3.z | ((unsigned long long)q3.w << 32);
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                }
            }
#else
            if (gslot && !created) {
                o.touched = ld_l2(&gslot->touched);
                o.count = ld_l2(&gslot->count);
                o.nspeed = ld_l2(&gslot->nspeed);
                o.sspeed = ld_l2(&gslot->sspeed);
                o.slat = ld_l2(&gslot->slat);
                o.slon = ld_l2(&gslot->slon);
            }
#endif
            return o;
        };
        auto line_of = [&](const MRec &p, const MLine &o, bool first, unsigned krow) __attribute__((always_inline)) -> MLine {
            MLine v;
            const unsigned long long acnt = S.scnt[t], ansp = S.snsp[t];
            v.count = o.count + acnt;
            v.nspeed = o.nspeed + ansp;
            v.sspeed = ansp ? o.sspeed + S.sssp[t] : o.sspeed;
            v.slat = o.slat + S.sslat[t];
            v.slon = o.slon + S.sslon[t];
            if constexpr (rehash) v.touched = p.touched;
            else v.touched = first ? ((unsigned long long)seq << 32) | krow : o.touched;
            return v;
        };
        // row index of a key's first touch in this batch: one LDS add per wave
        auto touch_rows = [&](bool first) __attribute__((always_inline)) -> unsigned {
            const unsigned long long fb = __ballot(first);
            unsigned tbase = 0;
            if (lane_id() == 0 && fb) tbase = atomicAdd(&S.n_touched, (unsigned)__popcll(fb));
            tbase = __shfl(tbase, 0, 64);
            return tbase + (unsigned)__popcll(fb & ((1ull << lane_id()) - 1));
        };
        auto count_created = [&](bool created, int r) __attribute__((always_inline)) {
            for (int q = 0; q < nres; q++) {
                const unsigned long long m = __ballot(created && r == q);
                if (m && lane_id() == 0) atomicAdd(&S.res_new[q], (unsigned)__popcll(m));
            }
        };
        // software pipeline: the next chunk's record is loaded while this chunk is merged
        Rec nxt;
        if (b0 + t < b1) nxt = ld_stream(parts + b0 + t);
        for (int64_t c0 = b0; c0 < b1; c0 += MO_THREADS) {
            // 1. stage this chunk's records in LDS
            const int64_t i = c0 + t;
            const bool has = i < b1;
            MRec p{};
            if constexpr (kWi) {
                if (has) p = mrec_of_wi(nxt, WI, winfo, cell_hi);
            } else {
                if (has) p = mrec_of(nxt, winfo, cell_hi);
            }
            if (i + MO_THREADS < b1) nxt = ld_stream(parts + i + MO_THREADS);
            if (has) {
                S.sc[t] = p.cell;
                S.sh[t] = p.hk;
                S.scnt[t] = p.cnt;
                S.snsp[t] = p.nsp;
                S.sssp[t] = p.ssp;
                S.sslat[t] = p.slat;
                S.sslon[t] = p.slon;
            }
            lds_barrier();
            // 2. find and claim the key's slot, or join the lane that holds it
            TileSlot *gslot = nullptr;
            bool created = false, preloaded = false;
            int r = -1, ci = -1;
            MLine pre{};
#if HM_MO_COOP_PROBE
            if constexpr (kResident && kCoop) probe_coop(p, has, gslot, created, r, ci, pre, preloaded);
            else if (has) probe(p, gslot, created, r, ci);
#else
            if (has) probe(p, gslot, created, r, ci);
#endif
            count_created(created, r);
#if HM_MO_EARLY_LINES
            // 3a. the claimed existing lines, loaded before the barrier (their slots' last stores were drained by an
            // earlier chunk's barrier, and no store of this chunk precedes step 4): the round trip overlaps the wait
            const MLine o = old_line(gslot, created, pre, preloaded);
            lds_barrier();
#else
            lds_barrier();
            const MLine o = old_line(gslot, created, pre, preloaded);
#endif
            // 3. the claimers' new lines
            MLine v{};
            const bool retouch = !rehash && gslot && !created && (unsigned)(o.touched >> 32) == seq;
            const bool first = !rehash && gslot && !retouch;
            unsigned krow = touch_rows(first);
            if (!first) krow = (unsigned)o.touched;
            if (gslot) v = line_of(p, o, first, krow);
            // 4. this chunk's stores: the state line (whole) and the key's row
#ifndef HM_ABL_NOSLOT   // ablation builds only: the state line stores priced by their absence
            {
                const uint64_t b0s = __builtin_bit_cast(uint64_t, v.sspeed), b1s = __builtin_bit_cast(uint64_t, v.slat);
                const uint64_t b2s = __builtin_bit_cast(uint64_t, v.slon);
                const uint4 q0 = make_uint4((unsigned)p.cell, (unsigned)(p.cell >> 32), (unsigned)p.we, (unsigned)(p.we >> 32));
                const uint4 q1 = make_uint4((unsigned)v.count, (unsigned)(v.count >> 32), (unsigned)v.nspeed, (unsigned)(v.nspeed >> 32));
                const uint4 q2 = make_uint4((unsigned)b0s, (unsigned)(b0s >> 32), (unsigned)b1s, (unsigned)(b1s >> 32));
                const uint4 q3 = make_uint4((unsigned)b2s, (unsigned)(b2s >> 32), (unsigned)v.touched, (unsigned)(v.touched >> 32));
#if HM_MO_COOP_LINES
                // whole lines per store instruction: in round k, the wave's lanes 16k..16k+15 put their lines in LDS
                // (the wave's slices of S.sc / S.sh, unused after the probe), then lane L stores part L & 3 of line
                // 16k + L / 4 -- each 16-B store instruction writes 16 whole 64-B lines instead of a quarter of 64
                // (each lane's own line: four instructions, each touching 64 different lines)
                uint4 *xa = (uint4 *)&S.sc[t & ~63], *xb = (uint4 *)&S.sh[t & ~63];
                const int ln = lane_id();
                const unsigned long long ga = (unsigned long long)gslot;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if ((ln >> 4) == k) {
                        const int e = (ln & 15) * 2;
                        xa[e] = q0;
                        xa[e + 1] = q1;
                        xb[e] = q2;
                        xb[e + 1] = q3;
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    const int src = k * 16 + (ln >> 2), part = ln & 3;
                    const unsigned long long sa = __shfl(ga, src, 64);
                    const uint4 val = ((part < 2) ? xa : xb)[(src & 15) * 2 + (part & 1)];
                    if (sa) st_g16((uint4 *)sa + part, val);
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                }
#else
                if (gslot) {
                    uint4 *d = (uint4 *)gslot;   // the whole 64-B line
                    d[0] = q0;
                    d[1] = q1;
                    d[2] = q2;
                    d[3] = q3;
                }
#endif
            }
#endif
            if (gslot) {
                if (created) created_cnt++;
#ifndef HM_ABL_NOROWS
                if (!rehash) put_row(rows, b0 + krow, p.cell, p.we, v.count, v.nspeed, v.sspeed, v.slat, v.slon);
#endif
            }
            // created keys of non-resident windows count for their window here (resident ones: res_new); rehash:
            // the host already carries the moved keys
            if constexpr (!kResident) {
                const bool count_here = created && !rehash && r < 0;
                if (__ballot(count_here) && !wave_count_windows(count_here, p.we, 1ull, WL, sink)) overflow = true;
            }
            // 5. drain this chunk's stores (visible to the next chunk's probes: a full barrier waits for every store of
            // the wave -- measured: draining them a chunk later instead, deferring the keys the previous chunk wrote,
            // cost 1.5 ms on the bench and 4.5 ms on the state-read leg); release the claims
            __syncthreads();
            if (ci >= 0) {
                if constexpr (kResident) ((unsigned *)S.claim)[ci] = 0u;
                else S.claim[ci] = 0;
            }
        }
        lds_barrier();
        // 6. write the resident regions' tags back
        if (t < nres && S.res_new[t] && !gmap_add(gm, S.res_we[t], S.res_new[t])) overflow = true;
        for (int r = 0; r < nres; r++) {
            if (!S.res_dirty[r]) continue;
            uint4 *dst = (uint4 *)S.res_gtags[r];
            const unsigned w0 = S.res_off[r] >> 4, nw = (S.res_mask[r] + 1) >> 4;
            for (unsigned q = t; q < nw; q += MO_THREADS) st_g16(dst + q, ((const uint4 *)mo_tags)[w0 + q]);
        }
        if (t == 0) { bin_cnt[bin] = S.n_touched; S.n_touched = 0; }
        lds_barrier();
    }
    if (!wl_flush(WL, sink)) overflow = true;
    created_cnt = wave_sum(created_cnt);
    unsigned long long ov = __ballot(overflow);
    if (lane_id() == 0) {
        if (created_cnt) atomicAdd(&st->n_state_new, created_cnt);
        if (ov) atomicAdd(&st->overflow, 1ull);
    }
}

// =====================================================================================================
// K4: close the gaps between the bins' row segments: bin b's rows [O(b), O(b) + cnt[b]) -> [off[b], ...)
// =====================================================================================================
// zero n16 16-B words (the window tables' tag bytes on pool reuse: hipMemsetAsync's fill kernel ran at ~0.3 TB/s
// on these 64-MB ranges, 0.68 ms per batch)
__global__ __launch_bounds__(256) void k_zero16(uint4 *__restrict__ p, int64_t n16) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) p[i] = make_uint4(0u, 0u, 0u, 0u);
}

// the start of a batch in one launch (was six memsets and a copy): the batch statistics (max ts / min window start
// at their identities), the fast-path exception and dedup give-up words, the window registry and its census
__global__ __launch_bounds__(256) void k_batch_reset(unsigned long long *__restrict__ st, unsigned long long *__restrict__ slow_word,
                                                     unsigned long long *__restrict__ giveup_word, unsigned long long *__restrict__ wreg2,
                                                     int n_wreg2) {
    static_assert(sizeof(DevStats) % 8 == 0 && offsetof(DevStats, min_wstart) == offsetof(DevStats, max_ts_ms) + 8, "DevStats");
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_wreg2) wreg2[i] = 0;
    if (i < (int)(sizeof(DevStats) / 8)) {
        const int mx = (int)(offsetof(DevStats, max_ts_ms) / 8);
        st[i] = i == mx ? (unsigned long long)INT64_MIN : i == mx + 1 ? (unsigned long long)INT64_MAX : 0ull;
    }
    if (i == 0) { *slow_word = 0; *giveup_word = 0; }
}

// In-place densification of the per-bin row segments: bin b's merged rows are [s_b, s_b + c_b) of the staging
// arrays (s_b = the bin's first partial, c_b its touched keys), so the rows [0, T) (T = sum c_b) are dense except
// for the gaps left by keys with several partials; each gap below T takes one row from above T (gap i <- the i-th
// row at or above T, both counted in bin order).  Moves only the ~2% gap rows instead of every row.
__global__ __launch_bounds__(256) void k_gap_counts(const unsigned long long *__restrict__ O, int64_t ntiles, int nbins,
                                                    const unsigned *__restrict__ cnt, const unsigned long long *__restrict__ T_ptr,
                                                    unsigned *__restrict__ g, unsigned *__restrict__ v) {
    const unsigned long long T = *T_ptr;
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < nbins; b += gridDim.x * blockDim.x) {
        const unsigned long long s = O[(int64_t)b * ntiles], e = O[(int64_t)(b + 1) * ntiles], c = cnt[b];
        const unsigned long long glo = s + c, ghi = e < T ? e : T;
        g[b] = ghi > glo ? (unsigned)(ghi - glo) : 0u;
        const unsigned long long vlo = s > T ? s : T, vhi = s + c;
        v[b] = vhi > vlo ? (unsigned)(vhi - vlo) : 0u;
    }
}
__global__ __launch_bounds__(256) void k_fill_gaps(RowsOut r, const unsigned long long *__restrict__ O, int64_t ntiles, int nbins,
                                                   const unsigned *__restrict__ cnt, const unsigned long long *__restrict__ T_ptr,
                                                   const unsigned *__restrict__ g, const unsigned long long *__restrict__ goff,
                                                   const unsigned long long *__restrict__ voff) {
    const unsigned long long T = *T_ptr;
    for (int b = blockIdx.x; b < nbins; b += gridDim.x) {
        const unsigned ng = g[b];
        if (!ng) continue;
        const unsigned long long dst0 = O[(int64_t)b * ntiles] + cnt[b], g0 = goff[b];
        int lo = -1;   // the donor bin: the last bin with voff <= i
        for (unsigned k = threadIdx.x; k < ng; k += blockDim.x) {
            const unsigned long long i = g0 + k;
            if (lo < 0) {   // a thread's first row: binary search (13 dependent loads)
                lo = 0;
                int hi = nbins;
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (voff[mid] <= i) lo = mid; else hi = mid;
                }
            } else {        // i grows by blockDim.x per row: the donor bin moves forward a few bins at most
                while (lo + 1 < nbins && voff[lo + 1] <= i) lo++;
            }
            const unsigned long long sb = O[(int64_t)lo * ntiles];
            const int64_t src = (int64_t)((sb > T ? sb : T) + (i - voff[lo])), dst = (int64_t)(dst0 + k);
            r.cell[dst] = r.cell[src];
            r.ws[dst] = r.ws[src];
            r.cnt[dst] = r.cnt[src];
            r.sp[dst] = r.sp[src];
            r.spnull[dst] = r.spnull[src];
            r.lon[dst] = r.lon[src];
            r.lat[dst] = r.lat[src];
        }
    }
}
// =====================================================================================================
// K5: latest position per (provider, vehicleId)
// =====================================================================================================
__device__ __forceinline__ long long find_or_claim_vkey(DedupSlot *tab, unsigned long long mask, unsigned long long v,
                                                        bool &claimed, unsigned long long max_probe) {
    unsigned long long h = vkey_hash(v) & mask;
    claimed = false;
    for (unsigned long long probe = 0; probe < max_probe; probe++) {
        unsigned long long cur = __hip_atomic_load(&tab[h].vkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == EMPTY_VKEY) {
            cur = atomicCAS(&tab[h].vkey, EMPTY_VKEY, v);
            if (cur == EMPTY_VKEY) { claimed = true; return (long long)h; }
        }
        if (cur == v) return (long long)h;
        h = (h + 1) & mask;
    }
    return -1;
}
// find_or_claim_vkey that also returns the slot's max ts, read together with its key (one round trip; a stale max
// is <= the true one and only costs the caller an extra atomicMax)
__device__ __forceinline__ long long find_or_claim_vkey_ts(DedupSlot *tab, unsigned long long mask, unsigned long long v,
                                                           bool &claimed, unsigned long long max_probe, long long &cur_max) {
    unsigned long long h = vkey_hash(v) & mask;
    claimed = false;
    for (unsigned long long probe = 0; probe < max_probe; probe++) {
        unsigned long long cur = __hip_atomic_load(&tab[h].vkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cur_max = __hip_atomic_load(&tab[h].maxts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == EMPTY_VKEY) {
            cur = atomicCAS(&tab[h].vkey, EMPTY_VKEY, v);
            if (cur == EMPTY_VKEY) { claimed = true; return (long long)h; }
        }
        if (cur == v) return (long long)h;
        h = (h + 1) & mask;
    }
    return -1;
}
__device__ __forceinline__ long long find_vkey(const DedupSlot *tab, unsigned long long mask, unsigned long long v) {
    unsigned long long h = vkey_hash(v) & mask;
    for (unsigned long long probe = 0; probe <= mask; probe++) {
        unsigned long long cur = tab[h].vkey;
        if (cur == v) return (long long)h;
        if (cur == EMPTY_VKEY) return -1;
        h = (h + 1) & mask;
    }
    return -1;
}

__global__ __launch_bounds__(256) void k_init_dedup(DedupSlot *tab, unsigned long long cap) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)cap; i += stride) {
        tab[i].vkey = EMPTY_VKEY;
        tab[i].maxts = INT64_MIN;
    }
}
__global__ __launch_bounds__(256) void k_clear_dedup(DedupSlot *tab, const unsigned int *used, const unsigned long long *n_used) {
    const int64_t n = (int64_t)*n_used;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        tab[used[i]].vkey = EMPTY_VKEY;
        tab[used[i]].maxts = INT64_MIN;
    }
}

// rows (or candidates) -> per-vkey max ts
__global__ __launch_bounds__(256) void k_dedup_max(const uint64_t *__restrict__ vkey, const int64_t *__restrict__ ts,
                                                   const uint8_t *__restrict__ flags, const Cand *__restrict__ cands, int64_t n,
                                                   DedupSlot *tab, unsigned long long mask, unsigned int *used,
                                                   unsigned long long *n_used, DevStats *st) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    bool overflow = false;
    unsigned long long bad = 0;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        int64_t i = base + threadIdx.x;
        bool claimed = false;
        long long h = -1;
        if (i < n) {
            bool take;
            unsigned long long v;
            long long t;
            if (cands) { take = true; v = cands[i].vkey; t = cands[i].ts; }
            else { take = (flags[i] & F_VALID) != 0; v = take ? vkey[i] : 0; t = take ? ts[i] : 0; }
            if (take && v == EMPTY_VKEY) { bad++; take = false; }
            if (take) {
                h = find_or_claim_vkey(tab, mask, v, claimed, mask + 1);
                if (h < 0) {
                    overflow = true;
                } else {
                    // a stale relaxed read is <= the true max: it can only cost an extra atomic
                    long long cur = __hip_atomic_load(&tab[h].maxts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (t > cur) atomicMax(&tab[h].maxts, t);
                }
            }
        }
        unsigned long long pos = wave_append(claimed, n_used);
        if (claimed) used[pos] = (unsigned int)h;
    }
    bad = wave_sum(bad);
    unsigned long long ov = __ballot(overflow);
    if (lane_id() == 0) {
        if (ov) atomicAdd(&st->overflow, 1ull);
        if (bad) atomicAdd(&st->bad_vkey, bad);
    }
}

// winner flag per row (or candidate): ts == max ts of its vkey.  DF_U rows per thread, their first probes
// issued together, each probe one 16-B slot load (key and max ts): the lookups' latencies overlap.
constexpr int DF_U = 4;
__global__ __launch_bounds__(256) void k_dedup_flag(const uint64_t *__restrict__ vkey, const int64_t *__restrict__ ts,
                                                    const uint8_t *__restrict__ flags, const Cand *__restrict__ cands, int64_t n,
                                                    const DedupSlot *__restrict__ tab, unsigned long long mask,
                                                    uint8_t *__restrict__ win, bool only_cand) {
    const int64_t step = (int64_t)blockDim.x * DF_U;
    for (int64_t base = (int64_t)blockIdx.x * step; base < n; base += (int64_t)gridDim.x * step) {
        unsigned long long v[DF_U], h[DF_U];
        long long t[DF_U];
        bool take[DF_U];
        for (int u = 0; u < DF_U; u++) {
            const int64_t i = base + u * blockDim.x + threadIdx.x;
            take[u] = false;
            v[u] = 0;
            t[u] = 0;
            if (i < n) {
                if (cands) { take[u] = true; v[u] = cands[i].vkey; t[u] = cands[i].ts; }
                else if (only_cand) {   // k_ingest's max saw every row: only its candidates can be at the max
                    take[u] = (flags[i] & F_CAND) != 0;
                    if (take[u]) { v[u] = vkey[i]; t[u] = ts[i]; }
                } else { v[u] = vkey[i]; t[u] = ts[i]; take[u] = (flags[i] & F_VALID) != 0; }   // (loads not waiting for the flag)
            }
            take[u] = take[u] && v[u] != EMPTY_VKEY;
            h[u] = vkey_hash(v[u]) & mask;
        }
        DedupSlot sl[DF_U];
        for (int u = 0; u < DF_U; u++)
            if (take[u]) sl[u] = tab[h[u]];
        for (int u = 0; u < DF_U; u++) {
            const int64_t i = base + u * blockDim.x + threadIdx.x;
            uint8_t w = 0;
            if (take[u]) {
                for (unsigned long long probe = 0; probe <= mask; probe++) {
                    if (sl[u].vkey == v[u]) { w = sl[u].maxts == t[u]; break; }
                    if (sl[u].vkey == EMPTY_VKEY) break;
                    h[u] = (h[u] + 1) & mask;
                    sl[u] = tab[h[u]];
                }
            }
            if (i < n) win[i] = w;
        }
    }
}

// =====================================================================================================
// K1: ingest. One pass over the events: the filter (heatmap_stream.py:96-104), latLngToCell (the UDF,
// :65-75), the tumbling window and late test (:107,115), the batch's window registry, the per-vkey max ts of the
// dedup (:200-203), and one event key per row (kernels.h ekey: cell + window slot; 0 = not aggregated) -- the
// input of both aggregation paths (direct: partition + merge; table: k_agg + k_bin_reduce).  The fp64 cell
// computation dominates; the dedup's table atomics overlap with it.
// =====================================================================================================
// The fused per-vkey max gives up on a key after DEDUP_FUSED_PROBES probes (its table was sized from the previous
// batch and is too small); the first give-up is published in *dgiveup, a word on a cache line of its own, polled
// every 16 rounds (polling a DevStats word every round, a line other atomics hit, made the ingest 4x slower), and
// later rounds skip the fused dedup, which phase_dedup then reruns over the whole batch on a full-size table.
constexpr unsigned long long DEDUP_FUSED_PROBES = 32;
constexpr int IG_THREADS = 256;
#ifndef HM_INGEST_PREFETCH
#define HM_INGEST_PREFETCH 1
#endif
#ifndef HM_INGEST_TLATE
#define HM_INGEST_TLATE 1
#endif

// wave-cooperative count: lanes with pred add 1 to cnt[slot] (one LDS add per distinct slot per wave)
__device__ __forceinline__ void wave_count_slots(bool pred, int slot, unsigned *cnt) {
    unsigned long long pend = __ballot(pred);
    while (pend) {
        const int leader = __ffsll((long long)pend) - 1;
        const int s = __shfl(slot, leader, 64);
        const unsigned long long m = __ballot(pred && slot == s);
        if (lane_id() == leader) atomicAdd(&cnt[s], (unsigned)__popcll(m));
        pend &= ~m;
    }
}

__global__ __launch_bounds__(IG_THREADS) HM_SNAP_ATTR void k_ingest(
    const double *__restrict__ lat, const double *__restrict__ lon, const int64_t *__restrict__ ts,
    const uint8_t *__restrict__ row_valid, const uint64_t *__restrict__ vkey, int64_t i_begin, int64_t n, int res, FloorDiv wdiv,
    int64_t late_end_us, uint8_t *__restrict__ flags_out, uint64_t *__restrict__ keys_out, DedupSlot *dtab,
    unsigned long long dmask, unsigned int *dused, unsigned long long *n_dused, unsigned int *__restrict__ slow,
    unsigned long long *n_slow, unsigned long long *dgiveup, unsigned long long *wreg, unsigned long long *wcount,
    DevStats *st) {
    __shared__ WinCacheL WC;
    __shared__ double Fc[20][3], Fu[20][2][3];   // the fast path's per-face tables (res parity): LDS reads
    __shared__ unsigned dskip;                    // the fused dedup has given up (*dgiveup) -- skip it
    __shared__ long long tmax_l[IG_THREADS];      // per-thread max ts (an LDS max per row instead of 2 live registers)
    for (int k = threadIdx.x; k < 60; k += IG_THREADS) (&Fc[0][0])[k] = (&c_tab.faceCenterPoint[0][0])[k];
    for (int k = threadIdx.x; k < 120; k += IG_THREADS) (&Fu[0][0][0])[k] = (&c_tab.fastU[res & 1][0][0][0])[k];
    // _faceIjkToH3's base-cell tables in LDS (7.7 KB): from __constant__ memory they were lane-indexed vector loads
    // at the end of every cell, each with a full wait that also waited for the next round's prefetched columns
    __shared__ H3BaseTables BT;
    for (int k = threadIdx.x; k < 20 * 27 * 2; k += IG_THREADS) (&BT.faceIjkBaseCells[0][0][0][0][0])[k] = (&c_tab.faceIjkBaseCells[0][0][0][0][0])[k];
    for (int k = threadIdx.x; k < 122 * 7; k += IG_THREADS) (&BT.baseCellData[0][0])[k] = (&c_tab.baseCellData[0][0])[k];
    wc_init(WC);
    if (threadIdx.x == 0) dskip = 0;
    __syncthreads();
    const int64_t tile_us = wdiv.d;
    // per-thread counters in 32 bits (a thread sees at most n / gstride < 2^32 rows): fewer registers live across
    // the cell computation, whose peak spilled the prefetched columns
    unsigned nvalid = 0, nlate = 0, bad = 0, wover = 0;
    tmax_l[threadIdx.x] = INT64_MIN;
    bool dretry = false;
    int round = 0;
    const int64_t gstride = (int64_t)gridDim.x * IG_THREADS;
#if HM_INGEST_PREFETCH
    // the next round's columns are loaded while this round computes its cells (software pipelining: the loads'
    // latency hides behind the fp64 work instead of stalling every round)
    double nla = 0.0, nlo = 0.0;
    int64_t nt = 0;
    unsigned long long nv = EMPTY_VKEY;
    uint8_t nrv = 1;
    {
        const int64_t i0 = i_begin + (int64_t)blockIdx.x * IG_THREADS + threadIdx.x;
        if (i0 < n) {
            nla = __builtin_nontemporal_load(&lat[i0]);
            nlo = __builtin_nontemporal_load(&lon[i0]);
#if !HM_INGEST_TLATE
            nt = __builtin_nontemporal_load(&ts[i0]);
#endif
            nv = __builtin_nontemporal_load(&vkey[i0]);
            if (row_valid) nrv = __builtin_nontemporal_load(&row_valid[i0]);
        }
    }
#endif
    for (int64_t base = i_begin + (int64_t)blockIdx.x * IG_THREADS; base < n; base += gstride, round++) {
        const int64_t i = base + threadIdx.x;
        const bool in = i < n;
#if HM_INGEST_PREFETCH
        const double la = nla, lo = nlo;
#if HM_INGEST_TLATE
        // ts is not prefetched: it is loaded now and first used after the cell, whose computation hides the load
        // (prefetched, the next round's ts was the register the cell computation's peak spilled -- a spill that
        // waited for every prefetched load mid-round)
        const int64_t t = in ? __builtin_nontemporal_load(&ts[i]) : 0;
        (void)nt;
#else
        const int64_t t = nt;
#endif
        const unsigned long long v = nv;
        const bool rv = nrv != 0;
#if HM_INGEST_TLATE
        {
            // unconditional (the row clamped to the last one; a row past n is never used): a conditional load keeps
            // the old value on the other path, and that register copy waited for every load in flight
            const int64_t j = i + gstride < n ? i + gstride : n - 1;
            nla = __builtin_nontemporal_load(&lat[j]);
            nlo = __builtin_nontemporal_load(&lon[j]);
            nv = __builtin_nontemporal_load(&vkey[j]);
            nrv = __builtin_nontemporal_load(   // (no branch: see above; global, not flat: a flat load's wait is a full one)
                (__attribute__((address_space(1))) const uint8_t *)(row_valid ? &row_valid[j] : &g_one_byte));
        }
#else
        if (i + gstride < n) {
            nla = __builtin_nontemporal_load(&lat[i + gstride]);
            nlo = __builtin_nontemporal_load(&lon[i + gstride]);
            nt = __builtin_nontemporal_load(&ts[i + gstride]);
            nv = __builtin_nontemporal_load(&vkey[i + gstride]);
            if (row_valid) nrv = __builtin_nontemporal_load(&row_valid[i + gstride]);
        }
#endif
#else
        double la = 0.0, lo = 0.0;
        int64_t t = 0;
        unsigned long long v = EMPTY_VKEY;
        bool rv = true;
        if (in) {
            la = lat[i];
            lo = lon[i];
            t = ts[i];
            v = vkey[i];
            if (row_valid) rv = row_valid[i] != 0;
        }
#endif
#if HM_INGEST_TLATE
        // the cell of every row in range, before the ts- and validity-dependent tests (late, invalid or
        // out-of-range-ts rows waste their cell): nothing loaded this round is waited for before the cell
        const bool geo0 = in && la >= -90.0 && la <= 90.0 && lo >= -180.0 && lo <= 180.0;
        bool exc = false;
        uint64_t cell = EMPTY_CELL;
#ifdef HM_ABL_NOCELL
        if (geo0) cell = mix64(__builtin_bit_cast(uint64_t, la) ^ mix64(__builtin_bit_cast(uint64_t, lo)));
#else
        if (geo0) exc = !latLngToCellFastP(la, lo, res, c_tab, Fc, Fu, cell, BT);
#endif
        const bool geo = geo0 && rv;
#else
        const bool geo = in && rv && la >= -90.0 && la <= 90.0 && lo >= -180.0 && lo <= 180.0;
#endif
        const bool ok = geo && t > INT64_MIN + 2 * tile_us && t < INT64_MAX - 2 * tile_us;
        // dedup: the vkey's home slot is loaded now, its latency hidden behind the cell computation (a plain load:
        // a stale copy can only show the slot empty or its max lower, both of which the atomics below correct)
#ifdef HM_ABL_NODEDUP
        const bool dd = false;
#else
        const bool dd = ok && v != EMPTY_VKEY && !__hip_atomic_load(&dskip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
        const unsigned long long dh0 = vkey_hash(v) & dmask;
        DedupSlot d0{EMPTY_VKEY, 0};
        if (dd) d0 = dtab[dh0];
        uint8_t fl = 0;
        int widx = -1, wslot = -1;
        if (ok) {
            const int64_t wq = floor_div(t, wdiv);   // tumbling window: floor(t / tile) (Spark TimeWindowing)
            const int64_t ws = wq * tile_us;
            const bool late = (ws + tile_us) <= late_end_us;
            fl = late ? (F_VALID | F_LATE) : (F_VALID | F_AGG);
            nvalid++;
            nlate += late;
            atomicMax(&tmax_l[threadIdx.x], (long long)t);
            if (!late) {
                widx = wc_lookup(WC, wreg, wq, wenc_of(ws), wslot);
                if (widx < 0) { wover++; fl = F_VALID; }   // registry full: the batch fails (hm_process_batch)
            }
        }
        // cell of the aggregated rows; margin exceptions go to k_ingest_exact (exact path), which fills their key
#if HM_INGEST_TLATE
        exc = exc && (fl & F_AGG) != 0;
#else
        bool exc = false;
        uint64_t cell = EMPTY_CELL;
#ifdef HM_ABL_NOCELL   // ablation builds (tools/ablate_ingest.sh): a hash stands in for the cell
        if (fl & F_AGG) cell = mix64(__builtin_bit_cast(uint64_t, la) ^ mix64(__builtin_bit_cast(uint64_t, lo)));
#else
        if (fl & F_AGG) exc = !latLngToCellFastP(la, lo, res, c_tab, Fc, Fu, cell, BT);
#endif
#endif
        {
            const unsigned long long pos = wave_append(exc, n_slow);
            if (exc) slow[pos] = (unsigned int)i;
        }
        // dedup: per-vkey max ts over the valid rows (late rows included, as in the reference's batch frame)
        bool claimed = false;
        long long dh = -1;
        bad += ok && v == EMPTY_VKEY;
        bool cand = false;
        if (dd) {
            long long cur = d0.maxts;
            if (d0.vkey == v) dh = (long long)dh0;   // the usual case: the key sits in its home slot
            else dh = find_or_claim_vkey_ts(dtab, dmask, v, claimed, DEDUP_FUSED_PROBES, cur);
            if (dh < 0) {
                if (!dretry) atomicExch(dgiveup, 1ull);
                dretry = true;
            } else {
                // (cur may be stale, i.e. below the slot's max: a superset of the rows at the final max)
                cand = t >= cur || claimed;
                if (t > cur) atomicMax(&dtab[dh].maxts, (long long)t);
            }
        }
        const bool agg = (fl & F_AGG) != 0;
        if (in) {
            flags_out[i] = fl | (cand ? F_CAND : 0);
            keys_out[i] = agg ? ekey_make(exc ? 0 : cell, (unsigned)widx) : 0;
        }
        const unsigned long long pos = wave_append(claimed, n_dused);
        if (claimed) dused[pos] = (unsigned int)dh;
        // census: aggregated rows per window (sizes the window tables of the direct path)
        wave_count_slots(agg && wslot >= 0, wslot, WC.cnt);
        if (agg && wslot < 0) atomicAdd(&wcount[widx], 1ull);
        // poll the give-up flag now and then (its own cache line)
        if (threadIdx.x == 0 && (round & 15) == 15 && !dskip)
            __hip_atomic_store(&dskip, __hip_atomic_load(dgiveup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ? 1u : 0u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < WC_SLOTS; q += IG_THREADS)
        if (WC.cnt[q]) atomicAdd(&wcount[(WC.e[q] & 0xfff) - 1], (unsigned long long)WC.cnt[q]);
    const unsigned long long wvalid = wave_sum((unsigned long long)nvalid), wlate = wave_sum((unsigned long long)nlate);
    const unsigned long long wbad = wave_sum((unsigned long long)bad), wwover = wave_sum((unsigned long long)wover);
    const long long tmax = wave_max(tmax_l[threadIdx.x]);
    const unsigned long long rt = __ballot(dretry);
    if (lane_id() == 0) {
        if (wvalid) atomicAdd(&st->n_valid, wvalid);
        if (wlate) atomicAdd(&st->n_late, wlate);
        if (tmax != INT64_MIN) atomicMax(&st->max_ts_ms, (long long)(tmax / 1000));   // trunc(max) = max(trunc)
        if (wbad) atomicAdd(&st->bad_vkey, wbad);
        if (wwover) atomicAdd(&st->win_overflow, wwover);
        if (rt) atomicAdd(&st->dedup_retry, 1ull);
    }
}

// exceptions of k_ingest's fast path: upstream's exact sequence; the cell bits go into the row's key (k_ingest
// wrote its window slot)
__global__ __launch_bounds__(256) void k_ingest_exact(const double *__restrict__ lat, const double *__restrict__ lon, int res,
                                                      const unsigned int *__restrict__ slow, const unsigned long long *n_slow,
                                                      uint64_t *__restrict__ keys) {
    const int64_t m = (int64_t)*n_slow;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
        const unsigned i = slow[q];
        keys[i] |= latLngToCellDeg(lat[i], lon[i], res, c_tab) & CELL_LO;
    }
}

// Heavy hitters in the batch's event keys, for the choice of the aggregation path when the last batch says nothing
// (the first batch, or a sudden change of the data): HS_SAMPLE keys at an even stride, the largest
// multiplicity among them -> DevStats.sample_max_run.  A key holding a few % of the rows would put that share of the
// batch through one merge workgroup (one bin) on the direct path; table mode aggregates it in LDS first.
constexpr int HS_SAMPLE = 4096, HS_THREADS = 1024, HS_SLOTS = 2 * HS_SAMPLE;
// (the multiplicities counted in an LDS hash table at load <= 1/2: was a bitonic sort of the sample, 78 barriers)
__global__ __launch_bounds__(HS_THREADS) void k_sample_heavy(const uint64_t *__restrict__ keys, int64_t n, DevStats *st) {
    __shared__ unsigned long long k[HS_SLOTS];
    __shared__ unsigned c[HS_SLOTS];
    __shared__ unsigned best;
    const int t = threadIdx.x;
    const int64_t stride = n / HS_SAMPLE > 0 ? n / HS_SAMPLE : 1;
    constexpr int PER = HS_SAMPLE / HS_THREADS;
    uint64_t v[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {   // every load in flight before the table is cleared
        const int64_t i = (int64_t)(t + u * HS_THREADS) * stride;
        v[u] = i < n ? keys[i] : 0;
    }
    for (int q = t; q < HS_SLOTS; q += HS_THREADS) { k[q] = 0; c[q] = 0; }
    if (t == 0) best = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; u++) {
        if (!v[u]) continue;   // rows without a key are not counted
        unsigned h = (unsigned)mix64(v[u]) & (HS_SLOTS - 1);
        for (;;) {   // (at most HS_SAMPLE keys in 2 x as many slots: an empty or matching slot is always found)
            const unsigned long long prev = atomicCAS(&k[h], 0ull, (unsigned long long)v[u]);
            if (prev == 0 || prev == v[u]) { atomicAdd(&c[h], 1u); break; }
            h = (h + 1) & (HS_SLOTS - 1);
        }
    }
    __syncthreads();
    unsigned m = 0;
    for (int q = t; q < HS_SLOTS; q += HS_THREADS) m = c[q] > m ? c[q] : m;
    atomicMax(&best, m);
    __syncthreads();
    if (t == 0) st->sample_max_run = best;
}

// the read side's cellToBoundary (row f4; h3_boundary.h): up to 10 vertices per cell, lat/lng degrees
__global__ __launch_bounds__(256) void k_cells_boundary(const uint64_t *__restrict__ cells, int64_t n, double *__restrict__ lat,
                                                        double *__restrict__ lng, int32_t *__restrict__ nverts) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        double la[10], lo[10];
        const int nv = cellToBoundaryDeg(cells[i], c_tab, la, lo);
        nverts[i] = nv;
        for (int k = 0; k < 10; k++) {
            lat[10 * i + k] = k < nv ? la[k] : __builtin_nan("");
            lng[10 * i + k] = k < nv ? lo[k] : __builtin_nan("");
        }
    }
}

// =====================================================================================================
// K0: Kafka values -> batch columns (row f1: from_json + to_timestamp, heatmap_stream.py:88-93; json_decode.h),
// one thread per record; then the exact string dictionaries of provider and vehicleId (hash table keyed by a
// 64-bit string hash, every row verified byte for byte against its slot's representative; a hash collision
// reruns the dictionary with another seed) and vkey = provider_code * n_vehicles + vehicle_code.
// =====================================================================================================
constexpr int64_t SPAN_SCRATCH = INT64_C(1) << 62;   // span offset flag: the decoded bytes are in the scratch buffer
__global__ __launch_bounds__(256) void k_json_parse(const uint8_t *__restrict__ bytes, const int64_t *__restrict__ offs,
                                                    int64_t base, int64_t n, uint8_t *__restrict__ scratch,
                                                    double *__restrict__ lat, double *__restrict__ lon,
                                                    int64_t *__restrict__ ts, double *__restrict__ speed,
                                                    uint8_t *__restrict__ sv, uint8_t *__restrict__ rv,
                                                    int64_t *__restrict__ p_off, int32_t *__restrict__ p_len,
                                                    int64_t *__restrict__ v_off, int32_t *__restrict__ v_len,
                                                    unsigned long long *counts) {
    unsigned long long bad = 0, unsup = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        JsonRow r;
        parse_record(bytes, offs[i] - base, offs[i + 1] - base, scratch, r);
        const uint32_t f = r.flags;
        bad += (f & JF_MALFORMED) != 0;
        unsup += (f & JF_UNSUPPORTED) != 0;
        lat[i] = (f & JF_LAT) ? r.lat : __builtin_nan("");
        lon[i] = (f & JF_LON) ? r.lon : __builtin_nan("");
        ts[i] = (f & JF_TS) ? r.ts_us : 0;
        speed[i] = (f & JF_SPEED) ? r.speed : 0.0;
        sv[i] = (f & JF_SPEED) ? 1 : 0;
        rv[i] = (f & JF_PROV) && (f & JF_VEH) && (f & JF_TS) ? 1 : 0;
        p_off[i] = r.p_off | ((f & JF_PROV_ESC) ? SPAN_SCRATCH : 0);
        p_len[i] = (f & JF_PROV) ? r.p_len : -1;
        v_off[i] = r.v_off | ((f & JF_VEH_ESC) ? SPAN_SCRATCH : 0);
        v_len[i] = (f & JF_VEH) ? r.v_len : -1;
    }
    bad = wave_sum(bad);
    unsup = wave_sum(unsup);
    if (lane_id() == 0) {
        if (bad) atomicAdd(&counts[0], bad);
        if (unsup) atomicAdd(&counts[1], unsup);
    }
}

__device__ __forceinline__ const uint8_t *span_ptr(const uint8_t *bytes, const uint8_t *scratch, int64_t off) {
    return (off & SPAN_SCRATCH) ? scratch + (off & ~SPAN_SCRATCH) : bytes + off;
}
__device__ __forceinline__ uint64_t str_hash(const uint8_t *s, int n, uint64_t seed) {
    uint64_t h = mix64(seed ^ ((uint64_t)n * UINT64_C(0x9e3779b97f4a7c15)));
    for (int k = 0; k < n; k += 8) {
        uint64_t x = 0;
        for (int q = 0; q < 8 && k + q < n; q++) x |= (uint64_t)s[k + q] << (8 * q);
        h = mix64(h ^ x) + UINT64_C(0x632be59bd9b4e019);
    }
    return h & ~(UINT64_C(1) << 63);   // (never DICT_EMPTY)
}
struct DictSlot {   // cleared to all-ones bytes
    unsigned long long key;   // str_hash, < 2^63; ~0 = empty
    unsigned rep;             // the smallest row holding the string
    unsigned pad;
};
constexpr unsigned long long DICT_EMPTY = ~0ull;
constexpr int DICT_PROBES = 64;
__global__ __launch_bounds__(256) void k_dict_insert(const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ scratch,
                                                     const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                                                     int64_t n, DictSlot *tab, unsigned long long mask, uint64_t seed,
                                                     unsigned *__restrict__ slot_of, unsigned long long *overflow) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int32_t L = len[i];
        if (L < 0) { slot_of[i] = ~0u; continue; }
        const uint64_t h = str_hash(span_ptr(bytes, scratch, off[i]), L, seed);
        unsigned long long s = mix64(h ^ seed) & mask;
        unsigned got = ~0u;
        for (int p = 0; p < DICT_PROBES; p++) {
            unsigned long long k = __hip_atomic_load(&tab[s].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == DICT_EMPTY) k = atomicCAS(&tab[s].key, DICT_EMPTY, (unsigned long long)h);
            if (k == DICT_EMPTY || k == h) {
                atomicMin(&tab[s].rep, (unsigned)i);
                got = (unsigned)s;
                break;
            }
            s = (s + 1) & mask;
        }
        slot_of[i] = got;
        if (got == ~0u) atomicAdd(overflow, 1ull);
    }
}
// every row's bytes against its slot's representative: a mismatch is a 64-bit hash collision
__global__ __launch_bounds__(256) void k_dict_verify(const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ scratch,
                                                     const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                                                     int64_t n, const DictSlot *__restrict__ tab,
                                                     const unsigned *__restrict__ slot_of, unsigned long long *collide) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned s = slot_of[i];
        if (s == ~0u) continue;
        const unsigned r = tab[s].rep;
        if (r == (unsigned)i) continue;
        bool eq = len[r] == len[i];
        if (eq) {
            const uint8_t *a = span_ptr(bytes, scratch, off[i]), *b = span_ptr(bytes, scratch, off[r]);
            for (int k = 0; k < len[i] && eq; k++) eq = a[k] == b[k];
        }
        if (!eq) atomicAdd(collide, 1ull);
    }
}
__global__ __launch_bounds__(256) void k_dict_occ(const DictSlot *__restrict__ tab, int64_t cap, uint8_t *__restrict__ occ) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += stride) occ[s] = tab[s].key != DICT_EMPTY;
}
// code c = the c-th occupied slot (ascending): code_of_slot, and the code's string length
__global__ __launch_bounds__(256) void k_dict_codes(const int64_t *__restrict__ slots, const unsigned long long *n_codes,
                                                    const DictSlot *__restrict__ tab, const int32_t *__restrict__ len,
                                                    unsigned *__restrict__ code_of_slot, unsigned *__restrict__ clen) {
    const int64_t m = (int64_t)*n_codes;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += stride) {
        const int64_t s = slots[c];
        code_of_slot[s] = (unsigned)c;
        clen[c] = (unsigned)len[tab[s].rep];
    }
}
__global__ __launch_bounds__(256) void k_dict_gather(const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ scratch,
                                                     const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                                                     const int64_t *__restrict__ slots, const unsigned long long *n_codes,
                                                     const DictSlot *__restrict__ tab, const unsigned long long *__restrict__ coff,
                                                     uint8_t *__restrict__ out) {
    const int64_t m = (int64_t)*n_codes;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += stride) {
        const unsigned r = tab[slots[c]].rep;
        const uint8_t *a = span_ptr(bytes, scratch, off[r]);
        for (int k = 0; k < len[r]; k++) out[coff[c] + k] = a[k];
    }
}
__global__ __launch_bounds__(256) void k_json_vkey(const uint8_t *__restrict__ rv, const unsigned *__restrict__ pslot,
                                                   const unsigned *__restrict__ vslot, const unsigned *__restrict__ pcode,
                                                   const unsigned *__restrict__ vcode, int64_t n, uint64_t n_vehicles,
                                                   uint64_t *__restrict__ vkey) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        vkey[i] = rv[i] ? (uint64_t)pcode[pslot[i]] * n_vehicles + vcode[vslot[i]] : 0;
}
// the distinct 900-s buckets of the latest rows' eventTs (a set of int64, EMPTY = INT64_MIN), compacted into list
__global__ __launch_bounds__(256) void k_latest_buckets(const int64_t *__restrict__ rows, int64_t m,
                                                        const int64_t *__restrict__ ts, long long *set, unsigned long long mask,
                                                        long long *list, unsigned long long *n_list) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const long long b = (long long)floordiv(floordiv(ts[rows[q]], 1000000), 900);
        unsigned long long s = mix64((uint64_t)b) & mask;
        for (unsigned long long p = 0; p <= mask; p++) {
            long long k = __hip_atomic_load(&set[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == INT64_MIN) {
                k = atomicCAS((unsigned long long *)&set[s], (unsigned long long)INT64_MIN, (unsigned long long)b);
                if (k == INT64_MIN) { list[atomicAdd(n_list, 1ull)] = b; break; }
            }
            if (k == b) break;
            s = (s + 1) & mask;
        }
    }
}
__global__ __launch_bounds__(256) void k_fill_i64(long long *p, int64_t n, long long v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

// =====================================================================================================
// ordered compaction of a 0/1 byte array -> indices (deterministic, ascending)
// =====================================================================================================
constexpr int CP_THREADS = 256;
constexpr int CP_PER = 16;
constexpr int CP_TILE = CP_THREADS * CP_PER;

__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned &total, unsigned *sh) {
    unsigned incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        unsigned u = __shfl_up(incl, o, 64);
        if (lane_id() >= o) incl += u;
    }
    int wv = threadIdx.x >> 6;
    if (lane_id() == 63) sh[wv] = incl;
    __syncthreads();
    unsigned off = 0;
    total = 0;
    for (int q = 0; q < CP_THREADS / 64; q++) {
        if (q < wv) off += sh[q];
        total += sh[q];
    }
    __syncthreads();
    return off + incl - v;
}

__global__ __launch_bounds__(CP_THREADS) void k_cp_count(const uint8_t *__restrict__ f, int64_t n, unsigned *__restrict__ bc) {
    __shared__ unsigned sh[CP_THREADS / 64];
    int64_t b0 = (int64_t)blockIdx.x * CP_TILE + (int64_t)threadIdx.x * CP_PER;
    unsigned c = 0;
    for (int q = 0; q < CP_PER; q++) {
        int64_t i = b0 + q;
        c += (i < n) ? (f[i] != 0) : 0;
    }
    unsigned total;
    block_excl_scan(c, total, sh);
    if (threadIdx.x == 0) bc[blockIdx.x] = total;
}
// single block: exclusive scan of nb block counts (64-bit offsets), total -> *tot
__global__ __launch_bounds__(1024) void k_cp_scan(const unsigned *__restrict__ bc, int64_t nb, unsigned long long *__restrict__ off,
                                                  unsigned long long *tot) {
    int64_t per = (nb + 1023) / 1024;
    int64_t s0 = (int64_t)threadIdx.x * per;
    unsigned long long sum = 0;
    for (int64_t q = 0; q < per; q++) if (s0 + q < nb) sum += bc[s0 + q];
    unsigned long long total;
    unsigned long long run = block1024_exclusive(sum, &total);
    for (int64_t q = 0; q < per; q++)
        if (s0 + q < nb) { off[s0 + q] = run; run += bc[s0 + q]; }
    if (threadIdx.x == 1023) *tot = total;
}
__global__ __launch_bounds__(CP_THREADS) void k_cp_write(const uint8_t *__restrict__ f, int64_t n,
                                                         const unsigned long long *__restrict__ off, int64_t *__restrict__ out) {
    __shared__ unsigned sh[CP_THREADS / 64];
    int64_t b0 = (int64_t)blockIdx.x * CP_TILE + (int64_t)threadIdx.x * CP_PER;
    unsigned c = 0;
    uint8_t v[CP_PER];
    for (int q = 0; q < CP_PER; q++) {
        int64_t i = b0 + q;
        v[q] = (i < n) ? f[i] : 0;
        c += v[q] != 0;
    }
    unsigned total;
    unsigned ex = block_excl_scan(c, total, sh);
    unsigned long long pos = off[blockIdx.x] + ex;
    for (int q = 0; q < CP_PER; q++)
        if (v[q]) out[pos++] = b0 + q;
}

// =====================================================================================================
// owner partitioning of records for the multi-GPU exchange (counts, then ordered scatter)
// =====================================================================================================
template <typename Rec>
__device__ __forceinline__ int rec_owner(const Rec &r, int nranks);
template <>
__device__ __forceinline__ int rec_owner<TilePartial>(const TilePartial &r, int nranks) {
    return owner_of(tile_hash(r.cell, r.wstart), nranks);
}
template <>
__device__ __forceinline__ int rec_owner<Cand>(const Cand &r, int nranks) {
    return owner_of(vkey_hash(r.vkey), nranks);
}

template <typename Rec>
__global__ __launch_bounds__(256) void k_part_count(const Rec *__restrict__ recs, const unsigned long long *n_dev, int nranks,
                                                    unsigned long long *counts) {
    __shared__ unsigned long long sc[64];
    for (int r = threadIdx.x; r < nranks; r += blockDim.x) sc[r] = 0;
    __syncthreads();
    const int64_t n = (int64_t)*n_dev;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        atomicAdd(&sc[rec_owner(recs[i], nranks)], 1ull);
    __syncthreads();
    for (int r = threadIdx.x; r < nranks; r += blockDim.x)
        if (sc[r]) atomicAdd(&counts[r], sc[r]);
}
// scatter with per-owner cursors (order within an owner's segment is unspecified): per tile of 4096 records,
// LDS counts per owner, ONE global cursor reservation per (workgroup tile, owner), LDS ranks for the positions
constexpr int PS_PER = 16;
template <typename Rec>
__global__ __launch_bounds__(256) void k_part_scatter(const Rec *__restrict__ recs, const unsigned long long *n_dev, int nranks,
                                                      unsigned long long *cursor, Rec *__restrict__ out) {
    __shared__ unsigned cnt[64];
    __shared__ unsigned long long base[64];
    const int64_t n = (int64_t)*n_dev;
    const int64_t tile = 256 * PS_PER;
    for (int64_t t0 = (int64_t)blockIdx.x * tile; t0 < n; t0 += (int64_t)gridDim.x * tile) {
        if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
        __syncthreads();
        int own[PS_PER];
        unsigned loc[PS_PER];
        for (int q = 0; q < PS_PER; q++) {
            const int64_t i = t0 + q * 256 + threadIdx.x;
            own[q] = i < n ? rec_owner(recs[i], nranks) : -1;
            loc[q] = own[q] >= 0 ? atomicAdd(&cnt[own[q]], 1u) : 0u;
        }
        __syncthreads();
        if ((int)threadIdx.x < nranks && cnt[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
        __syncthreads();
        for (int q = 0; q < PS_PER; q++) {
            const int64_t i = t0 + q * 256 + threadIdx.x;
            if (own[q] >= 0) out[base[own[q]] + loc[q]] = recs[i];
        }
        __syncthreads();
    }
}

// rows flagged as local winners -> candidate records
__global__ __launch_bounds__(256) void k_make_cands(const int64_t *__restrict__ rows, const unsigned long long *n_dev,
                                                    const uint64_t *__restrict__ vkey, const int64_t *__restrict__ ts, int rank,
                                                    Cand *__restrict__ out) {
    const int64_t n = (int64_t)*n_dev;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int64_t r = rows[i];
        Cand c;
        c.vkey = vkey[r];
        c.ts = ts[r];
        c.row = r;
        c.origin = rank;
        out[i] = c;
    }
}
// owner-side winners: candidates with win flag -> (origin, row) records grouped by origin
__global__ __launch_bounds__(256) void k_winner_route(const Cand *__restrict__ cands, const int64_t *__restrict__ widx,
                                                      const unsigned long long *n_dev, int nranks, unsigned long long *counts_or_cursor,
                                                      int64_t *__restrict__ out, int pass) {
    const int64_t n = (int64_t)*n_dev;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const Cand c = cands[widx[i]];
        int o = (int)c.origin;
        if (o < 0 || o >= nranks) continue;
        unsigned long long p = atomicAdd(&counts_or_cursor[o], 1ull);
        if (pass == 1) out[p] = c.row;
    }
}

// =====================================================================================================
// host side
// =====================================================================================================
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

struct Inputs {   // a batch's device columns
    const double *lat, *lon, *sp;
    const int64_t *ts;
    const uint8_t *sv, *rv;
    const uint64_t *vk;
    int64_t n;
};

struct hm_ctx {
    hm_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    hipEvent_t ev[11] = {};
    // host inputs: their copies run on copy_stream in row chunks, k_ingest on each chunk as soon as it has arrived
    // (stage_inputs records the sources, phase_local issues copies and launches)
    static constexpr int H2D_CHUNKS = 16;
    hipStream_t copy_stream = nullptr;
    // hm_process_batch's dedup (flag + compaction) runs on side_stream while the main stream partitions and merges:
    // the two bind on different units (the dedup streams flags and probes a cache-resident table; the partition is
    // write-pattern bound, the merge instruction-issue bound)
    hipStream_t side_stream = nullptr;
    hipEvent_t side_ev[4] = {};   // [3]: the pooled tables' tags cleared (table_release)
    bool dedup_side = false;
    hipEvent_t h2d_ev[H2D_CHUNKS] = {};
    struct H2D { const void *src; void *dst; size_t el; };
    H2D h2d[7] = {};
    int n_h2d = 0;
    double timings[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // host side of the last batch call (hm_last_timings [8, 14)): wall ms of the call, ms blocked in stream
    // synchronizations, ms in device/pinned allocations and frees, the longest single synchronization and its source
    // line, allocations + frees made
    double host_ms[6] = {0, 0, 0, 0, 0, 0};
    // per-event
    DevBuf in_lat, in_lon, in_ts, in_speed, in_sv, in_vkey, in_rv;
    DevBuf cell, wstart, flags, win, rows, block_counts, block_offs;
    DevBuf partials, cands, parts_sorted, rp_H, rp_O, rp_btot, rp_boff;
    DevBuf slow;   // k_ingest's fast-path exceptions (event indices) for k_ingest_exact
    // persistent tile state: one table per live window (kernels.h: GenDesc); released tables are pooled and
    // reused without clearing
    struct Gen { unsigned long long wenc; TileSlot *tab; int log2cap; unsigned rbits; int64_t keys; int64_t batch_parts; };
    std::vector<Gen> gens;
    std::vector<std::pair<TileSlot *, int>> pool;   // (table, log2 slots)
    // state_arena_bytes: window tables carved from one zeroed reservation made at create (no driver allocation
    // inside a batch); carved tables are pooled like the others but never freed before the arena
    uint8_t *arena = nullptr;
    size_t arena_bytes = 0, arena_used = 0;
    GenDesc *d_gmap = nullptr, *h_gmap = nullptr;   // device map window -> table (host mirror)
    bool gmap_ready = false;                         // h_gmap holds the device map after this batch's merge
    GenDesc *d_glist = nullptr, *h_glist = nullptr; // the same descriptors as a dense list (kernels' LDS cache)
    int n_glist = 0;
    bool census_ready = false;                      // k_ingest filled d_cmap for this batch's partials
    WinCount *d_cmap = nullptr, *h_cmap = nullptr;  // census of the current batch's partials per window
    int64_t state_size = 0;           // live keys after the last batch
    DevBuf s_cell, s_ws, s_cnt, s_sp, s_spn, s_lon, s_lat;   // k_merge_owned's rows in per-bin segments (with gaps)
    DevBuf bin_cnt, bin_off;          // k_merge_owned: touched keys per bin, their output offsets
    DevBuf parts_regrow;              // growth: the old tables' keys as partial records
    DevBuf gapbuf;                    // k_gap_counts / k_fill_gaps: per-bin gap and donor counts + donor offsets
    unsigned long long seq = 0;
    // dedup table (persistent, cleared through its used list)
    // latest-position tables (16-B slots, cleared through their used lists): `fused` is k_ingest's, sized from the
    // last batch's distinct vkeys and kept small (cache residency is its speed); `full` serves the max pass when
    // the fused one gave up, and received candidates (multi-GPU): grow-only, so it is allocated once
    struct DedupTable {
        DedupSlot *tab = nullptr;
        unsigned long long cap = 0;
        DevBuf used;
        bool dirty = false;
        int used_word = 0;   // d_scratch word counting the used slots
    } dfused, dfull;
    DedupTable *dlast = nullptr;   // the table the last batch's flags were computed on
    int64_t dedup_seen = 0;
    int64_t n_partials_merged = 0;   // partial records of the last merge (hm_batch_out.n_partials)
    int ingest_grid = 0;             // k_ingest's persistent grid: resident workgroups per CU x CUs
    int n_cus = 0;
    // aggregation path: direct (event records -> partition -> merge) or table (k_agg + k_bin_reduce, low
    // cardinality); MOBHEAT_INGEST_MODE pins one (0 adaptive, 1 direct, 2 table)
    int ingest_mode = 0;
    // k_merge_owned's grid: 0 = one workgroup per bin; else that many persistent workgroups looping over the bins
    // (MOBHEAT_MERGE_GRID, tuning)
    int merge_grid = 0;
    int64_t prev_agg_rows = 0, prev_keys = 0;   // aggregated rows and distinct keys of the last batch
    bool merge_coop = false;   // the last batch's keys were mostly existing ones: the merge's cooperative probe
    bool last_table = false;
    int64_t last_counts[6] = {0, 0, 0, 0, 0, 0};   // hm_last_counts [0, 6) ([6], [7]: n_allocs, n_frees)
    int64_t n_allocs = 0, n_frees = 0;             // device + pinned-host allocations / frees since create
    int64_t table_evicted = 0;                   // table mode: aggregates k_agg evicted into its buckets (last batch)
    // hm_decode_json (row f1): the values on the device, the decoded columns, the string dictionaries
    struct Dict {
        DevBuf tab, slot_of, occ, slots, code_of_slot, clen, coff, cbytes, btot, boff;
        int64_t last_codes = 0;   // distinct strings of the last batch (sizes the next table: cache-resident)
        int64_t n_codes = 0;
        void *h_off = nullptr, *h_bytes = nullptr;   // pinned host copies of the dictionary
        size_t h_off_cap = 0, h_bytes_cap = 0;
    };
    DevBuf jd_bytes, jd_offs, jd_scratch, jd_lat, jd_lon, jd_ts, jd_speed, jd_sv, jd_rv, jd_vkey, jd_poff, jd_plen, jd_voff,
        jd_vlen;
    Dict jd_prov, jd_veh;
    DevBuf lb_set, lb_list;   // hm_last_latest_buckets
    DevBuf keys;                     // k_ingest's event key per row (kernels.h ekey)
    unsigned long long *d_wreg = nullptr, *h_wreg = nullptr;     // the batch's window registry (WREG_SLOTS wenc)
    unsigned long long *d_wcount = nullptr, *h_wcount = nullptr; // aggregated rows per registry slot (census)
    WInfo *d_winfo = nullptr, *h_winfo = nullptr;   // per registry slot: window parameters of the direct path
    hipEvent_t winfo_ev = nullptr;                    // recorded after the last upload from h_winfo
    DevBuf agg_bucket, agg_cursor;   // table mode: k_agg's buckets (AG_BINS x AG_SUB x cap AggRecs) + fill cursors
    unsigned agg_cap = 0;            // AggRecs per sub-bucket
    std::vector<unsigned long long> h_agg_cursor;
    // outputs (device + pinned host)
    DevBuf o_cell, o_ws, o_cnt, o_sp, o_spn, o_lon, o_lat;
    void *h_cell = nullptr, *h_ws = nullptr, *h_cnt = nullptr, *h_sp = nullptr, *h_spn = nullptr, *h_lon = nullptr,
         *h_lat = nullptr, *h_rows = nullptr;
    size_t h_tiles_cap = 0, h_rows_cap = 0;
    // stats
    DevStats *d_st = nullptr;
    DevStats *h_st = nullptr;
    unsigned long long *d_scratch = nullptr;   // 256 words: partition counts/cursors, totals
    unsigned long long *h_scratch = nullptr;
    // watermark (ms)
    int64_t wm_prev = 0, wm_cur = 0;
    int64_t epoch = -1;
    // tile update statements (hm_encode_tile_updates): the last batch's emitted tiles and their windows
    int64_t last_n_tiles = 0;
    int64_t last_n_latest = -1;   // the last hm_process_batch's latest rows (ctx->rows) and its input columns
    const uint64_t *last_vk = nullptr;
    const int64_t *last_ts = nullptr;
    const double *last_lat = nullptr, *last_lon = nullptr;
    std::vector<int64_t> batch_windows;
    DevBuf td_sizes, td_off, td_btot, td_boff, td_bytes, td_params;
    void *h_td_bytes = nullptr, *h_td_off = nullptr;
    size_t h_td_bytes_cap = 0, h_td_off_cap = 0;
    // stage API state (hm_stage_ingest -> hm_stage_send -> hm_stage_merge -> hm_stage_finish)
    int stage = 0;
    bool staged = false;                               // the last batch ran through the stage API
    int nranks = 1, rank = 0;
    int64_t stage_n_in = 0;
    int64_t stage_agg_rows = 0;
    hm_stage_sizes stage_sizes{};
    Inputs stage_I{};                                  // the batch's device columns (valid until hm_stage_send)
    DevStats stage_s1{};                               // this rank's ingest statistics
    bool stage_table = false;                          // the batch's aggregation path (the same on every rank)
    int64_t stage_gmax_ms = INT64_MIN;                 // the batch's max event time over all ranks
    int64_t stage_sent = 0;                            // tile records this rank sent
    std::vector<unsigned long long> stage_gwreg;       // the batch's global window registry (WREG_SLOTS wenc)
    std::vector<unsigned> stage_gslot;                 // this rank's registry slot -> global slot
};

static std::string g_create_err;
// d_scratch word layout: [0,64) tile partition counts/cursors, [64,128) candidate counts/cursors,
// DUSED_WORD: used-slot count of the persistent dedup table (survives until the table is cleared),
// 255: result count of the last ordered compaction
constexpr int DUSED_WORD = 253;
constexpr int FULL_USED_WORD = 240;   // used-slot count of the full dedup table
constexpr int SLOW_WORD = 252;
constexpr size_t REG_BLOCK_BYTES = 2 * (WREG_SLOTS + 1) * 8 + sizeof(DevStats);   // d_wreg | d_wcount | d_st (hm_create)   // number of k_ingest fast-path exceptions of the current batch
constexpr int REGROW_WORD = 251; // records dumped by k_dump_gen
constexpr int GIVEUP_WORD = 232;
constexpr int GAPS_WORD = 242;   // 242-243: totals of the gap / donor scans
constexpr int POSBAD_WORD = 241; // position statements: rows outside the caller's dictionaries
constexpr int JSON_WORD = 244;   // 244-248: hm_decode_json's malformed / unsupported counts, dictionary overflow /
                                 // collisions; hm_last_latest_buckets' bucket count
// (GIVEUP_WORD: k_ingest's fused dedup gave up, a cache line of its own: words 232-239)

#define HIPCHK(ctx, expr)                                                                             \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) {                                                                       \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                           \
            return HM_E_HIP;                                                                          \
        }                                                                                             \
    } while (0)

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
// hipStreamSynchronize on the context's stream, timed into host_ms (site: the caller's source line)
static hipError_t ctx_sync(hm_ctx *ctx, int site) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipStreamSynchronize(ctx->stream);
    const double ms = ms_since(t0);
    ctx->host_ms[1] += ms;
    if (ms > ctx->host_ms[3]) { ctx->host_ms[3] = ms; ctx->host_ms[4] = site; }
    return e;
}
static void host_batch_begin(hm_ctx *ctx) { for (double &x : ctx->host_ms) x = 0; }
struct BatchClock {   // the call's wall time into host_ms[0] on every return path
    hm_ctx *ctx;
    std::chrono::steady_clock::time_point t0;
    explicit BatchClock(hm_ctx *c) : ctx(c), t0(std::chrono::steady_clock::now()) {}
    ~BatchClock() { ctx->host_ms[0] = ms_since(t0); }
};
struct AllocTimer {   // times a device/pinned allocation or free into host_ms[2]
    hm_ctx *ctx;
    std::chrono::steady_clock::time_point t0;
    explicit AllocTimer(hm_ctx *c) : ctx(c), t0(std::chrono::steady_clock::now()) {}
    ~AllocTimer() { ctx->host_ms[2] += ms_since(t0); ctx->host_ms[5] += 1; }
};
static int set_err(hm_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    ctx->err = buf;
    return code;
}

// MOBHEAT_TRACE=1: every device allocation of the library (size, host wall time) to stderr
static bool g_trace = getenv("MOBHEAT_TRACE") && getenv("MOBHEAT_TRACE")[0] == '1';
static double wall_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}
static hipError_t dev_malloc(hm_ctx *ctx, void **p, size_t bytes, const char *what) {
    const double t0 = g_trace ? wall_ms() : 0;
    AllocTimer at_(ctx);
    const hipError_t e = hipMalloc(p, bytes);
    ctx->n_allocs++;
    if (g_trace) fprintf(stderr, "[mobheat] hipMalloc %-12s %10.3f GB %8.1f ms\n", what, bytes / 1e9, wall_ms() - t0);
    return e;
}

static int ensure(hm_ctx *ctx, DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return HM_OK;
    size_t want = std::max<size_t>(bytes, 256);
    // a regrowth takes 1.5x headroom: a size that creeps up over a window's life (the census of a growing window,
    // its regrow records) then reallocates O(log) times instead of in every batch that grows it
    if (b.p) want = std::max(want, b.bytes + b.bytes / 2);
    if (b.p) {
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        { AllocTimer at_(ctx); HIPCHK(ctx, hipFree(b.p)); }
        ctx->n_frees++;
        b.p = nullptr;
        b.bytes = 0;
    }
    want = (want + 4095) & ~(size_t)4095;
    if (dev_malloc(ctx, &b.p, want, "buffer") != hipSuccess) {
        (void)hipGetLastError();
        want = (std::max<size_t>(bytes, 256) + 4095) & ~(size_t)4095;   // without the headroom
        if (dev_malloc(ctx, &b.p, want, "buffer") != hipSuccess) {
            (void)hipGetLastError();
            b.p = nullptr;
            return set_err(ctx, HM_E_NOMEM, "hipMalloc(%zu) failed", want);
        }
    }
    b.bytes = want;
    return HM_OK;
}

static int grid_for(int64_t n, int threads, int max_blocks = 256 * 16) {
    int64_t b = (n + threads - 1) / threads;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (int)b;
}

static uint64_t next_pow2(uint64_t v) {
    uint64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

// ---- per-window state tables (kernels.h: GenDesc) ----
static int ilog2(uint64_t v) { return 63 - __builtin_clzll(v); }

// Geometry of a window's table for `keys` keys receiving `parts` partials per batch: load <= 1/2, regions of
// >= 2^REGION_MIN_BITS slots, and enough regions that one merge workgroup gets <= ~16k of the window's partials
// (a hot window with few keys is still merged in parallel).
// H3 cells at a resolution (2 + 120 * 7^res): no window can hold more keys than that
static int64_t h3_cells_at(int res) {
    int64_t c = 120;
    for (int r = 0; r < res; r++) c *= 7;
    return c + 2;
}

static void gen_geometry(const hm_ctx *ctx, int64_t keys, int64_t parts, int min_log2, int &log2cap, unsigned &rbits) {
    keys = std::min(keys, h3_cells_at(ctx->cfg.h3_res));   // (the census bounds keys by rows; the grid bounds them too)
    int L = ilog2(next_pow2((uint64_t)std::max<int64_t>(2 * keys, 1024)));
    const int want_rb = std::min(RP_BITS, ilog2(next_pow2((uint64_t)std::max<int64_t>((parts + 16383) / 16384, 1))));
    L = std::max({L, want_rb + REGION_MIN_BITS, min_log2});
    rbits = (unsigned)std::min(RP_BITS, L - REGION_MIN_BITS);
    log2cap = L;
}

static bool in_arena(const hm_ctx *ctx, const void *p) {
    return ctx->arena && (const uint8_t *)p >= ctx->arena && (const uint8_t *)p < ctx->arena + ctx->arena_bytes;
}

// A table of >= 2^log2cap slots: the smallest pooled table of 2^log2cap .. 2^(log2cap+2) slots (not cleared: see
// kernels.h; a window whose key count sits near a power of two must not miss the pool and pay a multi-GB hipMalloc
// every batch), else a new one zeroed once.  log2cap and rbits return the table's actual geometry.
static int table_acquire(hm_ctx *ctx, int &log2cap, unsigned &rbits, TileSlot **out) {
    int best = -1;
    for (size_t i = 0; i < ctx->pool.size(); i++) {
        const int l = ctx->pool[i].second;
        if (l >= log2cap && l <= log2cap + 2 && (best < 0 || l < ctx->pool[best].second)) best = (int)i;
    }
    if (best >= 0) {
        *out = ctx->pool[best].first;
        log2cap = ctx->pool[best].second;
        rbits = (unsigned)std::min(RP_BITS, log2cap - REGION_MIN_BITS);
        ctx->pool.erase(ctx->pool.begin() + best);
        // the slots keep the previous window's keys (never matched: other wenc), the tags were cleared at release
        HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[3], 0));
        return HM_OK;
    }
    const size_t bytes = (size_t(1) << log2cap) * (sizeof(TileSlot) + 1);   // slots, then one tag byte per slot
    TileSlot *t = nullptr;
    if (ctx->arena && ctx->arena_used + bytes <= ctx->arena_bytes) {   // zeroed at create, never handed out before
        *out = (TileSlot *)(ctx->arena + ctx->arena_used);
        ctx->arena_used += (bytes + 255) & ~(size_t)255;
        return HM_OK;
    }
    if (dev_malloc(ctx, (void **)&t, bytes, "state table") != hipSuccess) {
        (void)hipGetLastError();
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        HIPCHK(ctx, hipStreamSynchronize(ctx->side_stream));   // (pooled tags being cleared: table_release)
        std::vector<std::pair<TileSlot *, int>> keep;
        for (auto &pt : ctx->pool)
            if (in_arena(ctx, pt.first)) keep.push_back(pt); else { AllocTimer at_(ctx); (void)hipFree(pt.first); ctx->n_frees++; }
        ctx->pool.swap(keep);
        ctx->n_allocs++;
        if (hipMalloc(&t, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return set_err(ctx, HM_E_NOMEM, "state table of 2^%d slots: out of device memory", log2cap);
        }
    }
    HIPCHK(ctx, hipMemsetAsync(t, 0, bytes, ctx->stream));
    *out = t;
    return HM_OK;
}
// (the stream must have drained every kernel that reads the table).  The table's tags are cleared at once on the
// side stream -- behind the main stream's work so far, concurrent with the next batch's first kernels (k_ingest does
// not use the HBM bandwidth) -- and table_acquire waits for that (side_ev[3]).
static int table_release(hm_ctx *ctx, TileSlot *t, int log2cap) {
    const int64_t n16 = (int64_t(1) << log2cap) / 16;   // (2^log2cap >= 1024 tag bytes, 64-B aligned)
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[0], ctx->stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->side_ev[0], 0));
    hipLaunchKernelGGL(k_zero16, dim3(grid_for(n16, 256, 256 * 32)), dim3(256), 0, ctx->side_stream,
                       (uint4 *)(t + (size_t(1) << log2cap)), n16);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[3], ctx->side_stream));
    ctx->pool.emplace_back(t, log2cap);
    size_t own = 0;   // pooled tables of our own allocations (arena tables stay pooled)
    for (auto &pt : ctx->pool) own += !in_arena(ctx, pt.first);
    for (size_t i = 0; own > 8 && i < ctx->pool.size();) {
        if (in_arena(ctx, ctx->pool[i].first)) { i++; continue; }
        HIPCHK(ctx, hipStreamSynchronize(ctx->side_stream));   // (its tags may still be being cleared)
        { AllocTimer at_(ctx); (void)hipFree(ctx->pool[i].first); }
        ctx->n_frees++;
        ctx->pool.erase(ctx->pool.begin() + i);
        own--;
    }
    return HM_OK;
}

static int gens_upload(hm_ctx *ctx) {
    memset(ctx->h_gmap, 0, GMAP_SLOTS * sizeof(GenDesc));
    ctx->gmap_ready = false;   // (h_gmap is the upload's staging now)
    for (const auto &g : ctx->gens) {
        unsigned h = (unsigned)(mix64(g.wenc) & (GMAP_SLOTS - 1));
        while (ctx->h_gmap[h].wenc) h = (h + 1) & (GMAP_SLOTS - 1);
        GenDesc &d = ctx->h_gmap[h];
        d.wenc = g.wenc;
        d.tab = g.tab;
        d.rbits = g.rbits;
        d.rshift = (unsigned)g.log2cap - g.rbits;
        d.rmask = (UINT64_C(1) << d.rshift) - 1;
        d.count = (unsigned long long)g.keys;
        d.batch_parts = (unsigned long long)g.batch_parts;
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_gmap, ctx->h_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyHostToDevice, ctx->stream));
    ctx->n_glist = 0;
    for (int q = 0; q < GMAP_SLOTS; q++)
        if (ctx->h_gmap[q].wenc) ctx->h_glist[ctx->n_glist++] = ctx->h_gmap[q];
    if (ctx->n_glist)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_glist, ctx->h_glist, ctx->n_glist * sizeof(GenDesc), hipMemcpyHostToDevice, ctx->stream));
    return HM_OK;
}

// exclusive scan of the m = (nbins + 1) x ntiles tile histogram rp_H into rp_O (digit-major)
// exclusive scan of m u32 counts `in` into u64 offsets `out`
static int scan_counts(hm_ctx *ctx, const unsigned *in, int64_t m, unsigned long long *out) {
    const int64_t nb = (m + SC_PER - 1) / SC_PER;
    int rc;
    if ((rc = ensure(ctx, ctx->rp_btot, nb * 4)) || (rc = ensure(ctx, ctx->rp_boff, nb * 8))) return rc;
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, in, m, out, (unsigned *)ctx->rp_btot.p);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->rp_btot.p, nb,
                       (unsigned long long *)ctx->rp_boff.p, ctx->d_scratch + 254);
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, out, m,
                       (const unsigned long long *)ctx->rp_boff.p);
    return HM_OK;
}
static int rp_scan(hm_ctx *ctx, int64_t m) {
    return scan_counts(ctx, (const unsigned *)ctx->rp_H.p, m, (unsigned long long *)ctx->rp_O.p);
}

// radix partition of n partial records into RP_BINS bins (one per (window, region)); the sorted copy goes to
// ctx->parts_sorted, bin b starts at rp_O[b * ntiles]
// In -> Out: TilePartial -> SortedRec (table mode / stage merge, into parts_sorted), GrowRec -> GrowRec (growth, into
// parts_sorted), TilePartial -> TilePartial (the owner partition, into the caller's send buffer)
template <typename In, typename Out>
static int partition(hm_ctx *ctx, const In *parts, int64_t n, int64_t &ntiles, int nranks = 0, Out *dst = nullptr) {
    const int nbins = nranks > 0 ? nranks : RP_BINS;
    if (n >= (int64_t)UINT32_MAX) return set_err(ctx, HM_E_INVALID, "%lld partial records in one merge exceed 2^32-2", (long long)n);
    const int64_t tile = rp_tile_for(n);
    ntiles = std::max<int64_t>((n + tile - 1) / tile, 1);
    const int64_t m = (int64_t)(nbins + 1) * ntiles;   // digit nbins: gaps (cell 0), which the scatter drops
    int rc;
    if (!dst && (rc = ensure(ctx, ctx->parts_sorted, std::max<int64_t>(n, 1) * sizeof(Out)))) return rc;
    if ((rc = ensure(ctx, ctx->rp_H, m * 4)) || (rc = ensure(ctx, ctx->rp_O, m * 8))) return rc;
    hipLaunchKernelGGL(k_rp_hist<In>, dim3(ntiles), dim3(RP_THREADS), 0, ctx->stream, parts, n, tile, (const GenDesc *)ctx->d_gmap,
                       (const GenDesc *)ctx->d_glist, ctx->n_glist, nranks, nbins, (unsigned *)ctx->rp_H.p, ntiles, ctx->d_st);
    if ((rc = rp_scan(ctx, m))) return rc;
    hipLaunchKernelGGL((k_rp_scatter<In, Out>), dim3(ntiles), dim3(RP_THREADS), 0, ctx->stream, parts, n, tile,
                       (const GenDesc *)ctx->d_gmap, (const GenDesc *)ctx->d_glist, ctx->n_glist, nranks, nbins,
                       (const unsigned long long *)ctx->rp_O.p, ntiles, dst ? dst : (Out *)ctx->parts_sorted.p);
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

// the direct path's partition: n event keys with the batch's columns (I) or, on a multi-GPU owner, the received payload
// stream -> EventRecs in (window, region) bins (parts_sorted); or with nranks > 0 the wire streams grouped by owner rank
// (dst = key stream, payload_out); rows without a key fall into digit nbins (dropped)
static int phase_dedup(hm_ctx *ctx, const Inputs *I, const Cand *cands, int64_t n, bool rerun_max, hipStream_t st);
// the batch's dedup on the side stream (hm_process_batch): side_ev[1] / [2] bracket it
static int launch_side_dedup(hm_ctx *ctx, const Inputs *I) {
    int rc;
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[1], ctx->side_stream));
    if ((rc = phase_dedup(ctx, I, nullptr, I->n, false, ctx->side_stream))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[2], ctx->side_stream));
    return HM_OK;
}

template <typename Out>
static int ev_partition(hm_ctx *ctx, const uint64_t *keys, int64_t n, const Inputs *I, const uint64_t *payload_in,
                        int64_t &ntiles, int nranks = 0, Out *dst = nullptr, uint64_t *payload_out = nullptr) {
    const int nbins = nranks > 0 ? nranks : RP_BINS;
    const int64_t tile = rp_tile_for(n);
    ntiles = std::max<int64_t>((n + tile - 1) / tile, 1);
    const int64_t m = (int64_t)(nbins + 1) * ntiles;
    int rc;
    // (+ 64 slack records: k_ev_scatter_rec's lanes past a tile store there)
    if (!dst && (rc = ensure(ctx, ctx->parts_sorted, (std::max<int64_t>(n, 1) + 64) * sizeof(Out)))) return rc;
    if ((rc = ensure(ctx, ctx->rp_H, m * 4)) || (rc = ensure(ctx, ctx->rp_O, m * 8))) return rc;
    const uint64_t ch = cell_hi_of(ctx->cfg.h3_res);
    hipLaunchKernelGGL(k_ev_hist, dim3(ntiles), dim3(EV_THREADS), 0, ctx->stream, keys, n, tile, (const WInfo *)ctx->d_winfo, ch,
                       nranks, nbins, (unsigned *)ctx->rp_H.p, ntiles);
    if ((rc = rp_scan(ctx, m))) return rc;
    if constexpr (std::is_same<Out, EventRec>::value) {
        if (nranks != 0 || dst) return set_err(ctx, HM_E_STATE, "ev_partition: EventRecs go to the context's bins");
        if (payload_in)
            hipLaunchKernelGGL(k_ev_scatter_rec<true>, dim3(ntiles), dim3(SR_THREADS), 0, ctx->stream, keys, n, tile, nullptr,
                               nullptr, nullptr, nullptr, payload_in, (const WInfo *)ctx->d_winfo, ch, nbins,
                               (const unsigned long long *)ctx->rp_O.p, ntiles, (EventRec *)ctx->parts_sorted.p);
        else
            hipLaunchKernelGGL(k_ev_scatter_rec<false>, dim3(ntiles), dim3(SR_THREADS), 0, ctx->stream, keys, n, tile, I->sp, I->sv,
                               I->lat, I->lon, nullptr, (const WInfo *)ctx->d_winfo, ch, nbins,
                               (const unsigned long long *)ctx->rp_O.p, ntiles, (EventRec *)ctx->parts_sorted.p);
    } else {
        hipLaunchKernelGGL(k_ev_scatter<Out>, dim3(ntiles), dim3(EV_THREADS), 0, ctx->stream, keys, n, tile, I ? I->sp : nullptr,
                           I ? I->sv : nullptr, I ? I->lat : nullptr, I ? I->lon : nullptr, payload_in,
                           (const WInfo *)ctx->d_winfo, ch, nranks, nbins, (const unsigned long long *)ctx->rp_O.p, ntiles,
                           dst ? dst : (Out *)ctx->parts_sorted.p, payload_out);
    }
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

static RowsOut rows_of(DevBuf &cell, DevBuf &ws, DevBuf &cnt, DevBuf &sp, DevBuf &spn, DevBuf &lon, DevBuf &lat) {
    return RowsOut{(uint64_t *)cell.p, (int64_t *)ws.p, (int64_t *)cnt.p, (double *)sp.p, (uint8_t *)spn.p,
                   (double *)lon.p, (double *)lat.p};
}
static RowsOut staged_rows(hm_ctx *ctx) {
    return rows_of(ctx->s_cell, ctx->s_ws, ctx->s_cnt, ctx->s_sp, ctx->s_spn, ctx->s_lon, ctx->s_lat);
}

// the batch sequence number kept in the slots' touched words (32 bits, never 0: fresh slots hold 0)
static unsigned seq32(const hm_ctx *ctx) { return (unsigned)(ctx->seq % 0xffffffffull) + 1u; }

// merge the partitioned records (ctx->parts_sorted) of n_rows staging rows
template <typename Rec>
static int merge_sorted(hm_ctx *ctx, int64_t n_rows, int64_t ntiles) {
    constexpr bool rehash = std::is_same<Rec, GrowRec>::value;
    int rc;
    if ((rc = ensure(ctx, ctx->bin_cnt, RP_BINS * 4)) || (rc = ensure(ctx, ctx->bin_off, RP_BINS * 8)))
        return rc;
    if (!rehash) {
        const int64_t m = std::max<int64_t>(n_rows, 1);
        if ((rc = ensure(ctx, ctx->s_cell, m * 8)) || (rc = ensure(ctx, ctx->s_ws, m * 8)) || (rc = ensure(ctx, ctx->s_cnt, m * 8)) ||
            (rc = ensure(ctx, ctx->s_sp, m * 8)) || (rc = ensure(ctx, ctx->s_spn, m)) || (rc = ensure(ctx, ctx->s_lon, m * 8)) ||
            (rc = ensure(ctx, ctx->s_lat, m * 8)))
            return rc;
    }
    // resident tags: every window merged into this batch may have a region in a bin
    unsigned tag_bytes = 0;
    if (!rehash) {
        size_t need = 0;
        for (const auto &g : ctx->gens)
            if (g.batch_parts) need += size_t(1) << (g.log2cap - (int)g.rbits);
        tag_bytes = (unsigned)std::min<size_t>((need + 4095) & ~size_t(4095), MO_TAG_MAX);   // (attribute: hm_create)
    }
    const int grid = ctx->merge_grid > 0 ? std::min(ctx->merge_grid, RP_BINS) : RP_BINS;
    // every window of the batch resident in every bin (their regions' tags fit together): the variant without the
    // HBM-probing fallback
    bool resident = false;
    if (!rehash) {
        size_t need = 0;
        int nwin = 0;
        for (const auto &g : ctx->gens)
            if (g.batch_parts) { need += size_t(1) << (g.log2cap - (int)g.rbits); nwin++; }
        resident = need <= tag_bytes && nwin <= MO_RES_MAX && ctx->n_glist <= GC_MAX;
    }
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(MO_THREADS), tag_bytes, ctx->stream, (const Rec *)ctx->parts_sorted.p, n_rows,
                           (const unsigned long long *)ctx->rp_O.p, ntiles, RP_BINS, ctx->d_gmap, (const GenDesc *)ctx->d_glist,
                           ctx->n_glist, (const WInfo *)ctx->d_winfo, cell_hi_of(ctx->cfg.h3_res), seq32(ctx), staged_rows(ctx),
                           (unsigned *)ctx->bin_cnt.p, ctx->d_st, tag_bytes);
    };
    if constexpr (!rehash) {
        if (resident && ctx->merge_coop) launch(k_merge_owned<Rec, true, true>);
        else if (resident) launch(k_merge_owned<Rec, true>);
        else launch(k_merge_owned<Rec, false>);
    } else {
        launch(k_merge_owned<Rec, false>);
    }
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

// census of partial records per window (the stage merge's received partials; table mode counts its own)
static int census_of_partials(hm_ctx *ctx, const TilePartial *parts, int64_t n, std::vector<WinCount> &census) {
    if (!ctx->census_ready) {
        HIPCHK(ctx, hipMemsetAsync(ctx->d_cmap, 0, GMAP_SLOTS * sizeof(WinCount), ctx->stream));
        hipLaunchKernelGGL(k_census, dim3(grid_for(n, 256, 256 * 8)), dim3(256), 0, ctx->stream, parts, n, ctx->d_cmap, ctx->d_st);
        HIPCHK(ctx, hipGetLastError());
    }
    ctx->census_ready = false;
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_cmap, ctx->d_cmap, GMAP_SLOTS * sizeof(WinCount), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "more than %d windows in one batch", GMAP_SLOTS);
    census.clear();
    for (int q = 0; q < GMAP_SLOTS; q++)
        if (ctx->h_cmap[q].wenc) census.push_back(ctx->h_cmap[q]);
    return HM_OK;
}
// census of the direct path: the registry's windows and their aggregated rows (h_wreg / h_wcount, read back after
// k_ingest)
static void census_of_registry(const hm_ctx *ctx, std::vector<WinCount> &census) {
    census.clear();
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wreg[w] && ctx->h_wcount[w]) census.push_back(WinCount{ctx->h_wreg[w], ctx->h_wcount[w]});
}

// WInfo of every registry slot in use (after gens_prepare when with_bins: the radix bin parameters need the
// window's table geometry)
static int winfo_upload(hm_ctx *ctx, bool with_bins) {
    HIPCHK(ctx, hipEventSynchronize(ctx->winfo_ev));   // (h_winfo is reused: the previous upload must be done)
    WInfo *h = ctx->h_winfo;
    int lo = WREG_SLOTS, hi = -1;
    for (int w = 0; w < WREG_SLOTS; w++) {
        const unsigned long long we = ctx->h_wreg[w];
        if (!we) continue;
        WInfo &x = h[w];
        memset(&x, 0, sizeof x);
        x.wenc = we;
        x.inner = window_inner(wdec(we));
        x.gslot = ctx->stage_gslot.empty() ? (unsigned)w : ctx->stage_gslot[w];
        if (with_bins) {
            unsigned rbits = 0;
            bool found = false;
            for (const auto &g : ctx->gens)
                if (g.wenc == we) { rbits = g.rbits; found = true; break; }
            if (!found) return set_err(ctx, HM_E_STATE, "window without a state table");
            const unsigned sb = REGION_BITS - rbits;
            x.binp = (sb << 24) | (window_salt(we) & ((1u << sb) - 1));
        }
        lo = std::min(lo, w);
        hi = std::max(hi, w);
    }
    if (hi >= lo)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_winfo + lo, h + lo, (size_t)(hi - lo + 1) * sizeof(WInfo), hipMemcpyHostToDevice,
                                   ctx->stream));
    // the direct-mapped image the kernels keep in LDS (kernels.h WiCacheImg)
    WiCacheImg *img = (WiCacheImg *)(h + WREG_SLOTS + 1);
    for (int e = 0; e < WI_CACHE; e++) img->tag[e] = WI_NONE;
    for (int w = lo; w <= hi; w++) {
        if (!ctx->h_wreg[w]) continue;
        const int e = w & (WI_CACHE - 1);
        if (img->tag[e] == WI_NONE) {
            img->tag[e] = (unsigned)w;
            img->e[e] = h[w];
        } else {
            img->tag[e] = WI_CONFLICT;   // (both slots keep the global lookup)
        }
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_winfo + WREG_SLOTS + 1, img, sizeof(WiCacheImg), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipEventRecord(ctx->winfo_ev, ctx->stream));
    return HM_OK;
}

// Give every window of the census a table large enough for its keys after this batch (new windows: a new table;
// windows that would pass load 1/2: a larger table, filled by dumping the old one and merging the dump in rehash
// mode); upload the window map.
static int gens_prepare(hm_ctx *ctx, const std::vector<WinCount> &census) {
    std::vector<hm_ctx::Gen> old;   // tables being replaced by larger ones
    int rc;
    for (auto &g : ctx->gens) g.batch_parts = 0;
    for (const WinCount &w : census) {
        ctx->batch_windows.push_back(wdec(w.wenc));
        const int64_t c = (int64_t)w.count;
        auto it = std::find_if(ctx->gens.begin(), ctx->gens.end(), [&](const hm_ctx::Gen &g) { return g.wenc == w.wenc; });
        int L;
        unsigned rb;
        if (it == ctx->gens.end()) {
            gen_geometry(ctx, c, c, 0, L, rb);
            TileSlot *t = nullptr;
            if ((rc = table_acquire(ctx, L, rb, &t))) return rc;
            ctx->gens.push_back({w.wenc, t, L, rb, 0, c});
            continue;
        }
        if (std::min(it->keys + c, h3_cells_at(ctx->cfg.h3_res)) * 2 > (int64_t(1) << it->log2cap)) {
            gen_geometry(ctx, it->keys + c, c, it->log2cap + 1, L, rb);
            TileSlot *t = nullptr;
            if ((rc = table_acquire(ctx, L, rb, &t))) return rc;
            old.push_back(*it);
            it->tab = t;
            it->log2cap = L;
            it->rbits = rb;   // keys unchanged: the rehash merge moves them without counting
        }
        it->batch_parts = c;
    }
    if ((int)ctx->gens.size() > GMAP_SLOTS / 2)
        return set_err(ctx, HM_E_OVERFLOW, "%zu live windows exceed the window map (%d)", ctx->gens.size(), GMAP_SLOTS / 2);
    if ((rc = gens_upload(ctx))) return rc;
    if (!old.empty()) {
        int64_t moved = 0;
        for (const auto &g : old) moved += g.keys;
        if ((rc = ensure(ctx, ctx->parts_regrow, std::max<int64_t>(moved, 1) * sizeof(GrowRec)))) return rc;
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + REGROW_WORD, 0, 8, ctx->stream));
        for (const auto &g : old) {
            GenDesc d{};
            d.wenc = g.wenc;
            d.tab = g.tab;
            d.rbits = g.rbits;
            d.rshift = (unsigned)g.log2cap - g.rbits;
            d.rmask = (UINT64_C(1) << d.rshift) - 1;
            hipLaunchKernelGGL(k_dump_gen, dim3(grid_for(int64_t(1) << g.log2cap, 256)), dim3(256), 0, ctx->stream, d,
                               (GrowRec *)ctx->parts_regrow.p, ctx->d_scratch + REGROW_WORD);
        }
        HIPCHK(ctx, hipGetLastError());
        int64_t ntiles;
        if ((rc = partition<GrowRec, GrowRec>(ctx, (const GrowRec *)ctx->parts_regrow.p, moved, ntiles))) return rc;
        if ((rc = merge_sorted<GrowRec>(ctx, moved, ntiles))) return rc;
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        for (const auto &g : old)
            if ((rc = table_release(ctx, g.tab, g.log2cap))) return rc;
    }
    return HM_OK;
}

// After a batch: every window's key count from the device; windows whose end <= the eviction watermark are
// released whole (their rows are late from now on); n_state = keys of the live windows.
static int state_account(hm_ctx *ctx, int64_t evict_wm_ms) {
    if (!ctx->gmap_ready) {
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_gmap, ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    }
    ctx->gmap_ready = false;
    const int64_t dead_end_us = evict_wm_ms * 1000;
    int64_t live = 0;
    std::vector<hm_ctx::Gen> keep;
    for (auto &g : ctx->gens) {
        unsigned h = (unsigned)(mix64(g.wenc) & (GMAP_SLOTS - 1));
        for (int p = 0; p < GMAP_SLOTS && ctx->h_gmap[h].wenc; p++, h = (h + 1) & (GMAP_SLOTS - 1))
            if (ctx->h_gmap[h].wenc == g.wenc) { g.keys = (int64_t)ctx->h_gmap[h].count; break; }
        if (wdec(g.wenc) + ctx->cfg.tile_us <= dead_end_us) {
            if (int rc = table_release(ctx, g.tab, g.log2cap)) return rc;
        } else {
            live += g.keys;
            keep.push_back(g);
        }
    }
    ctx->gens.swap(keep);
    ctx->state_size = live;
    return HM_OK;
}

// Clear a dedup table through its used list and make sure it holds `n_keys` keys at <= 1/2 load; shrink: the
// table is also reallocated when it is more than twice the size needed (the fused table: cache residency).
static int dedup_prepare(hm_ctx *ctx, hm_ctx::DedupTable &d, int64_t n_keys, bool shrink) {
    if (d.dirty) {
        hipLaunchKernelGGL(k_clear_dedup, dim3(grid_for(d.cap, 256)), dim3(256), 0, ctx->stream, d.tab,
                           (const unsigned int *)d.used.p, ctx->d_scratch + d.used_word);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + d.used_word, 0, 8, ctx->stream));
        d.dirty = false;
    }
    unsigned long long want = next_pow2((unsigned long long)std::max<int64_t>(2 * n_keys, 1024));
    // (a 2 MB fused table stays in every XCD's L2, an 8 MB one does not: k_ingest 6.9 -> 28 ms on the bench)
    if (d.tab && d.cap >= want && (!shrink || d.cap <= 2 * want)) return HM_OK;
    if (d.tab) {
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        { AllocTimer at_(ctx); HIPCHK(ctx, hipFree(d.tab)); }
        ctx->n_frees++;
        d.tab = nullptr;
    }
    if (dev_malloc(ctx, (void **)&d.tab, want * sizeof(DedupSlot), "dedup table") != hipSuccess) {
        (void)hipGetLastError();
        return set_err(ctx, HM_E_NOMEM, "dedup table alloc failed");
    }
    d.cap = want;
    hipLaunchKernelGGL(k_init_dedup, dim3(grid_for(want, 256)), dim3(256), 0, ctx->stream, d.tab, want);
    HIPCHK(ctx, hipGetLastError());
    return ensure(ctx, d.used, want * sizeof(unsigned int));
}
// k_ingest's table: sized from the last batch's distinct vkeys (small and cache-resident), not from n; a batch
// with many more keys makes the fused probes give up and phase_dedup reruns the max pass on a full-size table.
static int64_t dedup_fused_keys(const hm_ctx *ctx, int64_t n) {
    const int64_t guess = ctx->dedup_seen > 0 ? ctx->dedup_seen + ctx->dedup_seen / 4 : int64_t(1) << 18;   // first batch
    return std::min<int64_t>(n, std::max<int64_t>(int64_t(1) << 15, guess));
}

// ordered compaction of byte flags -> int64 indices into ctx->rows; count into d_scratch[255]
static int compact_flags(hm_ctx *ctx, const uint8_t *f, int64_t n, int64_t *out, hipStream_t st) {
    int64_t nb = (n + CP_TILE - 1) / CP_TILE;
    if (nb < 1) nb = 1;
    int rc;
    if ((rc = ensure(ctx, ctx->block_counts, nb * sizeof(unsigned)))) return rc;
    if ((rc = ensure(ctx, ctx->block_offs, nb * sizeof(unsigned long long)))) return rc;
    hipLaunchKernelGGL(k_cp_count, dim3(nb), dim3(CP_THREADS), 0, st, f, n, (unsigned *)ctx->block_counts.p);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, st, (const unsigned *)ctx->block_counts.p, nb,
                       (unsigned long long *)ctx->block_offs.p, ctx->d_scratch + 255);
    hipLaunchKernelGGL(k_cp_write, dim3(nb), dim3(CP_THREADS), 0, st, f, n,
                       (const unsigned long long *)ctx->block_offs.p, out);
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

static int stage_inputs(hm_ctx *ctx, const hm_batch_in *in, const double **lat, const double **lon, const int64_t **ts,
                        const double **sp, const uint8_t **sv, const uint64_t **vk, const uint8_t **rv) {
    int64_t n = in->n;
    if (in->memory == HM_MEM_DEVICE || n == 0) {
        *lat = in->lat; *lon = in->lon; *ts = in->ts_us; *sp = in->speed; *sv = in->speed_valid; *vk = in->vkey;
        *rv = in->row_valid;
        return HM_OK;
    }
    struct { DevBuf *b; const void *src; size_t el; const void **dst; } items[] = {
        {&ctx->in_lat, in->lat, 8, (const void **)lat},     {&ctx->in_lon, in->lon, 8, (const void **)lon},
        {&ctx->in_ts, in->ts_us, 8, (const void **)ts},     {&ctx->in_speed, in->speed, 8, (const void **)sp},
        {&ctx->in_sv, in->speed_valid, 1, (const void **)sv}, {&ctx->in_vkey, in->vkey, 8, (const void **)vk},
        {&ctx->in_rv, in->row_valid, 1, (const void **)rv},
    };
    ctx->n_h2d = 0;
    for (auto &it : items) {
        if (!it.src) { *it.dst = nullptr; continue; }
        int rc = ensure(ctx, *it.b, n * it.el);
        if (rc) return rc;
        ctx->h2d[ctx->n_h2d++] = hm_ctx::H2D{it.src, it.b->p, it.el};   // copied by phase_local, chunk by chunk
        *it.dst = it.b->p;
    }
    return HM_OK;
}

// pinned host capacity for `need` elements, grown with 1.5x headroom (output row counts creep up as windows fill)
static size_t host_cap_for(size_t cap, size_t need) { return std::max<size_t>({need, cap + cap / 2, 1024}); }

static int ensure_host(hm_ctx *ctx, void **p, size_t &cap_el, size_t want_el, size_t el) {
    (void)cap_el;
    AllocTimer at_(ctx);
    if (*p) { HIPCHK(ctx, hipHostFree(*p)); ctx->n_frees++; }
    *p = nullptr;
    ctx->n_allocs++;
    HIPCHK(ctx, hipHostMalloc(p, std::max<size_t>(want_el, 1) * el, hipHostMallocDefault));
    return HM_OK;
}

// ---- batch phases shared by the single-GPU and stage paths ----
// k_ingest + k_ingest_exact: flags, event keys, the window registry and its census, dedup max, batch statistics
static int phase_local(hm_ctx *ctx, const Inputs &I, int64_t late_wm_ms) {
    int64_t n = I.n;
    int rc;
    if ((rc = ensure(ctx, ctx->flags, n)) || (rc = ensure(ctx, ctx->win, n)) || (rc = ensure(ctx, ctx->rows, n * 8)) ||
        (rc = ensure(ctx, ctx->keys, n * 8)) || (rc = ensure(ctx, ctx->slow, n * sizeof(unsigned int))))
        return rc;
    if ((rc = dedup_prepare(ctx, ctx->dfused, dedup_fused_keys(ctx, n), true))) return rc;
    {
        const int nw = 2 * (WREG_SLOTS + 1);   // d_wreg and d_wcount: one allocation (hm_create)
        hipLaunchKernelGGL(k_batch_reset, dim3((nw + 255) / 256), dim3(256), 0, ctx->stream, (unsigned long long *)ctx->d_st,
                           ctx->d_scratch + SLOW_WORD, ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg, nw);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[0], ctx->stream));
    if (n > 0) {
        // host inputs: row chunks copied on copy_stream, each chunk's k_ingest launched behind its copy (the copies
        // of later chunks overlap the ingest of earlier ones); device inputs: one launch
        const int nch = ctx->n_h2d ? (int)std::min<int64_t>(hm_ctx::H2D_CHUNKS, std::max<int64_t>(1, n >> 22)) : 1;
        if (ctx->n_h2d) {
            HIPCHK(ctx, hipEventRecord(ctx->h2d_ev[0], ctx->stream));   // (buffers free: the last batch is done)
            HIPCHK(ctx, hipStreamWaitEvent(ctx->copy_stream, ctx->h2d_ev[0], 0));
        }
        for (int c = 0; c < nch; c++) {
            const int64_t a = n * c / nch, b = n * (c + 1) / nch;
            if (ctx->n_h2d) {
                for (int q = 0; q < ctx->n_h2d; q++) {
                    const hm_ctx::H2D &h = ctx->h2d[q];
                    HIPCHK(ctx, hipMemcpyAsync((uint8_t *)h.dst + a * h.el, (const uint8_t *)h.src + a * h.el, (b - a) * h.el,
                                               hipMemcpyHostToDevice, ctx->copy_stream));
                }
                HIPCHK(ctx, hipEventRecord(ctx->h2d_ev[c], ctx->copy_stream));
                HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->h2d_ev[c], 0));
            }
            const int blocks = (int)std::min<int64_t>((b - a + IG_THREADS - 1) / IG_THREADS, ctx->ingest_grid);
            hipLaunchKernelGGL(k_ingest, dim3(blocks), dim3(IG_THREADS), 0, ctx->stream, I.lat, I.lon, I.ts, I.rv, I.vk, a, b,
                               ctx->cfg.h3_res, make_floor_div(ctx->cfg.tile_us), late_wm_ms * 1000, (uint8_t *)ctx->flags.p,
                               (uint64_t *)ctx->keys.p, ctx->dfused.tab, ctx->dfused.cap - 1, (unsigned int *)ctx->dfused.used.p,
                               ctx->d_scratch + ctx->dfused.used_word, (unsigned int *)ctx->slow.p, ctx->d_scratch + SLOW_WORD,
                               ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg, ctx->d_wcount, ctx->d_st);
        }
        ctx->n_h2d = 0;
        hipLaunchKernelGGL(k_ingest_exact, dim3(256), dim3(256), 0, ctx->stream, I.lat, I.lon, ctx->cfg.h3_res,
                           (const unsigned int *)ctx->slow.p, ctx->d_scratch + SLOW_WORD, (uint64_t *)ctx->keys.p);
        hipLaunchKernelGGL(k_sample_heavy, dim3(1), dim3(HS_THREADS), 0, ctx->stream, (const uint64_t *)ctx->keys.p, n, ctx->d_st);
        HIPCHK(ctx, hipGetLastError());
        ctx->dfused.dirty = true;
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], ctx->stream));
    // the batch statistics and the registry with its census, read back together
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_wreg, ctx->d_wreg, REG_BLOCK_BYTES, hipMemcpyDeviceToHost, ctx->stream));   // (+ h_wcount, h_st)
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->win_overflow)
        return set_err(ctx, HM_E_OVERFLOW, "more than %d distinct windows in one micro-batch (%llu rows)", WREG_SLOTS,
                       ctx->h_st->win_overflow);
    return HM_OK;
}

// Aggregation path of the batch: table mode when the last batches had few distinct keys that repeat a lot (their
// aggregates fit k_bin_reduce's LDS tables), or when this batch's key sample shows heavy hitters (a key in >= 1/256
// of the sampled rows: k_sample_heavy), else the direct path.
static bool choose_table(const hm_ctx *ctx, int64_t n_agg, unsigned long long sample_max_run) {
    if (ctx->ingest_mode) return ctx->ingest_mode == 2;
    if (n_agg < (int64_t(1) << 16)) return false;
    if (sample_max_run >= (unsigned long long)(HS_SAMPLE / 256)) return true;
    return ctx->prev_keys > 0 && ctx->prev_keys <= (int64_t)AG_BINS * (AG_SLOTS / 2) && ctx->prev_agg_rows >= 8 * ctx->prev_keys;
}

// table mode: k_agg + k_bin_reduce -> one partial record per key of the batch (ctx->partials, count *n_parts),
// census in d_cmap
static int phase_table(hm_ctx *ctx, const Inputs &I, int64_t n_agg, int64_t *n_parts) {
    int rc;
    const int64_t n = I.n;
    if ((rc = ensure(ctx, ctx->partials, std::max<int64_t>(n_agg, 1) * sizeof(TilePartial)))) return rc;
    const int nsub = AG_BINS * AG_SUB;
    if (ctx->agg_cap == 0)   // first table batch: room for about a quarter of the rows evicted twice over
        ctx->agg_cap = (unsigned)std::min<int64_t>(std::max<int64_t>(4096, n_agg / (2 * nsub)), int64_t(1) << 30);
    if ((rc = ensure(ctx, ctx->agg_bucket, (size_t)nsub * ctx->agg_cap * sizeof(AggRec))) ||
        (rc = ensure(ctx, ctx->agg_cursor, (size_t)nsub * 8)))
        return rc;
    HIPCHK(ctx, hipMemsetAsync(ctx->agg_cursor.p, 0, (size_t)nsub * 8, ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->d_cmap, 0, GMAP_SLOTS * sizeof(WinCount), ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(&ctx->d_st->n_partials, 0, 8, ctx->stream));
    if (n > 0) {
        const int64_t per = (n + ctx->n_cus - 1) / ctx->n_cus;
        const int64_t span = std::max<int64_t>((per + AG_THREADS - 1) / AG_THREADS, 1) * AG_THREADS;
        const uint64_t ch = cell_hi_of(ctx->cfg.h3_res);
        hipLaunchKernelGGL(k_agg, dim3((unsigned)((n + span - 1) / span)), dim3(AG_THREADS), 0, ctx->stream,
                           (const uint64_t *)ctx->keys.p, n, span, I.sp, I.sv, I.lat, I.lon, (AggRec *)ctx->agg_bucket.p,
                           (unsigned long long *)ctx->agg_cursor.p, ctx->agg_cap, (const unsigned long long *)ctx->d_wreg, ch,
                           (TilePartial *)ctx->partials.p, ctx->d_cmap, ctx->d_st);
        hipLaunchKernelGGL(k_bin_reduce, dim3(AG_BINS), dim3(AG_THREADS), 0, ctx->stream, (const AggRec *)ctx->agg_bucket.p,
                           (const unsigned long long *)ctx->agg_cursor.p, ctx->agg_cap, (const unsigned long long *)ctx->d_wreg,
                           ch, (TilePartial *)ctx->partials.p, ctx->d_cmap, ctx->d_st);
        HIPCHK(ctx, hipGetLastError());
    }
    ctx->h_agg_cursor.resize(nsub);
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_agg_cursor.data(), ctx->agg_cursor.p, (size_t)nsub * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "more than %d windows in one batch", GMAP_SLOTS);
    *n_parts = (int64_t)ctx->h_st->n_partials;
    ctx->table_evicted = (int64_t)ctx->h_st->n_evicted;
    // the next table batch's sub-bucket capacity: twice this batch's fullest one (shrinks slowly)
    unsigned long long mx = 0;
    for (unsigned long long c : ctx->h_agg_cursor) mx = std::max(mx, c);
    const unsigned want = (unsigned)std::min<unsigned long long>(std::max<unsigned long long>(4096, 2 * mx), 1ull << 30);
    if (want > ctx->agg_cap || want < ctx->agg_cap / 4) ctx->agg_cap = want;
    ctx->census_ready = true;
    return HM_OK;
}

// Dedup over the batch's rows (I != nullptr; the per-vkey max came from k_ingest unless its probes gave up:
// `rerun_max`) or over received candidates; result: ctx->rows indices, count in d_scratch[255].
static int phase_dedup(hm_ctx *ctx, const Inputs *I, const Cand *cands, int64_t n, bool rerun_max,
                       hipStream_t st = nullptr) {
    int rc;
    const bool need_max = cands != nullptr || rerun_max;
    if (!st) st = ctx->stream;
    hm_ctx::DedupTable &d = need_max ? ctx->dfull : ctx->dfused;
    if (need_max && (rc = dedup_prepare(ctx, d, n, false))) return rc;
    ctx->dlast = &d;
    if ((rc = ensure(ctx, ctx->win, std::max<int64_t>(n, 1))) || (rc = ensure(ctx, ctx->rows, std::max<int64_t>(n, 1) * 8)))
        return rc;
    if (n > 0) {
        if (need_max) {
            hipLaunchKernelGGL(k_dedup_max, dim3(grid_for(n, 256)), dim3(256), 0, st, I ? I->vk : nullptr,
                               I ? I->ts : nullptr, (const uint8_t *)ctx->flags.p, cands, n, d.tab, d.cap - 1,
                               (unsigned int *)d.used.p, ctx->d_scratch + d.used_word, ctx->d_st);
            d.dirty = true;
        }
        hipLaunchKernelGGL(k_dedup_flag, dim3(grid_for(n, 256)), dim3(256), 0, st, I ? I->vk : nullptr,
                           I ? I->ts : nullptr, (const uint8_t *)ctx->flags.p, cands, n, d.tab, d.cap - 1,
                           (uint8_t *)ctx->win.p, !need_max);
        HIPCHK(ctx, hipGetLastError());
        if ((rc = compact_flags(ctx, (const uint8_t *)ctx->win.p, n, (int64_t *)ctx->rows.p, st))) return rc;
    } else {
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + 255, 0, 8, st));
    }
    return HM_OK;
}

static int ensure_outputs(hm_ctx *ctx, int64_t n_rows) {
    int rc;
    int64_t m = std::max<int64_t>(n_rows, 1);
    if ((rc = ensure(ctx, ctx->o_cell, m * 8)) || (rc = ensure(ctx, ctx->o_ws, m * 8)) || (rc = ensure(ctx, ctx->o_cnt, m * 8)) ||
        (rc = ensure(ctx, ctx->o_sp, m * 8)) || (rc = ensure(ctx, ctx->o_spn, m)) || (rc = ensure(ctx, ctx->o_lon, m * 8)) ||
        (rc = ensure(ctx, ctx->o_lat, m * 8)))
        return rc;
    return HM_OK;
}

// densify the merge's per-bin row segments into the output rows (k_gap_counts / k_fill_gaps, then a buffer swap)
static int rows_densify(hm_ctx *ctx, int64_t ntiles) {
    int rc;
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->bin_cnt.p, (int64_t)RP_BINS,
                       (unsigned long long *)ctx->bin_off.p, &ctx->d_st->n_touched);
    if ((rc = ensure(ctx, ctx->gapbuf, (size_t)RP_BINS * 24))) return rc;
    unsigned *gg = (unsigned *)ctx->gapbuf.p, *gv = gg + RP_BINS;
    unsigned long long *gvo = (unsigned long long *)(gv + RP_BINS), *ggo = (unsigned long long *)ctx->bin_off.p;
    const unsigned long long *O = (const unsigned long long *)ctx->rp_O.p;
    hipLaunchKernelGGL(k_gap_counts, dim3(grid_for(RP_BINS, 256)), dim3(256), 0, ctx->stream, O, ntiles, RP_BINS,
                       (const unsigned *)ctx->bin_cnt.p, &ctx->d_st->n_touched, gg, gv);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, gg, (int64_t)RP_BINS, ggo, ctx->d_scratch + GAPS_WORD);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, gv, (int64_t)RP_BINS, gvo, ctx->d_scratch + GAPS_WORD + 1);
    hipLaunchKernelGGL(k_fill_gaps, dim3(RP_BINS), dim3(256), 0, ctx->stream, staged_rows(ctx), O, ntiles, RP_BINS,
                       (const unsigned *)ctx->bin_cnt.p, &ctx->d_st->n_touched, (const unsigned *)gg,
                       (const unsigned long long *)ggo, (const unsigned long long *)gvo);
    HIPCHK(ctx, hipGetLastError());
    std::swap(ctx->s_cell, ctx->o_cell);
    std::swap(ctx->s_ws, ctx->o_ws);
    std::swap(ctx->s_cnt, ctx->o_cnt);
    std::swap(ctx->s_sp, ctx->o_sp);
    std::swap(ctx->s_spn, ctx->o_spn);
    std::swap(ctx->s_lon, ctx->o_lon);
    std::swap(ctx->s_lat, ctx->o_lat);
    return HM_OK;
}

// counters_zero: the merge's counters are still as k_batch_reset left them (the direct path, right after phase_local)
static int merge_begin(hm_ctx *ctx, int64_t n_rows, bool counters_zero = false) {
    static_assert(offsetof(DevStats, n_state_new) == offsetof(DevStats, n_touched) + 8, "DevStats");
    if (!counters_zero) {
        HIPCHK(ctx, hipMemsetAsync(&ctx->d_st->n_touched, 0, 16, ctx->stream));   // (+ n_state_new)
        HIPCHK(ctx, hipMemsetAsync(&ctx->d_st->overflow, 0, 8, ctx->stream));
    }
    ctx->seq++;
    ctx->batch_windows.clear();
    return ensure_outputs(ctx, n_rows);
}
static int merge_nothing(hm_ctx *ctx) {
    for (int e : {3, 7, 4, 5}) HIPCHK(ctx, hipEventRecord(ctx->ev[e], ctx->stream));
    return HM_OK;
}

// partial records parts[0, n_parts) (table mode, stage merge): census -> window tables -> partition -> merge -> rows
static int merge_partials(hm_ctx *ctx, const TilePartial *parts, int64_t n_parts) {
    int rc;
    ctx->n_partials_merged = n_parts;
    if ((rc = merge_begin(ctx, n_parts))) return rc;
    if (n_parts == 0) { ctx->census_ready = false; return merge_nothing(ctx); }
    std::vector<WinCount> census;
    if ((rc = census_of_partials(ctx, parts, n_parts, census)) || (rc = gens_prepare(ctx, census))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    int64_t ntiles;
    if ((rc = partition<TilePartial, SortedRec>(ctx, parts, n_parts, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    if ((rc = merge_sorted<SortedRec>(ctx, n_parts, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if ((rc = rows_densify(ctx, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    return HM_OK;
}

// the direct path: the batch's event keys (k_ingest) -> census from the registry -> window tables -> event partition
// -> merge -> rows.  n_rec = aggregated rows (keys != 0)
static int merge_events(hm_ctx *ctx, const Inputs &I, int64_t n_rec) {
    int rc;
    ctx->n_partials_merged = n_rec;
    if ((rc = merge_begin(ctx, I.n, true))) return rc;   // (only k_ingest, k_sample_heavy and the side stream's
                                                          // k_dedup_flag ran since k_batch_reset: none counts these)
    if (n_rec == 0) return merge_nothing(ctx);
    std::vector<WinCount> census;
    census_of_registry(ctx, census);
    if ((rc = gens_prepare(ctx, census)) || (rc = winfo_upload(ctx, true))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    int64_t ntiles;
    if ((rc = ev_partition<EventRec>(ctx, (const uint64_t *)ctx->keys.p, I.n, &I, nullptr, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    if ((rc = merge_sorted<EventRec>(ctx, I.n, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if ((rc = rows_densify(ctx, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    return HM_OK;
}

static int finish_outputs(hm_ctx *ctx, int64_t n_tiles, int64_t n_rows, const int64_t *rows_dev, int32_t out_memory,
                          hm_batch_out *out) {
    out->n_tiles = n_tiles;
    out->n_latest = n_rows;
    ctx->last_n_tiles = n_tiles;
    std::sort(ctx->batch_windows.begin(), ctx->batch_windows.end());
    if (out_memory == HM_MEM_DEVICE) {
        out->cell = (const uint64_t *)ctx->o_cell.p;
        out->window_start_us = (const int64_t *)ctx->o_ws.p;
        out->count = (const int64_t *)ctx->o_cnt.p;
        out->avg_speed = (const double *)ctx->o_sp.p;
        out->speed_null = (const uint8_t *)ctx->o_spn.p;
        out->avg_lon = (const double *)ctx->o_lon.p;
        out->avg_lat = (const double *)ctx->o_lat.p;
        out->latest_row = rows_dev;
        return HM_OK;
    }
    int rc;
    if ((size_t)n_tiles > ctx->h_tiles_cap || !ctx->h_cell) {
        size_t want = host_cap_for(ctx->h_cell ? ctx->h_tiles_cap : 0, (size_t)n_tiles);
        size_t dummy = 0;
        if ((rc = ensure_host(ctx, &ctx->h_cell, dummy, want, 8)) || (rc = ensure_host(ctx, &ctx->h_ws, dummy, want, 8)) ||
            (rc = ensure_host(ctx, &ctx->h_cnt, dummy, want, 8)) || (rc = ensure_host(ctx, &ctx->h_sp, dummy, want, 8)) ||
            (rc = ensure_host(ctx, &ctx->h_spn, dummy, want, 1)) || (rc = ensure_host(ctx, &ctx->h_lon, dummy, want, 8)) ||
            (rc = ensure_host(ctx, &ctx->h_lat, dummy, want, 8)))
            return rc;
        ctx->h_tiles_cap = want;
    }
    if ((size_t)n_rows > ctx->h_rows_cap || !ctx->h_rows) {
        size_t want = host_cap_for(ctx->h_rows ? ctx->h_rows_cap : 0, (size_t)n_rows), dummy = 0;
        if ((rc = ensure_host(ctx, &ctx->h_rows, dummy, want, 8))) return rc;
        ctx->h_rows_cap = want;
    }
    if (n_tiles > 0) {
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_cell, ctx->o_cell.p, n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_ws, ctx->o_ws.p, n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_cnt, ctx->o_cnt.p, n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_sp, ctx->o_sp.p, n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_spn, ctx->o_spn.p, n_tiles, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_lon, ctx->o_lon.p, n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_lat, ctx->o_lat.p, n_tiles * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    if (n_rows > 0) HIPCHK(ctx, hipMemcpyAsync(ctx->h_rows, rows_dev, n_rows * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    out->cell = (const uint64_t *)ctx->h_cell;
    out->window_start_us = (const int64_t *)ctx->h_ws;
    out->count = (const int64_t *)ctx->h_cnt;
    out->avg_speed = (const double *)ctx->h_sp;
    out->speed_null = (const uint8_t *)ctx->h_spn;
    out->avg_lon = (const double *)ctx->h_lon;
    out->avg_lat = (const double *)ctx->h_lat;
    out->latest_row = (const int64_t *)ctx->h_rows;
    return HM_OK;
}

static void advance_watermark(hm_ctx *ctx, int64_t batch_max_ms) {
    // Spark WatermarkTracker: global = max(global, batch max event time - delay); starts at 0
    int64_t next = ctx->wm_cur;
    if (batch_max_ms != INT64_MIN) {
        int64_t cand = batch_max_ms - ctx->cfg.watermark_delay_ms;
        if (cand > next) next = cand;
    }
    ctx->wm_prev = ctx->wm_cur;
    ctx->wm_cur = next;
}

static void fill_stats(hm_ctx *ctx, hm_batch_out *out, int64_t n_in, const DevStats &s, int64_t late_wm) {
    out->n_in = n_in;
    out->n_valid = (int64_t)s.n_valid;
    out->n_late = (int64_t)s.n_late;
    out->n_state = ctx->state_size;
    out->batch_max_event_ms = s.max_ts_ms;
    out->watermark_ms = ctx->wm_cur;
    out->late_watermark_ms = late_wm;
    out->n_partials = ctx->n_partials_merged;
}

static void record_timings(hm_ctx *ctx) {
    float t;
    auto el = [&](int a, int b) -> double { return hipEventElapsedTime(&t, ctx->ev[a], ctx->ev[b]) == hipSuccess ? t : -1.0; };
    ctx->timings[0] = el(0, 1);
    ctx->timings[1] = ctx->staged ? el(10, 2) : el(1, 2);   // (stage API: table mode runs in hm_stage_send)
    ctx->timings[2] = el(3, 4);
    ctx->timings[3] = el(4, 5);
    ctx->timings[4] = el(5, 6);
    if (ctx->dedup_side && !ctx->staged)   // (concurrent with the merge path: its own span on the side stream)
        ctx->timings[4] = hipEventElapsedTime(&t, ctx->side_ev[1], ctx->side_ev[2]) == hipSuccess ? t : -1.0;
    ctx->timings[5] = el(0, 6);
    ctx->timings[2] = el(7, 4);   // merge proper
    ctx->timings[6] = el(3, 7);   // partition by table region
    ctx->timings[7] = el(8, 9);   // multi-GPU sender: partition by owner rank
    (void)hipGetLastError();      // (an event a path did not record: its timing reads -1, no sticky error)
}

extern "C" {

int32_t hm_abi_version(void) { return HM_ABI_VERSION; }

int hm_create(const hm_config *cfg, hm_ctx **out) {
    g_create_err.clear();
    if (!cfg || !out) { g_create_err = "null argument"; return HM_E_INVALID; }
    if (cfg->abi_version != HM_ABI_VERSION) { g_create_err = "ABI version mismatch"; return HM_E_INVALID; }
    if (cfg->h3_res < 0 || cfg->h3_res > 15) { g_create_err = "h3_res out of range"; return HM_E_INVALID; }
    // (windows of at least a second: TILE_MINUTES is whole minutes in the reference, heatmap_stream.py:29; the
    // window registry's LDS cache relies on |ts / tile_us| < 2^51)
    if (cfg->tile_us < 1000000 || cfg->watermark_delay_ms < 0) { g_create_err = "bad tile/watermark"; return HM_E_INVALID; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        g_create_err = "no HIP device available (the mobheat hot path requires an MI355X GPU)";
        return HM_E_HIP;
    }
    if (cfg->device < 0 || cfg->device >= ndev) { g_create_err = "device ordinal out of range"; return HM_E_INVALID; }
    hm_ctx *ctx = new hm_ctx();
    ctx->cfg = *cfg;
    ctx->device = cfg->device;
    auto fail = [&](const char *what) {
        g_create_err = std::string(what) + ": " + ctx->err;
        hm_destroy(ctx);
        return HM_E_HIP;
    };
    if (hipSetDevice(ctx->device) != hipSuccess) { ctx->err = "hipSetDevice"; return fail("create"); }
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->side_stream, hipStreamNonBlocking) != hipSuccess) { ctx->err = "stream"; return fail("create"); }
    for (auto &e : ctx->side_ev)
        if (hipEventCreate(&e) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    if (hipEventCreateWithFlags(&ctx->winfo_ev, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    for (auto &e : ctx->h2d_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    // k_merge_owned's resident tags live in dynamic LDS of up to MO_TAG_MAX bytes (merge_sorted)
    if (hipFuncSetAttribute((const void *)k_merge_owned<EventRec, false>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<SortedRec, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<SortedRec, false>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<SortedRec, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess) {
        ctx->err = "merge LDS attribute";
        return fail("create");
    }
    for (auto &e : ctx->ev)
        if (hipEventCreate(&e) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    if (upload_tables() != hipSuccess) { ctx->err = "tables"; return fail("create"); }
    {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)k_ingest, IG_THREADS, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) {
            ctx->err = "occupancy query";
            return fail("create");
        }
        // the occupancy API can report one block per CU more than fits (MI355X_MICROARCH.md, correctness
        // boundaries: SGPR counts 81-112); k_ingest is persistent, so an extra block per CU would only run once
        // a resident one finished.  Bound it by the LDS each block takes.
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, (const void *)k_ingest) == hipSuccess && fa.sharedSizeBytes > 0)
            per_cu = std::min<int>(per_cu, (int)(163840 / fa.sharedSizeBytes));
        if (getenv("MOBHEAT_DEBUG"))
            fprintf(stderr, "mobheat: k_ingest %d blocks/CU x %d CUs (LDS %zu B)\n", per_cu, cus, fa.sharedSizeBytes);
        ctx->ingest_grid = std::max(1, per_cu) * std::max(1, cus);
        ctx->n_cus = std::max(1, cus);
    }
    // MOBHEAT_INGEST_MODE=direct|table pins the aggregation path (tests); default: adaptive
    if (const char *m = getenv("MOBHEAT_INGEST_MODE")) ctx->ingest_mode = !strcmp(m, "direct") ? 1 : !strcmp(m, "table") ? 2 : 0;
    if (const char *m = getenv("MOBHEAT_MERGE_GRID")) ctx->merge_grid = std::max(0, atoi(m));
    // the registry, its census and the batch statistics side by side (one reset, one readback after k_ingest)
    if (hipMalloc(&ctx->d_wreg, REG_BLOCK_BYTES) != hipSuccess || !(ctx->d_wcount = ctx->d_wreg + WREG_SLOTS + 1) ||
        !(ctx->d_st = (DevStats *)(ctx->d_wreg + 2 * (WREG_SLOTS + 1))) ||
        hipHostMalloc(&ctx->h_wreg, REG_BLOCK_BYTES, hipHostMallocDefault) != hipSuccess ||
        !(ctx->h_wcount = ctx->h_wreg + WREG_SLOTS + 1) || !(ctx->h_st = (DevStats *)(ctx->h_wreg + 2 * (WREG_SLOTS + 1))) ||
        hipMalloc(&ctx->d_winfo, (WREG_SLOTS + 1) * sizeof(WInfo) + sizeof(WiCacheImg)) != hipSuccess ||
        hipHostMalloc(&ctx->h_winfo, (WREG_SLOTS + 1) * sizeof(WInfo) + sizeof(WiCacheImg), hipHostMallocDefault) != hipSuccess ||
        hipMemset(ctx->d_winfo, 0, (WREG_SLOTS + 1) * sizeof(WInfo)) != hipSuccess ||
        hipMemset(ctx->d_winfo + WREG_SLOTS + 1, 0xff, sizeof(WiCacheImg)) != hipSuccess) {
        ctx->err = "window registry alloc";
        return fail("create");
    }
    if (hipMalloc(&ctx->d_scratch, 256 * 8) != hipSuccess || hipHostMalloc(&ctx->h_scratch, 256 * 8) != hipSuccess) {
        ctx->err = "stats alloc";
        return fail("create");
    }
    if (hipMemset(ctx->d_scratch, 0, 256 * 8) != hipSuccess) { ctx->err = "scratch init"; return fail("create"); }
    if (hipMalloc(&ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc)) != hipSuccess ||
        hipHostMalloc(&ctx->h_gmap, GMAP_SLOTS * sizeof(GenDesc), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&ctx->d_cmap, GMAP_SLOTS * sizeof(WinCount)) != hipSuccess ||
        hipMalloc(&ctx->d_glist, GMAP_SLOTS * sizeof(GenDesc)) != hipSuccess ||
        hipHostMalloc(&ctx->h_glist, GMAP_SLOTS * sizeof(GenDesc), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&ctx->h_cmap, GMAP_SLOTS * sizeof(WinCount), hipHostMallocDefault) != hipSuccess ||
        hipMemset(ctx->d_gmap, 0, GMAP_SLOTS * sizeof(GenDesc)) != hipSuccess) {
        ctx->err = "window map alloc";
        return fail("create");
    }
    ctx->dfused.used_word = DUSED_WORD;
    ctx->dfull.used_word = FULL_USED_WORD;
    // batch_capacity_hint: reserve the per-batch buffers now (multi-GB allocations would otherwise land in the
    // first batches; each later batch only grows them when it is larger)
    if (cfg->batch_capacity_hint > 0) {
        const int64_t n = cfg->batch_capacity_hint;
        const size_t tp = sizeof(TilePartial);
        (void)tp;
        if (ensure(ctx, ctx->flags, n) || ensure(ctx, ctx->win, n) || ensure(ctx, ctx->rows, n * 8) ||
            ensure(ctx, ctx->keys, n * 8) || ensure(ctx, ctx->slow, n * 4) ||
            ensure(ctx, ctx->parts_sorted, n * sizeof(EventRec)) ||
            ensure(ctx, ctx->s_cell, n * 8) || ensure(ctx, ctx->s_ws, n * 8) || ensure(ctx, ctx->s_cnt, n * 8) ||
            ensure(ctx, ctx->s_sp, n * 8) || ensure(ctx, ctx->s_spn, n) || ensure(ctx, ctx->s_lon, n * 8) ||
            ensure(ctx, ctx->s_lat, n * 8) || ensure_outputs(ctx, n))
            return fail("create");
        // the full dedup table a batch of n rows may need (when k_ingest's cache-sized table gives up: C5's first
        // batch paid a 17-GB hipMalloc inside the batch)
        if (dedup_prepare(ctx, ctx->dfull, n, false)) return fail("create");
    }
    if (cfg->state_arena_bytes > 0) {
        ctx->arena_bytes = (size_t)cfg->state_arena_bytes & ~(size_t)255;
        if (dev_malloc(ctx, (void **)&ctx->arena, ctx->arena_bytes, "state arena") != hipSuccess) {
            (void)hipGetLastError();
            ctx->arena = nullptr;
            ctx->err = "state arena: out of device memory";
            return fail("create");
        }
        hipLaunchKernelGGL(k_zero16, dim3(256 * 32), dim3(256), 0, ctx->stream, (uint4 *)ctx->arena, (int64_t)(ctx->arena_bytes / 16));
    }
    // state_capacity_hint: one window table for that many keys, reserved now into the pool (a 70-GB table costs
    // ~2 s in hipMalloc: C5's first batch)
    if (cfg->state_capacity_hint > 0) {
        int L = ilog2(next_pow2((uint64_t)std::max<int64_t>(2 * cfg->state_capacity_hint, 1024)));
        unsigned rb = 0;
        TileSlot *t = nullptr;
        if (table_acquire(ctx, L, rb, &t) || table_release(ctx, t, L)) return fail("create");
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) { ctx->err = "sync"; return fail("create"); }
    *out = ctx;
    return HM_OK;
}

void hm_destroy(hm_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side_stream) (void)hipStreamSynchronize(ctx->side_stream);
    DevBuf *bufs[] = {&ctx->in_lat, &ctx->in_lon, &ctx->in_ts, &ctx->in_speed, &ctx->in_sv, &ctx->in_vkey, &ctx->in_rv,
                      &ctx->cell, &ctx->wstart, &ctx->flags, &ctx->win, &ctx->rows, &ctx->block_counts, &ctx->block_offs,
                      &ctx->partials, &ctx->cands, &ctx->slow, &ctx->parts_sorted, &ctx->parts_regrow, &ctx->rp_H, &ctx->rp_O,
                      &ctx->rp_btot, &ctx->rp_boff,
                      &ctx->s_cell, &ctx->s_ws, &ctx->s_cnt, &ctx->s_sp, &ctx->s_spn, &ctx->s_lon, &ctx->s_lat, &ctx->bin_cnt, &ctx->bin_off, &ctx->dfused.used, &ctx->dfull.used, &ctx->o_cell, &ctx->o_ws, &ctx->o_cnt, &ctx->o_sp, &ctx->o_spn,
                      &ctx->o_lon, &ctx->o_lat, &ctx->td_sizes, &ctx->td_off, &ctx->td_btot, &ctx->td_boff, &ctx->td_bytes,
                      &ctx->td_params, &ctx->gapbuf, &ctx->keys, &ctx->agg_bucket, &ctx->agg_cursor,
                      &ctx->jd_bytes, &ctx->jd_offs, &ctx->jd_scratch, &ctx->jd_lat, &ctx->jd_lon, &ctx->jd_ts, &ctx->jd_speed,
                      &ctx->jd_sv, &ctx->jd_rv, &ctx->jd_vkey, &ctx->jd_poff, &ctx->jd_plen, &ctx->jd_voff, &ctx->jd_vlen,
                      &ctx->lb_set, &ctx->lb_list};
    for (DevBuf *b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (hm_ctx::Dict *d : {&ctx->jd_prov, &ctx->jd_veh}) {
        for (DevBuf *b : {&d->tab, &d->slot_of, &d->occ, &d->slots, &d->code_of_slot, &d->clen, &d->coff, &d->cbytes, &d->btot, &d->boff})
            if (b->p) (void)hipFree(b->p);
        if (d->h_off) (void)hipHostFree(d->h_off);
        if (d->h_bytes) (void)hipHostFree(d->h_bytes);
    }
    for (auto &g : ctx->gens)
        if (!in_arena(ctx, g.tab)) (void)hipFree(g.tab);
    for (auto &pt : ctx->pool)
        if (!in_arena(ctx, pt.first)) (void)hipFree(pt.first);
    if (ctx->arena) (void)hipFree(ctx->arena);
    if (ctx->d_wreg) (void)hipFree(ctx->d_wreg);   // (d_wcount, d_st / h_wcount, h_st: inside these)
    if (ctx->h_wreg) (void)hipHostFree(ctx->h_wreg);
    if (ctx->d_winfo) (void)hipFree(ctx->d_winfo);
    if (ctx->h_winfo) (void)hipHostFree(ctx->h_winfo);
    if (ctx->d_gmap) (void)hipFree(ctx->d_gmap);
    if (ctx->h_gmap) (void)hipHostFree(ctx->h_gmap);
    if (ctx->d_cmap) (void)hipFree(ctx->d_cmap);
    if (ctx->d_glist) (void)hipFree(ctx->d_glist);
    if (ctx->h_glist) (void)hipHostFree(ctx->h_glist);
    if (ctx->h_cmap) (void)hipHostFree(ctx->h_cmap);
    if (ctx->dfused.tab) (void)hipFree(ctx->dfused.tab);
    if (ctx->dfull.tab) (void)hipFree(ctx->dfull.tab);
    void *hbufs[] = {ctx->h_cell, ctx->h_ws, ctx->h_cnt, ctx->h_sp, ctx->h_spn, ctx->h_lon, ctx->h_lat, ctx->h_rows,
                     ctx->h_td_bytes, ctx->h_td_off};
    for (void *p : hbufs)
        if (p) (void)hipHostFree(p);
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    if (ctx->h_scratch) (void)hipHostFree(ctx->h_scratch);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->h2d_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
    if (ctx->side_stream) (void)hipStreamDestroy(ctx->side_stream);
    for (auto &e : ctx->side_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->winfo_ev) (void)hipEventDestroy(ctx->winfo_ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *hm_last_error(const hm_ctx *ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int hm_last_timings(const hm_ctx *ctx, double *ms, int32_t n) {
    if (!ctx || !ms) return HM_E_INVALID;
    for (int i = 0; i < n && i < 8; i++) ms[i] = ctx->timings[i];
    for (int i = 8; i < n && i < 14; i++) ms[i] = ctx->host_ms[i - 8];
    return HM_OK;
}

// the state's version: bumped when a batch's merge begins (a failed call that left it unchanged did not touch the state)
int64_t hm_state_version(const hm_ctx *ctx) { return ctx ? (int64_t)ctx->seq : -1; }

int hm_last_counts(const hm_ctx *ctx, int64_t *c, int32_t n) {
    if (!ctx || !c) return HM_E_INVALID;
    for (int i = 0; i < n && i < 6; i++) c[i] = ctx->last_counts[i];
    if (n > 6) c[6] = ctx->n_allocs;
    if (n > 7) c[7] = ctx->n_frees;
    return HM_OK;
}

#ifdef HM_EXP_OVERLAP
// experiment build only (tools/gpurun/gpurun_r3ov.sh): after a direct-path batch, k_ingest (into scratch keys) and
// k_ev_scatter_rec (the batch's own records again) timed alone and on two streams together
static void exp_overlap(hm_ctx *ctx, const Inputs &I, int64_t late_wm_ms) {
    static DevBuf ek, ef;
    const int64_t n = I.n;
    if (n <= 0 || ensure(ctx, ek, n * 8) || ensure(ctx, ef, n)) return;
    const int64_t tile = rp_tile_for(n), ntiles = std::max<int64_t>((n + tile - 1) / tile, 1);
    hipEvent_t e[4];
    for (auto &x : e) hipEventCreate(&x);
    auto ingest = [&](hipStream_t st) {
        hipMemsetAsync(ctx->d_scratch + SLOW_WORD, 0, 8, st);
        const int blocks = (int)std::min<int64_t>((n + IG_THREADS - 1) / IG_THREADS, ctx->ingest_grid);
        hipLaunchKernelGGL(k_ingest, dim3(blocks), dim3(IG_THREADS), 0, st, I.lat, I.lon, I.ts, I.rv, I.vk, (int64_t)0, n,
                           ctx->cfg.h3_res, make_floor_div(ctx->cfg.tile_us), late_wm_ms * 1000, (uint8_t *)ef.p,
                           (uint64_t *)ek.p, ctx->dfused.tab, ctx->dfused.cap - 1, (unsigned int *)ctx->dfused.used.p,
                           ctx->d_scratch + ctx->dfused.used_word, (unsigned int *)ctx->slow.p, ctx->d_scratch + SLOW_WORD,
                           ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg, ctx->d_wcount, ctx->d_st);
    };
    auto scatter = [&](hipStream_t st) {
        hipLaunchKernelGGL(k_ev_scatter_rec<false>, dim3(ntiles), dim3(SR_THREADS), 0, st, (const uint64_t *)ctx->keys.p, n, tile,
                           I.sp, I.sv, I.lat, I.lon, nullptr, (const WInfo *)ctx->d_winfo, cell_hi_of(ctx->cfg.h3_res), RP_BINS,
                           (const unsigned long long *)ctx->rp_O.p, ntiles, (EventRec *)ctx->parts_sorted.p);
    };
    for (int rep = 0; rep < 3; rep++) {
        float ms[3];
        hipEventRecord(e[0], ctx->stream); ingest(ctx->stream); hipEventRecord(e[1], ctx->stream);
        hipStreamSynchronize(ctx->stream); hipEventElapsedTime(&ms[0], e[0], e[1]);
        hipEventRecord(e[0], ctx->stream); scatter(ctx->stream); hipEventRecord(e[1], ctx->stream);
        hipStreamSynchronize(ctx->stream); hipEventElapsedTime(&ms[1], e[0], e[1]);
        hipEventRecord(e[0], ctx->stream);
        hipStreamWaitEvent(ctx->side_stream, e[0], 0);
        ingest(ctx->stream);
        scatter(ctx->side_stream);
        hipEventRecord(e[2], ctx->side_stream);
        hipStreamWaitEvent(ctx->stream, e[2], 0);
        hipEventRecord(e[1], ctx->stream);
        hipStreamSynchronize(ctx->stream); hipEventElapsedTime(&ms[2], e[0], e[1]);
        fprintf(stderr, "exp_overlap ingest %.3f scatter %.3f both %.3f ms (sum %.3f)\n", ms[0], ms[1], ms[2], ms[0] + ms[1]);
    }
    for (auto &x : e) hipEventDestroy(x);
    ctx->dfused.dirty = true;
}
#endif

int hm_process_batch(hm_ctx *ctx, int64_t epoch_id, const hm_batch_in *in, int32_t out_memory, hm_batch_out *out) {
    if (!ctx || !in || !out || in->n < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (in->n > (int64_t)UINT32_MAX - 1) return set_err(ctx, HM_E_INVALID, "batch of %lld events exceeds 2^32-2", (long long)in->n);
    if (in->n > 0 && (!in->lat || !in->lon || !in->ts_us || !in->vkey))
        return set_err(ctx, HM_E_INVALID, "lat, lon, ts_us and vkey are required");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    host_batch_begin(ctx);
    const BatchClock clock_(ctx);
    memset(out, 0, sizeof(*out));
    ctx->gmap_ready = false;
    ctx->epoch = epoch_id;
    ctx->last_n_latest = -1;
    ctx->staged = false;
    ctx->stage = 0;
    int rc;
    // 1. evict with this batch's eviction watermark happened at the end of the previous batch (see below)
    int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    Inputs I;
    I.n = in->n;
    if ((rc = stage_inputs(ctx, in, &I.lat, &I.lon, &I.ts, &I.sp, &I.sv, &I.vk, &I.rv))) return rc;
    // 2. snap + window registry + event keys
    if ((rc = phase_local(ctx, I, late_wm))) return rc;
    DevStats s1 = *ctx->h_st;
    const int64_t n_agg = (int64_t)s1.n_valid - (int64_t)s1.n_late;
    // the aggregation path of this batch (table mode: two LDS passes first; direct: every row a record)
    const bool table = choose_table(ctx, n_agg, s1.sample_max_run);
    ctx->last_table = table;
    // 4. dedup over the batch's valid rows -- on the side stream, concurrently with step 3 (the rerun of the max on a
    // full table, after the fused one gave up, prepares that table on the main stream: it stays there)
    ctx->dedup_side = s1.dedup_retry == 0;
    // (launched here, ahead of the partition: 1-3% faster on the bench than launched after the merge path's kernels,
    // ~5% faster than overlapping the merge only, 2-4% faster than behind k_ev_hist -- profiles/r3/r3ab12/, r3ab13/)
    if (ctx->dedup_side) {
        HIPCHK(ctx, hipEventRecord(ctx->side_ev[0], ctx->stream));
        HIPCHK(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->side_ev[0], 0));
        if ((rc = launch_side_dedup(ctx, &I))) return rc;
    }
    // 3. aggregate, merge into state + emit (table mode: two LDS passes first; direct: every row a record)
    if (table) {
        int64_t n_parts = 0;
        if ((rc = phase_table(ctx, I, n_agg, &n_parts))) return rc;
        HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
        if ((rc = merge_partials(ctx, (const TilePartial *)ctx->partials.p, n_parts))) return rc;
    } else {
        HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
        if ((rc = merge_events(ctx, I, n_agg))) return rc;
    }
    if (!ctx->dedup_side) {
        if ((rc = phase_dedup(ctx, &I, nullptr, I.n, true))) return rc;
    } else {
        HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[2], 0));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[6], ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    // (the window map's key counts for state_account, read back in the same wait)
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_gmap, ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    ctx->gmap_ready = true;
    ctx->dedup_seen = (int64_t)ctx->h_scratch[ctx->dlast->used_word];   // distinct vkeys of this batch
    DevStats s2 = *ctx->h_st;
    if (s2.overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    if (s2.bad_vkey) return set_err(ctx, HM_E_INVALID, "vkey UINT64_MAX is reserved (%llu rows)", s2.bad_vkey);
    int64_t n_rows = (int64_t)ctx->h_scratch[255];
    ctx->last_n_latest = n_rows;
    ctx->last_vk = I.vk;
    ctx->last_ts = I.ts;
    ctx->last_lat = I.lat;
    ctx->last_lon = I.lon;
    record_timings(ctx);
    if ((rc = finish_outputs(ctx, (int64_t)s2.n_touched, n_rows, (const int64_t *)ctx->rows.p, out_memory, out))) return rc;
    ctx->last_counts[0] = (int64_t)s2.n_state_new;
    ctx->last_counts[1] = ctx->n_partials_merged;
    ctx->last_counts[2] = (int64_t)s2.n_touched;
    ctx->last_counts[3] = table ? 1 : 0;
    ctx->last_counts[4] = table ? ctx->table_evicted : 0;
    ctx->last_counts[5] = 0;
    // the next batch's aggregation path is chosen from this one's cardinality
    if (n_agg >= (int64_t(1) << 16)) {
        ctx->prev_agg_rows = n_agg;
        ctx->prev_keys = (int64_t)s2.n_touched;
        ctx->merge_coop = s2.n_touched > 0 && 2 * s2.n_state_new < s2.n_touched;
    }
    // 5. eviction after emission with this batch's watermark (lazy: see hm_ctx), then advance the watermark
    if ((rc = state_account(ctx, ctx->wm_cur))) return rc;
    fill_stats(ctx, out, in->n, s1, late_wm);
    advance_watermark(ctx, s1.max_ts_ms);
#ifdef HM_EXP_OVERLAP
    if (!table && getenv("MOBHEAT_EXP_OVERLAP")) exp_overlap(ctx, I, late_wm);
#endif
    return HM_OK;
}

// ---- context-free entry points (the standalone UDF and the read side): per-device tables, stream and scratch
// buffers made once and reused, behind one mutex ----
struct UdfState {
    bool ready = false;
    int64_t last_exact = 0;   // hm_latlng_to_cell: inputs the fast path handed to the exact path (last call)
    hipStream_t stream = nullptr;
    DevBuf in0, in1, out0, out1, out2, slow;
};
static std::mutex g_udf_mu;
static UdfState g_udf[64];
static hipError_t udf_buf(DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return hipSuccess;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    hipError_t e = hipMalloc(&b.p, want);
    if (e == hipSuccess) b.bytes = want;
    return e;
}
static int udf_begin(int32_t device, UdfState *&S) {   // (g_udf_mu held)
    int ndev = 0;
    if (device < 0 || device >= 64 || hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) return HM_E_HIP;
    if (hipSetDevice(device) != hipSuccess) return HM_E_HIP;
    S = &g_udf[device];
    if (!S->ready) {
        if (upload_tables() != hipSuccess) return HM_E_HIP;
        if (hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking) != hipSuccess) return HM_E_HIP;
        S->ready = true;
    }
    return HM_OK;
}

int hm_latlng_to_cell(const double *lat, const double *lon, int64_t n, int32_t res, int32_t memory, int32_t device,
                      uint64_t *out) {
    if (n < 0 || n > (int64_t)UINT32_MAX || res < 0 || res > 15) return HM_E_INVALID;
    if (n == 0) return HM_OK;
    std::lock_guard<std::mutex> lock(g_udf_mu);
    UdfState *S = nullptr;
    int rc;
    if ((rc = udf_begin(device, S))) return rc;
    const double *dlat = lat, *dlon = lon;
    uint64_t *dout = out;
    // exception list + its count (last 8 bytes)
    if (udf_buf(S->slow, n * 4 + 16) != hipSuccess) return HM_E_NOMEM;
    unsigned long long *n_slow = (unsigned long long *)((char *)S->slow.p + ((n * 4 + 7) & ~int64_t(7)));
    hipError_t e = hipSuccess;
    if (memory == HM_MEM_HOST) {
        if (udf_buf(S->in0, n * 8) || udf_buf(S->in1, n * 8) || udf_buf(S->out0, n * 8)) return HM_E_NOMEM;
        e = hipMemcpyAsync(S->in0.p, lat, n * 8, hipMemcpyHostToDevice, S->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(S->in1.p, lon, n * 8, hipMemcpyHostToDevice, S->stream);
        dlat = (const double *)S->in0.p;
        dlon = (const double *)S->in1.p;
        dout = (uint64_t *)S->out0.p;
    }
    if (e == hipSuccess) e = hipMemsetAsync(n_slow, 0, 8, S->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_cells, dim3(grid_for(n, 256, 256 * 32)), dim3(256), 0, S->stream, dlat, dlon, n, res, dout,
                           (unsigned int *)S->slow.p, n_slow);
        hipLaunchKernelGGL(k_cells_exact, dim3(256), dim3(256), 0, S->stream, dlat, dlon, res, dout, (const unsigned int *)S->slow.p,
                           (const unsigned long long *)n_slow);
        e = hipGetLastError();
    }
    if (e == hipSuccess && memory == HM_MEM_HOST) e = hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, S->stream);
    unsigned long long ne = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&ne, n_slow, 8, hipMemcpyDeviceToHost, S->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(S->stream);
    S->last_exact = (int64_t)ne;
    return e == hipSuccess ? HM_OK : HM_E_HIP;
}

int64_t hm_latlng_to_cell_last_exact(int32_t device) {
    std::lock_guard<std::mutex> lock(g_udf_mu);
    return device >= 0 && device < 64 ? g_udf[device].last_exact : -1;
}

int hm_cells_to_boundary(const uint64_t *cells, int64_t n, int32_t memory, int32_t device, double *lat, double *lng,
                         int32_t *nverts) {
    if (n < 0 || n > (int64_t)UINT32_MAX || (n > 0 && (!cells || !lat || !lng || !nverts))) return HM_E_INVALID;
    if (n == 0) return HM_OK;
    std::lock_guard<std::mutex> lock(g_udf_mu);
    UdfState *S = nullptr;
    int rc;
    if ((rc = udf_begin(device, S))) return rc;
    const uint64_t *dcells = cells;
    double *dlat = lat, *dlng = lng;
    int32_t *dnv = nverts;
    hipError_t e = hipSuccess;
    if (memory == HM_MEM_HOST) {
        if (udf_buf(S->in0, n * 8) || udf_buf(S->out0, n * 80) || udf_buf(S->out1, n * 80) || udf_buf(S->out2, n * 4))
            return HM_E_NOMEM;
        e = hipMemcpyAsync(S->in0.p, cells, n * 8, hipMemcpyHostToDevice, S->stream);
        dcells = (const uint64_t *)S->in0.p;
        dlat = (double *)S->out0.p;
        dlng = (double *)S->out1.p;
        dnv = (int32_t *)S->out2.p;
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_cells_boundary, dim3(grid_for(n, 256, 256 * 32)), dim3(256), 0, S->stream, dcells, n, dlat, dlng, dnv);
        e = hipGetLastError();
    }
    if (e == hipSuccess && memory == HM_MEM_HOST) {
        e = hipMemcpyAsync(lat, dlat, n * 80, hipMemcpyDeviceToHost, S->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(lng, dlng, n * 80, hipMemcpyDeviceToHost, S->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(nverts, dnv, n * 4, hipMemcpyDeviceToHost, S->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(S->stream);
    return e == hipSuccess ? HM_OK : HM_E_HIP;
}

int hm_selftest_cells_to_boundary_host(const uint64_t *cells, int64_t n, double *lat, double *lng, int32_t *nverts) {
    if (n < 0 || (n > 0 && (!cells || !lat || !lng || !nverts))) return HM_E_INVALID;
    static const H3Tables T = make_tables();
    for (int64_t i = 0; i < n; i++) {
        double la[10], lo[10];
        const int nv = cellToBoundaryDeg(cells[i], T, la, lo);
        nverts[i] = nv;
        for (int k = 0; k < 10; k++) {
            lat[10 * i + k] = k < nv ? la[k] : NAN;
            lng[10 * i + k] = k < nv ? lo[k] : NAN;
        }
    }
    return HM_OK;
}

// ---- multi-GPU stage API ----
// summary words of one rank (HM_STAGE_SUMMARY_WORDS int64, all-gathered by the caller between ingest and send)
enum : int {
    SW_N_IN = 0, SW_VALID, SW_LATE, SW_AGG, SW_MAX_MS, SW_SAMPLE_RUN, SW_PREV_AGG, SW_PREV_KEYS, SW_NWIN, SW_RESERVED,
    SW_WIN0   // then n_windows pairs (registry slot, wenc)
};
static_assert(SW_WIN0 + 2 * WREG_SLOTS <= HM_STAGE_SUMMARY_WORDS, "summary layout");

int hm_stage_ingest(hm_ctx *ctx, int64_t epoch_id, const hm_batch_in *in, int32_t nranks, int32_t rank, int64_t *summary) {
    if (!ctx || !in || !summary || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks)
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (in->n > (int64_t)UINT32_MAX - 1) return set_err(ctx, HM_E_INVALID, "batch of %lld events exceeds 2^32-2", (long long)in->n);
    if (in->n > 0 && (!in->lat || !in->lon || !in->ts_us || !in->vkey))
        return set_err(ctx, HM_E_INVALID, "lat, lon, ts_us and vkey are required");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    ctx->stage = 0;
    ctx->epoch = epoch_id;
    ctx->last_n_latest = -1;   // (hm_encode_position_updates: single-context batches only)
    ctx->nranks = nranks;
    ctx->rank = rank;
    const int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    Inputs I;
    I.n = in->n;
    if ((rc = stage_inputs(ctx, in, &I.lat, &I.lon, &I.ts, &I.sp, &I.sv, &I.vk, &I.rv))) return rc;
    if ((rc = phase_local(ctx, I, late_wm))) return rc;
    const DevStats s1 = *ctx->h_st;
    ctx->stage_I = I;
    ctx->stage_s1 = s1;
    ctx->staged = true;
    memset(summary, 0, HM_STAGE_SUMMARY_WORDS * sizeof(int64_t));
    summary[SW_N_IN] = I.n;
    summary[SW_VALID] = (int64_t)s1.n_valid;
    summary[SW_LATE] = (int64_t)s1.n_late;
    summary[SW_AGG] = (int64_t)s1.n_valid - (int64_t)s1.n_late;
    summary[SW_MAX_MS] = s1.max_ts_ms;
    summary[SW_SAMPLE_RUN] = (int64_t)s1.sample_max_run;
    summary[SW_PREV_AGG] = ctx->prev_agg_rows;
    summary[SW_PREV_KEYS] = ctx->prev_keys;
    int64_t nw = 0;
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wreg[w] && ctx->h_wcount[w]) {
            summary[SW_WIN0 + 2 * nw] = w;
            summary[SW_WIN0 + 2 * nw + 1] = (int64_t)ctx->h_wreg[w];
            nw++;
        }
    summary[SW_NWIN] = nw;
    ctx->stage_n_in = I.n;
    ctx->stage = 1;
    return HM_OK;
}

// The batch-wide decisions every rank derives identically from all ranks' summaries: the global max event time (the
// watermark's input), the aggregation path, and the global window registry (k_ingest's hashing -- slot wq mod
// WREG_SLOTS, linear probing -- over the union of the ranks' windows in ascending order).
static int stage_decide(hm_ctx *ctx, const int64_t *sums) {
    const int W = ctx->nranks;
    int64_t gmax = INT64_MIN, min_agg = INT64_MAX, prev_agg = 0, prev_keys = 0;
    unsigned long long max_run = 0;
    std::vector<unsigned long long> wins;
    for (int r = 0; r < W; r++) {
        const int64_t *S = sums + (size_t)r * HM_STAGE_SUMMARY_WORDS;
        gmax = std::max(gmax, S[SW_MAX_MS]);
        min_agg = std::min(min_agg, S[SW_AGG]);
        max_run = std::max(max_run, (unsigned long long)S[SW_SAMPLE_RUN]);
        prev_agg += S[SW_PREV_AGG];
        prev_keys += S[SW_PREV_KEYS];
        if (S[SW_NWIN] < 0 || S[SW_NWIN] > WREG_SLOTS) return set_err(ctx, HM_E_INVALID, "summary of rank %d is malformed", r);
        for (int64_t k = 0; k < S[SW_NWIN]; k++) wins.push_back((unsigned long long)S[SW_WIN0 + 2 * k + 1]);
    }
    std::sort(wins.begin(), wins.end());
    wins.erase(std::unique(wins.begin(), wins.end()), wins.end());
    ctx->stage_gwreg.assign(WREG_SLOTS, 0ull);
    for (unsigned long long we : wins) {
        const int64_t wq = wdec(we) / ctx->cfg.tile_us;   // (window starts are multiples of tile_us)
        unsigned h = (unsigned)((uint64_t)wq % (uint64_t)WREG_SLOTS);
        int p = 0;
        for (; p < WREG_SLOTS && ctx->stage_gwreg[h]; p++) h = h + 1 == (unsigned)WREG_SLOTS ? 0u : h + 1;
        if (p == WREG_SLOTS)
            return set_err(ctx, HM_E_OVERFLOW, "more than %d distinct windows in one micro-batch over all ranks", WREG_SLOTS);
        ctx->stage_gwreg[h] = we;
    }
    ctx->stage_gmax_ms = gmax;
    // aggregation path: the single-context rule (choose_table) on batch-wide numbers -- table mode when a rank's key
    // sample shows heavy hitters, or when the last batch's keys were few and repeated a lot on every rank
    bool table;
    if (ctx->ingest_mode) table = ctx->ingest_mode == 2;
    else if (min_agg < (int64_t(1) << 16)) table = false;
    else if (max_run >= (unsigned long long)(HS_SAMPLE / 256)) table = true;
    else table = prev_keys > 0 && prev_keys <= (int64_t)AG_BINS * (AG_SLOTS / 2) && prev_agg >= 8 * (int64_t)W * prev_keys;
    ctx->stage_table = table;
    return HM_OK;
}

int hm_stage_send(hm_ctx *ctx, const int64_t *summaries, void *tile_send_buf, void *payload_send_buf, int64_t tile_send_cap,
                  int64_t *tile_send_counts, void *cand_send_buf, int64_t cand_send_cap, int64_t *cand_send_counts,
                  hm_stage_sizes *sizes) {
    if (!ctx || !summaries || !tile_send_counts || !cand_send_counts)
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 1) return set_err(ctx, HM_E_STATE, "hm_stage_send before hm_stage_ingest");
    const Inputs &I = ctx->stage_I;
    if (I.n > 0 && (!tile_send_buf || !payload_send_buf || !cand_send_buf))
        return set_err(ctx, HM_E_INVALID, "send buffers are required");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const int W = ctx->nranks;
    if (summaries[(size_t)ctx->rank * HM_STAGE_SUMMARY_WORDS + SW_N_IN] != I.n)
        return set_err(ctx, HM_E_INVALID, "summaries[rank] is not this rank's summary");
    if ((rc = stage_decide(ctx, summaries))) return rc;
    const DevStats &s1 = ctx->stage_s1;
    const int64_t n_agg = (int64_t)s1.n_valid - (int64_t)s1.n_late;
    const bool table = ctx->stage_table;
    ctx->last_table = table;
    int64_t n_records = n_agg;
    HIPCHK(ctx, hipEventRecord(ctx->ev[10], ctx->stream));
    if (table && (rc = phase_table(ctx, I, n_agg, &n_records))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    ctx->census_ready = false;   // (the owner counts what it receives)
    // local dedup over rows -> local winners -> candidates
    if ((rc = phase_dedup(ctx, &I, nullptr, I.n, s1.dedup_retry != 0))) return rc;
    if ((rc = ensure(ctx, ctx->cands, std::max<int64_t>(I.n, 1) * sizeof(Cand)))) return rc;
    hipLaunchKernelGGL(k_make_cands, dim3(grid_for(std::max<int64_t>(I.n, 1), 256)), dim3(256), 0, ctx->stream,
                       (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, I.vk, I.ts, ctx->rank, (Cand *)ctx->cands.p);
    HIPCHK(ctx, hipGetLastError());
    // partition both record kinds by owner rank: candidates by counts + cursors here, tile records below
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch, 0, 128 * 8, ctx->stream));
    const int gb = grid_for(std::max<int64_t>(I.n, 1), 256);
    hipLaunchKernelGGL(k_part_count<Cand>, dim3(gb), dim3(256), 0, ctx->stream, (const Cand *)ctx->cands.p, ctx->d_scratch + 255,
                       W, ctx->d_scratch + 64);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    if (ctx->h_st->bad_vkey) return set_err(ctx, HM_E_INVALID, "vkey UINT64_MAX is reserved");
    ctx->dedup_seen = (int64_t)ctx->h_scratch[ctx->dlast->used_word];
    if (n_records > tile_send_cap || (int64_t)ctx->h_scratch[255] > cand_send_cap)
        return set_err(ctx, HM_E_INVALID, "send buffer too small (%lld tile records, %llu candidates)", (long long)n_records,
                       ctx->h_scratch[255]);
    // candidates: exclusive offsets -> cursors
    unsigned long long cur[128];
    unsigned long long acc = 0;
    for (int r = 0; r < W; r++) { cur[64 + r] = acc; cand_send_counts[r] = (int64_t)ctx->h_scratch[64 + r]; acc += ctx->h_scratch[64 + r]; }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_scratch + 64, cur + 64, 64 * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_part_scatter<Cand>, dim3(gb), dim3(256), 0, ctx->stream, (const Cand *)ctx->cands.p, ctx->d_scratch + 255,
                       W, ctx->d_scratch + 64, (Cand *)cand_send_buf);
    HIPCHK(ctx, hipGetLastError());
    // tile records: the radix partition with the owner rank as the digit, straight into the send streams
    HIPCHK(ctx, hipEventRecord(ctx->ev[8], ctx->stream));
    if (n_records > 0) {
        int64_t ntiles;
        if (table) {
            if ((rc = partition<TilePartial, TilePartial>(ctx, (const TilePartial *)ctx->partials.p, n_records, ntiles, W,
                                                          (TilePartial *)tile_send_buf)))
                return rc;
        } else {
            // this rank's registry slots -> the batch's global slots (WInfo.gslot), keys rewritten by the scatter
            ctx->stage_gslot.assign(WREG_SLOTS, 0u);
            for (int w = 0; w < WREG_SLOTS; w++) {
                const unsigned long long we = ctx->h_wreg[w];
                if (!we) continue;
                const auto it = std::find(ctx->stage_gwreg.begin(), ctx->stage_gwreg.end(), we);
                if (it == ctx->stage_gwreg.end() && ctx->h_wcount[w])
                    return set_err(ctx, HM_E_STATE, "a window of this rank is missing from the global registry");
                ctx->stage_gslot[w] = (unsigned)(it - ctx->stage_gwreg.begin());
            }
            rc = winfo_upload(ctx, false);
            ctx->stage_gslot.clear();
            if (rc || (rc = ev_partition<WireKey>(ctx, (const uint64_t *)ctx->keys.p, I.n, &I, nullptr, ntiles, W,
                                                  (WireKey *)tile_send_buf, (uint64_t *)payload_send_buf)))
                return rc;
        }
        hipLaunchKernelGGL(k_digit_starts, dim3(1), dim3(128), 0, ctx->stream, (const unsigned long long *)ctx->rp_O.p, ntiles,
                           W + 1, ctx->d_scratch);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, (W + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[9], ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    for (int r = 0; r < W; r++) {
        const int64_t start = n_records > 0 ? (int64_t)ctx->h_scratch[r] : 0;
        const int64_t end = n_records > 0 ? (int64_t)ctx->h_scratch[r + 1] : 0;   // [W]: the gaps' digit
        tile_send_counts[r] = end - start;
    }
    ctx->stage_agg_rows = n_agg;
    ctx->stage_sent = n_records;
    hm_stage_sizes z{};
    z.table_mode = table ? 1 : 0;
    z.n_tile_records = n_records;
    for (int r = 0; r < W; r++) z.n_cands += cand_send_counts[r];
    z.global_batch_max_event_ms = ctx->stage_gmax_ms;
    z.n_valid = (int64_t)s1.n_valid;
    z.n_late = (int64_t)s1.n_late;
    ctx->stage_sizes = z;
    if (sizes) *sizes = z;
    ctx->stage = 2;
    return HM_OK;
}

// the multi-GPU owner's direct path: the received key + payload streams (n rows of all ranks) -> census per global
// window -> window tables -> (window, region) partition into EventRecs -> merge -> rows
static int merge_received_events(hm_ctx *ctx, const uint64_t *keys, const uint64_t *payload, int64_t n) {
    int rc;
    ctx->n_partials_merged = n;
    if ((rc = merge_begin(ctx, n))) return rc;
    if (n == 0) return merge_nothing(ctx);
    memcpy(ctx->h_wreg, ctx->stage_gwreg.data(), WREG_SLOTS * sizeof(unsigned long long));
    HIPCHK(ctx, hipMemsetAsync(ctx->d_wcount, 0, (WREG_SLOTS + 1) * 8, ctx->stream));
    hipLaunchKernelGGL(k_key_census, dim3(grid_for(n, 256, 256 * 8)), dim3(256), 0, ctx->stream, keys, n, ctx->d_wcount);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_wcount, ctx->d_wcount, WREG_SLOTS * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wcount[w] && !ctx->h_wreg[w]) return set_err(ctx, HM_E_INVALID, "received a record of an unknown window slot");
    std::vector<WinCount> census;
    census_of_registry(ctx, census);
    if ((rc = gens_prepare(ctx, census)) || (rc = winfo_upload(ctx, true))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    int64_t ntiles;
    if ((rc = ev_partition<EventRec>(ctx, keys, n, nullptr, payload, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    if ((rc = merge_sorted<EventRec>(ctx, n, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if ((rc = rows_densify(ctx, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    return HM_OK;
}

int hm_stage_merge(hm_ctx *ctx, const void *tile_recv_dev, const void *payload_recv_dev, int64_t n_tile_recv,
                   const void *cand_recv_dev, int64_t n_cand_recv, int32_t out_memory, hm_batch_out *out,
                   void *winner_send_buf, int64_t winner_send_cap, int64_t *winner_send_counts) {
    if (!ctx || !out || !winner_send_counts || n_tile_recv < 0 || n_cand_recv < 0 || winner_send_cap < n_cand_recv ||
        (n_cand_recv > 0 && (!winner_send_buf || !cand_recv_dev)) || (n_tile_recv > 0 && !tile_recv_dev))
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 2) return set_err(ctx, HM_E_STATE, "hm_stage_merge before hm_stage_send");
    if (!ctx->stage_table && n_tile_recv > 0 && !payload_recv_dev)
        return set_err(ctx, HM_E_INVALID, "the direct path needs the received payload stream");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    memset(out, 0, sizeof(*out));
    const int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    if (ctx->stage_table) rc = merge_partials(ctx, (const TilePartial *)tile_recv_dev, n_tile_recv);
    else rc = merge_received_events(ctx, (const uint64_t *)tile_recv_dev, (const uint64_t *)payload_recv_dev, n_tile_recv);
    if (rc) return rc;
    // owner-side dedup over received candidates
    if ((rc = phase_dedup(ctx, nullptr, (const Cand *)cand_recv_dev, n_cand_recv, true))) return rc;
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch, 0, 128 * 8, ctx->stream));
    if (n_cand_recv > 0) {
        hipLaunchKernelGGL(k_winner_route, dim3(grid_for(n_cand_recv, 256)), dim3(256), 0, ctx->stream, (const Cand *)cand_recv_dev,
                           (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, ctx->nranks, ctx->d_scratch, (int64_t *)nullptr, 0);
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[6], ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    DevStats s2 = *ctx->h_st;
    if (s2.overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    unsigned long long cur[64];
    unsigned long long acc = 0;
    for (int r = 0; r < ctx->nranks; r++) { cur[r] = acc; winner_send_counts[r] = (int64_t)ctx->h_scratch[r]; acc += ctx->h_scratch[r]; }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_scratch, cur, 64 * 8, hipMemcpyHostToDevice, ctx->stream));
    if (n_cand_recv > 0) {
        hipLaunchKernelGGL(k_winner_route, dim3(grid_for(n_cand_recv, 256)), dim3(256), 0, ctx->stream, (const Cand *)cand_recv_dev,
                           (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, ctx->nranks, ctx->d_scratch,
                           (int64_t *)winner_send_buf, 1);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    record_timings(ctx);
    if ((rc = finish_outputs(ctx, (int64_t)s2.n_touched, 0, nullptr, out_memory, out))) return rc;
    // hm_last_counts: this rank's share of the batch (state keys created, records merged, tiles emitted, path)
    ctx->last_counts[0] = (int64_t)s2.n_state_new;
    ctx->last_counts[1] = n_tile_recv;
    ctx->last_counts[2] = (int64_t)s2.n_touched;
    ctx->last_counts[3] = ctx->stage_table ? 1 : 0;
    ctx->last_counts[4] = ctx->stage_table ? ctx->table_evicted : 0;
    ctx->last_counts[5] = ctx->stage_sent;
    if (ctx->stage_agg_rows >= (int64_t(1) << 16)) {   // this rank's rows and owned keys (summed over ranks next batch)
        ctx->prev_agg_rows = ctx->stage_agg_rows;
        ctx->prev_keys = (int64_t)s2.n_touched;
        ctx->merge_coop = s2.n_touched > 0 && 2 * s2.n_state_new < s2.n_touched;
    }
    if ((rc = state_account(ctx, ctx->wm_cur))) return rc;
    DevStats sf{};
    sf.n_valid = ctx->stage_sizes.n_valid;
    sf.n_late = ctx->stage_sizes.n_late;
    sf.max_ts_ms = ctx->stage_gmax_ms;
    fill_stats(ctx, out, ctx->stage_n_in, sf, late_wm);
    advance_watermark(ctx, ctx->stage_gmax_ms);
    ctx->stage = 3;
    return HM_OK;
}

int hm_stage_finish(hm_ctx *ctx, const void *winner_recv_dev, int64_t n_winner_recv, int32_t out_memory, hm_batch_out *out) {
    if (!ctx || !out || n_winner_recv < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 3) return set_err(ctx, HM_E_STATE, "hm_stage_finish before hm_stage_merge");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    out->n_latest = n_winner_recv;
    if (out_memory == HM_MEM_DEVICE) {
        out->latest_row = (const int64_t *)winner_recv_dev;
    } else {
        if ((size_t)n_winner_recv > ctx->h_rows_cap || !ctx->h_rows) {
            size_t want = host_cap_for(ctx->h_rows ? ctx->h_rows_cap : 0, (size_t)n_winner_recv), dummy = 0;
            if ((rc = ensure_host(ctx, &ctx->h_rows, dummy, want, 8))) return rc;
            ctx->h_rows_cap = want;
        }
        if (n_winner_recv > 0)
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_rows, winner_recv_dev, n_winner_recv * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        std::sort((int64_t *)ctx->h_rows, (int64_t *)ctx->h_rows + n_winner_recv);
        out->latest_row = (const int64_t *)ctx->h_rows;
    }
    ctx->stage = 0;
    return HM_OK;
}

// ---- tile-state checkpoint (Spark's state store behind checkpointLocation, heatmap_stream.py:37,244) ----
// Export: every live window's keys dumped by k_dump_gen (the growth path's kernel) into one GrowRec array, copied
// to the caller; the touched word (this context's batch sequence) is cleared -- it means nothing elsewhere.
static void state_info_of(const hm_ctx *ctx, hm_state_info *info, int64_t n_keys) {
    memset(info, 0, sizeof(*info));
    info->epoch_id = ctx->epoch;
    info->n_keys = n_keys;
    info->watermark_ms = ctx->wm_cur;
    info->prev_watermark_ms = ctx->wm_prev;
    info->tile_us = ctx->cfg.tile_us;
    info->watermark_delay_ms = ctx->cfg.watermark_delay_ms;
    info->h3_res = ctx->cfg.h3_res;
}

// every live window's keys (only_seq != 0: those the batch with that sequence touched) into recs[0, n)
static int state_dump(hm_ctx *ctx, hm_state_rec *recs, int64_t n, unsigned only_seq) {
    int rc;
    if ((rc = ensure(ctx, ctx->parts_regrow, std::max<int64_t>(n, 1) * sizeof(GrowRec)))) return rc;
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + REGROW_WORD, 0, 8, ctx->stream));
    for (const auto &g : ctx->gens) {
        GenDesc d{};
        d.wenc = g.wenc;
        d.tab = g.tab;
        d.rbits = g.rbits;
        d.rshift = (unsigned)g.log2cap - g.rbits;
        d.rmask = (UINT64_C(1) << d.rshift) - 1;
        hipLaunchKernelGGL(k_dump_gen, dim3(grid_for(int64_t(1) << g.log2cap, 256)), dim3(256), 0, ctx->stream, d,
                           (GrowRec *)ctx->parts_regrow.p, ctx->d_scratch + REGROW_WORD, only_seq);
    }
    HIPCHK(ctx, hipGetLastError());
    unsigned long long dumped = 0;
    HIPCHK(ctx, hipMemcpyAsync(&dumped, ctx->d_scratch + REGROW_WORD, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if ((int64_t)dumped != n) return set_err(ctx, HM_E_STATE, "state dump found %llu keys, expected %lld", dumped, (long long)n);
    if (n > 0) HIPCHK(ctx, hipMemcpy(recs, ctx->parts_regrow.p, n * sizeof(GrowRec), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) recs[i].reserved = 0;
    return HM_OK;
}

int hm_state_export(hm_ctx *ctx, hm_state_info *info, hm_state_rec *recs, int64_t cap) {
    static_assert(sizeof(hm_state_rec) == sizeof(GrowRec), "hm_state_rec mirrors GrowRec");
    if (!ctx || !info) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 0) return set_err(ctx, HM_E_STATE, "hm_state_export between stage calls");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int64_t n = 0;
    for (const auto &g : ctx->gens) n += g.keys;
    state_info_of(ctx, info, n);
    if (!recs) return HM_OK;
    if (cap < n) return set_err(ctx, HM_E_INVALID, "state of %lld keys does not fit %lld records", (long long)n, (long long)cap);
    return n == 0 ? HM_OK : state_dump(ctx, recs, n, 0);
}

// Incremental checkpoint (Spark's state store writes a delta file per version): the keys the last batch touched, with
// their cumulative values; together with an older full export and the deltas between, the state after this batch is
// the last-written record of every key whose window end > info.prev_watermark_ms (the batch's eviction watermark).
int hm_state_export_touched(hm_ctx *ctx, hm_state_info *info, hm_state_rec *recs, int64_t cap, int64_t *n_out) {
    if (!ctx || !info || !n_out) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 0) return set_err(ctx, HM_E_STATE, "hm_state_export_touched between stage calls");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int64_t live = 0;
    for (const auto &g : ctx->gens) live += g.keys;
    state_info_of(ctx, info, live);
    // the last batch's touched keys that are still live (a touched key of an evicted window went with its table)
    int64_t n = 0;
    if (ctx->seq > 0 && !ctx->gens.empty()) {
        int rc;
        if ((rc = ensure(ctx, ctx->parts_regrow, std::max<int64_t>(live, 1) * sizeof(GrowRec)))) return rc;
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + REGROW_WORD, 0, 8, ctx->stream));
        for (const auto &g : ctx->gens) {
            GenDesc d{};
            d.wenc = g.wenc;
            d.tab = g.tab;
            d.rbits = g.rbits;
            d.rshift = (unsigned)g.log2cap - g.rbits;
            d.rmask = (UINT64_C(1) << d.rshift) - 1;
            hipLaunchKernelGGL(k_dump_gen, dim3(grid_for(int64_t(1) << g.log2cap, 256)), dim3(256), 0, ctx->stream, d,
                               (GrowRec *)ctx->parts_regrow.p, ctx->d_scratch + REGROW_WORD, seq32(ctx));
        }
        HIPCHK(ctx, hipGetLastError());
        unsigned long long dumped = 0;
        HIPCHK(ctx, hipMemcpyAsync(&dumped, ctx->d_scratch + REGROW_WORD, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        n = (int64_t)dumped;
    }
    *n_out = n;
    if (!recs) return HM_OK;
    if (cap < n) return set_err(ctx, HM_E_INVALID, "%lld touched keys do not fit %lld records", (long long)n, (long long)cap);
    if (n > 0) HIPCHK(ctx, hipMemcpy(recs, ctx->parts_regrow.p, n * sizeof(GrowRec), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) recs[i].reserved = 0;
    return HM_OK;
}

// Import: the records' windows get tables sized as a batch's new windows would be, then the records are merged
// through the growth path (partition + k_merge_owned in rehash mode: no counting, no rows, no touched update).
int hm_state_import(hm_ctx *ctx, const hm_state_info *info, const hm_state_rec *recs) {
    if (!ctx || !info || info->n_keys < 0 || (info->n_keys > 0 && !recs))
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->epoch != -1 || ctx->stage != 0 || !ctx->gens.empty())
        return set_err(ctx, HM_E_STATE, "hm_state_import into a context that already processed a batch");
    if (info->h3_res != ctx->cfg.h3_res || info->tile_us != ctx->cfg.tile_us || info->watermark_delay_ms != ctx->cfg.watermark_delay_ms)
        return set_err(ctx, HM_E_INVALID, "checkpoint of res %d / window %lld us / delay %lld ms does not match the context",
                       info->h3_res, (long long)info->tile_us, (long long)info->watermark_delay_ms);
    const int64_t n = info->n_keys;
    if (n >= (int64_t)UINT32_MAX) return set_err(ctx, HM_E_INVALID, "%lld state records exceed 2^32-2", (long long)n);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    // census per window + record checks (the device trusts them: a zero cell is a gap, reserved is touched)
    std::vector<std::pair<unsigned long long, int64_t>> wins;
    size_t last = 0;
    const int64_t T = ctx->cfg.tile_us;
    for (int64_t i = 0; i < n; i++) {
        const hm_state_rec &r = recs[i];
        if (r.cell == 0 || r.reserved != 0 || r.count < 1 || r.n_speed < 0 || r.n_speed > r.count ||
            ((r.window_start_us % T) + T) % T != 0)
            return set_err(ctx, HM_E_INVALID, "state record %lld is malformed", (long long)i);
        const unsigned long long we = wenc_of(r.window_start_us);
        if (last >= wins.size() || wins[last].first != we) {
            last = 0;
            while (last < wins.size() && wins[last].first != we) last++;
            if (last == wins.size()) {
                if ((int)wins.size() >= GMAP_SLOTS / 2)
                    return set_err(ctx, HM_E_OVERFLOW, "checkpoint holds more than %d windows", GMAP_SLOTS / 2);
                wins.emplace_back(we, 0);
            }
        }
        wins[last].second++;
    }
    int rc;
    for (const auto &w : wins) {
        int L;
        unsigned rb;
        gen_geometry(ctx, w.second, w.second, 0, L, rb);
        TileSlot *t = nullptr;
        if ((rc = table_acquire(ctx, L, rb, &t))) return rc;
        ctx->gens.push_back({w.first, t, L, rb, w.second, 0});
    }
    if ((rc = gens_upload(ctx))) return rc;
    if (n > 0) {
        if ((rc = ensure(ctx, ctx->parts_regrow, n * sizeof(GrowRec)))) return rc;
        HIPCHK(ctx, hipMemcpy(ctx->parts_regrow.p, recs, n * sizeof(GrowRec), hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemsetAsync(&ctx->d_st->overflow, 0, 8, ctx->stream));
        int64_t ntiles;
        if ((rc = partition<GrowRec, GrowRec>(ctx, (const GrowRec *)ctx->parts_regrow.p, n, ntiles))) return rc;
        if ((rc = merge_sorted<GrowRec>(ctx, n, ntiles))) return rc;
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow while restoring the state");
    }
    ctx->state_size = n;
    ctx->wm_cur = info->watermark_ms;
    ctx->wm_prev = info->prev_watermark_ms;
    ctx->epoch = info->epoch_id;
    return HM_OK;
}

// ---- tiles as MongoDB update statements (bson_docs.h; reference heatmap_stream.py:164-196) ----
int hm_last_windows(hm_ctx *ctx, int64_t *window_start_us, int64_t cap, int64_t *n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !window_start_us)) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    *n = (int64_t)ctx->batch_windows.size();
    for (int64_t i = 0; i < *n && i < cap; i++) window_start_us[i] = ctx->batch_windows[i];
    return HM_OK;
}

static int64_t civil_year(int64_t s) {   // proleptic Gregorian year of a second count since 1970 (host)
    int64_t z = s / 86400 - ((s % 86400) < 0) + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097, doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365, doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    return yoe + era * 400 + (mp >= 10);
}

// the statements in ctx->td_bytes / td_off: handed out on the device or copied to pinned host buffers
static int statements_out(hm_ctx *ctx, int64_t n, int64_t total, int32_t out_memory, const uint8_t **bytes,
                          const int64_t **offsets, int64_t *n_docs) {
    int rc;
    unsigned long long *off = (unsigned long long *)ctx->td_off.p;
    *n_docs = n;
    if (out_memory == HM_MEM_DEVICE) {
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        *bytes = (const uint8_t *)ctx->td_bytes.p;
        *offsets = (const int64_t *)ctx->td_off.p;
        return HM_OK;
    }
    size_t dummy = 0;
    if ((size_t)total + 16 > ctx->h_td_bytes_cap || !ctx->h_td_bytes) {
        const size_t want = (size_t)total + total / 4 + 4096;
        if ((rc = ensure_host(ctx, &ctx->h_td_bytes, dummy, want, 1))) return rc;
        ctx->h_td_bytes_cap = want;
    }
    if ((size_t)n + 1 > ctx->h_td_off_cap || !ctx->h_td_off) {
        const size_t want = (size_t)n + n / 4 + 1024;
        if ((rc = ensure_host(ctx, &ctx->h_td_off, dummy, want, 8))) return rc;
        ctx->h_td_off_cap = want;
    }
    if (total) HIPCHK(ctx, hipMemcpyAsync(ctx->h_td_bytes, ctx->td_bytes.p, total, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_td_off, off, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    *bytes = (const uint8_t *)ctx->h_td_bytes;
    *offsets = (const int64_t *)ctx->h_td_off;
    return HM_OK;
}

int hm_encode_tile_updates(hm_ctx *ctx, const hm_tile_doc_cfg *cfg, int32_t out_memory, const uint8_t **bytes,
                           const int64_t **offsets, int64_t *n_docs) {
    if (!ctx || !cfg || !bytes || !offsets || !n_docs || cfg->city_len < 0 || (cfg->city_len > 0 && !cfg->city) ||
        cfg->n_windows < 0 || (cfg->n_windows > 0 && (!cfg->window_start_us || !cfg->start_offset_s || !cfg->end_offset_s)))
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (cfg->city_len > (1 << 20)) return set_err(ctx, HM_E_INVALID, "city of %d bytes (at most 1 MiB)", cfg->city_len);
    const int64_t n = ctx->last_n_tiles;
    const auto &W = ctx->batch_windows;
    if (cfg->n_windows != (int64_t)W.size()) return set_err(ctx, HM_E_INVALID, "%lld window offsets for %zu windows", (long long)cfg->n_windows, W.size());
    for (size_t k = 0; k < W.size(); k++) {
        if (cfg->window_start_us[k] != W[k]) return set_err(ctx, HM_E_INVALID, "window offsets not in hm_last_windows order");
        const int64_t a = W[k] / 1000000 - (W[k] % 1000000 < 0) + cfg->start_offset_s[k];
        const int64_t b = (W[k] + ctx->cfg.tile_us) / 1000000 + cfg->end_offset_s[k];
        if (civil_year(a) < 1000 || civil_year(a) > 9999 || civil_year(b) > 9999)
            return set_err(ctx, HM_E_INVALID, "window start %lld us: year outside 1000-9999", (long long)W[k]);
        if (W[k] % 1000000 != 0) return set_err(ctx, HM_E_INVALID, "window start %lld us is not a whole second", (long long)W[k]);
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const int nw = (int)W.size();
    // parameters: city bytes (padded to 16), then the window table (3 x nw int64)
    const size_t cbytes = ((size_t)cfg->city_len + 15) & ~(size_t)15;
    const size_t pbytes = cbytes + (size_t)nw * 24 + 16;
    if ((rc = ensure(ctx, ctx->td_params, pbytes)) || (rc = ensure(ctx, ctx->td_off, (n + 1) * 8)) ||
        (rc = ensure(ctx, ctx->td_sizes, std::max<int64_t>(n, 1) * 4)))
        return rc;
    std::vector<uint8_t> hp(pbytes, 0);
    if (cfg->city_len) memcpy(hp.data(), cfg->city, cfg->city_len);
    if (nw) {
        memcpy(hp.data() + cbytes, W.data(), nw * 8);
        memcpy(hp.data() + cbytes + nw * 8, cfg->start_offset_s, nw * 8);
        memcpy(hp.data() + cbytes + nw * 16, cfg->end_offset_s, nw * 8);
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->td_params.p, hp.data(), pbytes, hipMemcpyHostToDevice, ctx->stream));
    TileDocParams P;
    P.city = (const uint8_t *)ctx->td_params.p;
    P.city_len = cfg->city_len;
    P.h3_res = ctx->cfg.h3_res;
    P.tile_us = ctx->cfg.tile_us;
    P.ttl_ms = cfg->ttl_ms;
    P.win_start_us = (const int64_t *)((uint8_t *)ctx->td_params.p + cbytes);
    P.off_start_s = P.win_start_us + nw;
    P.off_end_s = P.win_start_us + 2 * nw;
    P.n_win = nw;
    unsigned long long *off = (unsigned long long *)ctx->td_off.p;
    int64_t total = 0;
    if (n > 0) {
        if (nw == 0) return set_err(ctx, HM_E_STATE, "tiles without windows");
        hipLaunchKernelGGL(k_tile_doc_sizes, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, (const uint64_t *)ctx->o_cell.p,
                           (const int64_t *)ctx->o_ws.p, (const int64_t *)ctx->o_cnt.p, n, (unsigned *)ctx->td_sizes.p);
        const int64_t nb = (n + SC_PER - 1) / SC_PER;
        if ((rc = ensure(ctx, ctx->td_btot, nb * 4)) || (rc = ensure(ctx, ctx->td_boff, nb * 8))) return rc;
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_sizes.p, n, off,
                           (unsigned *)ctx->td_btot.p);
        hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_btot.p, nb,
                           (unsigned long long *)ctx->td_boff.p, off + n);
        hipLaunchKernelGGL(k_scan_add, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, off, n, (const unsigned long long *)ctx->td_boff.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(&total, off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if ((rc = ensure(ctx, ctx->td_bytes, total + 16))) return rc;
        // LDS staging sized by the longest statement this city/resolution can produce (int64 count, 16 hex
        // digits): occupancy is bounded by it (~400 B per statement -> 3 workgroups per CU)
        TileDocParams Ph = P;
        Ph.city = (const uint8_t *)cfg->city;
        Ph.win_start_us = W.data();
        Ph.off_start_s = cfg->start_offset_s;
        Ph.off_end_s = cfg->end_offset_s;
        const int max_doc = tile_statement(nullptr, Ph, ~0ull, W[0], INT64_MAX, 0.0, 1, 0.0, 0.0);
        if (max_doc > TD_MAX_DOC) {   // a long CITY: no LDS staging
            hipLaunchKernelGGL(k_tile_docs_direct, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, (const uint64_t *)ctx->o_cell.p,
                               (const int64_t *)ctx->o_ws.p, (const int64_t *)ctx->o_cnt.p, (const double *)ctx->o_sp.p,
                               (const uint8_t *)ctx->o_spn.p, (const double *)ctx->o_lon.p, (const double *)ctx->o_lat.p, n,
                               (const unsigned long long *)off, (uint8_t *)ctx->td_bytes.p);
        } else {
            const size_t lds = (size_t)TD_THREADS * ((max_doc + 15) & ~15) + 32;
            if (lds > 65536)
                HIPCHK(ctx, hipFuncSetAttribute((const void *)k_tile_docs, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(k_tile_docs, dim3(grid_for(n, TD_THREADS)), dim3(TD_THREADS), lds, ctx->stream, P, (const uint64_t *)ctx->o_cell.p,
                               (const int64_t *)ctx->o_ws.p, (const int64_t *)ctx->o_cnt.p, (const double *)ctx->o_sp.p,
                               (const uint8_t *)ctx->o_spn.p, (const double *)ctx->o_lon.p, (const double *)ctx->o_lat.p, n,
                               (const unsigned long long *)off, (uint8_t *)ctx->td_bytes.p);
        }
        HIPCHK(ctx, hipGetLastError());
    } else {
        HIPCHK(ctx, hipMemsetAsync(off, 0, 8, ctx->stream));
        if ((rc = ensure(ctx, ctx->td_bytes, 16))) return rc;
    }
    return statements_out(ctx, n, total, out_memory, bytes, offsets, n_docs);
}

// latest positions of the last hm_process_batch as positions_latest update statements (bson_docs.h)
static int pos_params(hm_ctx *ctx, const hm_position_doc_cfg *cfg, PosDocParams &P, std::vector<uint8_t> &hp) {
    const int64_t np_ = cfg->n_providers, nv = cfg->n_vehicles, nb = cfg->n_buckets;
    if (np_ < 0 || nv < 0 || nb < 0 || (np_ && (!cfg->provider_offsets || !cfg->provider_bytes)) ||
        (nv && (!cfg->vehicle_offsets || !cfg->vehicle_bytes)) || (nb && (!cfg->bucket_ids || !cfg->bucket_offset_s)))
        return set_err(ctx, HM_E_INVALID, "bad position dictionaries");
    for (int64_t k = 1; k < nb; k++)
        if (cfg->bucket_ids[k - 1] >= cfg->bucket_ids[k]) return set_err(ctx, HM_E_INVALID, "bucket ids not ascending");
    const int64_t pb = np_ ? cfg->provider_offsets[np_] : 0, vb = nv ? cfg->vehicle_offsets[nv] : 0;
    for (int64_t k = 0; k < np_; k++)
        if (cfg->provider_offsets[k] < 0 || cfg->provider_offsets[k] > cfg->provider_offsets[k + 1] ||
            cfg->provider_offsets[k + 1] - cfg->provider_offsets[k] > (1 << 20))
            return set_err(ctx, HM_E_INVALID, "provider offsets");
    for (int64_t k = 0; k < nv; k++)
        if (cfg->vehicle_offsets[k] < 0 || cfg->vehicle_offsets[k] > cfg->vehicle_offsets[k + 1] ||
            cfg->vehicle_offsets[k + 1] - cfg->vehicle_offsets[k] > (1 << 20))
            return set_err(ctx, HM_E_INVALID, "vehicle offsets");
    // one device block: offsets (8-B aligned) first, then the string bytes
    const size_t o_p = 0, o_v = o_p + (np_ + 1) * 8, o_bi = o_v + (nv + 1) * 8, o_b = o_bi + nb * 8, o_ps = o_b + nb * 8,
                 o_vs = o_ps + pb;
    hp.assign(o_vs + vb + 8, 0);
    if (np_) memcpy(hp.data() + o_p, cfg->provider_offsets, (np_ + 1) * 8);
    if (nv) memcpy(hp.data() + o_v, cfg->vehicle_offsets, (nv + 1) * 8);
    if (nb) memcpy(hp.data() + o_bi, cfg->bucket_ids, nb * 8);
    if (nb) memcpy(hp.data() + o_b, cfg->bucket_offset_s, nb * 8);
    if (pb) memcpy(hp.data() + o_ps, cfg->provider_bytes, pb);
    if (vb) memcpy(hp.data() + o_vs, cfg->vehicle_bytes, vb);
    int rc;
    if ((rc = ensure(ctx, ctx->td_params, hp.size()))) return rc;
    HIPCHK(ctx, hipMemcpyAsync(ctx->td_params.p, hp.data(), hp.size(), hipMemcpyHostToDevice, ctx->stream));
    uint8_t *d = (uint8_t *)ctx->td_params.p;
    P.p_off = (const int64_t *)(d + o_p);
    P.v_off = (const int64_t *)(d + o_v);
    P.bucket_id = (const int64_t *)(d + o_bi);
    P.bucket_off = (const int64_t *)(d + o_b);
    P.p_bytes = d + o_ps;
    P.v_bytes = d + o_vs;
    P.n_providers = np_;
    P.n_vehicles = nv;
    P.n_buckets = nb;
    return HM_OK;
}

int hm_encode_position_updates(hm_ctx *ctx, const hm_position_doc_cfg *cfg, int32_t out_memory, const uint8_t **bytes,
                               const int64_t **offsets, int64_t *n_docs) {
    if (!ctx || !cfg || !bytes || !offsets || !n_docs) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->last_n_latest < 0) return set_err(ctx, HM_E_STATE, "no hm_process_batch latest rows to encode");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int64_t n = ctx->last_n_latest;
    int rc;
    PosDocParams P;
    std::vector<uint8_t> hp;
    if ((rc = pos_params(ctx, cfg, P, hp))) return rc;
    if ((rc = ensure(ctx, ctx->td_off, (n + 1) * 8)) || (rc = ensure(ctx, ctx->td_sizes, std::max<int64_t>(n, 1) * 4))) return rc;
    unsigned long long *off = (unsigned long long *)ctx->td_off.p;
    int64_t total = 0;
    if (n > 0) {
        const int64_t *rows = (const int64_t *)ctx->rows.p;
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + POSBAD_WORD, 0, 8, ctx->stream));
        hipLaunchKernelGGL(k_pos_doc_sizes, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, rows, n, ctx->last_vk,
                           ctx->last_ts, (unsigned *)ctx->td_sizes.p, ctx->d_scratch + POSBAD_WORD);
        const int64_t nb = (n + SC_PER - 1) / SC_PER;
        if ((rc = ensure(ctx, ctx->td_btot, nb * 4)) || (rc = ensure(ctx, ctx->td_boff, nb * 8))) return rc;
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_sizes.p, n, off,
                           (unsigned *)ctx->td_btot.p);
        hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_btot.p, nb,
                           (unsigned long long *)ctx->td_boff.p, off + n);
        hipLaunchKernelGGL(k_scan_add, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, off, n, (const unsigned long long *)ctx->td_boff.p);
        HIPCHK(ctx, hipGetLastError());
        unsigned long long hb[2] = {0, 0};
        HIPCHK(ctx, hipMemcpyAsync(&hb[0], off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(&hb[1], ctx->d_scratch + POSBAD_WORD, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hb[1]) return set_err(ctx, HM_E_INVALID, "%llu latest rows outside the provider/vehicle dictionaries or time buckets", hb[1]);
        total = (int64_t)hb[0];
        if ((rc = ensure(ctx, ctx->td_bytes, total + 16))) return rc;
        hipLaunchKernelGGL(k_pos_docs, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, rows, n, ctx->last_vk, ctx->last_ts,
                           ctx->last_lat, ctx->last_lon, (const unsigned long long *)off, (uint8_t *)ctx->td_bytes.p);
        HIPCHK(ctx, hipGetLastError());
    } else {
        HIPCHK(ctx, hipMemsetAsync(off, 0, 8, ctx->stream));
        if ((rc = ensure(ctx, ctx->td_bytes, 16))) return rc;
    }
    return statements_out(ctx, n, total, out_memory, bytes, offsets, n_docs);
}

// ---- Kafka values -> batch columns (row f1; json_decode.h) ----
__global__ __launch_bounds__(256) void k_check_offsets(const int64_t *__restrict__ offs, int64_t n, int64_t lo, int64_t hi,
                                                       unsigned long long *bad) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        b += offs[i] < lo || offs[i] > offs[i + 1] || offs[i + 1] > hi;
    b = wave_sum(b);
    if (b && lane_id() == 0) atomicAdd(bad, b);
}

static int host_pinned(hm_ctx *ctx, void **p, size_t &cap, size_t want) {
    if (*p && cap >= want) return HM_OK;
    AllocTimer at_(ctx);
    if (*p) { HIPCHK(ctx, hipHostFree(*p)); ctx->n_frees++; }
    cap = *p ? host_cap_for(cap, want) : std::max<size_t>(want, 4096);
    *p = nullptr;
    ctx->n_allocs++;
    HIPCHK(ctx, hipHostMalloc(p, cap, hipHostMallocDefault));
    return HM_OK;
}

// the exact dictionary of one string column (spans off/len into bytes or scratch; len -1 = null): slot_of per row,
// code_of_slot, and the strings (Arrow offsets + bytes) in the Dict's pinned host buffers
static int dict_build(hm_ctx *ctx, hm_ctx::Dict &d, const uint8_t *bytes, const uint8_t *scratch, const int64_t *off,
                      const int32_t *len, int64_t n) {
    int rc;
    const unsigned long long full = next_pow2((unsigned long long)std::max<int64_t>(2 * n, 1024));
    unsigned long long cap = d.last_codes > 0 ? next_pow2((unsigned long long)std::max<int64_t>(4 * d.last_codes, 1024))
                                              : (1ull << 16);
    cap = std::min(cap, full);
    uint64_t seed = UINT64_C(0x8f1bbcdcca62c1d6);
    unsigned long long *words = ctx->d_scratch + JSON_WORD + 2;   // overflow, collisions
    for (int attempt = 0;; attempt++) {
        if (attempt == 6) return set_err(ctx, HM_E_OVERFLOW, "string dictionary: repeated hash collisions");
        if ((rc = ensure(ctx, d.tab, cap * sizeof(DictSlot))) || (rc = ensure(ctx, d.slot_of, std::max<int64_t>(n, 1) * 4)))
            return rc;
        HIPCHK(ctx, hipMemsetAsync(d.tab.p, 0xff, cap * sizeof(DictSlot), ctx->stream));
        HIPCHK(ctx, hipMemsetAsync(words, 0, 16, ctx->stream));
        hipLaunchKernelGGL(k_dict_insert, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, bytes, scratch, off, len, n,
                           (DictSlot *)d.tab.p, cap - 1, seed, (unsigned *)d.slot_of.p, words);
        hipLaunchKernelGGL(k_dict_verify, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, bytes, scratch, off, len, n,
                           (const DictSlot *)d.tab.p, (const unsigned *)d.slot_of.p, words + 1);
        HIPCHK(ctx, hipGetLastError());
        unsigned long long hw[2];
        HIPCHK(ctx, hipMemcpyAsync(hw, words, 16, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hw[0]) {   // probes ran out (more distinct strings than the last batch): a full-size table
            if (cap == full) return set_err(ctx, HM_E_OVERFLOW, "string dictionary table overflow");
            cap = full;
            continue;
        }
        if (hw[1]) {   // a 64-bit hash collision: another seed
            seed = mix64(seed + (uint64_t)attempt + 1);
            continue;
        }
        break;
    }
    // codes: the occupied slots in ascending order
    if ((rc = ensure(ctx, d.occ, cap)) || (rc = ensure(ctx, d.slots, cap * 8)) || (rc = ensure(ctx, d.code_of_slot, cap * 4)))
        return rc;
    hipLaunchKernelGGL(k_dict_occ, dim3(grid_for((int64_t)cap, 256)), dim3(256), 0, ctx->stream, (const DictSlot *)d.tab.p,
                       (int64_t)cap, (uint8_t *)d.occ.p);
    if ((rc = compact_flags(ctx, (const uint8_t *)d.occ.p, (int64_t)cap, (int64_t *)d.slots.p, ctx->stream))) return rc;
    unsigned long long nc = 0;
    HIPCHK(ctx, hipMemcpyAsync(&nc, ctx->d_scratch + 255, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    const int64_t m = (int64_t)nc;
    if ((rc = ensure(ctx, d.clen, std::max<int64_t>(m, 1) * 4)) || (rc = ensure(ctx, d.coff, (m + 1) * 8))) return rc;
    hipLaunchKernelGGL(k_dict_codes, dim3(grid_for(std::max<int64_t>(m, 1), 256)), dim3(256), 0, ctx->stream,
                       (const int64_t *)d.slots.p, ctx->d_scratch + 255, (const DictSlot *)d.tab.p, len,
                       (unsigned *)d.code_of_slot.p, (unsigned *)d.clen.p);
    unsigned long long *coff = (unsigned long long *)d.coff.p;
    int64_t total = 0;
    if (m > 0) {
        const int64_t nb = (m + SC_PER - 1) / SC_PER;
        if ((rc = ensure(ctx, d.btot, nb * 4)) || (rc = ensure(ctx, d.boff, nb * 8))) return rc;
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, (const unsigned *)d.clen.p, m, coff,
                           (unsigned *)d.btot.p);
        hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)d.btot.p, nb,
                           (unsigned long long *)d.boff.p, coff + m);
        hipLaunchKernelGGL(k_scan_add, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, coff, m, (const unsigned long long *)d.boff.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(&total, coff + m, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    } else {
        HIPCHK(ctx, hipMemsetAsync(coff, 0, 8, ctx->stream));
    }
    if ((rc = ensure(ctx, d.cbytes, std::max<int64_t>(total, 1)))) return rc;
    if (m > 0)
        hipLaunchKernelGGL(k_dict_gather, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, bytes, scratch, off, len,
                           (const int64_t *)d.slots.p, ctx->d_scratch + 255, (const DictSlot *)d.tab.p,
                           (const unsigned long long *)coff, (uint8_t *)d.cbytes.p);
    HIPCHK(ctx, hipGetLastError());
    if ((rc = host_pinned(ctx, &d.h_off, d.h_off_cap, (size_t)(m + 1) * 8)) ||
        (rc = host_pinned(ctx, &d.h_bytes, d.h_bytes_cap, (size_t)std::max<int64_t>(total, 1))))
        return rc;
    HIPCHK(ctx, hipMemcpyAsync(d.h_off, coff, (m + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (total) HIPCHK(ctx, hipMemcpyAsync(d.h_bytes, d.cbytes.p, total, hipMemcpyDeviceToHost, ctx->stream));
    d.n_codes = m;
    d.last_codes = m;
    return HM_OK;
}

int hm_decode_json(hm_ctx *ctx, const hm_json_in *in, hm_json_out *out) {
    if (!ctx || !in || !out || in->n < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    const int64_t n = in->n;
    if (n > (int64_t)UINT32_MAX - 2) return set_err(ctx, HM_E_INVALID, "%lld records exceed 2^32-2", (long long)n);
    if (n > 0 && (!in->bytes || !in->offsets)) return set_err(ctx, HM_E_INVALID, "bytes and offsets are required");
    if (in->memory != HM_MEM_HOST && in->memory != HM_MEM_DEVICE) return set_err(ctx, HM_E_INVALID, "bad memory kind");
    memset(out, 0, sizeof(*out));
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const size_t m = (size_t)std::max<int64_t>(n, 1);
    if ((rc = ensure(ctx, ctx->jd_lat, m * 8)) || (rc = ensure(ctx, ctx->jd_lon, m * 8)) || (rc = ensure(ctx, ctx->jd_ts, m * 8)) ||
        (rc = ensure(ctx, ctx->jd_speed, m * 8)) || (rc = ensure(ctx, ctx->jd_sv, m)) || (rc = ensure(ctx, ctx->jd_rv, m)) ||
        (rc = ensure(ctx, ctx->jd_vkey, m * 8)) || (rc = ensure(ctx, ctx->jd_poff, m * 8)) || (rc = ensure(ctx, ctx->jd_plen, m * 4)) ||
        (rc = ensure(ctx, ctx->jd_voff, m * 8)) || (rc = ensure(ctx, ctx->jd_vlen, m * 4)))
        return rc;
    int64_t o0 = 0, on = 0;
    const uint8_t *dbytes = nullptr;
    const int64_t *doffs = nullptr;
    if (n > 0) {
        if (in->memory == HM_MEM_HOST) {
            o0 = in->offsets[0];
            on = in->offsets[n];
            if (o0 < 0 || on < o0) return set_err(ctx, HM_E_INVALID, "bad offsets");
            if ((rc = ensure(ctx, ctx->jd_bytes, (size_t)(on - o0) + 16)) || (rc = ensure(ctx, ctx->jd_offs, (size_t)(n + 1) * 8))) return rc;
            if (on > o0) HIPCHK(ctx, hipMemcpyAsync(ctx->jd_bytes.p, in->bytes + o0, on - o0, hipMemcpyHostToDevice, ctx->stream));
            HIPCHK(ctx, hipMemcpyAsync(ctx->jd_offs.p, in->offsets, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
            dbytes = (const uint8_t *)ctx->jd_bytes.p;
            doffs = (const int64_t *)ctx->jd_offs.p;
        } else {
            HIPCHK(ctx, hipMemcpyAsync(&o0, in->offsets, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, hipMemcpyAsync(&on, in->offsets + n, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, ctx_sync(ctx, __LINE__));
            if (o0 < 0 || on < o0) return set_err(ctx, HM_E_INVALID, "bad offsets");
            dbytes = in->bytes + o0;
            doffs = in->offsets;
        }
        // every record inside [o0, on] with non-decreasing offsets (a bad offset would read out of bounds)
        unsigned long long *w = ctx->d_scratch + JSON_WORD;
        HIPCHK(ctx, hipMemsetAsync(w, 0, 16, ctx->stream));
        hipLaunchKernelGGL(k_check_offsets, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, doffs, n, o0, on, w);
        unsigned long long hb = 0;
        HIPCHK(ctx, hipMemcpyAsync(&hb, w, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hb) return set_err(ctx, HM_E_INVALID, "%llu offsets out of order or out of range", hb);
        if ((rc = ensure(ctx, ctx->jd_scratch, (size_t)(on - o0) + 16))) return rc;
        hipLaunchKernelGGL(k_json_parse, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, dbytes, doffs, o0, n,
                           (uint8_t *)ctx->jd_scratch.p, (double *)ctx->jd_lat.p, (double *)ctx->jd_lon.p, (int64_t *)ctx->jd_ts.p,
                           (double *)ctx->jd_speed.p, (uint8_t *)ctx->jd_sv.p, (uint8_t *)ctx->jd_rv.p, (int64_t *)ctx->jd_poff.p,
                           (int32_t *)ctx->jd_plen.p, (int64_t *)ctx->jd_voff.p, (int32_t *)ctx->jd_vlen.p, w);
        HIPCHK(ctx, hipGetLastError());
        unsigned long long counts[2];
        HIPCHK(ctx, hipMemcpyAsync(counts, w, 16, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        out->n_malformed = (int64_t)counts[0];
        out->n_unsupported = (int64_t)counts[1];
        if (counts[1])
            return set_err(ctx, HM_E_UNSUPPORTED, "%llu records outside the device decoder (a number of more than 19 significant "
                           "digits on a rounding boundary, or a float/object/array as a string field)", counts[1]);
    }
    const uint8_t *scratch = (const uint8_t *)ctx->jd_scratch.p;
    if ((rc = dict_build(ctx, ctx->jd_prov, dbytes, scratch, (const int64_t *)ctx->jd_poff.p, (const int32_t *)ctx->jd_plen.p, n)) ||
        (rc = dict_build(ctx, ctx->jd_veh, dbytes, scratch, (const int64_t *)ctx->jd_voff.p, (const int32_t *)ctx->jd_vlen.p, n)))
        return rc;
    const int64_t nv = std::max<int64_t>(ctx->jd_veh.n_codes, 1);
    if (n > 0)
        hipLaunchKernelGGL(k_json_vkey, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, (const uint8_t *)ctx->jd_rv.p,
                           (const unsigned *)ctx->jd_prov.slot_of.p, (const unsigned *)ctx->jd_veh.slot_of.p,
                           (const unsigned *)ctx->jd_prov.code_of_slot.p, (const unsigned *)ctx->jd_veh.code_of_slot.p, n,
                           (uint64_t)nv, (uint64_t *)ctx->jd_vkey.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    hm_batch_in &b = out->batch;
    b.n = n;
    b.memory = HM_MEM_DEVICE;
    b.lat = (const double *)ctx->jd_lat.p;
    b.lon = (const double *)ctx->jd_lon.p;
    b.ts_us = (const int64_t *)ctx->jd_ts.p;
    b.speed = (const double *)ctx->jd_speed.p;
    b.speed_valid = (const uint8_t *)ctx->jd_sv.p;
    b.vkey = (const uint64_t *)ctx->jd_vkey.p;
    b.row_valid = (const uint8_t *)ctx->jd_rv.p;
    out->n_providers = ctx->jd_prov.n_codes;
    out->provider_offsets = (const int64_t *)ctx->jd_prov.h_off;
    out->provider_bytes = (const uint8_t *)ctx->jd_prov.h_bytes;
    out->n_vehicles = ctx->jd_veh.n_codes;
    out->vehicle_offsets = (const int64_t *)ctx->jd_veh.h_off;
    out->vehicle_bytes = (const uint8_t *)ctx->jd_veh.h_bytes;
    return HM_OK;
}

int hm_last_latest_buckets(hm_ctx *ctx, int64_t *bucket_ids, int64_t cap, int64_t *n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !bucket_ids)) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->last_n_latest < 0) return set_err(ctx, HM_E_STATE, "no hm_process_batch latest rows");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int64_t m = ctx->last_n_latest;
    *n = 0;
    if (m == 0) return HM_OK;
    int rc;
    const unsigned long long scap = next_pow2((unsigned long long)std::max<int64_t>(2 * m, 1024));
    if ((rc = ensure(ctx, ctx->lb_set, scap * 8)) || (rc = ensure(ctx, ctx->lb_list, (size_t)m * 8))) return rc;
    unsigned long long *w = ctx->d_scratch + JSON_WORD + 4;
    hipLaunchKernelGGL(k_fill_i64, dim3(grid_for((int64_t)scap, 256)), dim3(256), 0, ctx->stream, (long long *)ctx->lb_set.p,
                       (int64_t)scap, (long long)INT64_MIN);
    HIPCHK(ctx, hipMemsetAsync(w, 0, 8, ctx->stream));
    hipLaunchKernelGGL(k_latest_buckets, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, (const int64_t *)ctx->rows.p, m,
                       ctx->last_ts, (long long *)ctx->lb_set.p, scap - 1, (long long *)ctx->lb_list.p, w);
    HIPCHK(ctx, hipGetLastError());
    unsigned long long k = 0;
    HIPCHK(ctx, hipMemcpyAsync(&k, w, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    std::vector<int64_t> ids(k);
    if (k) HIPCHK(ctx, hipMemcpy(ids.data(), ctx->lb_list.p, k * 8, hipMemcpyDeviceToHost));
    std::sort(ids.begin(), ids.end());
    *n = (int64_t)k;
    for (int64_t i = 0; i < (int64_t)k && i < cap; i++) bucket_ids[i] = ids[i];
    return HM_OK;
}

int hm_selftest_json_records(const uint8_t *bytes, const int64_t *offsets, int64_t n, uint8_t *scratch, double *lat,
                             double *lon, double *speed, int64_t *ts_us, int32_t *bearing, int32_t *accuracy,
                             int64_t *p_off, int32_t *p_len, int64_t *v_off, int32_t *v_len, uint32_t *flags) {
    if (n < 0 || (n > 0 && (!bytes || !offsets || !scratch))) return HM_E_INVALID;
    for (int64_t i = 0; i < n; i++) {
        JsonRow r;
        parse_record(bytes, offsets[i], offsets[i + 1], scratch, r);
        lat[i] = r.lat;
        lon[i] = r.lon;
        speed[i] = r.speed;
        ts_us[i] = r.ts_us;
        bearing[i] = r.bearing;
        accuracy[i] = r.accuracy;
        p_off[i] = r.p_off;
        p_len[i] = r.p_len;
        v_off[i] = r.v_off;
        v_len[i] = r.v_len;
        flags[i] = r.flags;
    }
    return HM_OK;
}

int hm_selftest_decimal_to_double(const uint64_t *w, const int64_t *q, int64_t n, uint64_t *bits) {
    if (n < 0 || (n > 0 && (!w || !q || !bits))) return HM_E_INVALID;
    for (int64_t i = 0; i < n; i++) bits[i] = decimal_to_double_bits(q[i], w[i]);
    return HM_OK;
}

int hm_device_alloc(int32_t device, int64_t bytes, void **ptr) {
    if (!ptr || bytes < 0) return HM_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return HM_E_HIP;
    return hipMalloc(ptr, std::max<int64_t>(bytes, 16)) == hipSuccess ? HM_OK : HM_E_NOMEM;
}
int hm_device_free(int32_t device, void *ptr) {
    if (hipSetDevice(device) != hipSuccess) return HM_E_HIP;
    return hipFree(ptr) == hipSuccess ? HM_OK : HM_E_HIP;
}
int hm_memcpy(void *dst, const void *src, int64_t bytes, int32_t kind) {
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    return hipMemcpy(dst, src, bytes, k) == hipSuccess ? HM_OK : HM_E_HIP;
}

// host execution of the statement encoder (bson_docs.h) on caller arrays: bytes (capacity cap) + offsets[n+1]
int hm_selftest_tile_statements(const hm_tile_doc_cfg *cfg, int32_t h3_res, int64_t tile_us, const uint64_t *cell,
                                const int64_t *ws, const int64_t *cnt, const double *sp, const uint8_t *spn,
                                const double *lon, const double *lat, int64_t n, uint8_t *bytes, int64_t cap,
                                int64_t *offsets) {
    if (!cfg || n < 0 || !offsets || cfg->n_windows <= 0 || cfg->city_len < 0 || cfg->city_len > (1 << 20)) return HM_E_INVALID;
    TileDocParams P;
    P.city = (const uint8_t *)cfg->city;
    P.city_len = cfg->city_len;
    P.h3_res = h3_res;
    P.tile_us = tile_us;
    P.ttl_ms = cfg->ttl_ms;
    P.win_start_us = cfg->window_start_us;
    P.off_start_s = cfg->start_offset_s;
    P.off_end_s = cfg->end_offset_s;
    P.n_win = (int)cfg->n_windows;
    int64_t o = 0;
    for (int64_t i = 0; i < n; i++) {
        offsets[i] = o;
        const int len = tile_statement(nullptr, P, cell[i], ws[i], cnt[i], sp[i], spn[i], lon[i], lat[i]);
        if (o + len > cap) return HM_E_INVALID;
        tile_statement(bytes + o, P, cell[i], ws[i], cnt[i], sp[i], spn[i], lon[i], lat[i]);
        o += len;
    }
    offsets[n] = o;
    return HM_OK;
}

// host execution of the positions statement encoder (bson_docs.h) on caller rows (vkey, ts, lat, lon per row)
int hm_selftest_position_statements(const hm_position_doc_cfg *cfg, const uint64_t *vkey, const int64_t *ts,
                                    const double *lat, const double *lon, int64_t n, uint8_t *bytes, int64_t cap,
                                    int64_t *offsets) {
    if (!cfg || n < 0 || !offsets) return HM_E_INVALID;
    PosDocParams P;
    P.p_off = cfg->provider_offsets;
    P.p_bytes = (const uint8_t *)cfg->provider_bytes;
    P.v_off = cfg->vehicle_offsets;
    P.v_bytes = (const uint8_t *)cfg->vehicle_bytes;
    P.n_providers = cfg->n_providers;
    P.n_vehicles = cfg->n_vehicles;
    P.n_buckets = cfg->n_buckets;
    P.bucket_id = cfg->bucket_ids;
    P.bucket_off = cfg->bucket_offset_s;
    int64_t o = 0;
    for (int64_t i = 0; i < n; i++) {
        offsets[i] = o;
        if (!position_ok(P, vkey[i], ts[i])) return HM_E_INVALID;
        const int len = position_statement(nullptr, P, vkey[i], ts[i], lat[i], lon[i]);
        if (o + len > cap) return HM_E_INVALID;
        position_statement(bytes + o, P, vkey[i], ts[i], lat[i], lon[i]);
        o += len;
    }
    offsets[n] = o;
    return HM_OK;
}

int hm_selftest_ld_ops(const double *a, int64_t n, int32_t op, double *out) {
    if (!a || !out || n < 0) return HM_E_INVALID;
    for (int64_t i = 0; i < n; i++) {
        double x = a[i], r;
        switch (op) {
            case 0: r = XMUL(x, PI_180); break;
            case 1: r = XMUL(x, SQRT7); break;
            case 2: r = XMUL(x, RSIN60); break;
            case 3: r = XADD(x, false, 2PI); break;
            case 4: r = XADD(x, true, 2PI); break;
            case 5: r = XADD(x, true, AP7_ROT); break;
            case 6: r = XADD(x, false, AP7_ROT); break;
            case 7: r = XMUL(x, SQRT3_2); break;
            case 8: r = XMUL(x, RSQRT7); break;
            case 9: r = XMUL(x, ONETHIRD); break;
            case 17: r = XMUL(x, 180_PI); break;
            case 10: r = xld_mul(x, HM_LD_PI_180_M, HM_LD_PI_180_E); break;
            case 11: r = xld_mul(x, HM_LD_SQRT7_M, HM_LD_SQRT7_E); break;
            case 12: r = xld_mul(x, HM_LD_RSIN60_M, HM_LD_RSIN60_E); break;
            case 13: r = xld_add(x, false, HM_LD_2PI_M, HM_LD_2PI_E); break;
            case 14: r = xld_add(x, true, HM_LD_2PI_M, HM_LD_2PI_E); break;
            case 15: r = xld_add(x, true, HM_LD_AP7_ROT_M, HM_LD_AP7_ROT_E); break;
            case 16: r = xld_add(x, false, HM_LD_AP7_ROT_M, HM_LD_AP7_ROT_E); break;
            default: return HM_E_INVALID;
        }
        out[i] = r;
    }
    return HM_OK;
}

int hm_selftest_floor_div(const int64_t *t, int64_t n, int64_t d, int64_t *out) {
    if (!t || !out || n < 0 || d < 1) return HM_E_INVALID;
    const FloorDiv D = make_floor_div(d);
    for (int64_t i = 0; i < n; i++) out[i] = floor_div(t[i], D);
    return HM_OK;
}

int hm_selftest_latlng_to_cell_host(const double *lat, const double *lon, int64_t n, int32_t res, uint64_t *out) {
    if (!lat || !lon || !out || n < 0 || res < 0 || res > 15) return HM_E_INVALID;
    static const H3Tables T = make_tables();
    for (int64_t i = 0; i < n; i++) out[i] = latLngToCellDeg(lat[i], lon[i], res, T);
    return HM_OK;
}

int hm_selftest_latlng_to_cell_fast_host(const double *lat, const double *lon, int64_t n, int32_t res, uint64_t *out,
                                         uint8_t *fell_back) {
    if (!lat || !lon || !out || n < 0 || res < 0 || res > 15) return HM_E_INVALID;
    static const H3Tables T = make_tables();
    for (int64_t i = 0; i < n; i++) {
        const bool ok = latLngToCellFast(lat[i], lon[i], res, T, out[i]);
        if (!ok) out[i] = latLngToCellDeg(lat[i], lon[i], res, T);
        if (fell_back) fell_back[i] = !ok;
    }
    return HM_OK;
}

// glibc's sincos / acos / atan2 / tan as restated in glibc_libm.h (fn 0 sincos: out = sin, out2 = cos; 1 acos(a);
// 2 atan2(a, b); 3 tan(a)), executed on the host and on the GPU (test entry points; tests/test_glibc_libm.py)
static int glm_check(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2) {
    if (!a || !out || n < 0 || fn < 0 || fn > 3 || (fn == 0 && !out2) || (fn == 2 && !b)) return HM_E_INVALID;
    return HM_OK;
}
HM_HD void glm_eval(int32_t fn, int64_t i, const double *a, const double *b, double *out, double *out2,
                    const glm::Tables &G) {
    switch (fn) {
        case 0: glm::sincos(a[i], out[i], out2[i], G); break;
        case 1: out[i] = glm::acos(a[i], G); break;
        case 2: out[i] = glm::atan2(a[i], b[i], G); break;
        default: out[i] = glm::tan(a[i], G); break;
    }
}
__global__ __launch_bounds__(256) void k_glibc_libm(int32_t fn, const double *a, const double *b, int64_t n,
                                                    double *out, double *out2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        glm_eval(fn, i, a, b, out, out2, g_glm);
}

int hm_selftest_glibc_libm_host(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2) {
    if (int e = glm_check(fn, a, b, n, out, out2)) return e;
    for (int64_t i = 0; i < n; i++) glm_eval(fn, i, a, b, out, out2, hm_glm_host);
    return HM_OK;
}

int hm_selftest_glibc_libm_device(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2,
                                  int32_t device) {
    if (int e = glm_check(fn, a, b, n, out, out2)) return e;
    int ndev = 0;
    if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev || hipSetDevice(device) != hipSuccess)
        return HM_E_HIP;
    if (n == 0) return HM_OK;
    const size_t B = (size_t)n * sizeof(double);
    double *d[4] = {nullptr, nullptr, nullptr, nullptr};
    int rc = HM_OK;
    for (int k = 0; k < 4 && rc == HM_OK; k++)
        if (hipMalloc((void **)&d[k], B) != hipSuccess) rc = HM_E_NOMEM;
    if (rc == HM_OK && (hipMemcpy(d[0], a, B, hipMemcpyHostToDevice) != hipSuccess ||
                        (b && hipMemcpy(d[1], b, B, hipMemcpyHostToDevice) != hipSuccess)))
        rc = HM_E_HIP;
    if (rc == HM_OK) {
        hipLaunchKernelGGL(k_glibc_libm, dim3(grid_for(n, 256)), dim3(256), 0, 0, fn, d[0], d[1], n, d[2], d[3]);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(out, d[2], B, hipMemcpyDeviceToHost) != hipSuccess ||
            (fn == 0 && hipMemcpy(out2, d[3], B, hipMemcpyDeviceToHost) != hipSuccess))
            rc = HM_E_HIP;
    }
    for (double *p : d)
        if (p) (void)hipFree(p);
    return rc;
}

}  // extern "C"
