// Device helpers shared by the kernels: wave primitives, per-window state-table lookups, census sinks, the batch's window registry.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

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
    return ((unsigned long long)((region_field(h) >> g.sb) - g.rbase) << g.rshift) | inreg_slot(h, g.rmask);
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
    const unsigned sb = g->sb;
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
    unsigned long long inner[WC_SLOTS];   // window_inner of the cached window, 0 until a row has computed it
    unsigned cnt[WC_SLOTS];   // aggregated rows per cached window (the direct path's census)
};
__device__ __forceinline__ void wc_init(WinCacheL &C) {
    for (int q = threadIdx.x; q < WC_SLOTS; q += blockDim.x) { C.e[q] = 0; C.inner[q] = 0; C.cnt[q] = 0; }
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
