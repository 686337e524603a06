// Radix partition kernels: (window, region) bins of the merge, owner ranks of the multi-GPU exchange (heatmap_stream.py:112-133; Spark's shuffle, :44).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// =====================================================================================================
// K2b: radix partition of the partials into RP_BINS bins (kernels.h: one bin per (window, region)), so that
// one merge workgroup owns each region: tile histogram (LDS) -> digit-major exclusive scan -> LDS-cursor
// scatter.  Records are one 64-B line each, so the scattered writes are whole lines.
// =====================================================================================================
constexpr int RP_BITS = REGION_BITS;
constexpr int RP_BINS = 1 << RP_BITS;
constexpr int RP_TILE = 131072;    // partials per tile (one workgroup) at most (65536 / 262144: within noise, r1 tune2)
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
    if (nranks > 0) return (unsigned)tile_owner_of(h, nranks);
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

typedef unsigned hm_v4u __attribute__((ext_vector_type(4)));
// (non-temporal record loads in the merge measured +1.1 ms, profiles/r1/nt2/: plain loads)
template <typename Rec>
__device__ __forceinline__ Rec ld_stream(const Rec *p) { return *p; }

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
                    d = (unsigned)tile_owner_of(h, nranks);
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
                if (rec < nrec && p != ~0u) d4[(int64_t)p * QO + q] = rp_part<In, Out>(ws, rec, q, (uint64_t)hl | ((uint64_t)hh << 32));
            }
            __builtin_amdgcn_wave_barrier();
        } else {
            for (int r = 0; r < QO; r++) {
                const int idx = r * 64 + ln, rec = idx / QO, q = idx % QO;
                const unsigned p = __shfl(pos, rec, 64);
                if (rec < nrec && p != ~0u) d4[(int64_t)p * QO + q] = src[(i0 + rec) * QI + q];
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
    if (nranks > 0) return (unsigned)tile_owner_of(h, nranks);
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

// The direct path's (window, region) bins: each aggregated row's 32-B EventRec (its key, speed, lat, lon) at its bin's
// cursor; a wave builds its 64 records in LDS and writes them as rounds of 16-B parts, consecutive lanes covering
// consecutive parts of one record (whole 32-B sectors at random places), with no wait for the stores or the next
// round's loads inside the loop.  Rounds alternate between two register sets (no loop-carried copy: a register copy of
// a pending load waits for it); every load is unconditional (the row clamped into the tile, absent columns read from
// one-element device constants), and every lane stores a record each round -- a row without a key goes
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
// workgroup size of k_ev_scatter_rec (its LDS: the 8193 cursors + a 32-B record per lane)
constexpr int SR_THREADS = 512;
__global__ __launch_bounds__(SR_THREADS) void k_ev_scatter_rec(const uint64_t *__restrict__ keys, int64_t n, int64_t tile,
                                                              const double *__restrict__ speed, const uint8_t *__restrict__ speed_valid,
                                                              const double *__restrict__ lat, const double *__restrict__ lon,
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
        r.sp = __builtin_bit_cast(uint64_t, __builtin_nontemporal_load((gcd *)(speed ? &speed[j] : &g_zero_double)));
        r.sv = __builtin_nontemporal_load((gcu8 *)(speed_valid ? &speed_valid[j] : speed ? &g_one_byte : &g_zero_byte));
        r.la = __builtin_nontemporal_load((gcd *)&lat[j]);
        r.lo = __builtin_nontemporal_load((gcd *)&lon[j]);
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
        const uint64_t spb = r.sv == 0 ? SPEED_NULL_BITS
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
            st_g16(&d4[(int64_t)p * 2 + part], ws[idx]);
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
