// Table-mode aggregation kernels (low-cardinality batches): k_agg + k_bin_reduce (Spark's partial HashAggregate, heatmap_stream.py:112-123).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

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
// 40 B each: 150 KB of LDS, one workgroup per CU.  A prime, so that every double-hashing step visits every slot.
constexpr int AG_SLOTS = 3833;
constexpr int AG_PER = AG_SLOTS / AG_THREADS + (AG_SLOTS % AG_THREADS != 0);
// flush when fewer than 640 slots are free.  A round adds at most AG_THREADS keys, ~360 on C3; when one
// adds more than the headroom, probes fail and those rows go out as partial records (exact, just not pre-aggregated).
// C3 shard (profiles/r2/abh/): headroom 1024 -> k_agg + k_bin_reduce 4.01 ms, 640 -> 3.89 ms (~200 such partials
// per batch), 400 -> 4.1 ms (13k)
constexpr int AG_FLUSH_AT = AG_SLOTS - 640;
// aggregates kept resident by a flush.  Fewer kept = more room per flush = fewer flushes, which cost more than the
// extra evicted aggregates (C3 shard, profiles/r2/abk*/: keep 1/2 -> k_agg + k_bin_reduce 6.4 ms, 1/3 -> 4.9,
// 1/5 -> 4.35, 1/8 -> 4.0, 1/12 and 1/24 -> 4.0; evicted aggregates 30.1M / 33.7M / 37.5M / 40.1M / 41.9M / 44.1M)
constexpr int AG_KEEP_MAX = AG_SLOTS / 8;
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
    return 1u + (unsigned)(((mix64(k) & 0xffffffffu) * (uint64_t)(AG_SLOTS - 1)) >> 32);
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
