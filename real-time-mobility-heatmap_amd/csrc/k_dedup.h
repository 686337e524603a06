// Latest position per (provider, vehicleId) (heatmap_stream.py:198-207) and the ordered compaction of flags into row indices.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

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
// issued together, each probe one 16-B slot load (key and max ts): the lookups' latencies overlap.  dense_cap > 0
// (only_cand: k_ingest's fused max): a vkey below it has its max in dense[vkey] (k_ingest.h DENSE_SIGN)
constexpr int DF_U = 4;
__global__ __launch_bounds__(256) void k_dedup_flag(const uint64_t *__restrict__ vkey, const int64_t *__restrict__ ts,
                                                    const uint8_t *__restrict__ flags, const Cand *__restrict__ cands, int64_t n,
                                                    const DedupSlot *__restrict__ tab, unsigned long long mask,
                                                    uint8_t *__restrict__ win, bool only_cand,
                                                    const unsigned long long *__restrict__ dense, unsigned long long dense_cap) {
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
        unsigned long long dn[DF_U];
        for (int u = 0; u < DF_U; u++) {
            dn[u] = 0;
            if (take[u]) {
                if (v[u] < dense_cap) dn[u] = dense[v[u]];
                else sl[u] = tab[h[u]];
            }
        }
        for (int u = 0; u < DF_U; u++) {
            const int64_t i = base + u * blockDim.x + threadIdx.x;
            uint8_t w = 0;
            if (take[u] && v[u] < dense_cap) {
                w = (long long)(dn[u] ^ DENSE_SIGN) == t[u];
            } else if (take[u]) {
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

// a thread's CP_PER = 16 flag bytes: one 16-B load (the flags of a whole 64-lane wave in one 1-KB access; byte loads
// ran the compaction's two passes at ~0.3 TB/s, 0.28-0.37 ms each on 1e8 rows, profiles/r5/r5tl/)
__device__ __forceinline__ void cp_load(const uint8_t *__restrict__ f, int64_t n, int64_t b0, uint8_t (&v)[CP_PER]) {
    static_assert(CP_PER == 16, "one 16-B load per thread");
    if (b0 + CP_PER <= n && ((uintptr_t)f & 15) == 0) {
        const uint4 w = *(const uint4 *)(f + b0);
        __builtin_memcpy(v, &w, 16);
    } else {
        for (int q = 0; q < CP_PER; q++) v[q] = b0 + q < n ? f[b0 + q] : 0;
    }
}
__global__ __launch_bounds__(CP_THREADS) void k_cp_count(const uint8_t *__restrict__ f, int64_t n, unsigned *__restrict__ bc) {
    __shared__ unsigned sh[CP_THREADS / 64];
    int64_t b0 = (int64_t)blockIdx.x * CP_TILE + (int64_t)threadIdx.x * CP_PER;
    uint8_t v[CP_PER];
    cp_load(f, n, b0, v);
    unsigned c = 0;
    for (int q = 0; q < CP_PER; q++) c += v[q] != 0;
    unsigned total;
    block_excl_scan(c, total, sh);
    if (threadIdx.x == 0) bc[blockIdx.x] = total;
}
// single block: exclusive scan of nb block counts (64-bit offsets), total -> *tot; 4096 counts per pass, four
// consecutive ones per thread (one thread's serial run of nb / 1024 counts took 0.12-0.34 ms on 24k counts)
__global__ __launch_bounds__(1024) void k_cp_scan(const unsigned *__restrict__ bc, int64_t nb, unsigned long long *__restrict__ off,
                                                  unsigned long long *tot) {
    unsigned long long carry = 0;
    for (int64_t t0 = 0; t0 < nb; t0 += 4096) {
        const int64_t b = t0 + (int64_t)threadIdx.x * 4;
        unsigned v[4];
        unsigned long long sum = 0;
        for (int q = 0; q < 4; q++) { v[q] = b + q < nb ? bc[b + q] : 0u; sum += v[q]; }
        unsigned long long total;
        unsigned long long run = carry + block1024_exclusive(sum, &total);
        for (int q = 0; q < 4; q++)
            if (b + q < nb) { off[b + q] = run; run += v[q]; }
        carry += total;
        __syncthreads();   // (block1024_exclusive's LDS totals are rewritten by the next pass)
    }
    if (threadIdx.x == 0) *tot = carry;
}
__global__ __launch_bounds__(CP_THREADS) void k_cp_write(const uint8_t *__restrict__ f, int64_t n,
                                                         const unsigned long long *__restrict__ off, int64_t *__restrict__ out) {
    __shared__ unsigned sh[CP_THREADS / 64];
    int64_t b0 = (int64_t)blockIdx.x * CP_TILE + (int64_t)threadIdx.x * CP_PER;
    uint8_t v[CP_PER];
    cp_load(f, n, b0, v);
    unsigned c = 0;
    for (int q = 0; q < CP_PER; q++) c += v[q] != 0;
    unsigned total;
    unsigned ex = block_excl_scan(c, total, sh);
    unsigned long long pos = off[blockIdx.x] + ex;
    for (int q = 0; q < CP_PER; q++)
        if (v[q]) out[pos++] = b0 + q;
}
