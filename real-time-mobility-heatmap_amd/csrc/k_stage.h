// Multi-GPU exchange helpers: owner partitioning of candidates, winner routing.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

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
