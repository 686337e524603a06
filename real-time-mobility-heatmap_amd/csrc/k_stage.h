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
    return tile_owner_of(tile_hash(r.cell, r.wstart), nranks);
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
    // one atomic per (wave, destination): the lanes with the same origin rank take consecutive positions (a returned
    // atomic per winner on a few counters serialised at ~12 ns each: 0.6 ms per pass for the bench's 50k vehicles)
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        Cand c{};
        int o = -1;
        if (i < n) {
            c = cands[widx[i]];
            o = (int)c.origin;
        }
        const bool ok = o >= 0 && o < nranks;
        unsigned long long pend = __ballot(ok);
        while (pend) {
            const int leader = __ffsll((long long)pend) - 1;
            const int d = __shfl(o, leader, 64);
            const unsigned long long m = __ballot(ok && o == d);
            unsigned long long b = 0;
            if (lane_id() == leader) b = atomicAdd(&counts_or_cursor[d], (unsigned long long)__popcll(m));
            b = __shfl(b, leader, 64);
            if (pass == 1 && ok && o == d) out[b + (unsigned long long)__popcll(m & ((1ull << lane_id()) - 1))] = c.row;
            pend &= ~m;
        }
    }
}

// =====================================================================================================
// The multi-GPU exchange: ONE chunk per (sender, destination) rank, moved by one all_to_all (hm_stage_send ->
// hm_stage_merge).  Every part 32-B aligned:
//   ChunkHdr (64 B)
//   direct path:  u32 counts[bins] -- the records of each region field the destination owns (shard_lo range, in
//                 order); u32 census[CENSUS_WORDS] -- records per global window slot (the destination's table sizes)
//   records       direct: EventRec with the batch's GLOBAL window slot in the key, grouped by region field;
//                 table mode: TilePartial
//   candidates    Cand (latest positions, to the vkey's owner)
// A record's destination is tile_owner_of(its key hash): contiguous ranges of region fields, so the sender's (window,
// region) bins -- k_ingest's fused binning, or the partition with one bin per region field -- are already grouped by
// destination, and the owner merges each bin from its senders' segments (no second partition).
// =====================================================================================================
constexpr int64_t CHUNK_MAGIC = 0x314b4e5548434d48ll;   // "HMCHUNK1"
constexpr int CENSUS_WORDS = WREG_SLOTS + 1;
struct ChunkHdr {
    int64_t magic;
    int64_t records;
    int64_t cands;
    int64_t rec_bytes;   // 32 (EventRec) or 48 (TilePartial)
    int64_t bins;        // direct path: the destination's region fields; table mode: 0
    int64_t recs_off;    // bytes from the chunk's start
    int64_t cands_off;
    int64_t bytes;       // the whole chunk
};
static_assert(sizeof(ChunkHdr) == 64, "ChunkHdr is 64 B");
HM_HD int64_t pad32(int64_t b) { return (b + 31) & ~int64_t(31); }
// the layout of a chunk of `records` records (rec_bytes each) and `cands` candidates; bins > 0: the direct path's
// counts and census precede the records
HM_HD ChunkHdr chunk_layout(int64_t records, int64_t cands, int64_t rec_bytes, int64_t bins) {
    ChunkHdr h{};
    h.magic = CHUNK_MAGIC;
    h.records = records;
    h.cands = cands;
    h.rec_bytes = rec_bytes;
    h.bins = bins;
    h.recs_off = (int64_t)sizeof(ChunkHdr) + (bins > 0 ? pad32(bins * 4) + pad32((int64_t)CENSUS_WORDS * 4) : 0);
    h.cands_off = h.recs_off + pad32(records * rec_bytes);
    h.bytes = h.cands_off + cands * (int64_t)sizeof(Cand);
    return h;
}
HM_HD int64_t chunk_census_off(int64_t bins) { return (int64_t)sizeof(ChunkHdr) + pad32(bins * 4); }

// Sender, direct path: one workgroup per region field b -- its records (slab b of k_ingest's fused binning, or the
// partition's bin b: [S[b * stride] - S[lo]) ...) copied into its owner's chunk with the key's window slot rewritten to
// the batch's global slot; the bin's count and the records' census into the chunk.  slab > 0: bin b's records start at
// src + b * slab, else at src + S[b * stride].  S: exclusive scan of the bins' record counts (stride words apart).
// self_rank >= 0: the bins this rank owns itself stay in its slabs (self-held: the local and global window slots are
// the same, hm_stage_send) -- only their counts and census go into the chunk it addresses to itself, whose header
// then counts no records; the owner merges those bins' own segment from the slabs (k_stage_segments).  self_census 0:
// the host writes that chunk's census (a world of one: the ingest's own census), the bins' counts only here.
__global__ __launch_bounds__(256) void k_stage_pack(const EventRec *__restrict__ src, int64_t slab,
                                                    const unsigned long long *__restrict__ S, int64_t stride,
                                                    const unsigned short *__restrict__ gslot_of, int nranks, int self_rank,
                                                    int self_census, const int64_t *__restrict__ chunk_start,
                                                    uint8_t *__restrict__ out) {
    __shared__ unsigned cc[CENSUS_WORDS];
    for (int q = threadIdx.x; q < CENSUS_WORDS; q += blockDim.x) cc[q] = 0;
    __syncthreads();
    const int b = blockIdx.x;
    const int o = (int)(((unsigned)b * (unsigned)nranks) >> REGION_BITS);
    const unsigned lo = shard_lo(o, nranks), hi = shard_lo(o + 1, nranks);
    const int64_t s0 = (int64_t)S[(int64_t)b * stride], cnt = (int64_t)S[(int64_t)(b + 1) * stride] - s0;
    const int64_t dst0 = s0 - (int64_t)S[(int64_t)lo * stride];
    uint8_t *chunk = out + chunk_start[o];
    const int64_t census_off = chunk_census_off((int64_t)(hi - lo));
    const ChunkHdr lay = chunk_layout(0, 0, (int64_t)sizeof(EventRec), (int64_t)(hi - lo));
    if (threadIdx.x == 0) ((unsigned *)(chunk + sizeof(ChunkHdr)))[b - lo] = (unsigned)cnt;
    const EventRec *in = src + (slab > 0 ? (int64_t)b * slab : s0);
    if (o == self_rank) {   // self-held: the census only (keys read, nothing copied)
        if (!self_census) return;
        for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) atomicAdd(&cc[gslot_of[ekey_widx(in[i].key)]], 1u);
    } else {
        EventRec *dst = (EventRec *)(chunk + lay.recs_off) + dst0;
        for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) {
            EventRec r = in[i];
            const unsigned g = gslot_of[ekey_widx(r.key)];
            r.key = (r.key & CELL_LO) | ((uint64_t)(g + 1) << 52);
            dst[i] = r;
            atomicAdd(&cc[g], 1u);
        }
    }
    __syncthreads();
    unsigned *census = (unsigned *)(chunk + census_off);
    for (int q = threadIdx.x; q < CENSUS_WORDS; q += blockDim.x)
        if (cc[q]) atomicAdd(&census[q], cc[q]);
}

// Owner, direct path: the segments of every region field it owns.  For bin b (global numbering, in [lo, hi)) and
// sender s: its records start at address SO[b * nseg + s] (in the receive buffer; the owner's own segment, self-held,
// in its slab: self_slab + b * slab_cap) and hold C[s][b - lo] of them (the chunk's counts); SP[b * nseg + s] = the
// records of b from senders < s; T[b] = all of them.  C is read from each chunk (chunk_off[s]: its byte offset);
// prefix: the exclusive scan of k_stage_counts' rows.
__global__ __launch_bounds__(256) void k_stage_segments(const uint8_t *__restrict__ recv, const int64_t *__restrict__ chunk_off,
                                                        const unsigned long long *__restrict__ prefix, int nseg, unsigned lo,
                                                        unsigned bins, int self_rank, const EventRec *self_slab, int64_t slab_cap,
                                                        unsigned long long *__restrict__ SO, unsigned *__restrict__ SP,
                                                        unsigned *__restrict__ T) {
    for (unsigned k = blockIdx.x * blockDim.x + threadIdx.x; k < (unsigned)RP_BINS; k += gridDim.x * blockDim.x) {
        if (k < lo || k >= lo + bins) {
            T[k] = 0;
            continue;
        }
        const unsigned j = k - lo;
        unsigned acc = 0;
        for (int s = 0; s < nseg; s++) {
            const uint8_t *chunk = recv + chunk_off[s];
            const ChunkHdr lay = chunk_layout(0, 0, (int64_t)sizeof(EventRec), (int64_t)bins);
            const unsigned c = ((const unsigned *)(chunk + sizeof(ChunkHdr)))[j];
            const unsigned long long *P = prefix + (int64_t)s * (bins + 1);   // (one scan over all senders' rows)
            const EventRec *base = s == self_rank ? self_slab + (int64_t)k * slab_cap
                                                  : (const EventRec *)(chunk + lay.recs_off) + (P[j] - P[0]);
            SO[(int64_t)k * nseg + s] = (unsigned long long)(uintptr_t)base;
            SP[(int64_t)k * nseg + s] = acc;
            acc += c;
        }
        T[k] = acc;
    }
}
// One GPU's binned batch in sub-bins (k_ingest sub_bits = SUB_BITS): bin k's 2^SUB_BITS sub-slabs as the segments of
// k_merge_owned's kSeg variant, in sub-region order -- SO the sub-slab's address, SP the bin's records in earlier
// sub-slabs, T[k] the bin's records (scan input; T[RP_BINS] = 0)
__global__ __launch_bounds__(256) void k_sub_segments(const unsigned *__restrict__ cur, const EventRec *slabs, int64_t slab_cap,
                                                      unsigned long long *__restrict__ SO, unsigned *__restrict__ SP,
                                                      unsigned *__restrict__ T) {
    constexpr int NS = 1 << SUB_BITS;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k <= RP_BINS; k += gridDim.x * blockDim.x) {
        if (k == RP_BINS) { T[k] = 0; continue; }
        unsigned acc = 0;
        for (int s = 0; s < NS; s++) {
            const int64_t q = (int64_t)k * NS + s;
            SO[q] = (unsigned long long)(uintptr_t)(slabs + q * slab_cap);
            SP[q] = acc;
            acc += cur[q];
        }
        T[k] = acc;
    }
}
// ---- a pipelined batch (host_pipe.h): chunk k's records are the part of every bin slab written since chunk k - 1 ----
// after chunk k's k_ingest<true> (+ its exceptions): the bin cursors (nbins + 1 words) into this chunk's snapshot, and
// the exception count, so that the next chunk's k_ingest_exact starts after this chunk's exceptions
__global__ __launch_bounds__(256) void k_pipe_snap(const unsigned *__restrict__ cur, int n, unsigned *__restrict__ snap,
                                                   const unsigned long long *__restrict__ slow_word, unsigned long long *slow_snap) {
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) snap[q] = cur[q];
    if (slow_snap && blockIdx.x == 0 && threadIdx.x == 0) *slow_snap = *slow_word;
}
// chunk k's segments of bin b (k_merge_owned's kSeg variant): for each of the bin's 2^sub_bits (sub-)slabs, the records
// between the previous chunk's cursor and this chunk's -- SO the first one's address, SP the bin's records in earlier
// segments, T[b] the bin's records of this chunk (scan input; T[RP_BINS] = 0).  A cursor past the slab (overflow: the
// host re-partitions) is clamped, so no segment reads past its slab.
__global__ __launch_bounds__(256) void k_chunk_segments(const unsigned *__restrict__ prev, const unsigned *__restrict__ cur,
                                                        const EventRec *slabs, int64_t slab_cap, unsigned sub_bits,
                                                        unsigned long long *__restrict__ SO, unsigned *__restrict__ SP,
                                                        unsigned *__restrict__ T) {
    const int ns = 1 << sub_bits;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k <= RP_BINS; k += gridDim.x * blockDim.x) {
        if (k == RP_BINS) { T[k] = 0; continue; }
        unsigned acc = 0;
        for (int s = 0; s < ns; s++) {
            const int64_t q = (int64_t)k * ns + s;
            const unsigned lo = prev ? min(prev[q], (unsigned)slab_cap) : 0u, hi = min(cur[q], (unsigned)slab_cap);
            SO[q] = (unsigned long long)(uintptr_t)(slabs + q * slab_cap + lo);
            SP[q] = acc;
            acc += hi > lo ? hi - lo : 0u;
        }
        T[k] = acc;
    }
}
// exclusive scan of m u32 counts after a base: out[i] = out[0] (as found) + sum(c[0, i)) -- chunk k's row offsets
// continue where chunk k - 1's ended (its scan's last word is this one's out[0]); one workgroup
__global__ __launch_bounds__(1024) void k_seg_scan(const unsigned *__restrict__ c, int64_t m, unsigned long long *out) {
    __shared__ unsigned long long base;
    if (threadIdx.x == 0) base = out[0];
    __syncthreads();
    unsigned long long carry = base;
    for (int64_t t0 = 0; t0 < m; t0 += 4096) {
        const int64_t b = t0 + (int64_t)threadIdx.x * 4;
        unsigned v[4];
        unsigned long long sum = 0;
        for (int q = 0; q < 4; q++) { v[q] = b + q < m ? c[b + q] : 0u; sum += v[q]; }
        unsigned long long total;
        unsigned long long run = carry + block1024_exclusive(sum, &total);
        for (int q = 0; q < 4; q++)
            if (b + q < m) { out[b + q] = run; run += v[q]; }
        carry += total;
        __syncthreads();
    }
}
// the fallback of a pipelined batch whose slab overflowed in chunk k (host_pipe.h): the rest of the batch partitioned
// by ev_partition (rp_O, digit-major over ntiles) -- its rows moved to start at base = out[0] (ev_partition's offsets
// start at 0), and the bins' starts gathered into the chunk's flat segment offsets out[0, RP_BINS] (ntiles 1)
__global__ __launch_bounds__(256) void k_seg_rebase(unsigned long long *__restrict__ rpO, int64_t m, int64_t ntiles,
                                                    unsigned long long *out) {
    const unsigned long long base = out[0];   // (read before any write: every thread writes out[b] = base + ..., out[0] = base)
    __syncthreads();
    for (int64_t q = threadIdx.x; q < m; q += blockDim.x) rpO[q] += base;
    __syncthreads();
    for (int b = threadIdx.x; b <= RP_BINS; b += blockDim.x) out[b] = rpO[(int64_t)b * ntiles];
}
// the chunks' counts as one u32 array per sender (scan input: [s][0, bins])
__global__ __launch_bounds__(256) void k_stage_counts(const uint8_t *__restrict__ recv, const int64_t *__restrict__ chunk_off,
                                                      int nseg, unsigned bins, unsigned *__restrict__ C) {
    const int64_t m = (int64_t)nseg * (bins + 1);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
        const int s = (int)(q / (bins + 1));
        const unsigned j = (unsigned)(q % (bins + 1));
        C[q] = j < bins ? ((const unsigned *)(recv + chunk_off[s] + sizeof(ChunkHdr)))[j] : 0u;
    }
}
// sender: every chunk's header, and its counts and census zeroed (one workgroup per destination)
__global__ __launch_bounds__(256) void k_stage_chunk_init(const ChunkHdr *__restrict__ hdr, const int64_t *__restrict__ chunk_start,
                                                          uint8_t *__restrict__ out) {
    const int o = blockIdx.x;
    uint8_t *chunk = out + chunk_start[o];
    const ChunkHdr h = hdr[o];
    if (threadIdx.x == 0) *(ChunkHdr *)chunk = h;
    unsigned *z = (unsigned *)(chunk + sizeof(ChunkHdr));
    const int64_t nz = (h.recs_off - (int64_t)sizeof(ChunkHdr)) / 4;
    for (int64_t q = threadIdx.x; q < nz; q += blockDim.x) z[q] = 0u;
}
// the region-field bin starts at the destinations' range starts: out[o] = S[shard_lo(o) * stride], o = 0..nranks
__global__ void k_shard_starts(const unsigned long long *__restrict__ S, int64_t stride, int nranks, unsigned long long *out) {
    for (int o = threadIdx.x; o <= nranks; o += blockDim.x) out[o] = S[(int64_t)shard_lo(o, nranks) * stride];
}
// owner: the senders' headers gathered (one 64-B header per chunk) and their census summed (per global window slot)
__global__ __launch_bounds__(256) void k_stage_headers(const uint8_t *__restrict__ recv, const int64_t *__restrict__ chunk_off,
                                                       const int64_t *__restrict__ chunk_bytes, int nseg, ChunkHdr *__restrict__ hdr,
                                                       int64_t census_off, unsigned long long *__restrict__ census) {
    for (int s = threadIdx.x; s < nseg; s += blockDim.x) {
        if (chunk_bytes[s] >= (int64_t)sizeof(ChunkHdr)) hdr[s] = *(const ChunkHdr *)(recv + chunk_off[s]);
        else hdr[s] = ChunkHdr{};
    }
    if (census_off <= 0) return;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < CENSUS_WORDS; q += gridDim.x * blockDim.x) {
        unsigned long long a = 0;
        for (int s = 0; s < nseg; s++)
            if (chunk_bytes[s] >= census_off + CENSUS_WORDS * 4) a += ((const unsigned *)(recv + chunk_off[s] + census_off))[q];
        census[q] = a;
    }
}
