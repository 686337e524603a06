// State-table kernels: census, growth dump, the region-owned merge into the update-mode state (heatmap_stream.py:111-133,243) and the row densification.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

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
// (clear_touched: a checkpoint export -- the touched word means nothing outside this context)
// Each workgroup iteration reads DUMP_PER x 256 consecutive slots (coalesced: slot k * 256 + tid) and appends its live
// keys with ONE atomic on the shared counter: a wave-aggregated append still made one same-address atomic per wave --
// 1.5 M of them over three 2^25-slot windows serialised at the L2 (12.7 ms for a 1e7-key delta, profiles/r6/r6w2);
// the record order in `out` is irrelevant to every caller (growth re-partitions, checkpoints are key sets).
constexpr int DUMP_PER = 8;
__global__ __launch_bounds__(256) void k_dump_gen(GenDesc g, GrowRec *__restrict__ out, unsigned long long *n_out,
                                                  unsigned only_seq = 0, bool clear_touched = false) {
    __shared__ unsigned wave_n[4];
    __shared__ unsigned long long blk_base;
    const int64_t cap = (int64_t)((g.rmask + 1) << g.rbits);
    const int64_t tile = 256 * DUMP_PER;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const unsigned long long below = (UINT64_C(1) << lane) - 1;
    for (int64_t base = (int64_t)blockIdx.x * tile; base < cap; base += (int64_t)gridDim.x * tile) {
        bool live[DUMP_PER];
        unsigned long long m[DUMP_PER];
        unsigned wtot = 0;
#pragma unroll
        for (int k = 0; k < DUMP_PER; k++) {
            const int64_t i = base + k * 256 + threadIdx.x;
            live[k] = false;
            if (i < cap) {
                const unsigned long long we = g.tab[i].wenc;
                live[k] = we == g.wenc && (only_seq == 0 || (unsigned)(g.tab[i].touched >> 32) == only_seq);
            }
            m[k] = __ballot(live[k]);
            wtot += __popcll(m[k]);
        }
        // the wave's k-th records go after its records of earlier k, in lane order
        if (lane == 0) wave_n[wave] = wtot;
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned tot = wave_n[0] + wave_n[1] + wave_n[2] + wave_n[3];
            blk_base = tot ? atomicAdd(n_out, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        unsigned long long pos = blk_base;
        for (int w = 0; w < wave; w++) pos += wave_n[w];
#pragma unroll
        for (int k = 0; k < DUMP_PER; k++) {
            if (live[k]) {
                const TileSlot sl = g.tab[base + k * 256 + threadIdx.x];
                GrowRec p;
                p.cell = sl.cell;
                p.wstart = wdec(sl.wenc);
                p.count = sl.count;
                p.nspeed = sl.nspeed;
                p.sspeed = sl.sspeed;
                p.slat = sl.slat;
                p.slon = sl.slon;
                p.touched = clear_touched ? 0ull : sl.touched;
                out[pos + __popcll(m[k] & below)] = p;
            }
            pos += __popcll(m[k]);
        }
        __syncthreads();   // (wave_n / blk_base reused by the next iteration)
    }
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
// in the bin; the slot's `touched` word keeps (batch seq, b0 + k)), and rewritten in place when a later chunk -- of
// this launch, or a later merge of the same batch -- updates the key again; k_fill_gaps closes the gaps left by keys
// that had several partials.
// rehash != 0: growth (k_dump_gen records, unique keys, into the window's new table): created slots keep the
// record's touched word, no rows are written.
// =====================================================================================================
constexpr int MO_THREADS = 512;      // partials per chunk (one per lane)
// the resident-only merge's wave-cooperative probe (needs the early-lines scratch)
// claim-set entries per record of a chunk (the resident-only merge: 2x as many 32-bit entries; 2 + the early old-line
// scratch fit the same LDS as 4 without it)
constexpr int MO_CLAIM = 2 * MO_THREADS;   // claim-set entries (load <= 1/2)
// LDS for resident region tags per workgroup: dynamic, sized per launch to the regions a bin can receive (the sum
// over the batch's windows of slots per region, 1 B each) up to MO_TAG_MAX -- 24 KB on the bench (3 windows x 8 K
// slots: two workgroups per CU), 32 KB for a res-7 window of 2^28 slots, which would otherwise probe through HBM
constexpr int MO_TAG_MAX = 90112;
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
    uint4 xline[MO_THREADS / 64][64];     // per wave: one round of the cooperative old-line loads (16 lines)
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
__device__ __forceinline__ MRec mrec_of_wi(const EventRec &p, const WInfo &wi, uint64_t cell_hi) {
    const uint64_t cell = (p.key & CELL_LO) | cell_hi;
    const bool sv = __builtin_bit_cast(uint64_t, p.speed) != SPEED_NULL_BITS;
    return MRec{cell, wi.wenc, mix64(cell ^ wi.inner), 1ull, sv ? 1ull : 0ull, sv ? p.speed : 0.0, p.lat, p.lon, 0ull};
}
__device__ __forceinline__ MRec mrec_of(const EventRec &p, const WInfo *winfo, uint64_t cell_hi) {
    const WInfo &wi = winfo[ekey_widx(p.key)];   // (an LDS copy measured no faster here: the chunk loop hides it)
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
    o.cell[t] = cell;
    o.ws[t] = wdec(we);
    o.cnt[t] = (int64_t)count;
    o.sp[t] = asp;
    o.spnull[t] = null_sp;
    o.lon[t] = alon;
    o.lat[t] = alat;
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
// kSeg (the multi-GPU owner): bin b's records are nseg segments, one per sender -- segment s at address SO[b * nseg + s]
// (the receive buffer, or the owner's own slab), after SP[b * nseg + s] records of the bin (k_stage_segments)
constexpr int MO_SEG_MAX = 64;
// Debug build (make libmobheat_dbg.so: MOBHEAT_BOUNDS_CHECK=1): every segment read of the kSeg variant must lie in one
// of the two ranges the host declared for the launch (merge_sorted: the receive buffer, the owner's slabs) -- else the
// kernel prints the bin, segment and address and traps, so that a fault names its access
#ifndef MOBHEAT_BOUNDS_CHECK
#define MOBHEAT_BOUNDS_CHECK 0
#endif
struct SegBounds {
    unsigned long long lo[2], hi[2];
};
#if MOBHEAT_BOUNDS_CHECK
__device__ SegBounds g_seg_bounds;
#endif
template <typename Rec, bool kResident = false, bool kCoop = false, bool kSeg = false>
__global__ __launch_bounds__(MO_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_merge_owned(const Rec *__restrict__ parts, int64_t slab,
                                                            const unsigned long long *__restrict__ SO, const unsigned *__restrict__ SP, int nseg,
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
    __shared__ unsigned long long seg_base[kSeg ? MO_SEG_MAX : 1];
    __shared__ unsigned seg_pre[kSeg ? MO_SEG_MAX + 1 : 1];
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
                    const unsigned sb = g.sb, smask = (1u << sb) - 1;
                    if (((unsigned)bin & smask) != (window_salt(g.wenc) & smask)) continue;
                    const unsigned reg = ((unsigned)bin >> sb) - g.rbase;   // (a shard's table: its range only)
                    if (reg >= (1u << g.rbits)) continue;
                    const unsigned slots = (unsigned)g.rmask + 1;
                    if (nr == MO_RES_MAX || off + slots > tag_bytes) continue;
                    const unsigned long long first = (unsigned long long)reg << g.rshift;
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
        if constexpr (kSeg) {
            for (int q = t; q < nseg; q += MO_THREADS) {
                seg_base[q] = SO[(int64_t)bin * nseg + q];
                seg_pre[q] = SP[(int64_t)bin * nseg + q];
            }
            if (t == 0) seg_pre[nseg] = (unsigned)(b1 - b0);
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
                unsigned s = (unsigned)inreg_slot(hk, rmask);
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
                s = (unsigned)inreg_slot(hk, rmask);
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
        // the new state line of a claimed slot (old values read here: the slot's last store is visible) and its
        // update-mode row index
        // the slot's current line (all loads of a lane issued together; created slots read nothing)
        auto old_line = [&](TileSlot *gslot, bool created, const MLine &pre, bool preloaded) __attribute__((always_inline)) -> MLine {
            MLine o{};
            if (preloaded) o = pre;
            created = created || preloaded;   // (the probe loaded it: nothing to load here)
            // whole lines per load instruction (the mirror of step 4's stores): in round k, lane L loads part L & 3 of
            // the line of lane 16k + L / 4 (16-B non-temporal loads: L2-served, like ld_l2) into the wave's LDS slice,
            // and lanes 16k..16k+15 take their lines from there.  Every lane of the wave runs it (shuffles).
            const bool need = gslot && !created;
            if (__ballot(need)) {
                // (its own scratch: the lines are loaded before the barrier, while other waves' joiners still read
                // this wave's staged keys in S.sc / S.sh)
                uint4 *xa = &S.xline[t >> 6][0], *xb = &S.xline[t >> 6][32];
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
        // (one LDS add per created key: a ballot per resident region measured 0.17 ms slower on the bench, r4j/)
        auto count_created = [&](bool created, int r) __attribute__((always_inline)) {
            if (created && r >= 0) atomicAdd(&S.res_new[r], 1u);
        };
        // software pipeline: the next chunk's record is loaded while this chunk is merged
        Rec nxt;
        // the bin's records: [b0, b1) of the partitioned array, or (slab != 0: k_ingest's fused binning) the first
        // b1 - b0 records of the bin's slab; either way row k of the bin goes to b0 + k
        const Rec *__restrict__ bp = slab ? parts + ((int64_t)bin * slab - b0) : parts;
        // kSeg: the record at bin index v = i - b0 is in the last segment starting at or before v (binary search)
        auto rec_at = [&](int64_t i) __attribute__((always_inline)) -> const Rec * {
            if constexpr (kSeg) {
                const unsigned v = (unsigned)(i - b0);
                int lo = 0, hi = nseg;   // seg_pre[lo] <= v < seg_pre[hi]
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (seg_pre[mid] <= v) lo = mid; else hi = mid;
                }
                const Rec *rp = (const Rec *)(uintptr_t)seg_base[lo] + (v - seg_pre[lo]);
#if MOBHEAT_BOUNDS_CHECK
                const unsigned long long a = (unsigned long long)(uintptr_t)rp, e = a + sizeof(Rec);
                const SegBounds &B = g_seg_bounds;
                if (!((a >= B.lo[0] && e <= B.hi[0]) || (a >= B.lo[1] && e <= B.hi[1]))) {
                    printf("k_merge_owned: bin %d segment %d record %u at 0x%llx outside [0x%llx, 0x%llx) and [0x%llx, 0x%llx)\n",
                           bin, lo, v, a, B.lo[0], B.hi[0], B.lo[1], B.hi[1]);
                    __builtin_trap();
                }
#endif
                return rp;
            } else {
                return bp + i;
            }
        };
        constexpr bool kEv = std::is_same<Rec, EventRec>::value;
        // EventRec: the next chunk's window parameters are loaded with the chunk's store drain, so that the record's
        // hash needs no dependent load at the chunk's start (state-read leg's merge -0.27 ms, bench leg unchanged:
        // profiles/r4/r4v7/)
        WInfo nwi{};
        if (b0 + t < b1) nxt = ld_stream(rec_at(b0 + t));
        if constexpr (kEv) { if (b0 + t < b1) nwi = winfo[ekey_widx(nxt.key)]; }
        for (int64_t c0 = b0; c0 < b1; c0 += MO_THREADS) {
            // 1. stage this chunk's records in LDS
            const int64_t i = c0 + t;
            const bool has = i < b1;
            MRec p{};
            if (has) {
                if constexpr (kEv) p = mrec_of_wi(nxt, nwi, cell_hi);
                else p = mrec_of(nxt, winfo, cell_hi);
            }
            if (i + MO_THREADS < b1) nxt = ld_stream(rec_at(i + MO_THREADS));
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
            if constexpr (kResident && kCoop) probe_coop(p, has, gslot, created, r, ci, pre, preloaded);
            else if (has) probe(p, gslot, created, r, ci);
            count_created(created, r);
            // 3a. the claimed existing lines, loaded before the barrier (their slots' last stores were drained by an
            // earlier chunk's barrier, and no store of this chunk precedes step 4): the round trip overlaps the wait
            const MLine o = old_line(gslot, created, pre, preloaded);
            lds_barrier();
            // 3. the claimers' new lines
            MLine v{};
            const bool retouch = !rehash && gslot && !created && (unsigned)(o.touched >> 32) == seq;
            const bool first = !rehash && gslot && !retouch;
            // (the row index is absolute -- the bin's first row b0 + its touch order -- so that a later merge of the same
            // batch, whose segment of the bin starts elsewhere, rewrites the row in place: a pipelined batch's chunks)
            unsigned krow = (unsigned)b0 + touch_rows(first);
            if (!first) krow = (unsigned)o.touched;
            if (gslot) v = line_of(p, o, first, krow);
            // 4. this chunk's stores: the state line (whole) and the key's row
            {
                const uint64_t b0s = __builtin_bit_cast(uint64_t, v.sspeed), b1s = __builtin_bit_cast(uint64_t, v.slat);
                const uint64_t b2s = __builtin_bit_cast(uint64_t, v.slon);
                const uint4 q0 = make_uint4((unsigned)p.cell, (unsigned)(p.cell >> 32), (unsigned)p.we, (unsigned)(p.we >> 32));
                const uint4 q1 = make_uint4((unsigned)v.count, (unsigned)(v.count >> 32), (unsigned)v.nspeed, (unsigned)(v.nspeed >> 32));
                const uint4 q2 = make_uint4((unsigned)b0s, (unsigned)(b0s >> 32), (unsigned)b1s, (unsigned)(b1s >> 32));
                const uint4 q3 = make_uint4((unsigned)b2s, (unsigned)(b2s >> 32), (unsigned)v.touched, (unsigned)(v.touched >> 32));
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
            }
            if (gslot) {
                if (created) created_cnt++;
                if (!rehash) put_row(rows, (int64_t)krow, p.cell, p.we, v.count, v.nspeed, v.sspeed, v.slat, v.slon);
            }
            // created keys of non-resident windows count for their window here (resident ones: res_new); rehash:
            // the host already carries the moved keys
            if constexpr (!kResident) {
                const bool count_here = created && !rehash && r < 0;
                if (__ballot(count_here) && !wave_count_windows(count_here, p.we, 1ull, WL, sink)) overflow = true;
            }
            if constexpr (kEv) { if (i + MO_THREADS < b1) nwi = winfo[ekey_widx(nxt.key)]; }
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
// up to ZR_MAX ranges in one launch (blockIdx.y = range): a batch's released tables
constexpr int ZR_MAX = 8;
struct ZeroRanges {
    uint4 *p[ZR_MAX];
    int64_t n16[ZR_MAX];
};
__global__ __launch_bounds__(256) void k_zero16_ranges(ZeroRanges r) {
    uint4 *__restrict__ p = r.p[blockIdx.y];
    const int64_t n16 = r.n16[blockIdx.y], stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) p[i] = make_uint4(0u, 0u, 0u, 0u);
}

// the start of a batch in one launch (was six memsets and a copy): the batch statistics (max ts / min window start
// at their identities), the fast-path exception and dedup give-up words, the window registry and its census
__global__ __launch_bounds__(256) void k_batch_reset(unsigned long long *__restrict__ st, unsigned long long *__restrict__ slow_word,
                                                     unsigned long long *__restrict__ giveup_word, unsigned long long *__restrict__ wreg2,
                                                     int n_wreg2, unsigned *__restrict__ bin_cur, int n_bin) {
    static_assert(sizeof(DevStats) % 8 == 0 && offsetof(DevStats, min_wstart) == offsetof(DevStats, max_ts_ms) + 8, "DevStats");
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_wreg2) wreg2[i] = 0;
    if (i < n_bin) bin_cur[i] = 0;
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
