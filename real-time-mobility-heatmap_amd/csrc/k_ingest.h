// The per-event pass: filter + latLngToCell + window + late test + dedup max + event keys (heatmap_stream.py:65-75,96-115,200-203); the standalone UDF and cellToBoundary kernels.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// =====================================================================================================
// K1: latLngToCell.  The per-event kernels run latLngToCellFast (h3_device.h: direct gnomonic projection,
// ~60 VGPRs) and append the rare events whose decision margins are below the error bound to an exception
// list; a second kernel runs upstream's exact sequence (latLngToCellDeg, ~170 VGPRs) on that list only, so
// the register footprint of the exact path never limits the occupancy of the streaming kernel.
// =====================================================================================================
// waves per SIMD for k_ingest: 6 (<= 80 VGPRs, no spills; 7 or 8 spill and only lengthen the waits, profiles/r3/r3ab15/,
// profiles/r4/r4wv/)
#define HM_SNAP_ATTR __attribute__((amdgpu_waves_per_eu(6)))
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
// K1: ingest. One pass over the events: the filter (heatmap_stream.py:96-104), latLngToCell (the UDF,
// :65-75), the tumbling window and late test (:107,115), the batch's window registry, the per-vkey max ts of the
// dedup (:200-203), and one event key per row (kernels.h ekey: cell + window slot; 0 = not aggregated) -- the
// input of both aggregation paths (direct: partition + merge; table: k_agg + k_bin_reduce).  The fp64 cell
// computation dominates; the dedup's table atomics overlap with it.
// =====================================================================================================
// Dense vkeys (the boundary's are dictionary codes, pcode * n_vehicles + vcode: stream.batch_columns, k_json_vkey):
// a vkey below dense_cap keeps its max ts in dense[vkey] -- the ts with its sign bit flipped, so that unsigned order is
// signed order and 0 (memset) is "no row yet" -- one 8-B load and, when the ts is a new max, one atomicMax; no probing,
// no claims.  Larger vkeys take the hash table below.  (The hash table's probe path -- a key not in its home slot, a
// quarter of them at load 1/2, and one such lane makes its whole wave probe with a full wait per step -- cost the bench
// ~0.9 ms of k_ingest's 6.7: tools/variants/ingest_ddload.patch, profiles/r5/r5ab6/.)
// The fused per-vkey max gives up on a key after DEDUP_FUSED_PROBES probes (its table was sized from the previous
// batch and is too small); the first give-up is published in *dgiveup, a word on a cache line of its own, polled
// every 16 rounds (polling a DevStats word every round, a line other atomics hit, made the ingest 4x slower), and
// later rounds skip the fused dedup, which phase_dedup then reruns over the whole batch on a full-size table.
constexpr unsigned long long DEDUP_FUSED_PROBES = 32;
constexpr int IG_THREADS = 256;

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

// kBin: the direct path's (window, region) binning fused in (hm_process_batch, large batches): every aggregated row's
// 32-B EventRec goes straight to its bin's slab -- bin = the key hash's region field (every window of such a batch
// has 2^REGION_BITS regions, so region = bin, kernels.h) at slab b * slab_cap + a returned atomic on the bin's
// cursor -- instead of a later histogram + scatter pass over the keys and columns.  A bin past slab_cap counts in
// DevStats.bin_overflow and the host partitions the batch from its keys instead.  sub_bits (hm_process_batch: SUB_BITS;
// the stage API: 0): each bin split into the key's sub-regions (kernels.h inreg_slot), slab (bin << sub_bits) | sub.
// (one kernel for every resolution: per-resolution specialisations of this kernel, measured no faster once the digits
// came from the step tables, were miscompiled at res 3 by this compiler -- wrong cells, caught by
// test_ingest_cells_every_resolution, profiles/r4/r4w/)
// k_sample_heavy's row stride for a batch of n rows: the largest power of two <= n / HS_SAMPLE (so that k_ingest<true>
// can write the sampled rows' keys with a mask test)
constexpr int HS_SAMPLE = 4096, HS_THREADS = 1024, HS_SLOTS = 2 * HS_SAMPLE;
__host__ __device__ inline int64_t hs_stride(int64_t n) {
    int64_t s = 1;
    while (s * 2 <= n / HS_SAMPLE) s *= 2;
    return s;
}
// kBin writes an event key only where something reads it before the merge: exception rows (k_ingest_exact completes
// them) and k_sample_heavy's rows (i & smask == 0) -- the binned records carry their own keys.  A batch that then
// needs every row's key (the key sample asks for table mode, or a slab overflowed and the batch re-partitions) runs
// kKeys: the same rows again, writing only the keys of the non-exception rows (no flags, dedup, census, statistics,
// bins), so that the keys read as one k_ingest<false> would have written them (keys_complete).
template <bool kBin, bool kKeys = false>
__global__ __launch_bounds__(IG_THREADS) HM_SNAP_ATTR void k_ingest(
    const double *__restrict__ lat, const double *__restrict__ lon, const int64_t *__restrict__ ts,
    const uint8_t *__restrict__ row_valid, const uint64_t *__restrict__ vkey, int64_t i_begin, int64_t n, int res_arg, FloorDiv wdiv,
    int64_t late_end_us, uint8_t *__restrict__ flags_out, uint64_t *__restrict__ keys_out, DedupSlot *dtab,
    unsigned long long dmask, unsigned int *dused, unsigned long long *n_dused, unsigned int *__restrict__ slow,
    unsigned long long *n_slow, unsigned long long *dgiveup, unsigned long long *wreg, unsigned long long *wcount,
    DevStats *st, const double *__restrict__ speed, const uint8_t *__restrict__ speed_valid, unsigned *__restrict__ bin_cur,
    EventRec *__restrict__ slabs, unsigned slab_cap, unsigned long long *__restrict__ dense, unsigned long long dense_cap,
    unsigned sub_bits, int64_t smask) {
    static_assert(!(kBin && kKeys), "k_ingest: kKeys runs unbinned");
    const int res = res_arg;
    __shared__ WinCacheL WC;
    __shared__ double Fc[20][3], Fu[20][2][3];   // the fast path's per-face tables (res parity): LDS reads
    __shared__ unsigned dskip;                    // the fused dedup has given up (*dgiveup) -- skip it
    __shared__ long long tmax_l[IG_THREADS];      // per-thread max ts (an LDS max per row instead of 2 live registers)
    __shared__ long long vmax_l[IG_THREADS];      // per-thread max vkey + 1 of the deduplicated rows (the same way)
    for (int k = threadIdx.x; k < 60; k += IG_THREADS) (&Fc[0][0])[k] = (&c_tab.faceCenterPoint[0][0])[k];
    for (int k = threadIdx.x; k < 120; k += IG_THREADS) (&Fu[0][0][0])[k] = (&c_tab.fastU[res & 1][0][0][0])[k];
    // _faceIjkToH3's packed base-cell and digit tables in LDS (11.2 KB): from __constant__ memory they were lane-indexed vector loads
    // at the end of every cell, each with a full wait that also waited for the next round's prefetched columns
    __shared__ H3BaseTables BT;
    for (int k = threadIdx.x; k < 20 * 27; k += IG_THREADS) BT.fijkPacked[k] = c_tab.fijkPacked[k];
    for (int k = threadIdx.x; k < 122; k += IG_THREADS) BT.bcdPacked[k] = c_tab.bcdPacked[k];
    for (int k = threadIdx.x; k < AP7_QUAD; k += IG_THREADS) BT.ap7Quad[k] = c_tab.ap7Quad[k];
    for (int k = threadIdx.x; k < AP7_PAIR; k += IG_THREADS) BT.ap7Pair[k] = c_tab.ap7Pair[k];
    wc_init(WC);
    if (threadIdx.x == 0) dskip = 0;
    __syncthreads();
    const int64_t tile_us = wdiv.d;
    // per-thread counters in 32 bits (a thread sees at most n / gstride < 2^32 rows): fewer registers live across
    // the cell computation, whose peak spilled the prefetched columns
    unsigned nvalid = 0, nlate = 0, bad = 0, wover = 0, binover = 0;
    tmax_l[threadIdx.x] = INT64_MIN;
    vmax_l[threadIdx.x] = 0;
    bool dretry = false;
    int round = 0;
    const int64_t gstride = (int64_t)gridDim.x * IG_THREADS;
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
            nv = __builtin_nontemporal_load(&vkey[i0]);
            if (row_valid) nrv = __builtin_nontemporal_load(&row_valid[i0]);
        }
    }
    for (int64_t base = i_begin + (int64_t)blockIdx.x * IG_THREADS; base < n; base += gstride, round++) {
        const int64_t i = base + threadIdx.x;
        const bool in = i < n;
        const double la = nla, lo = nlo;
        // ts is not prefetched: it is loaded now and first used after the cell, whose computation hides the load
        // (prefetched, the next round's ts was the register the cell computation's peak spilled -- a spill that
        // waited for every prefetched load mid-round)
        const int64_t t = in ? __builtin_nontemporal_load(&ts[i]) : 0;
        (void)nt;
        // kBin: the row's speed the same way (first used after the cell); absent columns read one-element constants
        uint64_t spb = 0;
        uint8_t svb = 0;
        if constexpr (kBin) {
            typedef __attribute__((address_space(1))) const uint64_t gcu64;
            typedef __attribute__((address_space(1))) const uint8_t gcu8;
            const int64_t j = in ? i : n - 1;
            spb = __builtin_nontemporal_load((gcu64 *)(speed ? (const uint64_t *)&speed[j] : (const uint64_t *)&g_zero_double));
            svb = __builtin_nontemporal_load((gcu8 *)(speed_valid ? &speed_valid[j] : speed ? &g_one_byte : &g_zero_byte));
        }
        const unsigned long long v = nv;
        const bool rv = nrv != 0;
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
        // the cell of every row in range, before the ts- and validity-dependent tests (late, invalid or
        // out-of-range-ts rows waste their cell): nothing loaded this round is waited for before the cell
        const bool geo0 = in && la >= -90.0 && la <= 90.0 && lo >= -180.0 && lo <= 180.0;
        bool exc = false;
        uint64_t cell = EMPTY_CELL;
        if (geo0) exc = !latLngToCellFastP(la, lo, res, c_tab, Fc, Fu, cell, BT);
        const bool geo = geo0 && rv;
        const bool ok = geo && t > INT64_MIN + 2 * tile_us && t < INT64_MAX - 2 * tile_us;
        // dedup: the vkey's home slot is loaded now, its latency hidden behind the cell computation (a plain load:
        // a stale copy can only show the slot empty or its max lower, both of which the atomics below correct)
        const bool dd = !kKeys && ok && v != EMPTY_VKEY && !__hip_atomic_load(&dskip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const bool dv = v < dense_cap;   // (dense_cap < 2^64 - 1: EMPTY_VKEY is never dense)
        const unsigned long long dh0 = vkey_hash(v) & dmask;
        DedupSlot d0{EMPTY_VKEY, 0};
        unsigned long long dn = 0;
        if (dd) {
            if (dv) dn = dense[v];
            else d0 = dtab[dh0];
        }
        uint8_t fl = 0;
        int widx = -1, wslot = -1;
        int64_t ws = 0;
        if (ok) {
            const int64_t wq = floor_div(t, wdiv);   // tumbling window: floor(t / tile) (Spark TimeWindowing)
            ws = wq * tile_us;
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
        exc = exc && (fl & F_AGG) != 0;
        if constexpr (!kKeys) {
            const unsigned long long pos = wave_append(exc, n_slow);
            if (exc) slow[pos] = (unsigned int)i;
        }
        // dedup: per-vkey max ts over the valid rows (late rows included, as in the reference's batch frame)
        bool claimed = false;
        long long dh = -1;
        bad += ok && v == EMPTY_VKEY;
        bool cand = false;
        if (dd) atomicMax(&vmax_l[threadIdx.x], (long long)(v < (1ull << 62) ? v + 1 : (1ull << 62)));
        if (dd && dv) {
            const long long cur = (long long)(dn ^ DENSE_SIGN);   // (0: INT64_MIN, no row yet)
            cand = t >= cur;
            if (t > cur) atomicMax(&dense[v], (unsigned long long)t ^ DENSE_SIGN);
        } else if (dd) {
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
        const uint64_t key = agg ? ekey_make(exc ? 0 : cell, (unsigned)widx) : 0;
        if (in) {
            if constexpr (!kKeys) flags_out[i] = fl | (cand ? F_CAND : 0);
            if (kKeys ? !exc : !kBin || exc || (i & smask) == 0) keys_out[i] = key;
        }
        if constexpr (kBin) {
            // the row's EventRec into its bin (exceptions: k_ingest_exact, once their cell is known)
            if (agg && !exc) {
                // the window's hash constant from the window cache (computed by the first rows that find it unset:
                // every writer stores the same value)
                uint64_t inner = wslot >= 0 ? __hip_atomic_load(&WC.inner[wslot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
                if (inner == 0) {
                    inner = window_inner(ws);
                    if (wslot >= 0) __hip_atomic_store(&WC.inner[wslot], inner, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                const uint64_t h = mix64(cell ^ inner);
                const unsigned b = (region_field(h) << sub_bits) | (sub_field(h) & ((1u << sub_bits) - 1));
                const unsigned p = atomicAdd(&bin_cur[b], 1u);
                if (p < slab_cap) {
                    const uint64_t sp = svb == 0 ? SPEED_NULL_BITS
                                                 : __builtin_bit_cast(double, spb) != __builtin_bit_cast(double, spb) ? CANON_NAN_BITS : spb;
                    const uint64_t lab = __builtin_bit_cast(uint64_t, la), lob = __builtin_bit_cast(uint64_t, lo);
                    uint4 *d = (uint4 *)&slabs[(size_t)b * slab_cap + p];
                    st_g16(d, make_uint4((unsigned)key, (unsigned)(key >> 32), (unsigned)sp, (unsigned)(sp >> 32)));
                    st_g16(d + 1, make_uint4((unsigned)lab, (unsigned)(lab >> 32), (unsigned)lob, (unsigned)(lob >> 32)));
                } else {
                    binover++;
                }
            }
        }
        if constexpr (!kKeys) {
            const unsigned long long pos = wave_append(claimed, n_dused);
            if (claimed) dused[pos] = (unsigned int)dh;
            // census: aggregated rows per window (sizes the window tables of the direct path)
            wave_count_slots(agg && wslot >= 0, wslot, WC.cnt);
            if (agg && wslot < 0) atomicAdd(&wcount[widx], 1ull);
        }
        // poll the give-up flag now and then (its own cache line)
        if (threadIdx.x == 0 && (round & 15) == 15 && !dskip)
            __hip_atomic_store(&dskip, __hip_atomic_load(dgiveup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ? 1u : 0u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if constexpr (kKeys) return;   // (no census, no statistics: the batch's first pass counted them)
    __syncthreads();
    for (int q = threadIdx.x; q < WC_SLOTS; q += IG_THREADS)
        if (WC.cnt[q]) atomicAdd(&wcount[(WC.e[q] & 0xfff) - 1], (unsigned long long)WC.cnt[q]);
    const unsigned long long wvalid = wave_sum((unsigned long long)nvalid), wlate = wave_sum((unsigned long long)nlate);
    const unsigned long long wbad = wave_sum((unsigned long long)bad), wwover = wave_sum((unsigned long long)wover);
    const unsigned long long wbinover = kBin ? wave_sum((unsigned long long)binover) : 0ull;
    const long long tmax = wave_max(tmax_l[threadIdx.x]);
    const long long vmax = wave_max(vmax_l[threadIdx.x]);
    const unsigned long long rt = __ballot(dretry);
    if (lane_id() == 0) {
        if (wvalid) atomicAdd(&st->n_valid, wvalid);
        if (wlate) atomicAdd(&st->n_late, wlate);
        if (tmax != INT64_MIN) atomicMax(&st->max_ts_ms, (long long)(tmax / 1000));   // trunc(max) = max(trunc)
        if (vmax > 0) atomicMax(&st->vkey_max1, (unsigned long long)vmax);
        if (wbad) atomicAdd(&st->bad_vkey, wbad);
        if (wwover) atomicAdd(&st->win_overflow, wwover);
        if (rt) atomicAdd(&st->dedup_retry, 1ull);
        if (wbinover) atomicAdd(&st->bin_overflow, wbinover);
    }
}


// exceptions of k_ingest's fast path: upstream's exact sequence; the cell bits go into the row's key (k_ingest
// wrote its window slot); with slabs (k_ingest<true>) the row's EventRec into its bin as k_ingest does
// (n_slow_begin: the first exception to complete -- a pipelined batch completes each chunk's own, k_pipe_snap; null: 0)
__global__ __launch_bounds__(256) void k_ingest_exact(const double *__restrict__ lat, const double *__restrict__ lon, int res,
                                                      const unsigned int *__restrict__ slow, const unsigned long long *n_slow,
                                                      uint64_t *__restrict__ keys, const double *__restrict__ speed,
                                                      const uint8_t *__restrict__ speed_valid, const unsigned long long *wreg,
                                                      unsigned *__restrict__ bin_cur, EventRec *__restrict__ slabs, unsigned slab_cap,
                                                      DevStats *st, unsigned sub_bits,
                                                      const unsigned long long *n_slow_begin = nullptr) {
    const int64_t m = (int64_t)*n_slow, q0 = n_slow_begin ? (int64_t)*n_slow_begin : 0;
    for (int64_t q = q0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += (int64_t)gridDim.x * blockDim.x) {
        const unsigned i = slow[q];
        const uint64_t cell = latLngToCellDeg(lat[i], lon[i], res, c_tab);
        const uint64_t key = keys[i] | (cell & CELL_LO);
        keys[i] = key;
        if (slabs) {
            const uint64_t h = mix64(cell ^ window_inner(wdec(wreg[ekey_widx(key)])));
            const unsigned b = (region_field(h) << sub_bits) | (sub_field(h) & ((1u << sub_bits) - 1));
            const unsigned p = atomicAdd(&bin_cur[b], 1u);
            if (p >= slab_cap) { atomicAdd(&st->bin_overflow, 1ull); continue; }
            const bool sv = speed && (!speed_valid || speed_valid[i]);
            const double sp = sv ? speed[i] : 0.0;
            EventRec r;
            r.key = key;
            r.speed = __builtin_bit_cast(double, !sv ? SPEED_NULL_BITS : sp != sp ? CANON_NAN_BITS : __builtin_bit_cast(uint64_t, sp));
            r.lat = lat[i];
            r.lon = lon[i];
            slabs[(size_t)b * slab_cap + p] = r;
        }
    }
}

// Heavy hitters in the batch's event keys, for the choice of the aggregation path when the last batch says nothing
// (the first batch, or a sudden change of the data): HS_SAMPLE keys spread evenly over the batch, the largest
// multiplicity among them -> DevStats.sample_max_run.  A key holding a few % of the rows would put that share of the
// batch through one merge workgroup (one bin) on the direct path; table mode aggregates it in LDS first.
// (the multiplicities counted in an LDS hash table at load <= 1/2: was a bitonic sort of the sample, 78 barriers)
// stride: the rows k_ingest<true> wrote keys for (multiples of it; hs_stride of the whole batch), n: the rows sampled
// ([0, n): the batch, or a pipelined batch's first chunk -- fewer than HS_SAMPLE multiples of the stride then, and the
// largest multiplicity is scaled to HS_SAMPLE samples)
__global__ __launch_bounds__(HS_THREADS) void k_sample_heavy(const uint64_t *__restrict__ keys, int64_t n, int64_t stride,
                                                             DevStats *st) {
    __shared__ unsigned long long k[HS_SLOTS];
    __shared__ unsigned c[HS_SLOTS];
    __shared__ unsigned best;
    const int t = threadIdx.x;
    const int64_t ns = n / stride < HS_SAMPLE ? (n / stride > 0 ? n / stride : 1) : HS_SAMPLE;
    constexpr int PER = HS_SAMPLE / HS_THREADS;
    uint64_t v[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {   // every load in flight before the table is cleared
        // (spread over the rows -- sample q at q n / ns, rounded down to the stride k_ingest<true> writes keys at (ns <=
        // n / stride: distinct rows): the stride alone covered only the first HS_SAMPLE x stride rows, as little as half
        // the batch, and a hot key late in a time-ordered batch went unseen -- ADVICE r5)
        const int64_t q = t + u * HS_THREADS;
        const int64_t i = q < ns ? (q * n / ns) & ~(stride - 1) : n;
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
    if (t == 0) st->sample_max_run = ns < HS_SAMPLE ? ((unsigned long long)best * HS_SAMPLE + ns - 1) / ns : best;
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
