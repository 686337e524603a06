// Host side: the pipelined micro-batch (round 6).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
//
// A binned direct-path batch (k_ingest<true>: every aggregated row's 32-B record into its (window, region) bin slab)
// used to run as two kernels in series: the ingest over all rows, then the merge of every bin into the state.  The two
// bind on different units -- the ingest on its scattered record stores and bin-cursor atomics, the merge on the latency
// of its chain of LDS steps -- so here the batch's rows are split into K chunks: chunk k's k_ingest<true> runs on the
// main stream while chunk k - 1's records merge on merge_stream.  A chunk's records are the part of each bin slab
// written since the previous chunk (the cursors are snapshotted after every chunk, k_pipe_snap), so chunks share the
// slabs and one k_merge_owned<kSeg> merges each chunk's segments of its bins.  Rows are absolute (the slot's touched
// word keeps the key's row), so a key that several chunks touch rewrites its one row in place, and the chunks' rows are
// consecutive segment groups that k_fill_gaps densifies as one.  Spark's update mode sees the batch as before: each key
// touched by the batch emits one row with its cumulative values after the batch (heatmap_stream.py:112-133,243).
#pragma once

constexpr int PIPE_CHUNKS = 4;                          // chunks of an automatically pipelined batch
constexpr int64_t PIPE_MIN_ROWS = int64_t(1) << 24;     // rows from which a binned batch is pipelined (auto)

// the chunks this batch is pipelined in (0: not pipelined)
static int pipe_chunks_for(const hm_ctx *ctx, const Inputs &I) {
    if (ctx->pipe_mode == 0 || I.n <= 0) return 0;
    if (!choose_binned(ctx, I.n)) return 0;
    if (ctx->pipe_mode > 0) return ctx->pipe_mode >= 2 && I.n >= ctx->pipe_mode ? ctx->pipe_mode : 0;
    return I.n >= PIPE_MIN_ROWS ? PIPE_CHUNKS : 0;
}

// MOBHEAT_PIPE_DEBUG=1: the device drained and its error checked after every step of a pipelined batch, the step named
// in the error (a fault then names the step that launched it)
static bool g_pipe_debug = getenv("MOBHEAT_PIPE_DEBUG") && getenv("MOBHEAT_PIPE_DEBUG")[0] == '1';
#define PIPE_STEP(ctx, what, k)                                                                                   \
    do {                                                                                                          \
        if (g_pipe_debug) {                                                                                       \
            const hipError_t e_ = hipDeviceSynchronize();                                                         \
            const hipError_t l_ = hipGetLastError();                                                              \
            fprintf(stderr, "[mobheat pipe] %s chunk %d: %s\n", what, (int)(k), hipGetErrorString(e_ ? e_ : l_)); \
            if (e_ || l_) return set_err(ctx, HM_E_HIP, "pipelined batch: %s of chunk %d: %s", what, (int)(k),  \
                                         hipGetErrorString(e_ ? e_ : l_));                                        \
        }                                                                                                         \
    } while (0)

// host wait for an event, timed into host_ms like ctx_sync
static hipError_t ev_sync(hm_ctx *ctx, hipEvent_t e, int site) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t r = hipEventSynchronize(e);
    const double ms = ms_since(t0);
    ctx->host_ms[1] += ms;
    if (ms > ctx->host_ms[3]) { ctx->host_ms[3] = ms; ctx->host_ms[4] = site; }
    return r;
}

// would gens_prepare change the window tables for this census (a new window, a window not yet merging this batch, a
// table past load 1/2 or of the wrong geometry)?
static bool gens_need_change(const hm_ctx *ctx, const std::vector<WinCount> &census) {
    unsigned lo = 0, hi = 0;
    range_of(ctx, lo, hi);
    for (const WinCount &w : census) {
        auto it = std::find_if(ctx->gens.begin(), ctx->gens.end(), [&](const hm_ctx::Gen &g) { return g.wenc == w.wenc; });
        if (it == ctx->gens.end() || it->batch_parts == 0) return true;
        if (std::min(it->keys + (int64_t)w.count, h3_cells_at(ctx->cfg.h3_res)) * 2 > usable_slots(ctx, *it)) return true;
        if (it->sb != 0 || it->rbase != lo || (int64_t(1) << it->rbits) < (int64_t)(hi - lo)) return true;
    }
    return false;
}

// Runs the main-stream calls of fn with ctx->stream = the merge stream (every launcher of the merge path enqueues on
// ctx->stream), then restores it.
template <typename F>
static int on_merge_stream(hm_ctx *ctx, F &&fn) {
    hipStream_t main = ctx->stream;
    ctx->stream = ctx->merge_stream;
    const int rc = fn();
    ctx->stream = main;
    return rc;
}

// the device's key counts per window (the merges so far) into the host's tables, before a window map upload
// (gens_upload writes the host's counts) -- the caller's stream must have drained the merges
static int gens_sync_counts(hm_ctx *ctx) {
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_gmap, ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    for (auto &g : ctx->gens) {
        unsigned h = (unsigned)(mix64(g.wenc) & (GMAP_SLOTS - 1));
        for (int p = 0; p < GMAP_SLOTS && ctx->h_gmap[h].wenc; p++, h = (h + 1) & (GMAP_SLOTS - 1))
            if (ctx->h_gmap[h].wenc == g.wenc) { g.keys = (int64_t)ctx->h_gmap[h].count; break; }
    }
    return HM_OK;
}

// after the batch's last readback: the bins' fill against their mean (the next batch's slab room, as phase_local) and
// the largest vkey (the next batch's dense dedup table)
static void pipe_batch_stats(hm_ctx *ctx, int nbins) {
    unsigned long long tot = 0, mx = 0;
    for (int b = 0; b < nbins; b++) { tot += ctx->h_bincur[b]; mx = std::max<unsigned long long>(mx, ctx->h_bincur[b]); }
    if (tot) ctx->bin_skew = std::max(1.0, (double)mx * nbins / (double)tot);
    if (ctx->h_st->vkey_max1) ctx->vkey_bound = (int64_t)ctx->h_st->vkey_max1;
}

// A slab overflowed in chunk k (its fill went past the slab room the last batch's skew gave it): chunks < k are merged;
// the rest of the batch, rows [n k / K, n), is partitioned from its event keys (as phase_local's overflowing batch is)
// and merged as one more segment group, its rows after chunk k - 1's.  Every chunk is ingested (the caller waited).
static int pipe_overflow_rest(hm_ctx *ctx, const Inputs &I, int K, int k) {
    int rc;
    const int64_t n = I.n, a = n * k / K;
    unsigned long long *plO = (unsigned long long *)ctx->pl_O.p;
    unsigned *plN = (unsigned *)ctx->pl_cnt.p;
    HIPCHK(ctx, hipStreamSynchronize(ctx->merge_stream));
    // the event keys of rows [a, n) (k_ingest<true> wrote only the exception and sampled rows' keys)
    const int blocks = (int)std::min<int64_t>((n - a + IG_THREADS - 1) / IG_THREADS, ctx->ingest_grid);
    hipLaunchKernelGGL((k_ingest<false, true>), dim3(std::max(blocks, 1)), dim3(IG_THREADS), 0, ctx->stream, I.lat, I.lon, I.ts,
                       I.rv, I.vk, a, n, ctx->cfg.h3_res, make_floor_div(ctx->cfg.tile_us), ctx->keys_late_us,
                       (uint8_t *)ctx->flags.p, (uint64_t *)ctx->keys.p, ctx->dfused.tab, ctx->dfused.cap - 1,
                       (unsigned int *)ctx->dfused.used.p, ctx->d_scratch + ctx->dfused.used_word, (unsigned int *)ctx->slow.p,
                       ctx->d_scratch + SLOW_WORD, ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg, ctx->d_wcount, ctx->d_st, I.sp,
                       I.sv, (unsigned *)ctx->bin_cur.p, (EventRec *)nullptr, 0u, (unsigned long long *)ctx->dense.p, 0ull, 0u,
                       (int64_t)0);
    HIPCHK(ctx, hipGetLastError());
    PIPE_STEP(ctx, "overflow: keys", k);
    ctx->keys_partial = false;
    // the tables from the batch's exact census
    if (k == 0) {
        int r;
        if ((r = merge_begin(ctx, n, true))) return r;
        HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    } else if ((rc = gens_sync_counts(ctx))) {
        return rc;
    }
    std::vector<WinCount> census;
    census_of_registry(ctx, census);
    ctx->batch_windows.clear();
    if ((rc = gens_prepare(ctx, census, true)) || (rc = winfo_upload(ctx, true))) return rc;
    Inputs Ik = I;
    Ik.lat += a; Ik.lon += a; Ik.ts += a; Ik.vk += a;
    if (Ik.sp) Ik.sp += a;
    if (Ik.sv) Ik.sv += a;
    if (Ik.rv) Ik.rv += a;
    Ik.n = n - a;
    int64_t ntiles = 1;
    PIPE_STEP(ctx, "overflow: tables", k);
    if ((rc = ev_partition(ctx, (const uint64_t *)ctx->keys.p + a, n - a, &Ik, ntiles))) return rc;
    PIPE_STEP(ctx, "overflow: partition", k);
    if (k == 0) HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    // its rows after chunk k - 1's (the partition's offsets moved to start there), the bins' starts as chunk k's segments
    hipLaunchKernelGGL(k_seg_rebase, dim3(1), dim3(256), 0, ctx->stream, (unsigned long long *)ctx->rp_O.p,
                       (int64_t)(RP_BINS + 1) * ntiles, ntiles, plO + (size_t)k * RP_BINS);
    HIPCHK(ctx, hipGetLastError());
    unsigned long long base = 0;
    HIPCHK(ctx, hipMemcpyAsync(&base, plO + (size_t)k * RP_BINS, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    // (the merge reads record i of [b0, b1) at src + i: the partitioned records start at row `base`)
    if ((rc = merge_sorted<EventRec>(ctx, n, ntiles, 0, (const EventRec *)ctx->parts_sorted.p - base, Segs(),
                                     (const unsigned long long *)ctx->rp_O.p, plN + (size_t)k * RP_BINS)))
        return rc;
    PIPE_STEP(ctx, "overflow: merge", k);
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if ((rc = rows_densify(ctx, 1, plO, plN, (k + 1) * RP_BINS))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    ctx->binned = false;
    ctx->bin_offsets_ready = false;
    ctx->last_pipe_chunks = K;
    ctx->n_partials_merged = (int64_t)ctx->h_st->n_valid - (int64_t)ctx->h_st->n_late;
    return HM_OK;
}

// The pipelined batch: chunked ingest + per-chunk merges + the rows densified; the side-stream dedup launched behind
// the last chunk.  to_table: the first chunk's key sample asked for table mode -- every chunk is ingested (binned) and
// nothing merged, the caller continues as after phase_local.  On return h_st holds the batch's statistics.
static int process_pipelined(hm_ctx *ctx, const Inputs &I, int64_t late_wm_ms, bool sub, int K, bool early_dedup,
                             bool &to_table) {
    to_table = false;
    const int64_t n = I.n;
    int rc;
    if ((rc = prepare_local(ctx, n, late_wm_ms, true, sub))) return rc;
    const int nbins = RP_BINS << ctx->sub_bits;
    const int ns = 1 << ctx->sub_bits;
    if ((rc = ensure(ctx, ctx->pl_cur, (size_t)K * (nbins + 1) * 4)) || (rc = ensure(ctx, ctx->pl_slow, (size_t)(K + 1) * 8)) ||
        (rc = ensure(ctx, ctx->pl_O, ((size_t)K * RP_BINS + 1) * 8)) || (rc = ensure(ctx, ctx->pl_cnt, (size_t)K * RP_BINS * 4)) ||
        (rc = ensure(ctx, ctx->pl_T, (RP_BINS + 1) * 4)) || (rc = ensure(ctx, ctx->stage_SO, (size_t)RP_BINS * ns * 8)) ||
        (rc = ensure(ctx, ctx->stage_SP, (size_t)RP_BINS * ns * 4)) || (rc = ensure(ctx, ctx->rp_O, (RP_BINS + 1) * 8)))
        return rc;
    unsigned long long *plO = (unsigned long long *)ctx->pl_O.p, *plS = (unsigned long long *)ctx->pl_slow.p;
    unsigned *plC = (unsigned *)ctx->pl_cur.p, *plN = (unsigned *)ctx->pl_cnt.p;
    HIPCHK(ctx, hipMemsetAsync(plO, 0, 8, ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(plS, 0, 8, ctx->stream));
    HIPCHK(ctx, hipEventRecord(ctx->ev[0], ctx->stream));
    // the merge stream starts behind everything queued so far (the previous batch's work, this batch's reset)
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[0], ctx->stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->merge_stream, ctx->side_ev[0], 0));
    const int64_t stride = hs_stride(n);
    auto row_of = [&](int k) { return n * k / K; };
    // chunk k: its rows' k_ingest<true>, the exception count after it, its exceptions' exact cells and records, the
    // cursors after it
    // (host inputs: each chunk's rows copied on copy_stream, its ingest behind the copy -- the next chunk's copy overlaps
    // this chunk's ingest, as phase_local's row chunks do)
    const bool h2d = ctx->n_h2d > 0;
    if (h2d) {
        HIPCHK(ctx, hipEventRecord(ctx->h2d_ev[0], ctx->stream));   // (buffers free: the last batch is done)
        HIPCHK(ctx, hipStreamWaitEvent(ctx->copy_stream, ctx->h2d_ev[0], 0));
    }
    auto launch_chunk = [&](int k) -> int {
        if (h2d) {
            const int64_t a = row_of(k), b = row_of(k + 1);
            for (int q = 0; q < ctx->n_h2d; q++) {
                const hm_ctx::H2D &h = ctx->h2d[q];
                HIPCHK(ctx, hipMemcpyAsync((uint8_t *)h.dst + a * h.el, (const uint8_t *)h.src + a * h.el, (b - a) * h.el,
                                           hipMemcpyHostToDevice, ctx->copy_stream));
            }
            HIPCHK(ctx, hipEventRecord(ctx->h2d_ev[k], ctx->copy_stream));
            HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->h2d_ev[k], 0));
        }
        PIPE_STEP(ctx, "h2d", k);
        launch_ingest(ctx, I, row_of(k), row_of(k + 1), true, late_wm_ms);
        PIPE_STEP(ctx, "k_ingest", k);
        hipLaunchKernelGGL(k_pipe_snap, dim3(1), dim3(64), 0, ctx->stream, (const unsigned *)nullptr, 0, (unsigned *)nullptr,
                           ctx->d_scratch + SLOW_WORD, plS + k + 1);
        hipLaunchKernelGGL(k_ingest_exact, dim3(64), dim3(256), 0, ctx->stream, I.lat, I.lon, ctx->cfg.h3_res,
                           (const unsigned int *)ctx->slow.p, plS + k + 1, (uint64_t *)ctx->keys.p, I.sp, I.sv,
                           (const unsigned long long *)ctx->d_wreg, (unsigned *)ctx->bin_cur.p, (EventRec *)ctx->parts_sorted.p,
                           ctx->slab_cap, ctx->d_st, ctx->sub_bits, (const unsigned long long *)(plS + k));
        PIPE_STEP(ctx, "k_ingest_exact", k);
        hipLaunchKernelGGL(k_pipe_snap, dim3(grid_for(nbins + 1, 256)), dim3(256), 0, ctx->stream, (const unsigned *)ctx->bin_cur.p,
                           nbins + 1, plC + (size_t)k * (nbins + 1), ctx->d_scratch + SLOW_WORD, (unsigned long long *)nullptr);
        if (k == 0)   // (the aggregation path's key sample: the first chunk's rows)
            hipLaunchKernelGGL(k_sample_heavy, dim3(1), dim3(HS_THREADS), 0, ctx->stream, (const uint64_t *)ctx->keys.p, row_of(1),
                               stride, ctx->d_st);
        PIPE_STEP(ctx, "snapshot/sample", k);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipEventRecord(ctx->pipe_ev[k], ctx->stream));
        if (k == K - 1) {
            ctx->n_h2d = 0;
            HIPCHK(ctx, hipEventRecord(ctx->ev[1], ctx->stream));
            HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
            ctx->dfused.dirty = true;
            ctx->dedup_early = early_dedup;
            if (early_dedup) {
                HIPCHK(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->ev[1], 0));
                int r;
                if ((r = launch_side_dedup(ctx, &I))) return r;
                PIPE_STEP(ctx, "side dedup", k);
            }
        }
        return HM_OK;
    };
    // the registry, its census and the statistics after the chunks so far (+ the cursors after the last one)
    auto readback = [&](bool last) -> int {
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_wreg, ctx->d_wreg, REG_BLOCK_BYTES, hipMemcpyDeviceToHost, ctx->stream));
        if (last) HIPCHK(ctx, hipMemcpyAsync(ctx->h_bincur, ctx->bin_cur.p, (size_t)nbins * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipEventRecord(ctx->pipe_rb, ctx->stream));
        return HM_OK;
    };
    if ((rc = launch_chunk(0)) || (rc = readback(K == 1))) return rc;
    int launched = 1;
    int64_t regs_uploaded = -1;   // registry windows the last winfo upload covered
    for (int k = 0; k < K; k++) {
        if (launched < K) {   // the next chunk queued before this one's readback is waited for: the stream never idles
            if ((rc = launch_chunk(launched))) return rc;
            launched++;
        }
        HIPCHK(ctx, ev_sync(ctx, ctx->pipe_rb, __LINE__));
        const DevStats st = *ctx->h_st;
        if (st.win_overflow)
            return set_err(ctx, HM_E_OVERFLOW, "more than %d distinct windows in one micro-batch (%llu rows)", WREG_SLOTS,
                           st.win_overflow);
        const int64_t n_agg = (int64_t)st.n_valid - (int64_t)st.n_late;
        if (k == 0 && choose_table(ctx, n_agg * K, st.sample_max_run)) {
            // heavy hitters: table mode for the whole batch, as phase_local's batch would (nothing merged yet)
            to_table = true;
            while (launched < K) {
                if ((rc = launch_chunk(launched))) return rc;
                launched++;
            }
            if ((rc = readback(true))) return rc;
            HIPCHK(ctx, ev_sync(ctx, ctx->pipe_rb, __LINE__));
            break;
        }
        if (st.bin_overflow) {
            // a slab overflowed in chunk k: the rest of the batch is partitioned from its keys (chunks < k are merged)
            while (launched < K) {
                if ((rc = launch_chunk(launched))) return rc;
                launched++;
            }
            if ((rc = readback(true))) return rc;
            HIPCHK(ctx, ev_sync(ctx, ctx->pipe_rb, __LINE__));
            pipe_batch_stats(ctx, nbins);
            return pipe_overflow_rest(ctx, I, K, k);
        }
        // the tables: from the census so far, scaled to the whole batch (every later chunk then fits them: a table
        // that grows inside a batch dumps and re-merges its keys); the last chunk's census is exact
        std::vector<WinCount> census;
        census_of_registry(ctx, census);
        if (k < K - 1) {
            const double scale = 1.25 * (double)n / (double)row_of(k + 1);
            for (auto &w : census) w.count = (unsigned long long)((double)w.count * scale) + 1024;
        }
        int64_t regs = 0;
        for (int w = 0; w < WREG_SLOTS; w++) regs += ctx->h_wreg[w] != 0;
        rc = on_merge_stream(ctx, [&]() -> int {
            int r;
            if (k == 0 && (r = merge_begin(ctx, n, true))) return r;
            if (k == 0 || gens_need_change(ctx, census)) {
                // a later chunk needs another table: the device's key counts of the merges so far first (the window
                // map's upload rewrites them), so the merge stream drains here
                if (k > 0 && (r = gens_sync_counts(ctx))) return r;
                ctx->batch_windows.clear();
                if ((r = gens_prepare(ctx, census, true))) return r;
            }
            PIPE_STEP(ctx, "tables", k);
            if (regs != regs_uploaded) {
                if ((r = winfo_upload(ctx, true))) return r;
                regs_uploaded = regs;
            }
            HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->pipe_ev[k], 0));
            if (k == 0) {
                HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
                HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
            }
            // chunk k's segments of every bin, its rows after chunk k - 1's
            hipLaunchKernelGGL(k_chunk_segments, dim3(grid_for(RP_BINS + 1, 256)), dim3(256), 0, ctx->stream,
                               k ? (const unsigned *)plC + (size_t)(k - 1) * (nbins + 1) : (const unsigned *)nullptr,
                               (const unsigned *)plC + (size_t)k * (nbins + 1), (const EventRec *)ctx->parts_sorted.p,
                               (int64_t)ctx->slab_cap, ctx->sub_bits, (unsigned long long *)ctx->stage_SO.p,
                               (unsigned *)ctx->stage_SP.p, (unsigned *)ctx->pl_T.p);
            hipLaunchKernelGGL(k_seg_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->pl_T.p, (int64_t)RP_BINS + 1,
                               plO + (size_t)k * RP_BINS);
            PIPE_STEP(ctx, "segments", k);
            HIPCHK(ctx, hipGetLastError());
            Segs seg;
            seg.SO = (const unsigned long long *)ctx->stage_SO.p;
            seg.SP = (const unsigned *)ctx->stage_SP.p;
            seg.nseg = ns;
            const unsigned long long a = (unsigned long long)(uintptr_t)ctx->parts_sorted.p;
            seg.bounds = SegBounds{{a, a}, {a + ctx->parts_sorted.bytes, a + ctx->parts_sorted.bytes}};
            if ((r = merge_sorted<EventRec>(ctx, n, 1, 0, (const EventRec *)ctx->parts_sorted.p, seg, plO + (size_t)k * RP_BINS,
                                            plN + (size_t)k * RP_BINS)))
                return r;
            PIPE_STEP(ctx, "k_merge_owned", k);
            if (k == K - 1) {
                HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
                HIPCHK(ctx, hipEventRecord(ctx->pipe_done, ctx->stream));
            }
            return HM_OK;
        });
        if (rc) return rc;
        if (k + 1 < K && (rc = readback(k + 1 == K - 1))) return rc;
    }
    pipe_batch_stats(ctx, nbins);
    if (to_table) {   // (as phase_local leaves a binned batch: the caller takes table mode)
        ctx->binned = ctx->h_st->bin_overflow == 0;
        ctx->last_pipe_chunks = 0;
        return HM_OK;
    }
    ctx->binned = true;
    ctx->last_pipe_chunks = K;
    ctx->n_partials_merged = (int64_t)ctx->h_st->n_valid - (int64_t)ctx->h_st->n_late;
    // the rows of all chunks densified on the main stream, behind the last merge
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->pipe_done, 0));
    if ((rc = rows_densify(ctx, 1, plO, plN, K * RP_BINS))) return rc;
    PIPE_STEP(ctx, "densify", K);
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    return HM_OK;
}
