// Host side: the batch phases shared by the single-GPU path and the stage API.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// ---- batch phases shared by the single-GPU and stage paths ----
// Fused binning (k_ingest<true>) for a direct-path batch of at least BIN_MIN_ROWS rows: the last batch's numbers did
// not ask for table mode (the choice is made before the ingest here; a key sample that then shows heavy hitters still
// switches the batch to table mode, the binned records unused).  MOBHEAT_INGEST_MODE=direct pins the separate
// partition, =binned the fused one at any size.
constexpr int64_t BIN_MIN_ROWS = int64_t(1) << 22;
static bool prev_says_table(const hm_ctx *ctx) {
    return ctx->prev_keys > 0 && ctx->prev_keys <= (int64_t)AG_BINS * (AG_SLOTS / 2) && ctx->prev_agg_rows >= 8 * ctx->prev_keys;
}
static bool choose_binned(const hm_ctx *ctx, int64_t n) {
    if (ctx->ingest_mode) return ctx->ingest_mode == 3;
    return n >= BIN_MIN_ROWS && !prev_says_table(ctx);
}
// records per bin slab for n rows: the rows spread over the RP_BINS bins by a hash (binomial counts, ~sqrt(n / RP_BINS)
// wide), so the mean + 25% + 256 overflows only on skewed keys (then the batch re-partitions from its keys)
// (clustered keys -- a key's rows share its bin -- widen that; the last binned batch's fullest bin / mean, `skew`, with
// 10% room, covers a stream whose clustering is steady)
static unsigned slab_cap_for(int64_t n, double skew, int64_t nbins) {
    const int64_t m = (n + nbins - 1) / nbins;
    const int64_t c = std::max<int64_t>(m + m / 4 + 256, (int64_t)(skew * 1.1 * (double)m) + 256);
    return (unsigned)std::min<int64_t>((c + 1) & ~int64_t(1), (int64_t)UINT32_MAX / 2);   // (even: 64-B aligned slabs)
}

// k_ingest + k_ingest_exact: flags, event keys, the window registry and its census, dedup max, batch statistics;
// allow_bin: the batch may bin its rows in k_ingest; sub: in sub-bins (hm_process_batch; the stage API's senders keep
// whole bins, the unit its chunks and self-held segments are made of)
// early_dedup (hm_process_batch): the latest-position dedup launched on the side stream right behind the ingest, so
// that it runs while the host reads the batch statistics back and prepares the merge (it assumes the fused max did not
// give up; hm_process_batch reruns it on the main stream when it did)
// offsets: the binned batch's row offsets (bin_offsets) launched right behind k_ingest too, ahead of the side stream's
// dedup (hm_process_batch): launched after the readback they queued behind the dedup's grid, 75 us on the merge's
// critical path (profiles/r5/r5tl/)
static int launch_side_dedup(hm_ctx *ctx, const Inputs *I);
static int bin_offsets(hm_ctx *ctx);
// the batch's per-row buffers, dedup tables, bins and counters ready, k_batch_reset launched (phase_local, the
// pipelined batch)
static int prepare_local(hm_ctx *ctx, int64_t n, int64_t late_wm_ms, bool bin, bool sub) {
    int rc;
    // the previous call's side-stream dedup may still run (a stage batch that a peer's failure ended before
    // hm_stage_send waited for it -- ADVICE r5): nothing below touches its tables, flags or rows before it is done
    if (ctx->dedup_early) HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[2], 0));
    ctx->dedup_early = false;
    if ((rc = ensure(ctx, ctx->flags, n)) || (rc = ensure(ctx, ctx->win, n)) || (rc = ensure(ctx, ctx->rows, n * 8)) ||
        (rc = ensure(ctx, ctx->keys, n * 8)) || (rc = ensure(ctx, ctx->slow, n * sizeof(unsigned int))))
        return rc;
    if ((rc = dedup_prepare(ctx, ctx->dfused, dedup_fused_keys(ctx, n), true))) return rc;
    // the dense dedup table: room for the last batch's vkeys (first batch: 2^20), 2^16 .. 2^22 words; none when the
    // last batch's vkeys were not dense codes (above 2^24)
    {
        const int64_t b = ctx->vkey_bound;
        unsigned long long cap = 0;
        if (ctx->dense_ok && n > 0 && b <= (int64_t(1) << 24)) {
            cap = b < 0 ? (1ull << 20) : 1ull << 16;
            while (cap < (unsigned long long)b && cap < (1ull << 22)) cap <<= 1;
        }
        ctx->dense_cap = cap;
        if (cap) {
            if ((rc = ensure(ctx, ctx->dense, cap * 8))) return rc;
            HIPCHK(ctx, hipMemsetAsync(ctx->dense.p, 0, cap * 8, ctx->stream));
        }
    }
    ctx->keys_partial = bin;   // (k_ingest<true> writes the keys of the exception and sampled rows only)
    ctx->keys_late_us = late_wm_ms * 1000;
    ctx->sub_bits = bin && sub ? SUB_BITS : 0;
    const int nbins = RP_BINS << ctx->sub_bits;
    ctx->slab_cap = bin ? slab_cap_for(n, ctx->bin_skew, nbins) : 0;
    if (bin && ctx->test_slab_cap) ctx->slab_cap = std::min(ctx->slab_cap, ctx->test_slab_cap);
    ctx->binned = false;
    ctx->bin_offsets_ready = false;
    if ((rc = ensure(ctx, ctx->bin_cur, ((RP_BINS << SUB_BITS) + 1) * 4))) return rc;
    // (+ 64 slack records: k_ev_scatter_rec's, when a slab overflows and the batch is re-partitioned)
    if (bin && (rc = ensure(ctx, ctx->parts_sorted, ((size_t)nbins * ctx->slab_cap + 64) * sizeof(EventRec)))) return rc;
    {
        const int nw = 2 * (WREG_SLOTS + 1);   // d_wreg and d_wcount: one allocation (hm_create)
        hipLaunchKernelGGL(k_batch_reset, dim3((std::max(nw, nbins + 1) + 255) / 256), dim3(256), 0, ctx->stream,
                           (unsigned long long *)ctx->d_st, ctx->d_scratch + SLOW_WORD, ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg,
                           nw, (unsigned *)ctx->bin_cur.p, nbins + 1);
        HIPCHK(ctx, hipGetLastError());
    }
    return HM_OK;
}

// k_ingest over rows [a, b) of the batch I (bin: k_ingest<true>, the rows' records into their bin slabs)
static void launch_ingest(hm_ctx *ctx, const Inputs &I, int64_t a, int64_t b, bool bin, int64_t late_wm_ms) {
    const int blocks = (int)std::min<int64_t>((b - a + IG_THREADS - 1) / IG_THREADS, bin ? ctx->ingest_grid_bin : ctx->ingest_grid);
    auto kern = bin ? k_ingest<true> : k_ingest<false>;
    hipLaunchKernelGGL(kern, dim3(std::max(blocks, 1)), dim3(IG_THREADS), 0, ctx->stream, I.lat, I.lon, I.ts, I.rv, I.vk, a, b,
                       ctx->cfg.h3_res, make_floor_div(ctx->cfg.tile_us), late_wm_ms * 1000, (uint8_t *)ctx->flags.p,
                       (uint64_t *)ctx->keys.p, ctx->dfused.tab, ctx->dfused.cap - 1, (unsigned int *)ctx->dfused.used.p,
                       ctx->d_scratch + ctx->dfused.used_word, (unsigned int *)ctx->slow.p, ctx->d_scratch + SLOW_WORD,
                       ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg, ctx->d_wcount, ctx->d_st, I.sp, I.sv,
                       (unsigned *)ctx->bin_cur.p, bin ? (EventRec *)ctx->parts_sorted.p : nullptr, ctx->slab_cap,
                       (unsigned long long *)ctx->dense.p, ctx->dense_cap, ctx->sub_bits, hs_stride(I.n) - 1);
}

static int phase_local(hm_ctx *ctx, const Inputs &I, int64_t late_wm_ms, bool allow_bin = false, bool sub = false,
                       bool early_dedup = false, bool offsets = false) {
    int64_t n = I.n;
    int rc;
    const bool bin = allow_bin && n > 0 && choose_binned(ctx, n);
    if ((rc = prepare_local(ctx, n, late_wm_ms, bin, sub))) return rc;
    const int nbins = RP_BINS << ctx->sub_bits;
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
            launch_ingest(ctx, I, a, b, bin, late_wm_ms);
        }
        ctx->n_h2d = 0;
        hipLaunchKernelGGL(k_ingest_exact, dim3(256), dim3(256), 0, ctx->stream, I.lat, I.lon, ctx->cfg.h3_res,
                           (const unsigned int *)ctx->slow.p, ctx->d_scratch + SLOW_WORD, (uint64_t *)ctx->keys.p, I.sp, I.sv,
                           (const unsigned long long *)ctx->d_wreg, (unsigned *)ctx->bin_cur.p,
                           bin ? (EventRec *)ctx->parts_sorted.p : nullptr, ctx->slab_cap, ctx->d_st, ctx->sub_bits,
                           (const unsigned long long *)nullptr);
        hipLaunchKernelGGL(k_sample_heavy, dim3(1), dim3(HS_THREADS), 0, ctx->stream, (const uint64_t *)ctx->keys.p, n, hs_stride(n),
                           ctx->d_st);
        HIPCHK(ctx, hipGetLastError());
        ctx->dfused.dirty = true;
        // (a slab that overflowed makes the batch re-partition: these offsets then go unused)
        if (bin && offsets) {
            if ((rc = bin_offsets(ctx))) return rc;
            ctx->bin_offsets_ready = true;
        }
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], ctx->stream));
    ctx->dedup_early = early_dedup && n > 0;
    if (ctx->dedup_early) {
        HIPCHK(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->ev[1], 0));
        if ((rc = launch_side_dedup(ctx, &I))) return rc;
    }
    // the batch statistics and the registry with its census, read back together
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_wreg, ctx->d_wreg, REG_BLOCK_BYTES, hipMemcpyDeviceToHost, ctx->stream));   // (+ h_wcount, h_st)
    if (bin) HIPCHK(ctx, hipMemcpyAsync(ctx->h_bincur, ctx->bin_cur.p, (size_t)nbins * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (bin) {   // the fullest bin against the mean: the next batch's slab room
        unsigned long long tot = 0, mx = 0;
        for (int b = 0; b < nbins; b++) { tot += ctx->h_bincur[b]; mx = std::max<unsigned long long>(mx, ctx->h_bincur[b]); }
        if (tot) ctx->bin_skew = std::max(1.0, (double)mx * nbins / (double)tot);
    }
    if (ctx->h_st->win_overflow)
        return set_err(ctx, HM_E_OVERFLOW, "more than %d distinct windows in one micro-batch (%llu rows)", WREG_SLOTS,
                       ctx->h_st->win_overflow);
    ctx->binned = bin && ctx->h_st->bin_overflow == 0;
    if (ctx->h_st->vkey_max1) ctx->vkey_bound = (int64_t)ctx->h_st->vkey_max1;
    return HM_OK;
}

// every row's event key after a binned ingest (k_ingest<false, true>): for the table mode and the re-partition of a
// batch whose slab overflowed, the only readers of all the keys
static int keys_complete(hm_ctx *ctx, const Inputs &I) {
    if (!ctx->keys_partial) return HM_OK;
    ctx->keys_partial = false;
    if (I.n == 0) return HM_OK;
    const int blocks = (int)std::min<int64_t>((I.n + IG_THREADS - 1) / IG_THREADS, ctx->ingest_grid);
    hipLaunchKernelGGL((k_ingest<false, true>), dim3(blocks), dim3(IG_THREADS), 0, ctx->stream, I.lat, I.lon, I.ts, I.rv, I.vk,
                       (int64_t)0, I.n, ctx->cfg.h3_res, make_floor_div(ctx->cfg.tile_us), ctx->keys_late_us,
                       (uint8_t *)ctx->flags.p, (uint64_t *)ctx->keys.p, ctx->dfused.tab, ctx->dfused.cap - 1,
                       (unsigned int *)ctx->dfused.used.p, ctx->d_scratch + ctx->dfused.used_word, (unsigned int *)ctx->slow.p,
                       ctx->d_scratch + SLOW_WORD, ctx->d_scratch + GIVEUP_WORD, ctx->d_wreg, ctx->d_wcount, ctx->d_st, I.sp,
                       I.sv, (unsigned *)ctx->bin_cur.p, (EventRec *)nullptr, 0u, (unsigned long long *)ctx->dense.p, 0ull, 0u,
                       (int64_t)0);
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

// Aggregation path of the batch: table mode when the last batches had few distinct keys that repeat a lot (their
// aggregates fit k_bin_reduce's LDS tables), or when this batch's key sample shows heavy hitters (a key in >= 1/256
// of the sampled rows: k_sample_heavy), else the direct path.
static bool choose_table(const hm_ctx *ctx, int64_t n_agg, unsigned long long sample_max_run) {
    if (ctx->ingest_mode) return ctx->ingest_mode == 2;
    if (n_agg < (int64_t(1) << 16)) return false;
    if (sample_max_run >= (unsigned long long)(HS_SAMPLE / 256)) return true;
    return prev_says_table(ctx);
}

// table mode: k_agg + k_bin_reduce -> one partial record per key of the batch (ctx->partials, count *n_parts),
// census in d_cmap
static int phase_table(hm_ctx *ctx, const Inputs &I, int64_t n_agg, int64_t *n_parts) {
    int rc;
    const int64_t n = I.n;
    if ((rc = keys_complete(ctx, I))) return rc;
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
                           (uint8_t *)ctx->win.p, !need_max, (const unsigned long long *)ctx->dense.p,
                           need_max ? 0ull : ctx->dense_cap);
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
// (O / cnt / nseg: the segments' row offsets and touched-key counts; default rp_O and bin_cnt over the RP_BINS bins --
// a pipelined batch passes its chunks' segments, nseg = chunks x RP_BINS, ntiles 1)
static int rows_densify(hm_ctx *ctx, int64_t ntiles, const unsigned long long *O = nullptr, const unsigned *cnt = nullptr,
                        int nseg = RP_BINS) {
    int rc;
    if (!O) O = (const unsigned long long *)ctx->rp_O.p;
    if (!cnt) cnt = (const unsigned *)ctx->bin_cnt.p;
    if ((rc = ensure(ctx, ctx->bin_off, (size_t)nseg * 8)) || (rc = ensure(ctx, ctx->gapbuf, (size_t)nseg * 24))) return rc;
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, cnt, (int64_t)nseg, (unsigned long long *)ctx->bin_off.p,
                       &ctx->d_st->n_touched);
    unsigned *gg = (unsigned *)ctx->gapbuf.p, *gv = gg + nseg;
    unsigned long long *gvo = (unsigned long long *)(gv + nseg), *ggo = (unsigned long long *)ctx->bin_off.p;
    hipLaunchKernelGGL(k_gap_counts, dim3(grid_for(nseg, 256)), dim3(256), 0, ctx->stream, O, ntiles, nseg, cnt,
                       &ctx->d_st->n_touched, gg, gv);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, gg, (int64_t)nseg, ggo, ctx->d_scratch + GAPS_WORD);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, gv, (int64_t)nseg, gvo, ctx->d_scratch + GAPS_WORD + 1);
    hipLaunchKernelGGL(k_fill_gaps, dim3(nseg), dim3(256), 0, ctx->stream, staged_rows(ctx), O, ntiles, nseg, cnt,
                       &ctx->d_st->n_touched, (const unsigned *)gg, (const unsigned long long *)ggo, (const unsigned long long *)gvo);
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

// the binned batch's row offsets rp_O (the exclusive scan of the bins' counts); in sub-bins, each bin's sub-slabs as
// its segments first, in sub-region order (k_sub_segments: stage_SO / stage_SP, bin totals stage_T)
static int bin_offsets(hm_ctx *ctx) {
    int rc;
    if ((rc = ensure(ctx, ctx->rp_O, (RP_BINS + 1) * 8))) return rc;
    if (!ctx->sub_bits)
        return scan_counts(ctx, (const unsigned *)ctx->bin_cur.p, RP_BINS + 1, (unsigned long long *)ctx->rp_O.p);
    constexpr int NS = 1 << SUB_BITS;
    static_assert(SUB_BITS == 3, "k_sub_segments and the merge's segment table assume 8 sub-bins");
    if ((rc = ensure(ctx, ctx->stage_SO, (size_t)RP_BINS * NS * 8)) || (rc = ensure(ctx, ctx->stage_SP, (size_t)RP_BINS * NS * 4)) ||
        (rc = ensure(ctx, ctx->stage_T, (RP_BINS + 1) * 4)))
        return rc;
    hipLaunchKernelGGL(k_sub_segments, dim3(grid_for(RP_BINS + 1, 256)), dim3(256), 0, ctx->stream, (const unsigned *)ctx->bin_cur.p,
                       (const EventRec *)ctx->parts_sorted.p, (int64_t)ctx->slab_cap, (unsigned long long *)ctx->stage_SO.p,
                       (unsigned *)ctx->stage_SP.p, (unsigned *)ctx->stage_T.p);
    HIPCHK(ctx, hipGetLastError());
    return scan_counts(ctx, (const unsigned *)ctx->stage_T.p, RP_BINS + 1, (unsigned long long *)ctx->rp_O.p);
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
    // binned in k_ingest: every window's table in range geometry (a row's bin is its region), and the bins' row
    // offsets are the exclusive scan of their cursors -- no partition pass over the keys and columns
    const bool binned = ctx->binned;
    if ((rc = gens_prepare(ctx, census, binned)) || (rc = winfo_upload(ctx, true))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    int64_t ntiles = 1;
    const bool subs = binned && ctx->sub_bits;
    Segs seg;
    if (binned && !ctx->bin_offsets_ready && (rc = bin_offsets(ctx))) return rc;
    if (subs) {   // each bin's sub-slabs as its segments, in sub-region order (k_sub_segments)
        seg.SO = (const unsigned long long *)ctx->stage_SO.p;
        seg.SP = (const unsigned *)ctx->stage_SP.p;
        seg.nseg = 1 << SUB_BITS;
        const unsigned long long a = (unsigned long long)(uintptr_t)ctx->parts_sorted.p;
        seg.bounds = SegBounds{{a, a}, {a + ctx->parts_sorted.bytes, a + ctx->parts_sorted.bytes}};
    } else if (!binned && ((rc = keys_complete(ctx, I)) || (rc = ev_partition(ctx, (const uint64_t *)ctx->keys.p, I.n, &I, ntiles)))) {
        return rc;
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    if (subs) rc = merge_sorted<EventRec>(ctx, I.n, 1, 0, (const EventRec *)ctx->parts_sorted.p, seg);
    else rc = merge_sorted<EventRec>(ctx, I.n, ntiles, binned ? ctx->slab_cap : 0);
    if (rc) return rc;
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
