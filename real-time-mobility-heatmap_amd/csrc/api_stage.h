// C ABI: the multi-GPU stage API (hm_stage_ingest / send / merge / finish).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// ---- multi-GPU stage API ----
// summary words of one rank (HM_STAGE_SUMMARY_WORDS int64, all-gathered by the caller between ingest and send)
enum : int {
    SW_N_IN = 0, SW_VALID, SW_LATE, SW_AGG, SW_MAX_MS, SW_SAMPLE_RUN, SW_PREV_AGG, SW_PREV_KEYS, SW_NWIN, SW_RESERVED,
    SW_WIN0   // then n_windows pairs (registry slot, wenc)
};
static_assert(SW_WIN0 + 2 * WREG_SLOTS <= HM_STAGE_SUMMARY_WORDS, "summary layout");

int hm_stage_ingest(hm_ctx *ctx, int64_t epoch_id, const hm_batch_in *in, int32_t nranks, int32_t rank, int64_t *summary) {
    if (!ctx || !in || !summary || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks)
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (in->n > MAX_BATCH_ROWS) return set_err(ctx, HM_E_INVALID, "batch of %lld events exceeds %lld", (long long)in->n, (long long)MAX_BATCH_ROWS);
    if (in->n > 0 && (!in->lat || !in->lon || !in->ts_us || !in->vkey))
        return set_err(ctx, HM_E_INVALID, "lat, lon, ts_us and vkey are required");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    ctx->stage = 0;
    ctx->epoch = epoch_id;
    ctx->last_n_latest = -1;   // (set again by hm_stage_finish: this rank's latest rows)
    ctx->nranks = nranks;
    ctx->rank = rank;
    const int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    Inputs I;
    I.n = in->n;
    if ((rc = stage_inputs(ctx, in, &I.lat, &I.lon, &I.ts, &I.sp, &I.sv, &I.vk, &I.rv))) return rc;
    if ((rc = phase_local(ctx, I, late_wm))) return rc;
    const DevStats s1 = *ctx->h_st;
    ctx->stage_I = I;
    ctx->stage_s1 = s1;
    ctx->staged = true;
    memset(summary, 0, HM_STAGE_SUMMARY_WORDS * sizeof(int64_t));
    summary[SW_N_IN] = I.n;
    summary[SW_VALID] = (int64_t)s1.n_valid;
    summary[SW_LATE] = (int64_t)s1.n_late;
    summary[SW_AGG] = (int64_t)s1.n_valid - (int64_t)s1.n_late;
    summary[SW_MAX_MS] = s1.max_ts_ms;
    summary[SW_SAMPLE_RUN] = (int64_t)s1.sample_max_run;
    summary[SW_PREV_AGG] = ctx->prev_agg_rows;
    summary[SW_PREV_KEYS] = ctx->prev_keys;
    int64_t nw = 0;
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wreg[w] && ctx->h_wcount[w]) {
            summary[SW_WIN0 + 2 * nw] = w;
            summary[SW_WIN0 + 2 * nw + 1] = (int64_t)ctx->h_wreg[w];
            nw++;
        }
    summary[SW_NWIN] = nw;
    ctx->stage_n_in = I.n;
    ctx->stage = 1;
    return HM_OK;
}

// The batch-wide decisions every rank derives identically from all ranks' summaries: the global max event time (the
// watermark's input), the aggregation path, and the global window registry (k_ingest's hashing -- slot wq mod
// WREG_SLOTS, linear probing -- over the union of the ranks' windows in ascending order).
static int stage_decide(hm_ctx *ctx, const int64_t *sums) {
    const int W = ctx->nranks;
    int64_t gmax = INT64_MIN, min_agg = INT64_MAX, prev_agg = 0, prev_keys = 0;
    unsigned long long max_run = 0;
    std::vector<unsigned long long> wins;
    for (int r = 0; r < W; r++) {
        const int64_t *S = sums + (size_t)r * HM_STAGE_SUMMARY_WORDS;
        gmax = std::max(gmax, S[SW_MAX_MS]);
        min_agg = std::min(min_agg, S[SW_AGG]);
        max_run = std::max(max_run, (unsigned long long)S[SW_SAMPLE_RUN]);
        prev_agg += S[SW_PREV_AGG];
        prev_keys += S[SW_PREV_KEYS];
        if (S[SW_NWIN] < 0 || S[SW_NWIN] > WREG_SLOTS) return set_err(ctx, HM_E_INVALID, "summary of rank %d is malformed", r);
        for (int64_t k = 0; k < S[SW_NWIN]; k++) wins.push_back((unsigned long long)S[SW_WIN0 + 2 * k + 1]);
    }
    std::sort(wins.begin(), wins.end());
    wins.erase(std::unique(wins.begin(), wins.end()), wins.end());
    ctx->stage_gwreg.assign(WREG_SLOTS, 0ull);
    for (unsigned long long we : wins) {
        const int64_t wq = wdec(we) / ctx->cfg.tile_us;   // (window starts are multiples of tile_us)
        unsigned h = (unsigned)((uint64_t)wq % (uint64_t)WREG_SLOTS);
        int p = 0;
        for (; p < WREG_SLOTS && ctx->stage_gwreg[h]; p++) h = h + 1 == (unsigned)WREG_SLOTS ? 0u : h + 1;
        if (p == WREG_SLOTS)
            return set_err(ctx, HM_E_OVERFLOW, "more than %d distinct windows in one micro-batch over all ranks", WREG_SLOTS);
        ctx->stage_gwreg[h] = we;
    }
    ctx->stage_gmax_ms = gmax;
    // aggregation path: the single-context rule (choose_table) on batch-wide numbers -- table mode when a rank's key
    // sample shows heavy hitters, or when the last batch's keys were few and repeated a lot on every rank
    bool table;
    if (ctx->ingest_mode) table = ctx->ingest_mode == 2;
    else if (min_agg < (int64_t(1) << 16)) table = false;
    else if (max_run >= (unsigned long long)(HS_SAMPLE / 256)) table = true;
    else table = prev_keys > 0 && prev_keys <= (int64_t)AG_BINS * (AG_SLOTS / 2) && prev_agg >= 8 * (int64_t)W * prev_keys;
    ctx->stage_table = table;
    return HM_OK;
}

int hm_stage_send(hm_ctx *ctx, const int64_t *summaries, void *tile_send_buf, void *payload_send_buf, int64_t tile_send_cap,
                  int64_t *tile_send_counts, void *cand_send_buf, int64_t cand_send_cap, int64_t *cand_send_counts,
                  hm_stage_sizes *sizes) {
    if (!ctx || !summaries || !tile_send_counts || !cand_send_counts)
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 1) return set_err(ctx, HM_E_STATE, "hm_stage_send before hm_stage_ingest");
    const Inputs &I = ctx->stage_I;
    if (I.n > 0 && (!tile_send_buf || !payload_send_buf || !cand_send_buf))
        return set_err(ctx, HM_E_INVALID, "send buffers are required");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const int W = ctx->nranks;
    if (summaries[(size_t)ctx->rank * HM_STAGE_SUMMARY_WORDS + SW_N_IN] != I.n)
        return set_err(ctx, HM_E_INVALID, "summaries[rank] is not this rank's summary");
    if ((rc = stage_decide(ctx, summaries))) return rc;
    const DevStats &s1 = ctx->stage_s1;
    const int64_t n_agg = (int64_t)s1.n_valid - (int64_t)s1.n_late;
    const bool table = ctx->stage_table;
    ctx->last_table = table;
    int64_t n_records = n_agg;
    HIPCHK(ctx, hipEventRecord(ctx->ev[10], ctx->stream));
    if (table && (rc = phase_table(ctx, I, n_agg, &n_records))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
    ctx->census_ready = false;   // (the owner counts what it receives)
    // local dedup over rows -> local winners -> candidates
    if ((rc = phase_dedup(ctx, &I, nullptr, I.n, s1.dedup_retry != 0))) return rc;
    if ((rc = ensure(ctx, ctx->cands, std::max<int64_t>(I.n, 1) * sizeof(Cand)))) return rc;
    hipLaunchKernelGGL(k_make_cands, dim3(grid_for(std::max<int64_t>(I.n, 1), 256)), dim3(256), 0, ctx->stream,
                       (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, I.vk, I.ts, ctx->rank, (Cand *)ctx->cands.p);
    HIPCHK(ctx, hipGetLastError());
    // partition both record kinds by owner rank: candidates by counts + cursors here, tile records below
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch, 0, 128 * 8, ctx->stream));
    const int gb = grid_for(std::max<int64_t>(I.n, 1), 256);
    hipLaunchKernelGGL(k_part_count<Cand>, dim3(gb), dim3(256), 0, ctx->stream, (const Cand *)ctx->cands.p, ctx->d_scratch + 255,
                       W, ctx->d_scratch + 64);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    if (ctx->h_st->bad_vkey) return set_err(ctx, HM_E_INVALID, "vkey UINT64_MAX is reserved");
    ctx->dedup_seen = (int64_t)ctx->h_scratch[ctx->dlast->used_word];
    if (n_records > tile_send_cap || (int64_t)ctx->h_scratch[255] > cand_send_cap)
        return set_err(ctx, HM_E_INVALID, "send buffer too small (%lld tile records, %llu candidates)", (long long)n_records,
                       ctx->h_scratch[255]);
    // candidates: exclusive offsets -> cursors
    unsigned long long cur[128];
    unsigned long long acc = 0;
    for (int r = 0; r < W; r++) { cur[64 + r] = acc; cand_send_counts[r] = (int64_t)ctx->h_scratch[64 + r]; acc += ctx->h_scratch[64 + r]; }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_scratch + 64, cur + 64, 64 * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_part_scatter<Cand>, dim3(gb), dim3(256), 0, ctx->stream, (const Cand *)ctx->cands.p, ctx->d_scratch + 255,
                       W, ctx->d_scratch + 64, (Cand *)cand_send_buf);
    HIPCHK(ctx, hipGetLastError());
    // tile records: the radix partition with the owner rank as the digit, straight into the send streams
    HIPCHK(ctx, hipEventRecord(ctx->ev[8], ctx->stream));
    if (n_records > 0) {
        int64_t ntiles;
        if (table) {
            if ((rc = partition<TilePartial, TilePartial>(ctx, (const TilePartial *)ctx->partials.p, n_records, ntiles, W,
                                                          (TilePartial *)tile_send_buf)))
                return rc;
        } else {
            // this rank's registry slots -> the batch's global slots (WInfo.gslot), keys rewritten by the scatter
            ctx->stage_gslot.assign(WREG_SLOTS, 0u);
            for (int w = 0; w < WREG_SLOTS; w++) {
                const unsigned long long we = ctx->h_wreg[w];
                if (!we) continue;
                const auto it = std::find(ctx->stage_gwreg.begin(), ctx->stage_gwreg.end(), we);
                if (it == ctx->stage_gwreg.end() && ctx->h_wcount[w])
                    return set_err(ctx, HM_E_STATE, "a window of this rank is missing from the global registry");
                ctx->stage_gslot[w] = (unsigned)(it - ctx->stage_gwreg.begin());
            }
            rc = winfo_upload(ctx, false);
            ctx->stage_gslot.clear();
            if (rc || (rc = ev_partition<WireKey>(ctx, (const uint64_t *)ctx->keys.p, I.n, &I, nullptr, ntiles, W,
                                                  (WireKey *)tile_send_buf, (uint64_t *)payload_send_buf)))
                return rc;
        }
        hipLaunchKernelGGL(k_digit_starts, dim3(1), dim3(128), 0, ctx->stream, (const unsigned long long *)ctx->rp_O.p, ntiles,
                           W + 1, ctx->d_scratch);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, (W + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[9], ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    for (int r = 0; r < W; r++) {
        const int64_t start = n_records > 0 ? (int64_t)ctx->h_scratch[r] : 0;
        const int64_t end = n_records > 0 ? (int64_t)ctx->h_scratch[r + 1] : 0;   // [W]: the gaps' digit
        tile_send_counts[r] = end - start;
    }
    ctx->stage_agg_rows = n_agg;
    ctx->stage_sent = n_records;
    hm_stage_sizes z{};
    z.table_mode = table ? 1 : 0;
    z.n_tile_records = n_records;
    for (int r = 0; r < W; r++) z.n_cands += cand_send_counts[r];
    z.global_batch_max_event_ms = ctx->stage_gmax_ms;
    z.n_valid = (int64_t)s1.n_valid;
    z.n_late = (int64_t)s1.n_late;
    ctx->stage_sizes = z;
    if (sizes) *sizes = z;
    ctx->stage = 2;
    return HM_OK;
}

// the multi-GPU owner's direct path: the received key + payload streams (n rows of all ranks) -> census per global
// window -> window tables -> (window, region) partition into EventRecs -> merge -> rows
static int merge_received_events(hm_ctx *ctx, const uint64_t *keys, const uint64_t *payload, int64_t n) {
    int rc;
    if (n > MAX_BATCH_ROWS) return set_err(ctx, HM_E_INVALID, "%lld received records exceed %lld", (long long)n, (long long)MAX_BATCH_ROWS);
    ctx->n_partials_merged = n;
    if ((rc = merge_begin(ctx, n))) return rc;
    if (n == 0) return merge_nothing(ctx);
    memcpy(ctx->h_wreg, ctx->stage_gwreg.data(), WREG_SLOTS * sizeof(unsigned long long));
    HIPCHK(ctx, hipMemsetAsync(ctx->d_wcount, 0, (WREG_SLOTS + 1) * 8, ctx->stream));
    hipLaunchKernelGGL(k_key_census, dim3(grid_for(n, 256, 256 * 8)), dim3(256), 0, ctx->stream, keys, n, ctx->d_wcount);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_wcount, ctx->d_wcount, WREG_SLOTS * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wcount[w] && !ctx->h_wreg[w]) return set_err(ctx, HM_E_INVALID, "received a record of an unknown window slot");
    std::vector<WinCount> census;
    census_of_registry(ctx, census);
    if ((rc = gens_prepare(ctx, census)) || (rc = winfo_upload(ctx, true))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    int64_t ntiles;
    if ((rc = ev_partition<EventRec>(ctx, keys, n, nullptr, payload, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    if ((rc = merge_sorted<EventRec>(ctx, n, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if ((rc = rows_densify(ctx, ntiles))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    return HM_OK;
}

int hm_stage_merge(hm_ctx *ctx, const void *tile_recv_dev, const void *payload_recv_dev, int64_t n_tile_recv,
                   const void *cand_recv_dev, int64_t n_cand_recv, int32_t out_memory, hm_batch_out *out,
                   void *winner_send_buf, int64_t winner_send_cap, int64_t *winner_send_counts) {
    if (!ctx || !out || !winner_send_counts || n_tile_recv < 0 || n_cand_recv < 0 || winner_send_cap < n_cand_recv ||
        (n_cand_recv > 0 && (!winner_send_buf || !cand_recv_dev)) || (n_tile_recv > 0 && !tile_recv_dev))
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 2) return set_err(ctx, HM_E_STATE, "hm_stage_merge before hm_stage_send");
    if (!ctx->stage_table && n_tile_recv > 0 && !payload_recv_dev)
        return set_err(ctx, HM_E_INVALID, "the direct path needs the received payload stream");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    memset(out, 0, sizeof(*out));
    const int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    if (ctx->stage_table) rc = merge_partials(ctx, (const TilePartial *)tile_recv_dev, n_tile_recv);
    else rc = merge_received_events(ctx, (const uint64_t *)tile_recv_dev, (const uint64_t *)payload_recv_dev, n_tile_recv);
    if (rc) return rc;
    // owner-side dedup over received candidates
    if ((rc = phase_dedup(ctx, nullptr, (const Cand *)cand_recv_dev, n_cand_recv, true))) return rc;
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch, 0, 128 * 8, ctx->stream));
    if (n_cand_recv > 0) {
        hipLaunchKernelGGL(k_winner_route, dim3(grid_for(n_cand_recv, 256)), dim3(256), 0, ctx->stream, (const Cand *)cand_recv_dev,
                           (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, ctx->nranks, ctx->d_scratch, (int64_t *)nullptr, 0);
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[6], ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    DevStats s2 = *ctx->h_st;
    if (s2.overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    unsigned long long cur[64];
    unsigned long long acc = 0;
    for (int r = 0; r < ctx->nranks; r++) { cur[r] = acc; winner_send_counts[r] = (int64_t)ctx->h_scratch[r]; acc += ctx->h_scratch[r]; }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_scratch, cur, 64 * 8, hipMemcpyHostToDevice, ctx->stream));
    if (n_cand_recv > 0) {
        hipLaunchKernelGGL(k_winner_route, dim3(grid_for(n_cand_recv, 256)), dim3(256), 0, ctx->stream, (const Cand *)cand_recv_dev,
                           (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, ctx->nranks, ctx->d_scratch,
                           (int64_t *)winner_send_buf, 1);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    record_timings(ctx);
    if ((rc = finish_outputs(ctx, (int64_t)s2.n_touched, 0, nullptr, out_memory, out))) return rc;
    // hm_last_counts: this rank's share of the batch (state keys created, records merged, tiles emitted, path)
    ctx->last_counts[0] = (int64_t)s2.n_state_new;
    ctx->last_counts[1] = n_tile_recv;
    ctx->last_counts[2] = (int64_t)s2.n_touched;
    ctx->last_counts[3] = ctx->stage_table ? 1 : 0;
    ctx->last_counts[4] = ctx->stage_table ? ctx->table_evicted : 0;
    ctx->last_counts[5] = ctx->stage_sent;
    ctx->last_binned = 0;
    if (ctx->stage_agg_rows >= (int64_t(1) << 16)) {   // this rank's rows and owned keys (summed over ranks next batch)
        ctx->prev_agg_rows = ctx->stage_agg_rows;
        ctx->prev_keys = (int64_t)s2.n_touched;
        ctx->merge_coop = s2.n_touched > 0 && 2 * s2.n_state_new < s2.n_touched;
    }
    if ((rc = state_account(ctx, ctx->wm_cur))) return rc;
    DevStats sf{};
    sf.n_valid = ctx->stage_sizes.n_valid;
    sf.n_late = ctx->stage_sizes.n_late;
    sf.max_ts_ms = ctx->stage_gmax_ms;
    fill_stats(ctx, out, ctx->stage_n_in, sf, late_wm);
    advance_watermark(ctx, ctx->stage_gmax_ms);
    ctx->stage = 3;
    return HM_OK;
}

int hm_stage_finish(hm_ctx *ctx, const void *winner_recv_dev, int64_t n_winner_recv, int32_t out_memory, hm_batch_out *out) {
    if (!ctx || !out || n_winner_recv < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 3) return set_err(ctx, HM_E_STATE, "hm_stage_finish before hm_stage_merge");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    out->n_latest = n_winner_recv;
    // the rank's latest rows into the context (library-owned like hm_process_batch's), so that the positions sink
    // (hm_encode_position_updates, hm_last_latest_buckets) encodes this rank's winners from its own columns: the
    // origin rank writes the positions_latest statements of the rows it holds (heatmap_stream.py:209-235)
    if ((rc = ensure(ctx, ctx->rows, std::max<int64_t>(n_winner_recv, 1) * 8))) return rc;
    if (n_winner_recv > 0)
        HIPCHK(ctx, hipMemcpyAsync(ctx->rows.p, winner_recv_dev, n_winner_recv * 8, hipMemcpyDeviceToDevice, ctx->stream));
    ctx->last_n_latest = n_winner_recv;
    ctx->last_vk = ctx->stage_I.vk;
    ctx->last_ts = ctx->stage_I.ts;
    ctx->last_lat = ctx->stage_I.lat;
    ctx->last_lon = ctx->stage_I.lon;
    if (out_memory == HM_MEM_DEVICE) {
        out->latest_row = (const int64_t *)ctx->rows.p;
    } else {
        if ((size_t)n_winner_recv > ctx->h_rows_cap || !ctx->h_rows) {
            size_t want = host_cap_for(ctx->h_rows ? ctx->h_rows_cap : 0, (size_t)n_winner_recv), dummy = 0;
            if ((rc = ensure_host(ctx, &ctx->h_rows, dummy, want, 8))) return rc;
            ctx->h_rows_cap = want;
        }
        if (n_winner_recv > 0)
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_rows, winner_recv_dev, n_winner_recv * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        std::sort((int64_t *)ctx->h_rows, (int64_t *)ctx->h_rows + n_winner_recv);
        out->latest_row = (const int64_t *)ctx->h_rows;
    }
    ctx->stage = 0;
    return HM_OK;
}
