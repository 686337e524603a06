// C ABI: tile-state checkpoint export / import (Spark's state store, heatmap_stream.py:37,244).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// ---- tile-state checkpoint (Spark's state store behind checkpointLocation, heatmap_stream.py:37,244) ----
// Export: every live window's keys dumped by k_dump_gen (the growth path's kernel) into one GrowRec array, copied
// to the caller; the touched word (this context's batch sequence) is cleared on the device -- it means nothing
// elsewhere (a host loop over the records cost ~10 ms per 1e7 keys).
static void state_info_of(const hm_ctx *ctx, hm_state_info *info, int64_t n_keys) {
    memset(info, 0, sizeof(*info));
    info->epoch_id = ctx->epoch;
    info->n_keys = n_keys;
    info->watermark_ms = ctx->wm_cur;
    info->prev_watermark_ms = ctx->wm_prev;
    info->tile_us = ctx->cfg.tile_us;
    info->watermark_delay_ms = ctx->cfg.watermark_delay_ms;
    info->h3_res = ctx->cfg.h3_res;
}

// every live window's keys (only_seq != 0: those the batch with that sequence touched) into recs[0, n)
static int state_dump(hm_ctx *ctx, hm_state_rec *recs, int64_t n, unsigned only_seq) {
    int rc;
    ctx->touched_dump_seq = ctx->export_dump_n = -1;   // (parts_regrow is overwritten)
    if ((rc = ensure(ctx, ctx->parts_regrow, std::max<int64_t>(n, 1) * sizeof(GrowRec)))) return rc;
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + REGROW_WORD, 0, 8, ctx->stream));
    for (const auto &g : ctx->gens) {
        const GenDesc d = gen_desc(g);
        hipLaunchKernelGGL(k_dump_gen, dim3(grid_for(int64_t(1) << g.log2cap, 256 * DUMP_PER)), dim3(256), 0, ctx->stream, d,
                           (GrowRec *)ctx->parts_regrow.p, ctx->d_scratch + REGROW_WORD, only_seq, true);
    }
    HIPCHK(ctx, hipGetLastError());
    unsigned long long dumped = 0;
    HIPCHK(ctx, hipMemcpyAsync(&dumped, ctx->d_scratch + REGROW_WORD, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if ((int64_t)dumped != n) return set_err(ctx, HM_E_STATE, "state dump found %llu keys, expected %lld", dumped, (long long)n);
    if (n > 0 && recs) HIPCHK(ctx, hipMemcpy(recs, ctx->parts_regrow.p, n * sizeof(GrowRec), hipMemcpyDeviceToHost));
    return HM_OK;
}

int hm_state_export(hm_ctx *ctx, hm_state_info *info, hm_state_rec *recs, int64_t cap) {
    static_assert(sizeof(hm_state_rec) == sizeof(GrowRec), "hm_state_rec mirrors GrowRec");
    if (!ctx || !info) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 0) return set_err(ctx, HM_E_STATE, "hm_state_export between stage calls");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int64_t n = 0;
    for (const auto &g : ctx->gens) n += g.keys;
    state_info_of(ctx, info, n);
    if (!recs) return HM_OK;
    if (cap < n) return set_err(ctx, HM_E_INVALID, "state of %lld keys does not fit %lld records", (long long)n, (long long)cap);
    return n == 0 ? HM_OK : state_dump(ctx, recs, n, 0);
}

// Incremental checkpoint (Spark's state store writes a delta file per version): the keys the last batch touched, with
// their cumulative values; together with an older full export and the deltas between, the state after this batch is
// the last-written record of every key whose window end > info.prev_watermark_ms (the batch's eviction watermark).
int hm_state_export_touched(hm_ctx *ctx, hm_state_info *info, hm_state_rec *recs, int64_t cap, int64_t *n_out) {
    if (!ctx || !info || !n_out) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 0) return set_err(ctx, HM_E_STATE, "hm_state_export_touched between stage calls");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int64_t live = 0;
    for (const auto &g : ctx->gens) live += g.keys;
    state_info_of(ctx, info, live);
    // the last batch's touched keys that are still live (a touched key of an evicted window went with its table);
    // the dump is kept for the call that fetches it (the caller's first call sizes its buffer: one scan of the
    // tables per export, not two)
    int64_t n = 0;
    if (ctx->touched_dump_seq == (int64_t)ctx->seq) {
        n = ctx->touched_dump_n;
    } else if (ctx->seq > 0 && !ctx->gens.empty()) {
        int rc;
        if ((rc = ensure(ctx, ctx->parts_regrow, std::max<int64_t>(live, 1) * sizeof(GrowRec)))) return rc;
        ctx->export_dump_n = -1;   // (parts_regrow is overwritten)
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + REGROW_WORD, 0, 8, ctx->stream));
        for (const auto &g : ctx->gens) {
            const GenDesc d = gen_desc(g);
            hipLaunchKernelGGL(k_dump_gen, dim3(grid_for(int64_t(1) << g.log2cap, 256 * DUMP_PER)), dim3(256), 0, ctx->stream, d,
                               (GrowRec *)ctx->parts_regrow.p, ctx->d_scratch + REGROW_WORD, seq32(ctx), true);
        }
        HIPCHK(ctx, hipGetLastError());
        unsigned long long dumped = 0;
        HIPCHK(ctx, hipMemcpyAsync(&dumped, ctx->d_scratch + REGROW_WORD, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        n = (int64_t)dumped;
        ctx->touched_dump_seq = (int64_t)ctx->seq;
        ctx->touched_dump_n = n;
    }
    *n_out = n;
    if (!recs) return HM_OK;
    if (cap < n) return set_err(ctx, HM_E_INVALID, "%lld touched keys do not fit %lld records", (long long)n, (long long)cap);
    if (n > 0) HIPCHK(ctx, hipMemcpy(recs, ctx->parts_regrow.p, n * sizeof(GrowRec), hipMemcpyDeviceToHost));
    return HM_OK;
}

// The export in two halves, for a file writer that overlaps the copy with the statements' encode: begin dumps the
// state (every live key, or the last batch's touched keys) into the device dump buffer and returns its size; copy
// moves records [first, first + count) of that dump to host memory on copy_stream (idle between batches), so that it
// can run on another thread while hm_encode_* run on this context's stream.
int hm_state_export_begin(hm_ctx *ctx, hm_state_info *info, int32_t touched_only, int64_t *n_out) {
    if (!ctx || !info || !n_out) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 0) return set_err(ctx, HM_E_STATE, "hm_state_export_begin between stage calls");
    int rc;
    int64_t n = 0;
    if (touched_only) {
        if ((rc = hm_state_export_touched(ctx, info, nullptr, 0, &n))) return rc;
        if (n > 0 && ctx->touched_dump_seq != (int64_t)ctx->seq) return set_err(ctx, HM_E_STATE, "touched dump lost");
    } else {
        if ((rc = hm_state_export(ctx, info, nullptr, 0))) return rc;
        n = info->n_keys;
        if (n > 0) {
            if ((rc = state_dump(ctx, nullptr, n, 0))) return rc;
        }
    }
    ctx->export_dump_n = n;
    ctx->export_dump_seq = ctx->seq;
    *n_out = n;
    return HM_OK;
}

int hm_state_export_copy(hm_ctx *ctx, hm_state_rec *recs, int64_t first, int64_t count) {
    if (!ctx || first < 0 || count < 0 || (count > 0 && !recs)) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->export_dump_n < 0 || ctx->export_dump_seq != ctx->seq)
        return set_err(ctx, HM_E_STATE, "hm_state_export_copy without an hm_state_export_begin after the last batch");
    if (first + count > ctx->export_dump_n)
        return set_err(ctx, HM_E_INVALID, "records [%lld, %lld) outside the dump of %lld", (long long)first,
                       (long long)(first + count), (long long)ctx->export_dump_n);
    if (count == 0) return HM_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipMemcpyAsync(recs, (const GrowRec *)ctx->parts_regrow.p + first, (size_t)count * sizeof(GrowRec),
                               hipMemcpyDeviceToHost, ctx->copy_stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->copy_stream));
    return HM_OK;
}

// The copies enqueued up front (before the statements' encode is: one hardware queue serves both streams, so a copy
// enqueued after the encode's would land after all of its pieces), one event per slice; the writer waits slice by slice.
int hm_state_export_copy_async(hm_ctx *ctx, hm_state_rec *recs, int64_t first, int64_t count, int32_t slot) {
    if (!ctx || first < 0 || count < 0 || (count > 0 && !recs) || slot < 0 || slot >= hm_ctx::EXPORT_SLICES)
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->export_dump_n < 0 || ctx->export_dump_seq != ctx->seq)
        return set_err(ctx, HM_E_STATE, "hm_state_export_copy without an hm_state_export_begin after the last batch");
    if (first + count > ctx->export_dump_n)
        return set_err(ctx, HM_E_INVALID, "records [%lld, %lld) outside the dump of %lld", (long long)first,
                       (long long)(first + count), (long long)ctx->export_dump_n);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (count > 0)
        HIPCHK(ctx, hipMemcpyAsync(recs, (const GrowRec *)ctx->parts_regrow.p + first, (size_t)count * sizeof(GrowRec),
                                   hipMemcpyDeviceToHost, ctx->copy_stream));
    HIPCHK(ctx, hipEventRecord(ctx->export_ev[slot], ctx->copy_stream));
    return HM_OK;
}

int hm_state_export_copy_wait(hm_ctx *ctx, int32_t slot) {
    if (!ctx || slot < 0 || slot >= hm_ctx::EXPORT_SLICES) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipEventSynchronize(ctx->export_ev[slot]));
    return HM_OK;
}

// Import: the records' windows get tables sized as a batch's new windows would be, then the records are merged
// through the growth path (partition + k_merge_owned in rehash mode: no counting, no rows, no touched update).
int hm_state_import(hm_ctx *ctx, const hm_state_info *info, const hm_state_rec *recs) {
    if (!ctx || !info || info->n_keys < 0 || (info->n_keys > 0 && !recs))
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->epoch != -1 || ctx->stage != 0 || !ctx->gens.empty())
        return set_err(ctx, HM_E_STATE, "hm_state_import into a context that already processed a batch");
    if (info->h3_res != ctx->cfg.h3_res || info->tile_us != ctx->cfg.tile_us || info->watermark_delay_ms != ctx->cfg.watermark_delay_ms)
        return set_err(ctx, HM_E_INVALID, "checkpoint of res %d / window %lld us / delay %lld ms does not match the context",
                       info->h3_res, (long long)info->tile_us, (long long)info->watermark_delay_ms);
    const int64_t n = info->n_keys;
    if (n >= (int64_t)UINT32_MAX) return set_err(ctx, HM_E_INVALID, "%lld state records exceed 2^32-2", (long long)n);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    // census per window + record checks (the device trusts them: a zero cell is a gap, reserved is touched)
    std::vector<std::pair<unsigned long long, int64_t>> wins;
    size_t last = 0;
    const int64_t T = ctx->cfg.tile_us;
    for (int64_t i = 0; i < n; i++) {
        const hm_state_rec &r = recs[i];
        if (r.cell == 0 || r.reserved != 0 || r.count < 1 || r.n_speed < 0 || r.n_speed > r.count ||
            ((r.window_start_us % T) + T) % T != 0)
            return set_err(ctx, HM_E_INVALID, "state record %lld is malformed", (long long)i);
        // a shard context's tables cover only its own region fields (range geometry): a foreign key would index
        // below its table's first region
        if (ctx->shard_count > 1 && tile_owner_of(tile_hash(r.cell, r.window_start_us), ctx->shard_count) != ctx->shard_rank)
            return set_err(ctx, HM_E_INVALID, "state record %lld (cell %llx) belongs to rank %d, not to this shard %d of %d",
                           (long long)i, (unsigned long long)r.cell,
                           tile_owner_of(tile_hash(r.cell, r.window_start_us), ctx->shard_count), ctx->shard_rank,
                           ctx->shard_count);
        const unsigned long long we = wenc_of(r.window_start_us);
        if (last >= wins.size() || wins[last].first != we) {
            last = 0;
            while (last < wins.size() && wins[last].first != we) last++;
            if (last == wins.size()) {
                if ((int)wins.size() >= GMAP_SLOTS / 2)
                    return set_err(ctx, HM_E_OVERFLOW, "checkpoint holds more than %d windows", GMAP_SLOTS / 2);
                wins.emplace_back(we, 0);
            }
        }
        wins[last].second++;
    }
    int rc;
    for (const auto &w : wins) {
        Geo geo = gen_geometry(ctx, w.second, w.second, range_mode(ctx, false));
        TileSlot *t = nullptr;
        if ((rc = table_acquire(ctx, geo, &t))) return rc;
        ctx->gens.push_back(gen_of(w.first, t, geo, w.second, 0));
    }
    if ((rc = gens_upload(ctx))) return rc;
    if (n > 0) {
        ctx->touched_dump_seq = -1;
        if ((rc = ensure(ctx, ctx->parts_regrow, n * sizeof(GrowRec)))) return rc;
        HIPCHK(ctx, hipMemcpy(ctx->parts_regrow.p, recs, n * sizeof(GrowRec), hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemsetAsync(&ctx->d_st->overflow, 0, 8, ctx->stream));
        int64_t ntiles;
        if ((rc = partition<GrowRec, GrowRec>(ctx, (const GrowRec *)ctx->parts_regrow.p, n, ntiles))) return rc;
        if ((rc = merge_sorted<GrowRec>(ctx, n, ntiles))) return rc;
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow while restoring the state");
    }
    ctx->state_size = n;
    ctx->wm_cur = info->watermark_ms;
    ctx->wm_prev = info->prev_watermark_ms;
    ctx->epoch = info->epoch_id;
    return HM_OK;
}
