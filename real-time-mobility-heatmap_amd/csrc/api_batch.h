// C ABI: hm_create / hm_destroy / hm_process_batch and the timing / count queries (include/mobheat.h).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

int32_t hm_abi_version(void) { return HM_ABI_VERSION; }

int hm_create(const hm_config *cfg, hm_ctx **out) {
    g_create_err.clear();
    if (!cfg || !out) { g_create_err = "null argument"; return HM_E_INVALID; }
    if (cfg->abi_version != HM_ABI_VERSION) { g_create_err = "ABI version mismatch"; return HM_E_INVALID; }
    if (cfg->h3_res < 0 || cfg->h3_res > 15) { g_create_err = "h3_res out of range"; return HM_E_INVALID; }
    // (windows of at least a second: TILE_MINUTES is whole minutes in the reference, heatmap_stream.py:29; the
    // window registry's LDS cache relies on |ts / tile_us| < 2^51)
    if (cfg->tile_us < 1000000 || cfg->watermark_delay_ms < 0) { g_create_err = "bad tile/watermark"; return HM_E_INVALID; }
    if (cfg->shard_count < 0 || cfg->shard_count > 64 || cfg->shard_rank < 0 ||
        (cfg->shard_count > 0 && cfg->shard_rank >= cfg->shard_count) || (cfg->shard_count == 0 && cfg->shard_rank != 0)) {
        g_create_err = "bad shard_rank/shard_count";
        return HM_E_INVALID;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        g_create_err = "no HIP device available (the mobheat hot path requires an MI355X GPU)";
        return HM_E_HIP;
    }
    if (cfg->device < 0 || cfg->device >= ndev) { g_create_err = "device ordinal out of range"; return HM_E_INVALID; }
    hm_ctx *ctx = new hm_ctx();
    ctx->cfg = *cfg;
    ctx->device = cfg->device;
    ctx->shard_rank = cfg->shard_rank;
    ctx->shard_count = cfg->shard_count;
    auto fail = [&](const char *what) {
        g_create_err = std::string(what) + ": " + ctx->err;
        hm_destroy(ctx);
        return HM_E_HIP;
    };
    if (hipSetDevice(ctx->device) != hipSuccess) { ctx->err = "hipSetDevice"; return fail("create"); }
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->side_stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->merge_stream, hipStreamNonBlocking) != hipSuccess) { ctx->err = "stream"; return fail("create"); }
    for (auto &e : ctx->pipe_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    if (hipEventCreateWithFlags(&ctx->pipe_rb, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->pipe_done, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    for (auto &e : ctx->side_ev)
        if (hipEventCreate(&e) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    if (hipEventCreateWithFlags(&ctx->winfo_ev, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    for (auto &e : ctx->h2d_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    for (auto &e : ctx->export_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    for (auto &e : ctx->stm_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    // k_merge_owned's resident tags live in dynamic LDS of up to MO_TAG_MAX bytes (merge_sorted)
    if (hipFuncSetAttribute((const void *)k_merge_owned<EventRec, false>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<SortedRec, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<SortedRec, false>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<SortedRec, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess ||
        hipFuncSetAttribute((const void *)k_merge_owned<EventRec, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, MO_TAG_MAX) != hipSuccess) {
        ctx->err = "merge LDS attribute";
        return fail("create");
    }
    for (auto &e : ctx->ev)
        if (hipEventCreate(&e) != hipSuccess) { ctx->err = "event"; return fail("create"); }
    if (upload_tables() != hipSuccess) { ctx->err = "tables"; return fail("create"); }
    for (int variant = 0; variant < 2; variant++) {
        const void *kern = variant ? (const void *)k_ingest<true> : (const void *)k_ingest<false>;
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, IG_THREADS, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) {
            ctx->err = "occupancy query";
            return fail("create");
        }
        // the occupancy API can report one block per CU more than fits (MI355X_MICROARCH.md, correctness
        // boundaries: SGPR counts 81-112); k_ingest is persistent, so an extra block per CU would only run once
        // a resident one finished.  Bound it by the LDS each block takes.
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, kern) == hipSuccess && fa.sharedSizeBytes > 0)
            per_cu = std::min<int>(per_cu, (int)(163840 / fa.sharedSizeBytes));
        // k_ingest<true> (the binned ingest) runs 2 workgroups per CU, not the 6 that fit: its time is its records'
        // scattered stores and bin-cursor atomics, which fewer waves in flight contend less for -- 5.41-5.50 ms at 2
        // against 5.62-5.67 at 3 and 5.88-5.97 at 6 (profiles/r5/r5wg2/, r5wg3/; 1 per CU: ~7 ms); the unbinned
        // kernel keeps every resident block (VALU and latency bound).  MOBHEAT_INGEST_WG_PER_CU overrides (tuning)
        if (variant) per_cu = std::min(per_cu, 2);
        if (const char *m = getenv("MOBHEAT_INGEST_WG_PER_CU")) {
            int w = 0, cap = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&cap, kern, IG_THREADS, 0);
            if (fa.sharedSizeBytes > 0) cap = std::min<int>(cap, (int)(163840 / fa.sharedSizeBytes));
            w = atoi(m);
            if (w > 0) per_cu = std::max(1, std::min(cap, w));
        }
        if (getenv("MOBHEAT_DEBUG"))
            fprintf(stderr, "mobheat: k_ingest<%d> %d blocks/CU x %d CUs (LDS %zu B, %d VGPRs)\n", variant, per_cu, cus,
                    fa.sharedSizeBytes, fa.numRegs);
        (variant ? ctx->ingest_grid_bin : ctx->ingest_grid) = std::max(1, per_cu) * std::max(1, cus);
        ctx->n_cus = std::max(1, cus);
    }
    // MOBHEAT_INGEST_MODE=direct|table|binned pins the aggregation path (tests): the direct path with its partition
    // pass, table mode, or the direct path binned in k_ingest at any batch size; default: adaptive
    if (const char *m = getenv("MOBHEAT_INGEST_MODE"))
        ctx->ingest_mode = !strcmp(m, "direct") ? 1 : !strcmp(m, "table") ? 2 : !strcmp(m, "binned") ? 3 : 0;
    if (const char *m = getenv("MOBHEAT_MERGE_GRID")) ctx->merge_grid = std::max(0, atoi(m));
    // MOBHEAT_DEDUP_STREAM=main runs the dedup on the main stream after the merge path (its cost to the overlapped
    // kernels, measured by the bench with and without it); default: the side stream
    if (const char *m = getenv("MOBHEAT_DEDUP_STREAM")) ctx->dedup_main = !strcmp(m, "main");
    if (const char *m = getenv("MOBHEAT_DEDUP_EARLY")) ctx->early_ok = strcmp(m, "0") != 0;
    if (const char *m = getenv("MOBHEAT_OFFSETS_EARLY")) ctx->offsets_early = strcmp(m, "0") != 0;
    if (const char *m = getenv("MOBHEAT_STAGE_SELF")) ctx->self_hold_ok = strcmp(m, "copy") != 0;
    if (const char *m = getenv("MOBHEAT_DEDUP_DENSE")) ctx->dense_ok = strcmp(m, "0") != 0;
    if (const char *m = getenv("MOBHEAT_COOP_PREDICT")) ctx->coop_predict = strcmp(m, "0") != 0;
    if (const char *m = getenv("MOBHEAT_SUBBINS")) ctx->subbins_mode = !strcmp(m, "0") ? 0 : !strcmp(m, "1") ? 1 : 2;
    // MOBHEAT_PIPELINE: unset / 0 never pipelines a batch (the default: slower on the bench, host_pipe.h), K >= 2
    // pipelines every binned batch in K chunks (tests, A/B), "auto": batches of >= PIPE_MIN_ROWS rows in PIPE_CHUNKS chunks
    if (const char *m = getenv("MOBHEAT_PIPELINE")) ctx->pipe_mode = !strcmp(m, "auto") ? -1 : std::max(0, std::min(atoi(m), hm_ctx::PIPE_MAX));
    if (const char *m = getenv("MOBHEAT_TEST_SLAB_CAP")) ctx->test_slab_cap = (unsigned)std::max(0, atoi(m));
    // the registry, its census and the batch statistics side by side (one reset, one readback after k_ingest)
    if (hipMalloc(&ctx->d_wreg, REG_BLOCK_BYTES) != hipSuccess || !(ctx->d_wcount = ctx->d_wreg + WREG_SLOTS + 1) ||
        !(ctx->d_st = (DevStats *)(ctx->d_wreg + 2 * (WREG_SLOTS + 1))) ||
        hipHostMalloc(&ctx->h_wreg, REG_BLOCK_BYTES, hipHostMallocDefault) != hipSuccess ||
        !(ctx->h_wcount = ctx->h_wreg + WREG_SLOTS + 1) || !(ctx->h_st = (DevStats *)(ctx->h_wreg + 2 * (WREG_SLOTS + 1))) ||
        hipMalloc(&ctx->d_winfo, (WREG_SLOTS + 1) * sizeof(WInfo) + sizeof(WiCacheImg)) != hipSuccess ||
        hipHostMalloc(&ctx->h_winfo, (WREG_SLOTS + 1) * sizeof(WInfo) + sizeof(WiCacheImg), hipHostMallocDefault) != hipSuccess ||
        hipMemset(ctx->d_winfo, 0, (WREG_SLOTS + 1) * sizeof(WInfo)) != hipSuccess ||
        hipMemset(ctx->d_winfo + WREG_SLOTS + 1, 0xff, sizeof(WiCacheImg)) != hipSuccess) {
        ctx->err = "window registry alloc";
        return fail("create");
    }
    if (hipMalloc(&ctx->d_scratch, 256 * 8) != hipSuccess || hipHostMalloc(&ctx->h_scratch, 256 * 8) != hipSuccess ||
        hipHostMalloc(&ctx->h_bincur, ((RP_BINS << SUB_BITS) + 1) * 4, hipHostMallocDefault) != hipSuccess) {
        ctx->err = "stats alloc";
        return fail("create");
    }
    if (hipMemset(ctx->d_scratch, 0, 256 * 8) != hipSuccess) { ctx->err = "scratch init"; return fail("create"); }
    if (hipMalloc(&ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc)) != hipSuccess ||
        hipHostMalloc(&ctx->h_gmap, GMAP_SLOTS * sizeof(GenDesc), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&ctx->d_cmap, GMAP_SLOTS * sizeof(WinCount)) != hipSuccess ||
        hipMalloc(&ctx->d_glist, GMAP_SLOTS * sizeof(GenDesc)) != hipSuccess ||
        hipHostMalloc(&ctx->h_glist, GMAP_SLOTS * sizeof(GenDesc), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&ctx->h_cmap, GMAP_SLOTS * sizeof(WinCount), hipHostMallocDefault) != hipSuccess ||
        hipMemset(ctx->d_gmap, 0, GMAP_SLOTS * sizeof(GenDesc)) != hipSuccess) {
        ctx->err = "window map alloc";
        return fail("create");
    }
    ctx->dfused.used_word = DUSED_WORD;
    ctx->dfull.used_word = FULL_USED_WORD;
    // batch_capacity_hint: reserve the per-batch buffers now (multi-GB allocations would otherwise land in the
    // first batches; each later batch only grows them when it is larger)
    if (cfg->batch_capacity_hint > 0) {
        const int64_t n = cfg->batch_capacity_hint;
        const size_t tp = sizeof(TilePartial);
        (void)tp;
        if (ensure(ctx, ctx->flags, n) || ensure(ctx, ctx->win, n) || ensure(ctx, ctx->rows, n * 8) ||
            ensure(ctx, ctx->keys, n * 8) || ensure(ctx, ctx->slow, n * 4) ||
            ensure(ctx, ctx->parts_sorted, n * sizeof(EventRec)) ||
            ensure(ctx, ctx->s_cell, n * 8) || ensure(ctx, ctx->s_ws, n * 8) || ensure(ctx, ctx->s_cnt, n * 8) ||
            ensure(ctx, ctx->s_sp, n * 8) || ensure(ctx, ctx->s_spn, n) || ensure(ctx, ctx->s_lon, n * 8) ||
            ensure(ctx, ctx->s_lat, n * 8) || ensure_outputs(ctx, n))
            return fail("create");
        // the full dedup table a batch of n rows may need (when k_ingest's cache-sized table gives up: C5's first
        // batch paid a 17-GB hipMalloc inside the batch)
        if (dedup_prepare(ctx, ctx->dfull, n, false)) return fail("create");
    }
    if (cfg->state_arena_bytes > 0) {
        ctx->arena_bytes = (size_t)cfg->state_arena_bytes & ~(size_t)255;
        if (dev_malloc(ctx, (void **)&ctx->arena, ctx->arena_bytes, "state arena") != hipSuccess) {
            (void)hipGetLastError();
            ctx->arena = nullptr;
            ctx->err = "state arena: out of device memory";
            return fail("create");
        }
        hipLaunchKernelGGL(k_zero16, dim3(256 * 32), dim3(256), 0, ctx->stream, (uint4 *)ctx->arena, (int64_t)(ctx->arena_bytes / 16));
    }
    // state_capacity_hint: one window table for that many keys, reserved now into the pool (a 70-GB table costs
    // ~2 s in hipMalloc: C5's first batch)
    if (cfg->state_capacity_hint > 0) {
        Geo geo{};
        geo.log2cap = ilog2(next_pow2((uint64_t)std::max<int64_t>(2 * cfg->state_capacity_hint, 1024)));
        TileSlot *t = nullptr;
        if (table_acquire(ctx, geo, &t) || table_release(ctx, t, geo.log2cap)) return fail("create");
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) { ctx->err = "sync"; return fail("create"); }
    *out = ctx;
    return HM_OK;
}

void hm_destroy(hm_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side_stream) (void)hipStreamSynchronize(ctx->side_stream);
    if (ctx->merge_stream) (void)hipStreamSynchronize(ctx->merge_stream);
    DevBuf *bufs[] = {&ctx->pl_cur, &ctx->pl_slow, &ctx->pl_O, &ctx->pl_cnt, &ctx->pl_T, &ctx->in_lat, &ctx->in_lon, &ctx->in_ts, &ctx->in_speed, &ctx->in_sv, &ctx->in_vkey, &ctx->in_rv,
                      &ctx->cell, &ctx->wstart, &ctx->flags, &ctx->win, &ctx->rows, &ctx->block_counts, &ctx->block_offs,
                      &ctx->partials, &ctx->cands, &ctx->slow, &ctx->parts_sorted, &ctx->parts_regrow, &ctx->parts_regrow_sorted, &ctx->stage_meta, &ctx->stage_C, &ctx->stage_P,
                      &ctx->stage_SO, &ctx->stage_SP, &ctx->stage_T, &ctx->cands_recv, &ctx->stage_tmp, &ctx->rp_H, &ctx->rp_O,
                      &ctx->rp_btot, &ctx->rp_boff,
                      &ctx->s_cell, &ctx->s_ws, &ctx->s_cnt, &ctx->s_sp, &ctx->s_spn, &ctx->s_lon, &ctx->s_lat, &ctx->bin_cnt, &ctx->bin_off, &ctx->dfused.used, &ctx->dfull.used, &ctx->o_cell, &ctx->o_ws, &ctx->o_cnt, &ctx->o_sp, &ctx->o_spn,
                      &ctx->o_lon, &ctx->o_lat, &ctx->td_sizes, &ctx->td_off, &ctx->td_btot, &ctx->td_boff, &ctx->td_bytes,
                      &ctx->td_params, &ctx->gapbuf, &ctx->keys, &ctx->bin_cur, &ctx->agg_bucket, &ctx->agg_cursor,
                      &ctx->jd_bytes, &ctx->jd_offs, &ctx->jd_scratch, &ctx->jd_lat, &ctx->jd_lon, &ctx->jd_ts, &ctx->jd_speed,
                      &ctx->jd_sv, &ctx->jd_rv, &ctx->jd_vkey, &ctx->jd_poff, &ctx->jd_plen, &ctx->jd_voff, &ctx->jd_vlen,
                      &ctx->jd_un, &ctx->jd_unrows, &ctx->jd_patch,
                      &ctx->lb_set, &ctx->lb_list, &ctx->dense};
    for (DevBuf *b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (hm_ctx::Dict *d : {&ctx->jd_prov, &ctx->jd_veh}) {
        for (DevBuf *b : {&d->tab, &d->slot_of, &d->occ, &d->slots, &d->code_of_slot, &d->clen, &d->coff, &d->cbytes, &d->btot, &d->boff})
            if (b->p) (void)hipFree(b->p);
        if (d->h_off) (void)hipHostFree(d->h_off);
        if (d->h_bytes) (void)hipHostFree(d->h_bytes);
    }
    for (auto &g : ctx->gens)
        if (!in_arena(ctx, g.tab)) (void)hipFree(g.tab);
    for (auto &pt : ctx->pool)
        if (!in_arena(ctx, pt.first)) (void)hipFree(pt.first);
    if (ctx->arena) (void)hipFree(ctx->arena);
    if (ctx->d_wreg) (void)hipFree(ctx->d_wreg);   // (d_wcount, d_st / h_wcount, h_st: inside these)
    if (ctx->h_wreg) (void)hipHostFree(ctx->h_wreg);
    if (ctx->d_winfo) (void)hipFree(ctx->d_winfo);
    if (ctx->h_winfo) (void)hipHostFree(ctx->h_winfo);
    if (ctx->d_gmap) (void)hipFree(ctx->d_gmap);
    if (ctx->h_gmap) (void)hipHostFree(ctx->h_gmap);
    if (ctx->d_cmap) (void)hipFree(ctx->d_cmap);
    if (ctx->d_glist) (void)hipFree(ctx->d_glist);
    if (ctx->h_glist) (void)hipHostFree(ctx->h_glist);
    if (ctx->h_cmap) (void)hipHostFree(ctx->h_cmap);
    if (ctx->dfused.tab) (void)hipFree(ctx->dfused.tab);
    if (ctx->dfull.tab) (void)hipFree(ctx->dfull.tab);
    void *hbufs[] = {ctx->h_cell, ctx->h_ws, ctx->h_cnt, ctx->h_sp, ctx->h_spn, ctx->h_lon, ctx->h_lat, ctx->h_rows,
                     ctx->h_td_bytes, ctx->h_td_off};
    for (void *p : hbufs)
        if (p) (void)hipHostFree(p);
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    if (ctx->h_scratch) (void)hipHostFree(ctx->h_scratch);
    if (ctx->h_bincur) (void)hipHostFree(ctx->h_bincur);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->h2d_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
    for (auto &e : ctx->export_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->stm_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
    if (ctx->side_stream) (void)hipStreamDestroy(ctx->side_stream);
    if (ctx->merge_stream) (void)hipStreamDestroy(ctx->merge_stream);
    for (auto &e : ctx->pipe_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->pipe_rb) (void)hipEventDestroy(ctx->pipe_rb);
    if (ctx->pipe_done) (void)hipEventDestroy(ctx->pipe_done);
    for (auto &e : ctx->side_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->winfo_ev) (void)hipEventDestroy(ctx->winfo_ev);
    if (ctx->ext_ev) (void)hipEventDestroy(ctx->ext_ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *hm_last_error(const hm_ctx *ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int hm_last_timings(const hm_ctx *ctx, double *ms, int32_t n) {
    if (!ctx || !ms) return HM_E_INVALID;
    for (int i = 0; i < n && i < 8; i++) ms[i] = ctx->timings[i];
    for (int i = 8; i < n && i < 14; i++) ms[i] = ctx->host_ms[i - 8];
    return HM_OK;
}

// the state's version: bumped when a batch's merge begins (a failed call that left it unchanged did not touch the state)
int64_t hm_state_version(const hm_ctx *ctx) { return ctx ? (int64_t)ctx->seq : -1; }

int hm_last_counts(const hm_ctx *ctx, int64_t *c, int32_t n) {
    if (!ctx || !c) return HM_E_INVALID;
    for (int i = 0; i < n && i < 6; i++) c[i] = ctx->last_counts[i];
    if (n > 6) c[6] = ctx->n_allocs;
    if (n > 7) c[7] = ctx->n_frees;
    if (n > 8) c[8] = ctx->last_binned;
    if (n > 9) c[9] = ctx->staged ? ctx->stage_self_recs : 0;
    if (n > 10) c[10] = ctx->staged ? 0 : ctx->last_pipe_chunks;
    return HM_OK;
}


int hm_process_batch(hm_ctx *ctx, int64_t epoch_id, const hm_batch_in *in, int32_t out_memory, hm_batch_out *out) {
    if (!ctx || !in || !out || in->n < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (in->n > MAX_BATCH_ROWS) return set_err(ctx, HM_E_INVALID, "batch of %lld events exceeds %lld", (long long)in->n, (long long)MAX_BATCH_ROWS);
    if (in->n > 0 && (!in->lat || !in->lon || !in->ts_us || !in->vkey))
        return set_err(ctx, HM_E_INVALID, "lat, lon, ts_us and vkey are required");
    if (ctx->shard_count > 1)
        return set_err(ctx, HM_E_STATE, "a context of shard %d of %d runs the stage API (its state is that shard's keys)",
                       ctx->shard_rank, ctx->shard_count);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    host_batch_begin(ctx);
    const BatchClock clock_(ctx);
    memset(out, 0, sizeof(*out));
    ctx->gmap_ready = false;
    ctx->epoch = epoch_id;
    ctx->last_n_latest = -1;
    ctx->staged = false;
    ctx->stage = 0;
    int rc;
    // 1. evict with this batch's eviction watermark happened at the end of the previous batch (see below)
    int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    Inputs I;
    I.n = in->n;
    if ((rc = stage_inputs(ctx, in, &I.lat, &I.lon, &I.ts, &I.sp, &I.sv, &I.vk, &I.rv))) return rc;
    // 2. snap + window registry + event keys
    const bool sub = ctx->subbins_mode == 1 || (ctx->subbins_mode == 2 && ctx->merge_coop);
    const bool early = ctx->early_ok && !ctx->dedup_main;
    // a large binned batch is pipelined (host_pipe.h): its chunks' ingest overlaps the previous chunk's merge, and the
    // rows come back densified (piped); else the ingest, then the merge path below
    const int K = pipe_chunks_for(ctx, I);
    bool piped = false;
    ctx->last_pipe_chunks = 0;
    if (K > 1) {
        bool to_table = false;
        if ((rc = process_pipelined(ctx, I, late_wm, sub, K, early, to_table))) return rc;
        piped = !to_table;
    } else if ((rc = phase_local(ctx, I, late_wm, true, sub, early, ctx->offsets_early))) {
        return rc;
    }
    DevStats s1 = *ctx->h_st;
    const int64_t n_agg = (int64_t)s1.n_valid - (int64_t)s1.n_late;
    // the aggregation path of this batch (table mode: two LDS passes first; direct: every row a record)
    const bool table = !piped && choose_table(ctx, n_agg, s1.sample_max_run);
    ctx->last_table = table;
    // 4. dedup over the batch's valid rows -- on the side stream, concurrently with step 3 (the rerun of the max on a
    // full table, after the fused one gave up, prepares that table on the main stream: it stays there)
    ctx->dedup_side = s1.dedup_retry == 0 && !ctx->dedup_main;
    // (launched behind k_ingest -- phase_local, early_dedup -- or else here, ahead of the partition: 1-3% faster on the
    // bench than launched after the merge path's kernels, ~5% faster than overlapping the merge only, 2-4% faster than
    // behind k_ev_hist -- profiles/r3/r3ab12/, r3ab13/)
    if (ctx->dedup_early && !ctx->dedup_side)   // (the fused max gave up: the rerun below overwrites its outputs)
        HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[2], 0));
    if (ctx->dedup_side && !ctx->dedup_early) {
        HIPCHK(ctx, hipEventRecord(ctx->side_ev[0], ctx->stream));
        HIPCHK(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->side_ev[0], 0));
        if ((rc = launch_side_dedup(ctx, &I))) return rc;
    }
    // 3. aggregate, merge into state + emit (table mode: two LDS passes first; direct: every row a record)
    if (table) {
        int64_t n_parts = 0;
        if ((rc = phase_table(ctx, I, n_agg, &n_parts))) return rc;
        HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
        if ((rc = merge_partials(ctx, (const TilePartial *)ctx->partials.p, n_parts))) return rc;
    } else if (!piped) {
        HIPCHK(ctx, hipEventRecord(ctx->ev[2], ctx->stream));
        if ((rc = merge_events(ctx, I, n_agg))) return rc;
    }
    if (!ctx->dedup_side) {
        if ((rc = phase_dedup(ctx, &I, nullptr, I.n, true))) return rc;
    } else {
        HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[2], 0));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[6], ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    // (the window map's key counts for state_account, read back in the same wait)
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_gmap, ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    ctx->gmap_ready = true;
    ctx->dedup_seen = (int64_t)ctx->h_scratch[ctx->dlast->used_word];   // distinct vkeys of this batch
    DevStats s2 = *ctx->h_st;
    if (s2.overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    if (s2.bad_vkey) return set_err(ctx, HM_E_INVALID, "vkey UINT64_MAX is reserved (%llu rows)", s2.bad_vkey);
    int64_t n_rows = (int64_t)ctx->h_scratch[255];
    ctx->last_n_latest = n_rows;
    ctx->last_vk = I.vk;
    ctx->last_ts = I.ts;
    ctx->last_lat = I.lat;
    ctx->last_lon = I.lon;
    record_timings(ctx);
    if ((rc = finish_outputs(ctx, (int64_t)s2.n_touched, n_rows, (const int64_t *)ctx->rows.p, out_memory, out))) return rc;
    ctx->last_counts[0] = (int64_t)s2.n_state_new;
    ctx->last_counts[1] = ctx->n_partials_merged;
    ctx->last_counts[2] = (int64_t)s2.n_touched;
    ctx->last_counts[3] = table ? 1 : 0;
    ctx->last_counts[4] = table ? ctx->table_evicted : 0;
    ctx->last_counts[5] = 0;
    ctx->last_binned = !table && ctx->binned ? 1 : 0;
    // the next batch's aggregation path is chosen from this one's cardinality
    if (n_agg >= (int64_t(1) << 16)) {
        ctx->prev_agg_rows = n_agg;
        ctx->prev_keys = (int64_t)s2.n_touched;
        ctx->merge_coop = s2.n_touched > 0 && 2 * s2.n_state_new < s2.n_touched;
    }
    // 5. eviction after emission with this batch's watermark (lazy: see hm_ctx), then advance the watermark
    if ((rc = state_account(ctx, ctx->wm_cur))) return rc;
    fill_stats(ctx, out, in->n, s1, late_wm);
    advance_watermark(ctx, s1.max_ts_ms);
    return HM_OK;
}
