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
    if (ctx->shard_count == 0 && ctx->gens.empty()) {   // (fixed by the first batch; a context holding state keeps its own)
        ctx->shard_rank = rank;
        ctx->shard_count = nranks;
    }
    if (ctx->shard_count != nranks && !(ctx->shard_count <= 1 && nranks == 1))
        return set_err(ctx, HM_E_STATE, "the context is shard %d of %d, not %d of %d", ctx->shard_rank, ctx->shard_count, rank, nranks);
    if (ctx->shard_count > 1 && ctx->shard_rank != rank)
        return set_err(ctx, HM_E_STATE, "the context is shard %d of %d, not %d of %d", ctx->shard_rank, ctx->shard_count, rank, nranks);
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
    // (large batches: bins of region fields, fused; the local dedup launched on the side stream behind k_ingest, so that
    // it runs while the ranks all-gather their summaries -- hm_stage_send waits for it)
    if ((rc = phase_local(ctx, I, late_wm, true, false, ctx->early_ok && !ctx->dedup_main))) return rc;
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

int64_t hm_stage_send_capacity(int64_t n_rows, int32_t nranks) {
    if (n_rows < 0 || nranks < 1) return 0;
    // records (<= 48 B) and candidates (32 B) of every row, per chunk its header, counts, census and alignment
    return n_rows * (HM_TILE_REC_BYTES + HM_CAND_REC_BYTES) + (int64_t)nranks * (sizeof(ChunkHdr) + 96 + CENSUS_WORDS * 4) +
           (int64_t)RP_BINS * 4;
}

// chunk layouts of this rank's send: records and candidates per destination -> headers, starts, total bytes
static int stage_layout(hm_ctx *ctx, const int64_t *recs, const int64_t *cands, bool table, int64_t cap,
                        std::vector<ChunkHdr> &hdr, std::vector<int64_t> &start, int64_t *send_bytes) {
    const int W = ctx->nranks;
    hdr.resize(W);
    start.resize(W + 1);
    int64_t off = 0;
    for (int o = 0; o < W; o++) {
        const int64_t bins = table ? 0 : (int64_t)(shard_lo(o + 1, W) - shard_lo(o, W));
        hdr[o] = chunk_layout(recs[o], cands[o], table ? (int64_t)sizeof(TilePartial) : (int64_t)sizeof(EventRec), bins);
        start[o] = off;
        send_bytes[o] = hdr[o].bytes;
        off += hdr[o].bytes;
    }
    start[W] = off;
    if (off > cap) return set_err(ctx, HM_E_INVALID, "send buffer of %lld bytes too small (%lld needed)", (long long)cap, (long long)off);
    return HM_OK;
}

int hm_stage_send(hm_ctx *ctx, const int64_t *summaries, void *send_buf, int64_t send_cap, int64_t *send_bytes,
                  hm_stage_sizes *sizes) {
    if (!ctx || !summaries || !send_bytes || send_cap < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 1) return set_err(ctx, HM_E_STATE, "hm_stage_send before hm_stage_ingest");
    const Inputs &I = ctx->stage_I;
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
    // local dedup over rows -> local winners -> candidates, counted per owner (launched in hm_stage_ingest unless the
    // fused max gave up: then rerun here after it)
    if (ctx->dedup_early) HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[2], 0));
    if ((!ctx->dedup_early || s1.dedup_retry != 0) && (rc = phase_dedup(ctx, &I, nullptr, I.n, s1.dedup_retry != 0))) return rc;
    if ((rc = ensure(ctx, ctx->cands, std::max<int64_t>(I.n, 1) * sizeof(Cand)))) return rc;
    hipLaunchKernelGGL(k_make_cands, dim3(grid_for(std::max<int64_t>(I.n, 1), 256)), dim3(256), 0, ctx->stream,
                       (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, I.vk, I.ts, ctx->rank, (Cand *)ctx->cands.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch, 0, 128 * 8, ctx->stream));
    const int gb = grid_for(std::max<int64_t>(I.n, 1), 256);
    hipLaunchKernelGGL(k_part_count<Cand>, dim3(gb), dim3(256), 0, ctx->stream, (const Cand *)ctx->cands.p, ctx->d_scratch + 255,
                       W, ctx->d_scratch + 64);
    HIPCHK(ctx, hipGetLastError());
    // the tile records grouped by destination: table mode, the partials partitioned by owner (stage_tmp); direct path,
    // the records grouped by region field -- k_ingest's slabs, or the partition with one bin per region field -- whose
    // destinations are contiguous ranges of bins
    HIPCHK(ctx, hipEventRecord(ctx->ev[8], ctx->stream));
    int64_t stride = 1, slab = 0;
    if (table) {
        if ((rc = ensure(ctx, ctx->stage_tmp, std::max<int64_t>(n_records, 1) * sizeof(TilePartial)))) return rc;
        int64_t ntiles = 1;
        if (n_records > 0) {
            if ((rc = partition<TilePartial, TilePartial>(ctx, (const TilePartial *)ctx->partials.p, n_records, ntiles, W,
                                                          (TilePartial *)ctx->stage_tmp.p)))
                return rc;
            hipLaunchKernelGGL(k_digit_starts, dim3(1), dim3(128), 0, ctx->stream, (const unsigned long long *)ctx->rp_O.p, ntiles,
                               W + 1, ctx->d_scratch + 128);
        } else {
            HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + 128, 0, (W + 1) * 8, ctx->stream));
        }
    } else if (I.n > 0) {
        if (ctx->binned) {   // k_ingest's slabs: bin b's records at b * slab_cap, its count in bin_cur[b]
            slab = ctx->slab_cap;
            if ((rc = ensure(ctx, ctx->rp_O, (RP_BINS + 1) * 8)) ||
                (rc = scan_counts(ctx, (const unsigned *)ctx->bin_cur.p, RP_BINS + 1, (unsigned long long *)ctx->rp_O.p)))
                return rc;
        } else {             // the partition with one bin per region field (WInfo without table geometry: binp 0)
            int64_t ntiles;
            if ((rc = winfo_upload(ctx, false)) || (rc = keys_complete(ctx, I)) ||
                (rc = ev_partition(ctx, (const uint64_t *)ctx->keys.p, I.n, &I, ntiles)))
                return rc;
            stride = ntiles;
        }
        hipLaunchKernelGGL(k_shard_starts, dim3(1), dim3(128), 0, ctx->stream, (const unsigned long long *)ctx->rp_O.p, stride, W,
                           ctx->d_scratch + 128);
    } else {
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + 128, 0, (W + 1) * 8, ctx->stream));
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_scratch, ctx->d_scratch, 256 * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "device hash table overflow");
    if (ctx->h_st->bad_vkey) return set_err(ctx, HM_E_INVALID, "vkey UINT64_MAX is reserved");
    ctx->dedup_seen = (int64_t)ctx->h_scratch[ctx->dlast->used_word];
    std::vector<int64_t> recs(W), cands(W);
    int64_t n_sent = 0;
    for (int o = 0; o < W; o++) {
        recs[o] = (int64_t)(ctx->h_scratch[128 + o + 1] - ctx->h_scratch[128 + o]);
        cands[o] = (int64_t)ctx->h_scratch[64 + o];
        n_sent += recs[o];
    }
    // the local -> global window slot map
    std::vector<unsigned short> gmap(WREG_SLOTS, 0);
    bool same_slots = true;
    for (int w = 0; w < WREG_SLOTS; w++) {
        const unsigned long long we = ctx->h_wreg[w];
        if (!we) continue;
        const auto it = std::find(ctx->stage_gwreg.begin(), ctx->stage_gwreg.end(), we);
        if (it == ctx->stage_gwreg.end()) {
            if (ctx->h_wcount[w]) return set_err(ctx, HM_E_STATE, "a window of this rank is missing from the global registry");
            continue;
        }
        gmap[w] = (unsigned short)(it - ctx->stage_gwreg.begin());
        same_slots = same_slots && (gmap[w] == w || !ctx->h_wcount[w]);
    }
    // the records of the bins this rank owns stay in its slabs when their keys need no rewrite (binned; every local
    // window slot is its global one -- the registry hashes a window to the same slot on every rank unless two of the
    // batch's windows collide): the chunk it addresses to itself then carries their counts and census only
    const bool self_held = ctx->self_hold_ok && !table && ctx->binned && I.n > 0 && same_slots;
    ctx->stage_self_held = self_held;
    ctx->stage_self_recs = self_held ? recs[ctx->rank] : 0;
    std::vector<int64_t> chunk_recs(recs);
    if (self_held) chunk_recs[ctx->rank] = 0;
    std::vector<ChunkHdr> hdr;
    std::vector<int64_t> start;
    if ((rc = stage_layout(ctx, chunk_recs.data(), cands.data(), table, send_cap, hdr, start, send_bytes))) return rc;
    if (start[W] > 0 && !send_buf) return set_err(ctx, HM_E_INVALID, "send buffer is required");
    // headers, chunk starts, the window slot map -> device
    const size_t meta = (size_t)W * sizeof(ChunkHdr) + (size_t)(W + 1) * 8 + WREG_SLOTS * sizeof(unsigned short);
    if ((rc = ensure(ctx, ctx->stage_meta, meta))) return rc;
    std::vector<uint8_t> hm(meta);
    memcpy(hm.data(), hdr.data(), (size_t)W * sizeof(ChunkHdr));
    memcpy(hm.data() + (size_t)W * sizeof(ChunkHdr), start.data(), (size_t)(W + 1) * 8);
    memcpy(hm.data() + (size_t)W * sizeof(ChunkHdr) + (size_t)(W + 1) * 8, gmap.data(), WREG_SLOTS * sizeof(unsigned short));
    HIPCHK(ctx, hipMemcpyAsync(ctx->stage_meta.p, hm.data(), meta, hipMemcpyHostToDevice, ctx->stream));
    const ChunkHdr *d_hdr = (const ChunkHdr *)ctx->stage_meta.p;
    const int64_t *d_start = (const int64_t *)((uint8_t *)ctx->stage_meta.p + (size_t)W * sizeof(ChunkHdr));
    const unsigned short *d_gmap = (const unsigned short *)((uint8_t *)ctx->stage_meta.p + (size_t)W * sizeof(ChunkHdr) + (size_t)(W + 1) * 8);
    uint8_t *out = (uint8_t *)send_buf;
    if (start[W] > 0) {
        hipLaunchKernelGGL(k_stage_chunk_init, dim3(W), dim3(256), 0, ctx->stream, d_hdr, d_start, out);
        if (table) {
            for (int o = 0, first = 0; o < W; o++) {
                if (recs[o])
                    HIPCHK(ctx, hipMemcpyAsync(out + start[o] + hdr[o].recs_off, (const TilePartial *)ctx->stage_tmp.p + first,
                                               recs[o] * sizeof(TilePartial), hipMemcpyDeviceToDevice, ctx->stream));
                first += (int)recs[o];
            }
        } else if (n_sent > 0) {
            // (a world of one holds every bin itself: its census is the ingest's, written from the host)
            const bool census_host = self_held && W == 1;
            hipLaunchKernelGGL(k_stage_pack, dim3(RP_BINS), dim3(256), 0, ctx->stream, (const EventRec *)ctx->parts_sorted.p, slab,
                               (const unsigned long long *)ctx->rp_O.p, stride, d_gmap, W, self_held ? ctx->rank : -1,
                               census_host ? 0 : 1, d_start, out);
            if (census_host) {
                std::vector<unsigned> &cen = ctx->stage_cen;   // (kept until the send's synchronization below)
                cen.assign(CENSUS_WORDS, 0u);
                for (int w = 0; w < WREG_SLOTS; w++)
                    if (ctx->h_wcount[w]) cen[gmap[w]] += (unsigned)ctx->h_wcount[w];
                HIPCHK(ctx, hipMemcpyAsync(out + start[ctx->rank] + chunk_census_off((int64_t)RP_BINS), cen.data(),
                                           CENSUS_WORDS * 4, hipMemcpyHostToDevice, ctx->stream));
            }
        }
        // candidates: per-destination cursors (in Cand units) into the chunks
        unsigned long long cur[64];
        for (int o = 0; o < W; o++) cur[o] = (unsigned long long)((start[o] + hdr[o].cands_off) / (int64_t)sizeof(Cand));
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_scratch + 64, cur, W * 8, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_part_scatter<Cand>, dim3(gb), dim3(256), 0, ctx->stream, (const Cand *)ctx->cands.p, ctx->d_scratch + 255,
                           W, ctx->d_scratch + 64, (Cand *)out);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[9], ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));   // (the caller's collective reads the buffer on its own stream)
    ctx->stage_agg_rows = n_agg;
    ctx->stage_sent = n_sent;
    hm_stage_sizes z{};
    z.table_mode = table ? 1 : 0;
    z.n_tile_records = n_sent;
    z.n_self_records = ctx->stage_self_recs;
    for (int o = 0; o < W; o++) z.n_cands += cands[o];
    z.global_batch_max_event_ms = ctx->stage_gmax_ms;
    z.n_valid = (int64_t)s1.n_valid;
    z.n_late = (int64_t)s1.n_late;
    ctx->stage_sizes = z;
    if (sizes) *sizes = z;
    ctx->stage = 2;
    return HM_OK;
}

// the multi-GPU owner's direct path: every sender's chunk holds the records of the owner's region fields in order
// (counts per field) -> census per global window -> window tables (range geometry) -> each bin merged from its
// senders' segments -> rows
static int merge_received_chunks(hm_ctx *ctx, const uint8_t *recv, int64_t recv_total, const int64_t *d_off,
                                 const std::vector<ChunkHdr> &hdr, int64_t n) {
    int rc;
    const int W = ctx->nranks;
    if (n > MAX_BATCH_ROWS) return set_err(ctx, HM_E_INVALID, "%lld received records exceed %lld", (long long)n, (long long)MAX_BATCH_ROWS);
    ctx->n_partials_merged = n;
    if ((rc = merge_begin(ctx, n))) return rc;
    if (n == 0) return merge_nothing(ctx);
    memcpy(ctx->h_wreg, ctx->stage_gwreg.data(), WREG_SLOTS * sizeof(unsigned long long));
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wcount[w] && !ctx->h_wreg[w]) return set_err(ctx, HM_E_INVALID, "received a record of an unknown window slot");
    std::vector<WinCount> census;
    census_of_registry(ctx, census);
    if ((rc = gens_prepare(ctx, census, true)) || (rc = winfo_upload(ctx, true))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], ctx->stream));
    const unsigned lo = shard_lo(ctx->rank, W), bins = shard_lo(ctx->rank + 1, W) - lo;
    const int64_t m = (int64_t)W * (bins + 1);
    if ((rc = ensure(ctx, ctx->stage_C, m * 4)) || (rc = ensure(ctx, ctx->stage_P, m * 8)) ||
        (rc = ensure(ctx, ctx->stage_SO, (size_t)RP_BINS * W * 8)) || (rc = ensure(ctx, ctx->stage_SP, (size_t)RP_BINS * W * 4)) ||
        (rc = ensure(ctx, ctx->stage_T, (RP_BINS + 1) * 4)) || (rc = ensure(ctx, ctx->rp_O, (RP_BINS + 1) * 8)))
        return rc;
    hipLaunchKernelGGL(k_stage_counts, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, recv, d_off, W, bins, (unsigned *)ctx->stage_C.p);
    if ((rc = scan_counts(ctx, (const unsigned *)ctx->stage_C.p, m, (unsigned long long *)ctx->stage_P.p))) return rc;
    HIPCHK(ctx, hipMemsetAsync((unsigned *)ctx->stage_T.p + RP_BINS, 0, 4, ctx->stream));
    hipLaunchKernelGGL(k_stage_segments, dim3(grid_for(RP_BINS, 256)), dim3(256), 0, ctx->stream, recv, d_off,
                       (const unsigned long long *)ctx->stage_P.p, W, lo, bins, ctx->stage_self_held ? ctx->rank : -1,
                       (const EventRec *)ctx->parts_sorted.p, (int64_t)ctx->slab_cap, (unsigned long long *)ctx->stage_SO.p,
                       (unsigned *)ctx->stage_SP.p, (unsigned *)ctx->stage_T.p);
    if ((rc = scan_counts(ctx, (const unsigned *)ctx->stage_T.p, RP_BINS + 1, (unsigned long long *)ctx->rp_O.p))) return rc;
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], ctx->stream));
    Segs seg;
    seg.SO = (const unsigned long long *)ctx->stage_SO.p;
    seg.SP = (const unsigned *)ctx->stage_SP.p;
    seg.nseg = W;
    {   // (the senders' segments in the receive buffer, the self-held ones in this rank's slabs)
        const unsigned long long r0 = (unsigned long long)(uintptr_t)recv, s0 = (unsigned long long)(uintptr_t)ctx->parts_sorted.p;
        seg.bounds = SegBounds{{r0, s0}, {r0 + (unsigned long long)recv_total, s0 + ctx->parts_sorted.bytes}};
    }
    if ((rc = merge_sorted<EventRec>(ctx, n, 1, 0, (const EventRec *)recv, seg))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], ctx->stream));
    if ((rc = rows_densify(ctx, 1))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], ctx->stream));
    (void)hdr;
    return HM_OK;
}

int hm_stage_merge(hm_ctx *ctx, const void *recv_buf, const int64_t *recv_bytes, int32_t out_memory, hm_batch_out *out,
                   void *winner_send_buf, int64_t winner_send_cap, int64_t *winner_send_counts) {
    if (!ctx || !out || !winner_send_counts || !recv_bytes || winner_send_cap < 0)
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->stage != 2) return set_err(ctx, HM_E_STATE, "hm_stage_merge before hm_stage_send");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const int W = ctx->nranks;
    memset(out, 0, sizeof(*out));
    const int64_t late_wm = ctx->cfg.late_uses_prev_watermark ? ctx->wm_prev : ctx->wm_cur;
    // the chunks: offsets, headers (and the direct path's census) read back
    std::vector<int64_t> off(W + 1, 0);
    for (int s = 0; s < W; s++) {
        if (recv_bytes[s] < 0 || (recv_bytes[s] & 7)) return set_err(ctx, HM_E_INVALID, "chunk %d: %lld bytes", s, (long long)recv_bytes[s]);
        off[s + 1] = off[s] + recv_bytes[s];
    }
    if (off[W] > 0 && !recv_buf) return set_err(ctx, HM_E_INVALID, "receive buffer is required");
    const uint8_t *recv = (const uint8_t *)recv_buf;
    const bool table = ctx->stage_table;
    const unsigned bins = shard_lo(ctx->rank + 1, W) - shard_lo(ctx->rank, W);
    const size_t meta = (size_t)(2 * W + 1) * 8 + (size_t)W * sizeof(ChunkHdr);
    if ((rc = ensure(ctx, ctx->stage_meta, meta))) return rc;
    int64_t *d_off = (int64_t *)ctx->stage_meta.p;
    int64_t *d_bytes = d_off + W + 1;
    ChunkHdr *d_hdr = (ChunkHdr *)(d_bytes + W);
    HIPCHK(ctx, hipMemcpyAsync(d_off, off.data(), (W + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(d_bytes, recv_bytes, W * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_stage_headers, dim3(16), dim3(256), 0, ctx->stream, recv, d_off, d_bytes, W, d_hdr,
                       table ? (int64_t)0 : chunk_census_off(bins), ctx->d_wcount);
    HIPCHK(ctx, hipGetLastError());
    std::vector<ChunkHdr> hdr(W);
    HIPCHK(ctx, hipMemcpyAsync(hdr.data(), d_hdr, W * sizeof(ChunkHdr), hipMemcpyDeviceToHost, ctx->stream));
    if (!table) HIPCHK(ctx, hipMemcpyAsync(ctx->h_wcount, ctx->d_wcount, WREG_SLOTS * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    int64_t n_rec = 0, n_cand = 0;
    for (int s = 0; s < W; s++) {
        const ChunkHdr &h = hdr[s];
        const ChunkHdr want = chunk_layout(h.records, h.cands, table ? (int64_t)sizeof(TilePartial) : (int64_t)sizeof(EventRec),
                                           table ? 0 : (int64_t)bins);
        if (h.magic != CHUNK_MAGIC || h.records < 0 || h.cands < 0 || memcmp(&h, &want, sizeof h) != 0 || h.bytes != recv_bytes[s])
            return set_err(ctx, HM_E_INVALID, "chunk of rank %d is malformed", s);
        n_rec += h.records;
        n_cand += h.cands;
    }
    if (winner_send_cap < n_cand || (n_cand > 0 && !winner_send_buf))
        return set_err(ctx, HM_E_INVALID, "winner buffer of %lld rows for %lld candidates", (long long)winner_send_cap, (long long)n_cand);
    // the candidates (and table mode's partials) of all senders, contiguous
    if ((rc = ensure(ctx, ctx->cands_recv, std::max<int64_t>(n_cand, 1) * sizeof(Cand)))) return rc;
    if (table && (rc = ensure(ctx, ctx->stage_tmp, std::max<int64_t>(n_rec, 1) * sizeof(TilePartial)))) return rc;
    for (int s = 0, c = 0, r = 0; s < W; s++) {
        if (hdr[s].cands)
            HIPCHK(ctx, hipMemcpyAsync((Cand *)ctx->cands_recv.p + c, recv + off[s] + hdr[s].cands_off, hdr[s].cands * sizeof(Cand),
                                       hipMemcpyDeviceToDevice, ctx->stream));
        if (table && hdr[s].records)
            HIPCHK(ctx, hipMemcpyAsync((TilePartial *)ctx->stage_tmp.p + r, recv + off[s] + hdr[s].recs_off,
                                       hdr[s].records * sizeof(TilePartial), hipMemcpyDeviceToDevice, ctx->stream));
        c += (int)hdr[s].cands;
        r += (int)hdr[s].records;
    }
    const Cand *cands = (const Cand *)ctx->cands_recv.p;
    if (table) rc = merge_partials(ctx, (const TilePartial *)ctx->stage_tmp.p, n_rec);
    else rc = merge_received_chunks(ctx, recv, off[W], d_off, hdr, n_rec + ctx->stage_self_recs);   // (+ the self-held ones)
    if (rc) return rc;
    // owner-side dedup over received candidates
    if ((rc = phase_dedup(ctx, nullptr, cands, n_cand, true))) return rc;
    HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch, 0, 128 * 8, ctx->stream));
    if (n_cand > 0) {
        hipLaunchKernelGGL(k_winner_route, dim3(grid_for(n_cand, 256)), dim3(256), 0, ctx->stream, cands,
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
    if (n_cand > 0) {
        hipLaunchKernelGGL(k_winner_route, dim3(grid_for(n_cand, 256)), dim3(256), 0, ctx->stream, cands,
                           (const int64_t *)ctx->rows.p, ctx->d_scratch + 255, ctx->nranks, ctx->d_scratch,
                           (int64_t *)winner_send_buf, 1);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    record_timings(ctx);
    if ((rc = finish_outputs(ctx, (int64_t)s2.n_touched, 0, nullptr, out_memory, out))) return rc;
    // hm_last_counts: this rank's share of the batch (state keys created, records merged, tiles emitted, path)
    ctx->last_counts[0] = (int64_t)s2.n_state_new;
    ctx->last_counts[1] = n_rec + (table ? 0 : ctx->stage_self_recs);
    ctx->last_counts[2] = (int64_t)s2.n_touched;
    ctx->last_counts[3] = ctx->stage_table ? 1 : 0;
    ctx->last_counts[4] = ctx->stage_table ? ctx->table_evicted : 0;
    ctx->last_counts[5] = ctx->stage_sent;
    ctx->last_binned = ctx->binned ? 1 : 0;
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

// the caller's collective stream -> the library's stream, without a host synchronization (distributed.py: RCCL's
// all_to_all of the chunks on torch's current stream, then hm_stage_merge / hm_stage_finish reading what it received)
int hm_stream_wait(hm_ctx *ctx, void *stream) {
    if (!ctx) return HM_E_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (!ctx->ext_ev) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ext_ev, hipEventDisableTiming));
    HIPCHK(ctx, hipEventRecord(ctx->ext_ev, (hipStream_t)stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ext_ev, 0));
    return 0;
}
