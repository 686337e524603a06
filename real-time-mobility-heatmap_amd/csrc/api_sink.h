// C ABI: tiles and positions as MongoDB update statements encoded on the GPU (heatmap_stream.py:159-235).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// ---- tiles as MongoDB update statements (bson_docs.h; reference heatmap_stream.py:164-196) ----
int hm_last_windows(hm_ctx *ctx, int64_t *window_start_us, int64_t cap, int64_t *n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !window_start_us)) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    *n = (int64_t)ctx->batch_windows.size();
    for (int64_t i = 0; i < *n && i < cap; i++) window_start_us[i] = ctx->batch_windows[i];
    return HM_OK;
}

static int64_t civil_year(int64_t s) {   // proleptic Gregorian year of a second count since 1970 (host)
    int64_t z = s / 86400 - ((s % 86400) < 0) + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097, doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365, doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    return yoe + era * 400 + (mp >= 10);
}

// the statements in ctx->td_bytes / td_off: handed out on the device or copied to pinned host buffers
static int statements_out(hm_ctx *ctx, int64_t n, int64_t total, int32_t out_memory, const uint8_t **bytes,
                          const int64_t **offsets, int64_t *n_docs) {
    int rc;
    unsigned long long *off = (unsigned long long *)ctx->td_off.p;
    *n_docs = n;
    if (out_memory != HM_MEM_HOST && out_memory != HM_MEM_DEVICE && out_memory != HM_MEM_HOST_STREAM)
        return set_err(ctx, HM_E_INVALID, "bad memory kind %d", out_memory);
    if (ctx->stm_pieces) {   // (a streamed encode's pieces still landing: they finish before the buffers are reused)
        ctx->stm_pieces = 0;
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    }
    if (out_memory == HM_MEM_DEVICE) {
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        *bytes = (const uint8_t *)ctx->td_bytes.p;
        *offsets = (const int64_t *)ctx->td_off.p;
        return HM_OK;
    }
    size_t dummy = 0;
    if ((size_t)total + 16 > ctx->h_td_bytes_cap || !ctx->h_td_bytes) {
        const size_t want = (size_t)total + total / 4 + 4096;
        if ((rc = ensure_host(ctx, &ctx->h_td_bytes, dummy, want, 1))) return rc;
        ctx->h_td_bytes_cap = want;
    }
    if ((size_t)n + 1 > ctx->h_td_off_cap || !ctx->h_td_off) {
        const size_t want = (size_t)n + n / 4 + 1024;
        if ((rc = ensure_host(ctx, &ctx->h_td_off, dummy, want, 8))) return rc;
        ctx->h_td_off_cap = want;
    }
    *bytes = (const uint8_t *)ctx->h_td_bytes;
    *offsets = (const int64_t *)ctx->h_td_off;
    if (out_memory == HM_MEM_HOST_STREAM) {
        // the offsets first (the sink cuts its commands from them), then the bytes in at most 64 pieces of >= 32 MiB,
        // each marked by an event hm_statements_wait blocks on
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_td_off, off, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        const int64_t piece = std::max<int64_t>(int64_t(32) << 20, (total + hm_ctx::STM_PIECES - 1) / hm_ctx::STM_PIECES);
        int k = 0;
        for (int64_t o = 0; o < total; o += piece, k++) {
            HIPCHK(ctx, hipMemcpyAsync((uint8_t *)ctx->h_td_bytes + o, (const uint8_t *)ctx->td_bytes.p + o,
                                       (size_t)std::min(piece, total - o), hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, hipEventRecord(ctx->stm_ev[k], ctx->stream));
        }
        ctx->stm_pieces = k;
        ctx->stm_piece = piece;
        ctx->stm_total = total;
        return HM_OK;
    }
    // (in 128-MiB pieces: a checkpoint writer's export copies on copy_stream interleave with them instead of queueing
    // behind one 3.7-GB copy -- the state file's disk writes then start while the statements are still landing)
    constexpr int64_t PIECE = int64_t(128) << 20;
    for (int64_t o = 0; o < total; o += PIECE)
        HIPCHK(ctx, hipMemcpyAsync((uint8_t *)ctx->h_td_bytes + o, (const uint8_t *)ctx->td_bytes.p + o, (size_t)std::min(PIECE, total - o),
                                   hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_td_off, off, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    *bytes = (const uint8_t *)ctx->h_td_bytes;
    *offsets = (const int64_t *)ctx->h_td_off;
    return HM_OK;
}

int hm_statements_wait(hm_ctx *ctx, int64_t upto) {
    if (!ctx || upto < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    const int pieces = ctx->stm_pieces;
    if (!pieces) return upto == 0 ? HM_OK : set_err(ctx, HM_E_STATE, "hm_statements_wait without a streamed encode");
    if (upto > ctx->stm_total) return set_err(ctx, HM_E_INVALID, "%lld bytes of %lld", (long long)upto, (long long)ctx->stm_total);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int last = (int)std::min<int64_t>((upto + ctx->stm_piece - 1) / ctx->stm_piece, pieces);
    for (int k = 0; k < last; k++) HIPCHK(ctx, hipEventSynchronize(ctx->stm_ev[k]));
    return HM_OK;
}

int hm_encode_tile_updates(hm_ctx *ctx, const hm_tile_doc_cfg *cfg, int32_t out_memory, const uint8_t **bytes,
                           const int64_t **offsets, int64_t *n_docs) {
    if (!ctx || !cfg || !bytes || !offsets || !n_docs || cfg->city_len < 0 || (cfg->city_len > 0 && !cfg->city) ||
        cfg->n_windows < 0 || (cfg->n_windows > 0 && (!cfg->window_start_us || !cfg->start_offset_s || !cfg->end_offset_s)))
        return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (cfg->city_len > (1 << 20)) return set_err(ctx, HM_E_INVALID, "city of %d bytes (at most 1 MiB)", cfg->city_len);
    const int64_t n = ctx->last_n_tiles;
    const auto &W = ctx->batch_windows;
    if (cfg->n_windows != (int64_t)W.size()) return set_err(ctx, HM_E_INVALID, "%lld window offsets for %zu windows", (long long)cfg->n_windows, W.size());
    for (size_t k = 0; k < W.size(); k++) {
        if (cfg->window_start_us[k] != W[k]) return set_err(ctx, HM_E_INVALID, "window offsets not in hm_last_windows order");
        const int64_t a = W[k] / 1000000 - (W[k] % 1000000 < 0) + cfg->start_offset_s[k];
        const int64_t b = (W[k] + ctx->cfg.tile_us) / 1000000 + cfg->end_offset_s[k];
        if (civil_year(a) < 1000 || civil_year(a) > 9999 || civil_year(b) > 9999)
            return set_err(ctx, HM_E_INVALID, "window start %lld us: year outside 1000-9999", (long long)W[k]);
        if (W[k] % 1000000 != 0) return set_err(ctx, HM_E_INVALID, "window start %lld us is not a whole second", (long long)W[k]);
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const int nw = (int)W.size();
    // parameters: city bytes (padded to 16), then the window table (3 x nw int64)
    const size_t cbytes = ((size_t)cfg->city_len + 15) & ~(size_t)15;
    const size_t pbytes = cbytes + (size_t)nw * 24 + 16;
    if ((rc = ensure(ctx, ctx->td_params, pbytes)) || (rc = ensure(ctx, ctx->td_off, (n + 1) * 8)) ||
        (rc = ensure(ctx, ctx->td_sizes, std::max<int64_t>(n, 1) * 4)))
        return rc;
    std::vector<uint8_t> hp(pbytes, 0);
    if (cfg->city_len) memcpy(hp.data(), cfg->city, cfg->city_len);
    if (nw) {
        memcpy(hp.data() + cbytes, W.data(), nw * 8);
        memcpy(hp.data() + cbytes + nw * 8, cfg->start_offset_s, nw * 8);
        memcpy(hp.data() + cbytes + nw * 16, cfg->end_offset_s, nw * 8);
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->td_params.p, hp.data(), pbytes, hipMemcpyHostToDevice, ctx->stream));
    TileDocParams P;
    P.city = (const uint8_t *)ctx->td_params.p;
    P.city_len = cfg->city_len;
    P.h3_res = ctx->cfg.h3_res;
    P.tile_us = ctx->cfg.tile_us;
    P.ttl_ms = cfg->ttl_ms;
    P.win_start_us = (const int64_t *)((uint8_t *)ctx->td_params.p + cbytes);
    P.off_start_s = P.win_start_us + nw;
    P.off_end_s = P.win_start_us + 2 * nw;
    P.n_win = nw;
    unsigned long long *off = (unsigned long long *)ctx->td_off.p;
    int64_t total = 0;
    if (n > 0) {
        if (nw == 0) return set_err(ctx, HM_E_STATE, "tiles without windows");
        hipLaunchKernelGGL(k_tile_doc_sizes, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, (const uint64_t *)ctx->o_cell.p,
                           (const int64_t *)ctx->o_ws.p, (const int64_t *)ctx->o_cnt.p, n, (unsigned *)ctx->td_sizes.p);
        const int64_t nb = (n + SC_PER - 1) / SC_PER;
        if ((rc = ensure(ctx, ctx->td_btot, nb * 4)) || (rc = ensure(ctx, ctx->td_boff, nb * 8))) return rc;
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_sizes.p, n, off,
                           (unsigned *)ctx->td_btot.p);
        hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_btot.p, nb,
                           (unsigned long long *)ctx->td_boff.p, off + n);
        hipLaunchKernelGGL(k_scan_add, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, off, n, (const unsigned long long *)ctx->td_boff.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(&total, off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if ((rc = ensure(ctx, ctx->td_bytes, total + 16))) return rc;
        // LDS staging sized by the longest statement this city/resolution can produce (int64 count, 16 hex
        // digits): occupancy is bounded by it (~400 B per statement -> 3 workgroups per CU)
        TileDocParams Ph = P;
        Ph.city = (const uint8_t *)cfg->city;
        Ph.win_start_us = W.data();
        Ph.off_start_s = cfg->start_offset_s;
        Ph.off_end_s = cfg->end_offset_s;
        const int max_doc = tile_statement(nullptr, Ph, ~0ull, W[0], INT64_MAX, 0.0, 1, 0.0, 0.0);
        if (max_doc > TD_MAX_DOC) {   // a long CITY: no LDS staging
            hipLaunchKernelGGL(k_tile_docs_direct, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, (const uint64_t *)ctx->o_cell.p,
                               (const int64_t *)ctx->o_ws.p, (const int64_t *)ctx->o_cnt.p, (const double *)ctx->o_sp.p,
                               (const uint8_t *)ctx->o_spn.p, (const double *)ctx->o_lon.p, (const double *)ctx->o_lat.p, n,
                               (const unsigned long long *)off, (uint8_t *)ctx->td_bytes.p);
        } else {
            const size_t lds = (size_t)TD_THREADS * ((max_doc + 15) & ~15) + 32;
            if (lds > 65536)
                HIPCHK(ctx, hipFuncSetAttribute((const void *)k_tile_docs, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            hipLaunchKernelGGL(k_tile_docs, dim3(grid_for(n, TD_THREADS)), dim3(TD_THREADS), lds, ctx->stream, P, (const uint64_t *)ctx->o_cell.p,
                               (const int64_t *)ctx->o_ws.p, (const int64_t *)ctx->o_cnt.p, (const double *)ctx->o_sp.p,
                               (const uint8_t *)ctx->o_spn.p, (const double *)ctx->o_lon.p, (const double *)ctx->o_lat.p, n,
                               (const unsigned long long *)off, (uint8_t *)ctx->td_bytes.p);
        }
        HIPCHK(ctx, hipGetLastError());
    } else {
        HIPCHK(ctx, hipMemsetAsync(off, 0, 8, ctx->stream));
        if ((rc = ensure(ctx, ctx->td_bytes, 16))) return rc;
    }
    return statements_out(ctx, n, total, out_memory, bytes, offsets, n_docs);
}

// latest positions of the last hm_process_batch as positions_latest update statements (bson_docs.h)
static int pos_params(hm_ctx *ctx, const hm_position_doc_cfg *cfg, PosDocParams &P, std::vector<uint8_t> &hp) {
    const int64_t np_ = cfg->n_providers, nv = cfg->n_vehicles, nb = cfg->n_buckets;
    if (np_ < 0 || nv < 0 || nb < 0 || (np_ && (!cfg->provider_offsets || !cfg->provider_bytes)) ||
        (nv && (!cfg->vehicle_offsets || !cfg->vehicle_bytes)) || (nb && (!cfg->bucket_ids || !cfg->bucket_offset_s)))
        return set_err(ctx, HM_E_INVALID, "bad position dictionaries");
    for (int64_t k = 1; k < nb; k++)
        if (cfg->bucket_ids[k - 1] >= cfg->bucket_ids[k]) return set_err(ctx, HM_E_INVALID, "bucket ids not ascending");
    const int64_t pb = np_ ? cfg->provider_offsets[np_] : 0, vb = nv ? cfg->vehicle_offsets[nv] : 0;
    for (int64_t k = 0; k < np_; k++)
        if (cfg->provider_offsets[k] < 0 || cfg->provider_offsets[k] > cfg->provider_offsets[k + 1] ||
            cfg->provider_offsets[k + 1] - cfg->provider_offsets[k] > (1 << 20))
            return set_err(ctx, HM_E_INVALID, "provider offsets");
    for (int64_t k = 0; k < nv; k++)
        if (cfg->vehicle_offsets[k] < 0 || cfg->vehicle_offsets[k] > cfg->vehicle_offsets[k + 1] ||
            cfg->vehicle_offsets[k + 1] - cfg->vehicle_offsets[k] > (1 << 20))
            return set_err(ctx, HM_E_INVALID, "vehicle offsets");
    // one device block: offsets (8-B aligned) first, then the string bytes
    const size_t o_p = 0, o_v = o_p + (np_ + 1) * 8, o_bi = o_v + (nv + 1) * 8, o_b = o_bi + nb * 8, o_ps = o_b + nb * 8,
                 o_vs = o_ps + pb;
    hp.assign(o_vs + vb + 8, 0);
    if (np_) memcpy(hp.data() + o_p, cfg->provider_offsets, (np_ + 1) * 8);
    if (nv) memcpy(hp.data() + o_v, cfg->vehicle_offsets, (nv + 1) * 8);
    if (nb) memcpy(hp.data() + o_bi, cfg->bucket_ids, nb * 8);
    if (nb) memcpy(hp.data() + o_b, cfg->bucket_offset_s, nb * 8);
    if (pb) memcpy(hp.data() + o_ps, cfg->provider_bytes, pb);
    if (vb) memcpy(hp.data() + o_vs, cfg->vehicle_bytes, vb);
    int rc;
    if ((rc = ensure(ctx, ctx->td_params, hp.size()))) return rc;
    HIPCHK(ctx, hipMemcpyAsync(ctx->td_params.p, hp.data(), hp.size(), hipMemcpyHostToDevice, ctx->stream));
    uint8_t *d = (uint8_t *)ctx->td_params.p;
    P.p_off = (const int64_t *)(d + o_p);
    P.v_off = (const int64_t *)(d + o_v);
    P.bucket_id = (const int64_t *)(d + o_bi);
    P.bucket_off = (const int64_t *)(d + o_b);
    P.p_bytes = d + o_ps;
    P.v_bytes = d + o_vs;
    P.n_providers = np_;
    P.n_vehicles = nv;
    P.n_buckets = nb;
    return HM_OK;
}

int hm_encode_position_updates(hm_ctx *ctx, const hm_position_doc_cfg *cfg, int32_t out_memory, const uint8_t **bytes,
                               const int64_t **offsets, int64_t *n_docs) {
    if (!ctx || !cfg || !bytes || !offsets || !n_docs) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->last_n_latest < 0) return set_err(ctx, HM_E_STATE, "no hm_process_batch latest rows to encode");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int64_t n = ctx->last_n_latest;
    int rc;
    PosDocParams P;
    std::vector<uint8_t> hp;
    if ((rc = pos_params(ctx, cfg, P, hp))) return rc;
    if ((rc = ensure(ctx, ctx->td_off, (n + 1) * 8)) || (rc = ensure(ctx, ctx->td_sizes, std::max<int64_t>(n, 1) * 4))) return rc;
    unsigned long long *off = (unsigned long long *)ctx->td_off.p;
    int64_t total = 0;
    if (n > 0) {
        const int64_t *rows = (const int64_t *)ctx->rows.p;
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + POSBAD_WORD, 0, 8, ctx->stream));
        hipLaunchKernelGGL(k_pos_doc_sizes, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, rows, n, ctx->last_vk,
                           ctx->last_ts, (unsigned *)ctx->td_sizes.p, ctx->d_scratch + POSBAD_WORD);
        const int64_t nb = (n + SC_PER - 1) / SC_PER;
        if ((rc = ensure(ctx, ctx->td_btot, nb * 4)) || (rc = ensure(ctx, ctx->td_boff, nb * 8))) return rc;
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_sizes.p, n, off,
                           (unsigned *)ctx->td_btot.p);
        hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->td_btot.p, nb,
                           (unsigned long long *)ctx->td_boff.p, off + n);
        hipLaunchKernelGGL(k_scan_add, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, off, n, (const unsigned long long *)ctx->td_boff.p);
        HIPCHK(ctx, hipGetLastError());
        unsigned long long hb[2] = {0, 0};
        HIPCHK(ctx, hipMemcpyAsync(&hb[0], off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipMemcpyAsync(&hb[1], ctx->d_scratch + POSBAD_WORD, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hb[1]) return set_err(ctx, HM_E_INVALID, "%llu latest rows outside the provider/vehicle dictionaries or time buckets", hb[1]);
        total = (int64_t)hb[0];
        if ((rc = ensure(ctx, ctx->td_bytes, total + 16))) return rc;
        hipLaunchKernelGGL(k_pos_docs, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, P, rows, n, ctx->last_vk, ctx->last_ts,
                           ctx->last_lat, ctx->last_lon, (const unsigned long long *)off, (uint8_t *)ctx->td_bytes.p);
        HIPCHK(ctx, hipGetLastError());
    } else {
        HIPCHK(ctx, hipMemsetAsync(off, 0, 8, ctx->stream));
        if ((rc = ensure(ctx, ctx->td_bytes, 16))) return rc;
    }
    return statements_out(ctx, n, total, out_memory, bytes, offsets, n_docs);
}
