// C ABI: hm_decode_json and hm_last_latest_buckets (row f1).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// ---- Kafka values -> batch columns (row f1; json_decode.h) ----
__global__ __launch_bounds__(256) void k_check_offsets(const int64_t *__restrict__ offs, int64_t n, int64_t lo, int64_t hi,
                                                       unsigned long long *bad) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        b += offs[i] < lo || offs[i] > offs[i + 1] || offs[i + 1] > hi;
    b = wave_sum(b);
    if (b && lane_id() == 0) atomicAdd(bad, b);
}

static int host_pinned(hm_ctx *ctx, void **p, size_t &cap, size_t want) {
    if (*p && cap >= want) return HM_OK;
    AllocTimer at_(ctx);
    if (*p) { HIPCHK(ctx, hipHostFree(*p)); ctx->n_frees++; }
    cap = *p ? host_cap_for(cap, want) : std::max<size_t>(want, 4096);
    *p = nullptr;
    ctx->n_allocs++;
    HIPCHK(ctx, hipHostMalloc(p, cap, hipHostMallocDefault));
    return HM_OK;
}

// the exact dictionary of one string column (spans off/len into bytes or scratch; len -1 = null): slot_of per row,
// code_of_slot, and the strings (Arrow offsets + bytes) in the Dict's pinned host buffers
static int dict_build(hm_ctx *ctx, hm_ctx::Dict &d, const uint8_t *bytes, const uint8_t *scratch, const int64_t *off,
                      const int32_t *len, int64_t n) {
    int rc;
    const unsigned long long full = next_pow2((unsigned long long)std::max<int64_t>(2 * n, 1024));
    unsigned long long cap = d.last_codes > 0 ? next_pow2((unsigned long long)std::max<int64_t>(4 * d.last_codes, 1024))
                                              : (1ull << 16);
    cap = std::min(cap, full);
    uint64_t seed = UINT64_C(0x8f1bbcdcca62c1d6);
    unsigned long long *words = ctx->d_scratch + JSON_WORD + 2;   // overflow, collisions
    for (int attempt = 0;; attempt++) {
        if (attempt == 6) return set_err(ctx, HM_E_OVERFLOW, "string dictionary: repeated hash collisions");
        if ((rc = ensure(ctx, d.tab, cap * sizeof(DictSlot))) || (rc = ensure(ctx, d.slot_of, std::max<int64_t>(n, 1) * 4)))
            return rc;
        HIPCHK(ctx, hipMemsetAsync(d.tab.p, 0xff, cap * sizeof(DictSlot), ctx->stream));
        HIPCHK(ctx, hipMemsetAsync(words, 0, 16, ctx->stream));
        // the first rows' strings first, by one workgroup: the frequent strings of a column (a batch's one provider)
        // are then in the table, written back, when the full launch starts, so that its waves find them with plain
        // loads -- each XCD's L2 otherwise served its waves a stale empty slot and every wave of the first grid pass
        // re-read the slot past it (agent scope) and raced for it (1.6-2.1 ms per 1e7 rows; with this, 38 + 89 us: profiles/r6/r6p/dict_kernels.txt)
        hipLaunchKernelGGL(k_dict_insert, dim3(1), dim3(256), 0, ctx->stream, bytes, scratch, off, len,
                           std::min<int64_t>(n, 4096), (DictSlot *)d.tab.p, cap - 1, seed, (unsigned *)d.slot_of.p, words);
        hipLaunchKernelGGL(k_dict_insert, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, bytes, scratch, off, len, n,
                           (DictSlot *)d.tab.p, cap - 1, seed, (unsigned *)d.slot_of.p, words);
        hipLaunchKernelGGL(k_dict_verify, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, bytes, scratch, off, len, n,
                           (const DictSlot *)d.tab.p, (const unsigned *)d.slot_of.p, words + 1);
        HIPCHK(ctx, hipGetLastError());
        unsigned long long hw[2];
        HIPCHK(ctx, hipMemcpyAsync(hw, words, 16, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hw[0]) {   // probes ran out (more distinct strings than the last batch): a full-size table
            if (cap == full) return set_err(ctx, HM_E_OVERFLOW, "string dictionary table overflow");
            cap = full;
            continue;
        }
        if (hw[1]) {   // a 64-bit hash collision: another seed
            seed = mix64(seed + (uint64_t)attempt + 1);
            continue;
        }
        break;
    }
    // codes: the occupied slots in ascending order
    if ((rc = ensure(ctx, d.occ, cap)) || (rc = ensure(ctx, d.slots, cap * 8)) || (rc = ensure(ctx, d.code_of_slot, cap * 4)))
        return rc;
    hipLaunchKernelGGL(k_dict_occ, dim3(grid_for((int64_t)cap, 256)), dim3(256), 0, ctx->stream, (const DictSlot *)d.tab.p,
                       (int64_t)cap, (uint8_t *)d.occ.p);
    if ((rc = compact_flags(ctx, (const uint8_t *)d.occ.p, (int64_t)cap, (int64_t *)d.slots.p, ctx->stream))) return rc;
    unsigned long long nc = 0;
    HIPCHK(ctx, hipMemcpyAsync(&nc, ctx->d_scratch + 255, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    const int64_t m = (int64_t)nc;
    if ((rc = ensure(ctx, d.clen, std::max<int64_t>(m, 1) * 4)) || (rc = ensure(ctx, d.coff, (m + 1) * 8))) return rc;
    hipLaunchKernelGGL(k_dict_codes, dim3(grid_for(std::max<int64_t>(m, 1), 256)), dim3(256), 0, ctx->stream,
                       (const int64_t *)d.slots.p, ctx->d_scratch + 255, (const DictSlot *)d.tab.p, len,
                       (unsigned *)d.code_of_slot.p, (unsigned *)d.clen.p);
    unsigned long long *coff = (unsigned long long *)d.coff.p;
    int64_t total = 0;
    if (m > 0) {
        const int64_t nb = (m + SC_PER - 1) / SC_PER;
        if ((rc = ensure(ctx, d.btot, nb * 4)) || (rc = ensure(ctx, d.boff, nb * 8))) return rc;
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, (const unsigned *)d.clen.p, m, coff,
                           (unsigned *)d.btot.p);
        hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)d.btot.p, nb,
                           (unsigned long long *)d.boff.p, coff + m);
        hipLaunchKernelGGL(k_scan_add, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, coff, m, (const unsigned long long *)d.boff.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(&total, coff + m, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    } else {
        HIPCHK(ctx, hipMemsetAsync(coff, 0, 8, ctx->stream));
    }
    if ((rc = ensure(ctx, d.cbytes, std::max<int64_t>(total, 1)))) return rc;
    if (m > 0)
        hipLaunchKernelGGL(k_dict_gather, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, bytes, scratch, off, len,
                           (const int64_t *)d.slots.p, ctx->d_scratch + 255, (const DictSlot *)d.tab.p,
                           (const unsigned long long *)coff, (uint8_t *)d.cbytes.p);
    HIPCHK(ctx, hipGetLastError());
    if ((rc = host_pinned(ctx, &d.h_off, d.h_off_cap, (size_t)(m + 1) * 8)) ||
        (rc = host_pinned(ctx, &d.h_bytes, d.h_bytes_cap, (size_t)std::max<int64_t>(total, 1))))
        return rc;
    HIPCHK(ctx, hipMemcpyAsync(d.h_off, coff, (m + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (total) HIPCHK(ctx, hipMemcpyAsync(d.h_bytes, d.cbytes.p, total, hipMemcpyDeviceToHost, ctx->stream));
    d.n_codes = m;
    d.last_codes = m;
    return HM_OK;
}

int hm_decode_json(hm_ctx *ctx, const hm_json_in *in, hm_json_out *out) {
    if (!ctx || !in || !out || in->n < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    const int64_t n = in->n;
    if (n > (int64_t)UINT32_MAX - 2) return set_err(ctx, HM_E_INVALID, "%lld records exceed 2^32-2", (long long)n);
    if (n > 0 && (!in->bytes || !in->offsets)) return set_err(ctx, HM_E_INVALID, "bytes and offsets are required");
    if (in->memory != HM_MEM_HOST && in->memory != HM_MEM_DEVICE) return set_err(ctx, HM_E_INVALID, "bad memory kind");
    if (in->flags & ~HM_JSON_SPLICE) return set_err(ctx, HM_E_INVALID, "unknown flags %d", in->flags);
    memset(out, 0, sizeof(*out));
    ctx->jd_n = -1;
    ctx->jd_unsup.clear();
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const size_t m = (size_t)std::max<int64_t>(n, 1);
    if ((rc = ensure(ctx, ctx->jd_lat, m * 8)) || (rc = ensure(ctx, ctx->jd_lon, m * 8)) || (rc = ensure(ctx, ctx->jd_ts, m * 8)) ||
        (rc = ensure(ctx, ctx->jd_speed, m * 8)) || (rc = ensure(ctx, ctx->jd_sv, m)) || (rc = ensure(ctx, ctx->jd_rv, m)) ||
        (rc = ensure(ctx, ctx->jd_vkey, m * 8)) || (rc = ensure(ctx, ctx->jd_poff, m * 8)) || (rc = ensure(ctx, ctx->jd_plen, m * 4)) ||
        (rc = ensure(ctx, ctx->jd_voff, m * 8)) || (rc = ensure(ctx, ctx->jd_vlen, m * 4)) ||
        (rc = ensure(ctx, ctx->jd_un, m)))
        return rc;
    int64_t o0 = 0, on = 0;
    const uint8_t *dbytes = nullptr;
    const int64_t *doffs = nullptr;
    if (n > 0) {
        if (in->memory == HM_MEM_HOST) {
            o0 = in->offsets[0];
            on = in->offsets[n];
            if (o0 < 0 || on < o0) return set_err(ctx, HM_E_INVALID, "bad offsets");
            if ((rc = ensure(ctx, ctx->jd_bytes, (size_t)(on - o0) + 16)) || (rc = ensure(ctx, ctx->jd_offs, (size_t)(n + 1) * 8))) return rc;
            if (on > o0) HIPCHK(ctx, hipMemcpyAsync(ctx->jd_bytes.p, in->bytes + o0, on - o0, hipMemcpyHostToDevice, ctx->stream));
            HIPCHK(ctx, hipMemcpyAsync(ctx->jd_offs.p, in->offsets, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
            dbytes = (const uint8_t *)ctx->jd_bytes.p;
            doffs = (const int64_t *)ctx->jd_offs.p;
        } else {
            HIPCHK(ctx, hipMemcpyAsync(&o0, in->offsets, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, hipMemcpyAsync(&on, in->offsets + n, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, ctx_sync(ctx, __LINE__));
            if (o0 < 0 || on < o0) return set_err(ctx, HM_E_INVALID, "bad offsets");
            dbytes = in->bytes + o0;
            doffs = in->offsets;
        }
        // every record inside [o0, on] with non-decreasing offsets (a bad offset would read out of bounds)
        unsigned long long *w = ctx->d_scratch + JSON_WORD;
        HIPCHK(ctx, hipMemsetAsync(w, 0, 16, ctx->stream));
        hipLaunchKernelGGL(k_check_offsets, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, doffs, n, o0, on, w);
        unsigned long long hb = 0;
        HIPCHK(ctx, hipMemcpyAsync(&hb, w, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hb) return set_err(ctx, HM_E_INVALID, "%llu offsets out of order or out of range", hb);
        if ((rc = ensure(ctx, ctx->jd_scratch, (size_t)(on - o0) + 16))) return rc;
        hipLaunchKernelGGL(k_json_parse, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, dbytes, doffs, o0, n,
                           (uint8_t *)ctx->jd_scratch.p, (double *)ctx->jd_lat.p, (double *)ctx->jd_lon.p, (int64_t *)ctx->jd_ts.p,
                           (double *)ctx->jd_speed.p, (uint8_t *)ctx->jd_sv.p, (uint8_t *)ctx->jd_rv.p, (int64_t *)ctx->jd_poff.p,
                           (int32_t *)ctx->jd_plen.p, (int64_t *)ctx->jd_voff.p, (int32_t *)ctx->jd_vlen.p,
                           (uint8_t *)ctx->jd_un.p, w);
        HIPCHK(ctx, hipGetLastError());
        unsigned long long counts[2];
        HIPCHK(ctx, hipMemcpyAsync(counts, w, 16, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        out->n_malformed = (int64_t)counts[0];
        out->n_unsupported = (int64_t)counts[1];
        if (counts[1] && (in->flags & HM_JSON_SPLICE)) {   // the rows for the host to decode (hm_json_patch)
            if ((rc = ensure(ctx, ctx->jd_unrows, (size_t)n * 8))) return rc;
            if ((rc = compact_flags(ctx, (const uint8_t *)ctx->jd_un.p, n, (int64_t *)ctx->jd_unrows.p, ctx->stream))) return rc;
            ctx->jd_unsup.resize(counts[1]);
            HIPCHK(ctx, hipMemcpyAsync(ctx->jd_unsup.data(), ctx->jd_unrows.p, counts[1] * 8, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, ctx_sync(ctx, __LINE__));
            out->unsupported_rows = ctx->jd_unsup.data();
        } else if (counts[1])
            return set_err(ctx, HM_E_UNSUPPORTED, "%llu records outside the device decoder (a number of more than 19 significant "
                           "digits on a rounding boundary, or a float/object/array as a string field)", counts[1]);
    }
    const uint8_t *scratch = (const uint8_t *)ctx->jd_scratch.p;
    if ((rc = dict_build(ctx, ctx->jd_prov, dbytes, scratch, (const int64_t *)ctx->jd_poff.p, (const int32_t *)ctx->jd_plen.p, n)) ||
        (rc = dict_build(ctx, ctx->jd_veh, dbytes, scratch, (const int64_t *)ctx->jd_voff.p, (const int32_t *)ctx->jd_vlen.p, n)))
        return rc;
    const int64_t nv = std::max<int64_t>(ctx->jd_veh.n_codes, 1);
    if (n > 0)
        hipLaunchKernelGGL(k_json_vkey, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, (const uint8_t *)ctx->jd_rv.p,
                           (const unsigned *)ctx->jd_prov.slot_of.p, (const unsigned *)ctx->jd_veh.slot_of.p,
                           (const unsigned *)ctx->jd_prov.code_of_slot.p, (const unsigned *)ctx->jd_veh.code_of_slot.p, n,
                           (uint64_t)nv, (uint64_t *)ctx->jd_vkey.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    hm_batch_in &b = out->batch;
    b.n = n;
    b.memory = HM_MEM_DEVICE;
    b.lat = (const double *)ctx->jd_lat.p;
    b.lon = (const double *)ctx->jd_lon.p;
    b.ts_us = (const int64_t *)ctx->jd_ts.p;
    b.speed = (const double *)ctx->jd_speed.p;
    b.speed_valid = (const uint8_t *)ctx->jd_sv.p;
    b.vkey = (const uint64_t *)ctx->jd_vkey.p;
    b.row_valid = (const uint8_t *)ctx->jd_rv.p;
    out->n_providers = ctx->jd_prov.n_codes;
    out->provider_offsets = (const int64_t *)ctx->jd_prov.h_off;
    out->provider_bytes = (const uint8_t *)ctx->jd_prov.h_bytes;
    out->n_vehicles = ctx->jd_veh.n_codes;
    out->vehicle_offsets = (const int64_t *)ctx->jd_veh.h_off;
    out->vehicle_bytes = (const uint8_t *)ctx->jd_veh.h_bytes;
    ctx->jd_n = n;
    ctx->jd_nv = ctx->jd_veh.n_codes;
    ctx->jd_np = ctx->jd_prov.n_codes;
    return HM_OK;
}

// ---- Arrow columns -> batch columns (the boundary's Arrow / Spark / pandas frames) ----
// one column's host buffers -> device (values into dst, or the string offsets / bytes into the column's own buffers)
static int arrow_upload(hm_ctx *ctx, const hm_arrow_col &c, int64_t n, size_t elem, void *dst, DevBuf &bits, DevBuf &offs,
                        DevBuf &data, ArrowDevCol &d, bool is_string) {
    memset(&d, 0, sizeof(d));
    if (c.unit != 0 && (is_string || elem != 8 || dst != ctx->jd_ts.p || c.unit != 1))
        return set_err(ctx, HM_E_INVALID, "unit %d: only eventTs may be in nanoseconds (1)", c.unit);
    if (!c.values || n == 0) return HM_OK;
    d.present = 1;
    d.ns = c.unit;
    if (c.validity) {
        if (c.validity_offset < 0) return set_err(ctx, HM_E_INVALID, "negative validity offset");
        const int64_t b0 = c.validity_offset >> 3, nb = ((c.validity_offset & 7) + n + 7) >> 3;
        int rc;
        if ((rc = ensure(ctx, bits, (size_t)nb))) return rc;
        HIPCHK(ctx, hipMemcpyAsync(bits.p, c.validity + b0, (size_t)nb, hipMemcpyHostToDevice, ctx->stream));
        d.valid = (const uint8_t *)bits.p;
        d.bit0 = (int16_t)(c.validity_offset & 7);
    }
    if (!is_string) {
        HIPCHK(ctx, hipMemcpyAsync(dst, c.values, (size_t)n * elem, hipMemcpyHostToDevice, ctx->stream));
        return HM_OK;
    }
    if (c.offset_bytes != 4 && c.offset_bytes != 8) return set_err(ctx, HM_E_INVALID, "string offsets of %d bytes", c.offset_bytes);
    const int64_t o0 = c.offset_bytes == 4 ? ((const int32_t *)c.values)[0] : ((const int64_t *)c.values)[0];
    const int64_t on = c.offset_bytes == 4 ? ((const int32_t *)c.values)[n] : ((const int64_t *)c.values)[n];
    if (o0 < 0 || on < o0) return set_err(ctx, HM_E_INVALID, "bad string offsets");
    if (on > o0 && !c.data) return set_err(ctx, HM_E_INVALID, "string column without bytes");
    int rc;
    if ((rc = ensure(ctx, offs, (size_t)(n + 1) * c.offset_bytes)) || (rc = ensure(ctx, data, (size_t)(on - o0) + 16))) return rc;
    HIPCHK(ctx, hipMemcpyAsync(offs.p, c.values, (size_t)(n + 1) * c.offset_bytes, hipMemcpyHostToDevice, ctx->stream));
    if (on > o0) HIPCHK(ctx, hipMemcpyAsync(data.p, c.data + o0, (size_t)(on - o0), hipMemcpyHostToDevice, ctx->stream));
    d.offs = offs.p;
    d.base = o0;
    d.offset_bytes = c.offset_bytes;
    return HM_OK;
}

int hm_arrow_columns(hm_ctx *ctx, const hm_arrow_in *in, hm_json_out *out) {
    if (!ctx || !in || !out || in->n < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    const int64_t n = in->n;
    if (n > (int64_t)UINT32_MAX - 2) return set_err(ctx, HM_E_INVALID, "%lld rows exceed 2^32-2", (long long)n);
    memset(out, 0, sizeof(*out));
    ctx->jd_n = -1;   // (nothing to patch: hm_json_patch is the JSON decoder's)
    ctx->jd_unsup.clear();
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc;
    const size_t m = (size_t)std::max<int64_t>(n, 1);
    if ((rc = ensure(ctx, ctx->jd_lat, m * 8)) || (rc = ensure(ctx, ctx->jd_lon, m * 8)) || (rc = ensure(ctx, ctx->jd_ts, m * 8)) ||
        (rc = ensure(ctx, ctx->jd_speed, m * 8)) || (rc = ensure(ctx, ctx->jd_sv, m)) || (rc = ensure(ctx, ctx->jd_rv, m)) ||
        (rc = ensure(ctx, ctx->jd_vkey, m * 8)) || (rc = ensure(ctx, ctx->jd_poff, m * 8)) || (rc = ensure(ctx, ctx->jd_plen, m * 4)) ||
        (rc = ensure(ctx, ctx->jd_voff, m * 8)) || (rc = ensure(ctx, ctx->jd_vlen, m * 4)))
        return rc;
    ArrowDevCol dl, dn, ds, dt, dp, dv;
    if ((rc = arrow_upload(ctx, in->lat, n, 8, ctx->jd_lat.p, ctx->ar_bits[0], ctx->ar_offs[0], ctx->ar_data[0], dl, false)) ||
        (rc = arrow_upload(ctx, in->lon, n, 8, ctx->jd_lon.p, ctx->ar_bits[1], ctx->ar_offs[0], ctx->ar_data[0], dn, false)) ||
        (rc = arrow_upload(ctx, in->speed, n, 8, ctx->jd_speed.p, ctx->ar_bits[2], ctx->ar_offs[0], ctx->ar_data[0], ds, false)) ||
        (rc = arrow_upload(ctx, in->ts_us, n, 8, ctx->jd_ts.p, ctx->ar_bits[3], ctx->ar_offs[0], ctx->ar_data[0], dt, false)) ||
        (rc = arrow_upload(ctx, in->provider, n, 0, nullptr, ctx->ar_bits[4], ctx->ar_offs[0], ctx->ar_data[0], dp, true)) ||
        (rc = arrow_upload(ctx, in->vehicle, n, 0, nullptr, ctx->ar_bits[5], ctx->ar_offs[1], ctx->ar_data[1], dv, true)))
        return rc;
    if (n > 0) {
        // (absent columns: every row null -- the prep kernel writes their values; nothing was copied)
        unsigned long long *w = ctx->d_scratch + JSON_WORD;
        HIPCHK(ctx, hipMemsetAsync(w, 0, 8, ctx->stream));
        if (dp.present) hipLaunchKernelGGL(k_arrow_check_offsets, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, dp, n, w);
        if (dv.present) hipLaunchKernelGGL(k_arrow_check_offsets, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, dv, n, w);
        unsigned long long hb = 0;
        HIPCHK(ctx, hipMemcpyAsync(&hb, w, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        if (hb) return set_err(ctx, HM_E_INVALID, "%llu string offsets out of order", hb);
        hipLaunchKernelGGL(k_arrow_prep, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, n, dl, dn, ds, dt, dp, dv,
                           (double *)ctx->jd_lat.p, (double *)ctx->jd_lon.p, (double *)ctx->jd_speed.p, (uint8_t *)ctx->jd_sv.p,
                           (int64_t *)ctx->jd_ts.p, (uint8_t *)ctx->jd_rv.p, (int64_t *)ctx->jd_poff.p, (int32_t *)ctx->jd_plen.p,
                           (int64_t *)ctx->jd_voff.p, (int32_t *)ctx->jd_vlen.p);
        HIPCHK(ctx, hipGetLastError());
    }
    if ((rc = dict_build(ctx, ctx->jd_prov, (const uint8_t *)ctx->ar_data[0].p, nullptr, (const int64_t *)ctx->jd_poff.p,
                         (const int32_t *)ctx->jd_plen.p, n)) ||
        (rc = dict_build(ctx, ctx->jd_veh, (const uint8_t *)ctx->ar_data[1].p, nullptr, (const int64_t *)ctx->jd_voff.p,
                         (const int32_t *)ctx->jd_vlen.p, n)))
        return rc;
    const int64_t nv = std::max<int64_t>(ctx->jd_veh.n_codes, 1);
    if (ctx->jd_prov.n_codes > 0 && (uint64_t)ctx->jd_prov.n_codes > (UINT64_MAX - 1) / (uint64_t)nv)
        return set_err(ctx, HM_E_INVALID, "vkey space overflows");
    if (n > 0)
        hipLaunchKernelGGL(k_json_vkey, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, (const uint8_t *)ctx->jd_rv.p,
                           (const unsigned *)ctx->jd_prov.slot_of.p, (const unsigned *)ctx->jd_veh.slot_of.p,
                           (const unsigned *)ctx->jd_prov.code_of_slot.p, (const unsigned *)ctx->jd_veh.code_of_slot.p, n,
                           (uint64_t)nv, (uint64_t *)ctx->jd_vkey.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    hm_batch_in &b = out->batch;
    b.n = n;
    b.memory = HM_MEM_DEVICE;
    b.lat = (const double *)ctx->jd_lat.p;
    b.lon = (const double *)ctx->jd_lon.p;
    b.ts_us = (const int64_t *)ctx->jd_ts.p;
    b.speed = (const double *)ctx->jd_speed.p;
    b.speed_valid = (const uint8_t *)ctx->jd_sv.p;
    b.vkey = (const uint64_t *)ctx->jd_vkey.p;
    b.row_valid = (const uint8_t *)ctx->jd_rv.p;
    out->n_providers = ctx->jd_prov.n_codes;
    out->provider_offsets = (const int64_t *)ctx->jd_prov.h_off;
    out->provider_bytes = (const uint8_t *)ctx->jd_prov.h_bytes;
    out->n_vehicles = ctx->jd_veh.n_codes;
    out->vehicle_offsets = (const int64_t *)ctx->jd_veh.h_off;
    out->vehicle_bytes = (const uint8_t *)ctx->jd_veh.h_bytes;
    return HM_OK;
}

int hm_json_patch(hm_ctx *ctx, int64_t m, const int64_t *rows, const double *lat, const double *lon, const int64_t *ts_us,
                  const double *speed, const uint8_t *speed_valid, const uint8_t *row_valid, const int64_t *pcode,
                  const int64_t *vcode, int64_t n_providers, int64_t n_vehicles) {
    if (!ctx || m < 0) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->jd_n < 0) return set_err(ctx, HM_E_STATE, "no hm_decode_json batch to patch");
    if (m > 0 && (!rows || !lat || !lon || !ts_us || !speed || !speed_valid || !row_valid || !pcode || !vcode))
        return set_err(ctx, HM_E_INVALID, "null column");
    if (n_providers < ctx->jd_np || n_vehicles < ctx->jd_nv)
        return set_err(ctx, HM_E_INVALID, "dictionaries may only grow (%lld < %lld providers or %lld < %lld vehicles)",
                       (long long)n_providers, (long long)ctx->jd_np, (long long)n_vehicles, (long long)ctx->jd_nv);
    const uint64_t nv_old = (uint64_t)std::max<int64_t>(ctx->jd_nv, 1), nv_new = (uint64_t)std::max<int64_t>(n_vehicles, 1);
    if (n_providers > 0 && (uint64_t)n_providers > (UINT64_MAX - 1) / nv_new)
        return set_err(ctx, HM_E_INVALID, "vkey space overflows");
    std::vector<JsonPatchRow> P((size_t)m);
    for (int64_t k = 0; k < m; k++) {
        if (rows[k] < 0 || rows[k] >= ctx->jd_n) return set_err(ctx, HM_E_INVALID, "row %lld outside the batch", (long long)rows[k]);
        if (row_valid[k] && (pcode[k] < 0 || pcode[k] >= n_providers || vcode[k] < 0 || vcode[k] >= n_vehicles))
            return set_err(ctx, HM_E_INVALID, "row %lld: code outside the dictionaries", (long long)rows[k]);
        JsonPatchRow &p = P[k];
        memset(&p, 0, sizeof(p));
        p.row = rows[k];
        p.ts_us = ts_us[k];
        p.pcode = pcode[k];
        p.vcode = vcode[k];
        p.lat = lat[k];
        p.lon = lon[k];
        p.speed = speed[k];
        p.sv = speed_valid[k] ? 1 : 0;
        p.rv = row_valid[k] ? 1 : 0;
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int64_t n = ctx->jd_n;
    int rc;
    if (n > 0 && nv_new != nv_old)
        hipLaunchKernelGGL(k_json_rekey, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream, (const uint8_t *)ctx->jd_rv.p, n,
                           nv_old, nv_new, (uint64_t *)ctx->jd_vkey.p);
    if (m > 0) {
        if ((rc = ensure(ctx, ctx->jd_patch, (size_t)m * sizeof(JsonPatchRow)))) return rc;
        HIPCHK(ctx, hipMemcpyAsync(ctx->jd_patch.p, P.data(), (size_t)m * sizeof(JsonPatchRow), hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_json_patch, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, (const JsonPatchRow *)ctx->jd_patch.p,
                           m, nv_new, (double *)ctx->jd_lat.p, (double *)ctx->jd_lon.p, (int64_t *)ctx->jd_ts.p,
                           (double *)ctx->jd_speed.p, (uint8_t *)ctx->jd_sv.p, (uint8_t *)ctx->jd_rv.p, (uint64_t *)ctx->jd_vkey.p);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));   // (P is pageable host memory)
    ctx->jd_nv = n_vehicles;
    ctx->jd_np = n_providers;
    return HM_OK;
}

int hm_last_latest_buckets(hm_ctx *ctx, int64_t *bucket_ids, int64_t cap, int64_t *n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !bucket_ids)) return ctx ? set_err(ctx, HM_E_INVALID, "bad argument") : HM_E_INVALID;
    if (ctx->last_n_latest < 0) return set_err(ctx, HM_E_STATE, "no hm_process_batch latest rows");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int64_t m = ctx->last_n_latest;
    *n = 0;
    if (m == 0) return HM_OK;
    int rc;
    const unsigned long long scap = next_pow2((unsigned long long)std::max<int64_t>(2 * m, 1024));
    if ((rc = ensure(ctx, ctx->lb_set, scap * 8)) || (rc = ensure(ctx, ctx->lb_list, (size_t)m * 8))) return rc;
    unsigned long long *w = ctx->d_scratch + JSON_WORD + 4;
    hipLaunchKernelGGL(k_fill_i64, dim3(grid_for((int64_t)scap, 256)), dim3(256), 0, ctx->stream, (long long *)ctx->lb_set.p,
                       (int64_t)scap, (long long)INT64_MIN);
    HIPCHK(ctx, hipMemsetAsync(w, 0, 8, ctx->stream));
    hipLaunchKernelGGL(k_latest_buckets, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, (const int64_t *)ctx->rows.p, m,
                       ctx->last_ts, (long long *)ctx->lb_set.p, scap - 1, (long long *)ctx->lb_list.p, w);
    HIPCHK(ctx, hipGetLastError());
    unsigned long long k = 0;
    HIPCHK(ctx, hipMemcpyAsync(&k, w, 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    std::vector<int64_t> ids(k);
    if (k) HIPCHK(ctx, hipMemcpy(ids.data(), ctx->lb_list.p, k * 8, hipMemcpyDeviceToHost));
    std::sort(ids.begin(), ids.end());
    *n = (int64_t)k;
    for (int64_t i = 0; i < (int64_t)k && i < cap; i++) bucket_ids[i] = ids[i];
    return HM_OK;
}
