// C ABI: device-buffer helpers and the host-executed self-test entry points the CPU tests call.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

int hm_selftest_json_records(const uint8_t *bytes, const int64_t *offsets, int64_t n, uint8_t *scratch, double *lat,
                             double *lon, double *speed, int64_t *ts_us, int32_t *bearing, int32_t *accuracy,
                             int64_t *p_off, int32_t *p_len, int64_t *v_off, int32_t *v_len, uint32_t *flags) {
    if (n < 0 || (n > 0 && (!bytes || !offsets || !scratch))) return HM_E_INVALID;
    for (int64_t i = 0; i < n; i++) {
        JsonRow r;
        parse_record(bytes, offsets[i], offsets[i + 1], scratch, r);
        lat[i] = r.lat;
        lon[i] = r.lon;
        speed[i] = r.speed;
        ts_us[i] = r.ts_us;
        bearing[i] = r.bearing;
        accuracy[i] = r.accuracy;
        p_off[i] = r.p_off;
        p_len[i] = r.p_len;
        v_off[i] = r.v_off;
        v_len[i] = r.v_len;
        flags[i] = r.flags;
    }
    return HM_OK;
}

int hm_selftest_decimal_to_double(const uint64_t *w, const int64_t *q, int64_t n, uint64_t *bits) {
    if (n < 0 || (n > 0 && (!w || !q || !bits))) return HM_E_INVALID;
    for (int64_t i = 0; i < n; i++) bits[i] = decimal_to_double_bits(q[i], w[i]);
    return HM_OK;
}

int hm_device_memory(int32_t device, int64_t *free_bytes, int64_t *total_bytes) {
    if (!free_bytes || !total_bytes) return HM_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return HM_E_HIP;
    }
    size_t f = 0, t = 0;
    if (hipMemGetInfo(&f, &t) != hipSuccess) return HM_E_HIP;
    *free_bytes = (int64_t)f;
    *total_bytes = (int64_t)t;
    return HM_OK;
}
int hm_device_alloc(int32_t device, int64_t bytes, void **ptr) {
    if (!ptr || bytes < 0) return HM_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return HM_E_HIP;
    return hipMalloc(ptr, std::max<int64_t>(bytes, 16)) == hipSuccess ? HM_OK : HM_E_NOMEM;
}
int hm_device_free(int32_t device, void *ptr) {
    if (hipSetDevice(device) != hipSuccess) return HM_E_HIP;
    return hipFree(ptr) == hipSuccess ? HM_OK : HM_E_HIP;
}
int hm_host_alloc(int64_t bytes, void **ptr) {
    if (!ptr || bytes < 0) return HM_E_INVALID;
    return hipHostMalloc(ptr, std::max<int64_t>(bytes, 16), hipHostMallocDefault) == hipSuccess ? HM_OK : HM_E_NOMEM;
}
int hm_host_free(void *ptr) { return hipHostFree(ptr) == hipSuccess ? HM_OK : HM_E_HIP; }
int hm_memcpy(void *dst, const void *src, int64_t bytes, int32_t kind) {
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    return hipMemcpy(dst, src, bytes, k) == hipSuccess ? HM_OK : HM_E_HIP;
}

// host execution of the statement encoder (bson_docs.h) on caller arrays: bytes (capacity cap) + offsets[n+1]
int hm_selftest_tile_statements(const hm_tile_doc_cfg *cfg, int32_t h3_res, int64_t tile_us, const uint64_t *cell,
                                const int64_t *ws, const int64_t *cnt, const double *sp, const uint8_t *spn,
                                const double *lon, const double *lat, int64_t n, uint8_t *bytes, int64_t cap,
                                int64_t *offsets) {
    if (!cfg || n < 0 || !offsets || cfg->n_windows <= 0 || cfg->city_len < 0 || cfg->city_len > (1 << 20)) return HM_E_INVALID;
    TileDocParams P;
    P.city = (const uint8_t *)cfg->city;
    P.city_len = cfg->city_len;
    P.h3_res = h3_res;
    P.tile_us = tile_us;
    P.ttl_ms = cfg->ttl_ms;
    P.win_start_us = cfg->window_start_us;
    P.off_start_s = cfg->start_offset_s;
    P.off_end_s = cfg->end_offset_s;
    P.n_win = (int)cfg->n_windows;
    int64_t o = 0;
    for (int64_t i = 0; i < n; i++) {
        offsets[i] = o;
        const int len = tile_statement(nullptr, P, cell[i], ws[i], cnt[i], sp[i], spn[i], lon[i], lat[i]);
        if (o + len > cap) return HM_E_INVALID;
        tile_statement(bytes + o, P, cell[i], ws[i], cnt[i], sp[i], spn[i], lon[i], lat[i]);
        o += len;
    }
    offsets[n] = o;
    return HM_OK;
}

// host execution of the positions statement encoder (bson_docs.h) on caller rows (vkey, ts, lat, lon per row)
int hm_selftest_position_statements(const hm_position_doc_cfg *cfg, const uint64_t *vkey, const int64_t *ts,
                                    const double *lat, const double *lon, int64_t n, uint8_t *bytes, int64_t cap,
                                    int64_t *offsets) {
    if (!cfg || n < 0 || !offsets) return HM_E_INVALID;
    PosDocParams P;
    P.p_off = cfg->provider_offsets;
    P.p_bytes = (const uint8_t *)cfg->provider_bytes;
    P.v_off = cfg->vehicle_offsets;
    P.v_bytes = (const uint8_t *)cfg->vehicle_bytes;
    P.n_providers = cfg->n_providers;
    P.n_vehicles = cfg->n_vehicles;
    P.n_buckets = cfg->n_buckets;
    P.bucket_id = cfg->bucket_ids;
    P.bucket_off = cfg->bucket_offset_s;
    int64_t o = 0;
    for (int64_t i = 0; i < n; i++) {
        offsets[i] = o;
        if (!position_ok(P, vkey[i], ts[i])) return HM_E_INVALID;
        const int len = position_statement(nullptr, P, vkey[i], ts[i], lat[i], lon[i]);
        if (o + len > cap) return HM_E_INVALID;
        position_statement(bytes + o, P, vkey[i], ts[i], lat[i], lon[i]);
        o += len;
    }
    offsets[n] = o;
    return HM_OK;
}

int hm_selftest_ld_ops(const double *a, int64_t n, int32_t op, double *out) {
    if (!a || !out || n < 0) return HM_E_INVALID;
    for (int64_t i = 0; i < n; i++) {
        double x = a[i], r;
        switch (op) {
            case 0: r = XMUL(x, PI_180); break;
            case 1: r = XMUL(x, SQRT7); break;
            case 2: r = XMUL(x, RSIN60); break;
            case 3: r = XADD(x, false, 2PI); break;
            case 4: r = XADD(x, true, 2PI); break;
            case 5: r = XADD(x, true, AP7_ROT); break;
            case 6: r = XADD(x, false, AP7_ROT); break;
            case 7: r = XMUL(x, SQRT3_2); break;
            case 8: r = XMUL(x, RSQRT7); break;
            case 9: r = XMUL(x, ONETHIRD); break;
            case 17: r = XMUL(x, 180_PI); break;
            case 10: r = xld_mul(x, HM_LD_PI_180_M, HM_LD_PI_180_E); break;
            case 11: r = xld_mul(x, HM_LD_SQRT7_M, HM_LD_SQRT7_E); break;
            case 12: r = xld_mul(x, HM_LD_RSIN60_M, HM_LD_RSIN60_E); break;
            case 13: r = xld_add(x, false, HM_LD_2PI_M, HM_LD_2PI_E); break;
            case 14: r = xld_add(x, true, HM_LD_2PI_M, HM_LD_2PI_E); break;
            case 15: r = xld_add(x, true, HM_LD_AP7_ROT_M, HM_LD_AP7_ROT_E); break;
            case 16: r = xld_add(x, false, HM_LD_AP7_ROT_M, HM_LD_AP7_ROT_E); break;
            default: return HM_E_INVALID;
        }
        out[i] = r;
    }
    return HM_OK;
}

int hm_selftest_floor_div(const int64_t *t, int64_t n, int64_t d, int64_t *out) {
    if (!t || !out || n < 0 || d < 1) return HM_E_INVALID;
    const FloorDiv D = make_floor_div(d);
    for (int64_t i = 0; i < n; i++) out[i] = floor_div(t[i], D);
    return HM_OK;
}

int hm_selftest_latlng_to_cell_host(const double *lat, const double *lon, int64_t n, int32_t res, uint64_t *out) {
    if (!lat || !lon || !out || n < 0 || res < 0 || res > 15) return HM_E_INVALID;
    static const H3Tables T = make_tables();
    for (int64_t i = 0; i < n; i++) out[i] = latLngToCellDeg(lat[i], lon[i], res, T);
    return HM_OK;
}

int hm_selftest_latlng_to_cell_fast_host(const double *lat, const double *lon, int64_t n, int32_t res, uint64_t *out,
                                         uint8_t *fell_back) {
    if (!lat || !lon || !out || n < 0 || res < 0 || res > 15) return HM_E_INVALID;
    static const H3Tables T = make_tables();
    for (int64_t i = 0; i < n; i++) {
        const bool ok = latLngToCellFast(lat[i], lon[i], res, T, out[i]);
        if (!ok) out[i] = latLngToCellDeg(lat[i], lon[i], res, T);
        if (fell_back) fell_back[i] = !ok;
    }
    return HM_OK;
}

// glibc's sincos / acos / atan2 / tan / asin / atan as restated in glibc_libm.h (fn 0 sincos: out = sin, out2 = cos;
// 1 acos(a); 2 atan2(a, b); 3 tan(a); 4 asin(a); 5 atan(a)), executed on the host and on the GPU (test entry points; tests/test_glibc_libm.py)
static int glm_check(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2) {
    if (!a || !out || n < 0 || fn < 0 || fn > 5 || (fn == 0 && !out2) || (fn == 2 && !b)) return HM_E_INVALID;
    return HM_OK;
}
HM_HD void glm_eval(int32_t fn, int64_t i, const double *a, const double *b, double *out, double *out2,
                    const glm::Tables &G) {
    switch (fn) {
        case 0: glm::sincos(a[i], out[i], out2[i], G); break;
        case 1: out[i] = glm::acos(a[i], G); break;
        case 2: out[i] = glm::atan2(a[i], b[i], G); break;
        case 3: out[i] = glm::tan(a[i], G); break;
        case 4: out[i] = glm::asin(a[i], G); break;
        default: out[i] = glm::atan(a[i], G); break;
    }
}
__global__ __launch_bounds__(256) void k_glibc_libm(int32_t fn, const double *a, const double *b, int64_t n,
                                                    double *out, double *out2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        glm_eval(fn, i, a, b, out, out2, g_glm);
}

int hm_selftest_glibc_libm_host(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2) {
    if (int e = glm_check(fn, a, b, n, out, out2)) return e;
    for (int64_t i = 0; i < n; i++) glm_eval(fn, i, a, b, out, out2, hm_glm_host);
    return HM_OK;
}

int hm_selftest_glibc_libm_device(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2,
                                  int32_t device) {
    if (int e = glm_check(fn, a, b, n, out, out2)) return e;
    int ndev = 0;
    if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev || hipSetDevice(device) != hipSuccess)
        return HM_E_HIP;
    if (n == 0) return HM_OK;
    const size_t B = (size_t)n * sizeof(double);
    double *d[4] = {nullptr, nullptr, nullptr, nullptr};
    int rc = HM_OK;
    for (int k = 0; k < 4 && rc == HM_OK; k++)
        if (hipMalloc((void **)&d[k], B) != hipSuccess) rc = HM_E_NOMEM;
    if (rc == HM_OK && (hipMemcpy(d[0], a, B, hipMemcpyHostToDevice) != hipSuccess ||
                        (b && hipMemcpy(d[1], b, B, hipMemcpyHostToDevice) != hipSuccess)))
        rc = HM_E_HIP;
    if (rc == HM_OK) {
        hipLaunchKernelGGL(k_glibc_libm, dim3(grid_for(n, 256)), dim3(256), 0, 0, fn, d[0], d[1], n, d[2], d[3]);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(out, d[2], B, hipMemcpyDeviceToHost) != hipSuccess ||
            (fn == 0 && hipMemcpy(out2, d[3], B, hipMemcpyDeviceToHost) != hipSuccess))
            rc = HM_E_HIP;
    }
    for (double *p : d)
        if (p) (void)hipFree(p);
    return rc;
}
