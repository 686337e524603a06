// C ABI: the context-free entry points -- the standalone UDF (hm_latlng_to_cell) and the read side (hm_cells_to_boundary).
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// ---- context-free entry points (the standalone UDF and the read side): per-device tables, stream and scratch
// buffers made once and reused, behind one mutex ----
struct UdfState {
    bool ready = false;
    int64_t last_exact = 0;   // hm_latlng_to_cell: inputs the fast path handed to the exact path (last call)
    hipStream_t stream = nullptr;
    DevBuf in0, in1, out0, out1, out2, slow;
};
static std::mutex g_udf_mu;
static UdfState g_udf[64];
static hipError_t udf_buf(DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return hipSuccess;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    hipError_t e = hipMalloc(&b.p, want);
    if (e == hipSuccess) b.bytes = want;
    return e;
}
static int udf_begin(int32_t device, UdfState *&S) {   // (g_udf_mu held)
    int ndev = 0;
    if (device < 0 || device >= 64 || hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) return HM_E_HIP;
    if (hipSetDevice(device) != hipSuccess) return HM_E_HIP;
    S = &g_udf[device];
    if (!S->ready) {
        if (upload_tables() != hipSuccess) return HM_E_HIP;
        if (hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking) != hipSuccess) return HM_E_HIP;
        S->ready = true;
    }
    return HM_OK;
}

int hm_latlng_to_cell(const double *lat, const double *lon, int64_t n, int32_t res, int32_t memory, int32_t device,
                      uint64_t *out) {
    if (n < 0 || n > (int64_t)UINT32_MAX || res < 0 || res > 15) return HM_E_INVALID;
    if (n == 0) return HM_OK;
    std::lock_guard<std::mutex> lock(g_udf_mu);
    UdfState *S = nullptr;
    int rc;
    if ((rc = udf_begin(device, S))) return rc;
    const double *dlat = lat, *dlon = lon;
    uint64_t *dout = out;
    // exception list + its count (last 8 bytes)
    if (udf_buf(S->slow, n * 4 + 16) != hipSuccess) return HM_E_NOMEM;
    unsigned long long *n_slow = (unsigned long long *)((char *)S->slow.p + ((n * 4 + 7) & ~int64_t(7)));
    hipError_t e = hipSuccess;
    if (memory == HM_MEM_HOST) {
        if (udf_buf(S->in0, n * 8) || udf_buf(S->in1, n * 8) || udf_buf(S->out0, n * 8)) return HM_E_NOMEM;
        e = hipMemcpyAsync(S->in0.p, lat, n * 8, hipMemcpyHostToDevice, S->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(S->in1.p, lon, n * 8, hipMemcpyHostToDevice, S->stream);
        dlat = (const double *)S->in0.p;
        dlon = (const double *)S->in1.p;
        dout = (uint64_t *)S->out0.p;
    }
    if (e == hipSuccess) e = hipMemsetAsync(n_slow, 0, 8, S->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_cells, dim3(grid_for(n, 256, 256 * 32)), dim3(256), 0, S->stream, dlat, dlon, n, res, dout,
                           (unsigned int *)S->slow.p, n_slow);
        hipLaunchKernelGGL(k_cells_exact, dim3(256), dim3(256), 0, S->stream, dlat, dlon, res, dout, (const unsigned int *)S->slow.p,
                           (const unsigned long long *)n_slow);
        e = hipGetLastError();
    }
    if (e == hipSuccess && memory == HM_MEM_HOST) e = hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, S->stream);
    unsigned long long ne = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&ne, n_slow, 8, hipMemcpyDeviceToHost, S->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(S->stream);
    S->last_exact = (int64_t)ne;
    return e == hipSuccess ? HM_OK : HM_E_HIP;
}

int64_t hm_latlng_to_cell_last_exact(int32_t device) {
    std::lock_guard<std::mutex> lock(g_udf_mu);
    return device >= 0 && device < 64 ? g_udf[device].last_exact : -1;
}

int hm_cells_to_boundary(const uint64_t *cells, int64_t n, int32_t memory, int32_t device, double *lat, double *lng,
                         int32_t *nverts) {
    if (n < 0 || n > (int64_t)UINT32_MAX || (n > 0 && (!cells || !lat || !lng || !nverts))) return HM_E_INVALID;
    if (n == 0) return HM_OK;
    std::lock_guard<std::mutex> lock(g_udf_mu);
    UdfState *S = nullptr;
    int rc;
    if ((rc = udf_begin(device, S))) return rc;
    const uint64_t *dcells = cells;
    double *dlat = lat, *dlng = lng;
    int32_t *dnv = nverts;
    hipError_t e = hipSuccess;
    if (memory == HM_MEM_HOST) {
        if (udf_buf(S->in0, n * 8) || udf_buf(S->out0, n * 80) || udf_buf(S->out1, n * 80) || udf_buf(S->out2, n * 4))
            return HM_E_NOMEM;
        e = hipMemcpyAsync(S->in0.p, cells, n * 8, hipMemcpyHostToDevice, S->stream);
        dcells = (const uint64_t *)S->in0.p;
        dlat = (double *)S->out0.p;
        dlng = (double *)S->out1.p;
        dnv = (int32_t *)S->out2.p;
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_cells_boundary, dim3(grid_for(n, 256, 256 * 32)), dim3(256), 0, S->stream, dcells, n, dlat, dlng, dnv);
        e = hipGetLastError();
    }
    if (e == hipSuccess && memory == HM_MEM_HOST) {
        e = hipMemcpyAsync(lat, dlat, n * 80, hipMemcpyDeviceToHost, S->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(lng, dlng, n * 80, hipMemcpyDeviceToHost, S->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(nverts, dnv, n * 4, hipMemcpyDeviceToHost, S->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(S->stream);
    return e == hipSuccess ? HM_OK : HM_E_HIP;
}

int hm_selftest_cells_to_boundary_host(const uint64_t *cells, int64_t n, double *lat, double *lng, int32_t *nverts) {
    if (n < 0 || (n > 0 && (!cells || !lat || !lng || !nverts))) return HM_E_INVALID;
    static const H3Tables T = make_tables();
    for (int64_t i = 0; i < n; i++) {
        double la[10], lo[10];
        const int nv = cellToBoundaryDeg(cells[i], T, la, lo);
        nverts[i] = nv;
        for (int k = 0; k < 10; k++) {
            lat[10 * i + k] = k < nv ? la[k] : NAN;
            lng[10 * i + k] = k < nv ? lo[k] : NAN;
        }
    }
    return HM_OK;
}
