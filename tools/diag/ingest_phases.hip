// k_ingest's VALU instructions by phase (VERDICT r3 "What's weak" 4 / item 6), on the bench's workload: 1e8 events
// uniform on the sphere, res 8.  A diagnostic build that includes the product translation unit and runs, besides
// the product's own k_ingest (both variants, through hm_process_batch), kernels that stop after successive phases of
// its per-event work -- the same device functions, the same loads and LDS tables:
//   ph_load     the row loads (lat, lon, ts, vkey, row_valid) and the loop            -> the skeleton
//   ph_sincos   + sin/cos of lat and lng (sincos_small) and the unit vector           -> + trigonometry
//   ph_face     + the closest face (closestFaceDodeca)                                 -> + face choice
//   ph_cell     + the whole fast path (projection, hex2d margins, _faceIjkToH3)        -> + hex2d and digits
//   ph_digits   _faceIjkToH3 alone on the rows' (face, ijk), loaded (16 B per row)     -> the digit loop's share
// Run under
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64
//             SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -- ./ingest_phases
// and reduce with tools/diag/ingest_phases.py (per-64-event instruction counts per phase, differences, durations).
// Build (tools/diag/Makefile-free): hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics
//   -o tools/diag/ingest_phases tools/diag/ingest_phases.hip
#include "../../real-time-mobility-heatmap_amd/csrc/mobheat.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

namespace diag {

constexpr int RES = 8;

__global__ void k_gen(double *lat, double *lon, int64_t *ts, uint64_t *vk, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h1 = mix64((uint64_t)i * 2 + 1), h2 = mix64((uint64_t)i * 2 + 2);
        const double u = (double)(h1 >> 11) * 0x1p-53, v = (double)(h2 >> 11) * 0x1p-53;
        lat[i] = asin(2.0 * u - 1.0) * 57.29577951308232;
        lon[i] = v * 360.0 - 180.0;
        ts[i] = 1759572000000000LL + (int64_t)(h1 % 900000000ull);
        vk[i] = h2 % 50000;
    }
}

// the LDS tables k_ingest keeps
struct Lds {
    double Fc[20][3], Fu[20][2][3];
    H3BaseTables BT;
};
__device__ void lds_load(Lds &L) {
    for (int k = threadIdx.x; k < 60; k += IG_THREADS) (&L.Fc[0][0])[k] = (&c_tab.faceCenterPoint[0][0])[k];
    for (int k = threadIdx.x; k < 120; k += IG_THREADS) (&L.Fu[0][0][0])[k] = (&c_tab.fastU[RES & 1][0][0][0])[k];
    for (int k = threadIdx.x; k < 20 * 27; k += IG_THREADS) L.BT.fijkPacked[k] = c_tab.fijkPacked[k];
    for (int k = threadIdx.x; k < 122; k += IG_THREADS) L.BT.bcdPacked[k] = c_tab.bcdPacked[k];
    for (int k = threadIdx.x; k < AP7_QUAD; k += IG_THREADS) L.BT.ap7Quad[k] = c_tab.ap7Quad[k];
    for (int k = threadIdx.x; k < AP7_PAIR; k += IG_THREADS) L.BT.ap7Pair[k] = c_tab.ap7Pair[k];
    __syncthreads();
}

// PH: 0 load, 1 sincos, 2 face, 3 cell
template <int PH>
__global__ __launch_bounds__(IG_THREADS) HM_SNAP_ATTR void k_phase(const double *__restrict__ lat, const double *__restrict__ lon,
                                                                   const int64_t *__restrict__ ts, const uint64_t *__restrict__ vk,
                                                                   int64_t n, unsigned long long *sink) {
    __shared__ Lds L;
    lds_load(L);
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * IG_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * IG_THREADS) {
        const double la = __builtin_nontemporal_load(&lat[i]), lo = __builtin_nontemporal_load(&lon[i]);
        const int64_t t = __builtin_nontemporal_load(&ts[i]);
        const uint64_t v = __builtin_nontemporal_load(&vk[i]);
        acc += (uint64_t)t ^ v;
        if constexpr (PH == 0) {
            acc += __builtin_bit_cast(uint64_t, la) ^ __builtin_bit_cast(uint64_t, lo);
        } else if constexpr (PH == 1 || PH == 2) {
            double sl, cl, sg, cg;
            sincos_small(la * 0.017453292519943295, sl, cl);
            sincos_small(lo * 0.017453292519943295, sg, cg);
            const double px = cg * cl, py = sg * cl, pz = sl;
            if constexpr (PH == 1) {
                acc += __builtin_bit_cast(uint64_t, px + py + pz);
            } else {
                int face = 0;
                const bool ok = closestFaceDodeca((float)px, (float)py, (float)pz, face);
                acc += (uint64_t)face + ok;
            }
        } else {
            uint64_t cell = 0;
            const bool ok = latLngToCellFastP(la, lo, RES, c_tab, L.Fc, L.Fu, cell, L.BT);
            acc += cell + ok;
        }
    }
    if (acc == 0x123456789ull) atomicAdd(sink, 1ull);
}

// the rows' (face, ijk) for ph_digits, from upstream's own sequence (not measured)
__global__ void k_face_ijk(const double *lat, const double *lon, int64_t n, int4 *fijk) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double sl, cl, sg, cg;
        sincos_small(lat[i] * 0.017453292519943295, sl, cl);
        sincos_small(lon[i] * 0.017453292519943295, sg, cg);
        const double px = cg * cl, py = sg * cl, pz = sl;
        int face = 0;
        (void)closestFaceDodeca((float)px, (float)py, (float)pz, face);
        const double *c = c_tab.faceCenterPoint[face];
        const double pc = fma(px, c[0], fma(py, c[1], pz * c[2]));
        const double(*u)[3] = c_tab.fastU[RES & 1][face];
        const double inv = c_tab.fastScale[RES] / pc;
        const double vx = fma(px, u[0][0], fma(py, u[0][1], pz * u[0][2])) * inv;
        const double vy = fma(px, u[1][0], fma(py, u[1][1], pz * u[1][2])) * inv;
        const IJK h = hex2dToCoordIJK(vx, vy);
        fijk[i] = make_int4(face, h.i, h.j, h.k);
    }
}

__global__ __launch_bounds__(IG_THREADS) HM_SNAP_ATTR void k_phase_digits(const int4 *__restrict__ fijk, int64_t n,
                                                                          unsigned long long *sink) {
    __shared__ Lds L;
    lds_load(L);
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * IG_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * IG_THREADS) {
        const int4 f = fijk[i];
        IJK h{f.y, f.z, f.w};
        acc += faceIjkToH3(f.x, h, RES, L.BT);
    }
    if (acc == 0x123456789ull) atomicAdd(sink, 1ull);
}

}  // namespace diag

int main() {
    const int64_t n = 100000000;
    CK(hipSetDevice(0));
    CK(upload_tables());
    double *lat, *lon;
    int64_t *ts;
    uint64_t *vk;
    int4 *fijk;
    unsigned long long *sink;
    CK(hipMalloc(&lat, n * 8));
    CK(hipMalloc(&lon, n * 8));
    CK(hipMalloc(&ts, n * 8));
    CK(hipMalloc(&vk, n * 8));
    CK(hipMalloc(&fijk, n * 16));
    CK(hipMalloc(&sink, 8));
    hipLaunchKernelGGL(diag::k_gen, dim3(4096), dim3(256), 0, 0, lat, lon, ts, vk, n);
    hipLaunchKernelGGL(diag::k_face_ijk, dim3(4096), dim3(256), 0, 0, lat, lon, n, fijk);
    CK(hipDeviceSynchronize());
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = ncu * 6 * 4 / (IG_THREADS / 64) * 1;   // 6 waves per SIMD, as k_ingest's occupancy
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(diag::k_phase<0>, dim3(grid), dim3(IG_THREADS), 0, 0, lat, lon, ts, vk, n, sink);
        hipLaunchKernelGGL(diag::k_phase<1>, dim3(grid), dim3(IG_THREADS), 0, 0, lat, lon, ts, vk, n, sink);
        hipLaunchKernelGGL(diag::k_phase<2>, dim3(grid), dim3(IG_THREADS), 0, 0, lat, lon, ts, vk, n, sink);
        hipLaunchKernelGGL(diag::k_phase<3>, dim3(grid), dim3(IG_THREADS), 0, 0, lat, lon, ts, vk, n, sink);
        hipLaunchKernelGGL(diag::k_phase_digits, dim3(grid), dim3(IG_THREADS), 0, 0, fijk, n, sink);
    }
    CK(hipDeviceSynchronize());
    // the product's k_ingest, both variants (MOBHEAT_INGEST_MODE direct = k_ingest<false>, binned = k_ingest<true>)
    for (const char *mode : {"direct", "binned"}) {
        setenv("MOBHEAT_INGEST_MODE", mode, 1);
        hm_config cfg{};
        cfg.abi_version = HM_ABI_VERSION;
        cfg.h3_res = diag::RES;
        cfg.device = 0;
        cfg.late_uses_prev_watermark = 1;
        cfg.tile_us = 300000000;
        cfg.watermark_delay_ms = 600000;
        cfg.batch_capacity_hint = n;
        cfg.state_arena_bytes = (int64_t)40 << 30;
        hm_ctx *ctx = nullptr;
        if (hm_create(&cfg, &ctx) != HM_OK) { printf("hm_create: %s\n", hm_last_error(nullptr)); return 1; }
        for (int step = 0; step < 2; step++) {
            hm_batch_in in{};
            in.n = n;
            in.memory = HM_MEM_DEVICE;
            in.lat = lat;
            in.lon = lon;
            in.ts_us = ts;
            in.vkey = vk;
            hm_batch_out out{};
            if (hm_process_batch(ctx, step, &in, HM_MEM_DEVICE, &out) != HM_OK) { printf("batch: %s\n", hm_last_error(ctx)); return 1; }
            printf("%s step %d: %lld tiles\n", mode, step, (long long)out.n_tiles);
        }
        hm_destroy(ctx);
    }
    printf("done\n");
    return 0;
}
