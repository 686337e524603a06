// BSON `update` statements for the tiles collection, encoded on the GPU.
//
// The reference builds one UpdateOne per emitted tile in a driver-side Python loop (heatmap_stream.py:164-188):
//   _id = f"{CITY}|h3r{H3_RES}|{cellId}|{windowStart:%Y-%m-%dT%H:%M:%SZ}", the $set document
//   {_id, city, grid, cellId, windowStart, windowEnd, count, avgSpeedKmh, centroid {type, coordinates [lon, lat]},
//   staleAt = windowEnd + TTL}, UpdateOne({_id}, {$set: doc}, upsert=True), written with unordered bulk_write
//   (:191-196).  pymongo turns each UpdateOne into the statement {q, u, multi: false, upsert: true} of an `update`
//   command (pymongo/synchronous/bulk.py add_update).  This file writes exactly those statement bytes, one
//   document per tile, so the host only slices the buffer into the command batches.
//
// Value rules reproduced (bson 4.x encoder, Python semantics of the reference's expressions):
//   * datetimes are pyspark's naive LOCAL wall times (TimestampType.fromInternal); bson encodes a naive datetime
//     as if it were UTC, so a field's int64 is (utc seconds + the local offset at that instant) x 1000; the
//     offsets of each window's start and end are computed by the host (hm_tile_doc_cfg) -- staleAt is the naive
//     windowEnd + timedelta(TTL), i.e. the end's local value + TTL;
//   * count: Python int -> int32 (0x10) when it fits, else int64 (0x12);
//   * `float(x or 0.0)`: a zero of either sign becomes +0.0, NaN is kept (truthy); avg(speed) null -> 0.0;
//   * strings: int32 length (bytes + 1), bytes, NUL; cellId = format(cell, "x").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"   // HM_HD

namespace hm {

constexpr int TD_THREADS = 128;
constexpr int TD_MAX_DOC = 576;    // statements up to this size go through k_tile_docs' LDS staging (a city of <= 64
                                   // bytes); longer ones (a long CITY) are written by k_tile_docs_direct

struct TileDocParams {
    const uint8_t *city;          // device copy, city_len bytes
    int city_len;
    int h3_res;
    int64_t tile_us;
    int64_t ttl_ms;
    const int64_t *win_start_us;  // n_win sorted window starts of the batch, and the local offsets (s) of
    const int64_t *off_start_s;   // each window's start and end instants
    const int64_t *off_end_s;
    int n_win;
};

// writer: measure mode (p == nullptr) only counts
struct BsonW {
    uint8_t *p;
    int n;
    HM_HD void u8(uint8_t v) { if (p) p[n] = v; n++; }
    HM_HD void i32(int32_t v) { for (int k = 0; k < 4; k++) u8((uint8_t)((uint32_t)v >> (8 * k))); }
    HM_HD void i64(int64_t v) { for (int k = 0; k < 8; k++) u8((uint8_t)((uint64_t)v >> (8 * k))); }
    HM_HD void f64(double v) { int64_t b; __builtin_memcpy(&b, &v, 8); i64(b); }
    HM_HD void key(uint8_t type, const char *k) {
        u8(type);
        for (int q = 0; k[q]; q++) u8((uint8_t)k[q]);
        u8(0);
    }
    HM_HD int begin() { const int at = n; i32(0); return at; }   // a document's length, patched by end()
    HM_HD void end(int at) {
        u8(0);
        if (p) { const int32_t len = n - at; for (int k = 0; k < 4; k++) p[at + k] = (uint8_t)((uint32_t)len >> (8 * k)); }
    }
};

HM_HD double py_or_zero(double v) { return v == 0.0 ? 0.0 : v; }   // float(v or 0.0)

// proleptic Gregorian civil date of a day count since 1970-01-01 (days_from_civil inverse)
HM_HD void civil_from_days(int64_t z, int64_t &y, int &m, int &d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    d = (int)(doy - (153 * mp + 2) / 5 + 1);
    m = (int)(mp < 10 ? mp + 3 : mp - 9);
    y = yoe + era * 400 + (m <= 2);
}

HM_HD int64_t floordiv(int64_t a, int64_t b) { return a / b - ((a % b != 0) && ((a < 0) != (b < 0))); }

// the _id string's bytes (without NUL): city|h3r{res}|{hex cell}|YYYY-MM-DDTHH:MM:SSZ of the local start
HM_HD void tile_id(BsonW &w, const TileDocParams &P, uint64_t cell, int64_t local_start_s) {
    for (int q = 0; q < P.city_len; q++) w.u8(P.city[q]);
    w.u8('|'); w.u8('h'); w.u8('3'); w.u8('r');
    if (P.h3_res >= 10) w.u8((uint8_t)('0' + P.h3_res / 10));
    w.u8((uint8_t)('0' + P.h3_res % 10));
    w.u8('|');
    int nd = 1;
    while (nd < 16 && (cell >> (4 * nd))) nd++;
    for (int q = nd - 1; q >= 0; q--) {
        const unsigned v = (unsigned)(cell >> (4 * q)) & 15u;
        w.u8((uint8_t)(v < 10 ? '0' + v : 'a' + v - 10));
    }
    w.u8('|');
    const int64_t days = floordiv(local_start_s, 86400);
    const int64_t sod = local_start_s - days * 86400;
    int64_t y;
    int mo, d;
    civil_from_days(days, y, mo, d);
    const int hh = (int)(sod / 3600), mi = (int)(sod / 60 % 60), ss = (int)(sod % 60);
    w.u8((uint8_t)('0' + y / 1000 % 10)); w.u8((uint8_t)('0' + y / 100 % 10)); w.u8((uint8_t)('0' + y / 10 % 10));
    w.u8((uint8_t)('0' + y % 10)); w.u8('-');
    w.u8((uint8_t)('0' + mo / 10)); w.u8((uint8_t)('0' + mo % 10)); w.u8('-');
    w.u8((uint8_t)('0' + d / 10)); w.u8((uint8_t)('0' + d % 10)); w.u8('T');
    w.u8((uint8_t)('0' + hh / 10)); w.u8((uint8_t)('0' + hh % 10)); w.u8(':');
    w.u8((uint8_t)('0' + mi / 10)); w.u8((uint8_t)('0' + mi % 10)); w.u8(':');
    w.u8((uint8_t)('0' + ss / 10)); w.u8((uint8_t)('0' + ss % 10)); w.u8('Z');
}

HM_HD void tile_str(BsonW &w, const char *k, const TileDocParams &P, uint64_t cell, int64_t local_start_s) {
    w.key(0x02, k);
    int nd = 1;
    while (nd < 16 && (cell >> (4 * nd))) nd++;
    w.i32(P.city_len + 5 + (P.h3_res >= 10) + 1 + nd + 1 + 20 + 1);   // city|h3r{res}|{hex}|{date} + NUL
    tile_id(w, P, cell, local_start_s);
    w.u8(0);
}

HM_HD void str_field(BsonW &w, const char *k, const uint8_t *s, int len) {
    w.key(0x02, k);
    w.i32(len + 1);
    for (int q = 0; q < len; q++) w.u8(s[q]);
    w.u8(0);
}

// one statement {q: {_id}, u: {$set: doc}, multi: false, upsert: true}; returns its length
HM_HD int tile_statement(uint8_t *dst, const TileDocParams &P, uint64_t cell, int64_t ws_us, int64_t count,
                              double avg_speed, uint8_t speed_null, double avg_lon, double avg_lat) {
    // the window's local offsets (binary search over the batch's few windows)
    int lo = 0, hi = P.n_win - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P.win_start_us[mid] < ws_us) lo = mid + 1; else hi = mid;
    }
    const int64_t start_s = floordiv(ws_us, 1000000), end_s = floordiv(ws_us + P.tile_us, 1000000);
    const int64_t ls = start_s + P.off_start_s[lo], le = end_s + P.off_end_s[lo];
    uint8_t grid[8] = {'h', '3', 'r', 0, 0, 0, 0, 0};
    int glen = 3;
    if (P.h3_res >= 10) grid[glen++] = (uint8_t)('0' + P.h3_res / 10);
    grid[glen++] = (uint8_t)('0' + P.h3_res % 10);
    // cellId = format(cell, "x")
    uint8_t hex[16];
    int nd = 1;
    while (nd < 16 && (cell >> (4 * nd))) nd++;
    for (int q = 0; q < nd; q++) {
        const unsigned v = (unsigned)(cell >> (4 * (nd - 1 - q))) & 15u;
        hex[q] = (uint8_t)(v < 10 ? '0' + v : 'a' + v - 10);
    }
    BsonW w{dst, 0};
    const int top = w.begin();
    w.key(0x03, "q");
    const int q = w.begin();
    tile_str(w, "_id", P, cell, ls);
    w.end(q);
    w.key(0x03, "u");
    const int u = w.begin();
    w.key(0x03, "$set");
    const int set = w.begin();
    tile_str(w, "_id", P, cell, ls);
    str_field(w, "city", P.city, P.city_len);
    str_field(w, "grid", grid, glen);
    str_field(w, "cellId", hex, nd);
    w.key(0x09, "windowStart");
    w.i64(ls * 1000);
    w.key(0x09, "windowEnd");
    w.i64(le * 1000);
    if (count >= INT32_MIN && count <= INT32_MAX) {
        w.key(0x10, "count");
        w.i32((int32_t)count);
    } else {
        w.key(0x12, "count");
        w.i64(count);
    }
    w.key(0x01, "avgSpeedKmh");
    w.f64(speed_null ? 0.0 : py_or_zero(avg_speed));
    w.key(0x03, "centroid");
    const int c = w.begin();
    str_field(w, "type", (const uint8_t *)"Point", 5);
    w.key(0x04, "coordinates");
    const int a = w.begin();
    w.key(0x01, "0");
    w.f64(py_or_zero(avg_lon));
    w.key(0x01, "1");
    w.f64(py_or_zero(avg_lat));
    w.end(a);
    w.end(c);
    w.key(0x09, "staleAt");
    w.i64(le * 1000 + P.ttl_ms);
    w.end(set);
    w.end(u);
    w.key(0x08, "multi");
    w.u8(0);
    w.key(0x08, "upsert");
    w.u8(1);
    w.end(top);
    return w.n;
}

// pass 1: statement sizes (u32) for the offsets scan
__global__ __launch_bounds__(256) void k_tile_doc_sizes(TileDocParams P, const uint64_t *__restrict__ cell, const int64_t *__restrict__ ws,
                                                        const int64_t *__restrict__ cnt, int64_t n, unsigned *__restrict__ sizes) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        sizes[i] = (unsigned)tile_statement(nullptr, P, cell[i], ws[i], cnt[i], 0.0, 1, 0.0, 0.0);
}

// pass 2: each thread writes its statement into LDS at its final offset relative to the block's first byte
// (shifted so LDS and HBM agree modulo 16), then the block stores its contiguous byte range with 16-B stores
// (bytes at the two edge lines, which neighbouring blocks share)
__global__ __launch_bounds__(TD_THREADS) void k_tile_docs(TileDocParams P, const uint64_t *__restrict__ cell, const int64_t *__restrict__ ws,
                                                          const int64_t *__restrict__ cnt, const double *__restrict__ sp,
                                                          const uint8_t *__restrict__ spn, const double *__restrict__ lon,
                                                          const double *__restrict__ lat, int64_t n,
                                                          const unsigned long long *__restrict__ off, uint8_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t buf[];   // TD_THREADS x (the launch's max statement) + 32
    for (int64_t b0 = (int64_t)blockIdx.x * TD_THREADS; b0 < n; b0 += (int64_t)gridDim.x * TD_THREADS) {
        const int64_t b1 = b0 + TD_THREADS < n ? b0 + TD_THREADS : n;
        const unsigned long long first = off[b0], last = off[b1];
        const unsigned long long base = first & ~15ull;
        const int64_t i = b0 + threadIdx.x;
        if (i < b1) tile_statement(buf + (off[i] - base), P, cell[i], ws[i], cnt[i], sp[i], spn[i], lon[i], lat[i]);
        __syncthreads();
        const unsigned long long endb = last - base;   // LDS bytes [first - base, endb) are this block's
        const unsigned long long nlines = (endb + 15) >> 4;
        for (unsigned long long L = threadIdx.x; L < nlines; L += TD_THREADS) {
            const unsigned long long s = L << 4;
            if (s >= first - base && s + 16 <= endb) {
                *(uint4 *)(out + base + s) = *(const uint4 *)(buf + s);
            } else {
                for (int k = 0; k < 16; k++) {
                    const unsigned long long x = s + k;
                    if (x >= first - base && x < endb) out[base + x] = buf[x];
                }
            }
        }
        __syncthreads();
    }
}

// statements longer than TD_MAX_DOC (a long CITY): each thread writes its own statement straight to HBM
__global__ __launch_bounds__(256) void k_tile_docs_direct(TileDocParams P, const uint64_t *__restrict__ cell, const int64_t *__restrict__ ws,
                                                          const int64_t *__restrict__ cnt, const double *__restrict__ sp,
                                                          const uint8_t *__restrict__ spn, const double *__restrict__ lon,
                                                          const double *__restrict__ lat, int64_t n,
                                                          const unsigned long long *__restrict__ off, uint8_t *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        tile_statement(out + off[i], P, cell[i], ws[i], cnt[i], sp[i], spn[i], lon[i], lat[i]);
}

// ---- positions_latest statements (reference heatmap_stream.py:211-228) ----
// UpdateOne({"_id": f"{provider}|{vehicleId}", "$or": [{"ts": {"$exists": False}}, {"ts": {"$lt": ts}}]},
//           {"$set": {provider, vehicleId, ts, loc: {type: "Point", coordinates: [lon, lat]}}}, upsert=True)
// for each latest row; provider / vehicleId come from the batch's string dictionaries (the host's factorization:
// vkey = provider_code * n_vehicles + vehicle_code), ts is pyspark's naive local datetime of eventTs (the local
// offset of the row's 900-s bucket floor(ts_s / 900), looked up in the caller's sorted list of the buckets the rows
// use), lat/lon the row's values as float().
struct PosDocParams {
    const int64_t *p_off;   // n_p + 1 offsets into p_bytes
    const uint8_t *p_bytes;
    const int64_t *v_off;
    const uint8_t *v_bytes;
    int64_t n_vehicles;
    int64_t n_providers;
    int64_t n_buckets;      // distinct 900-s buckets floor(ts_s / 900) of the rows, ascending, and the local
    const int64_t *bucket_id;   // offset (s) of each
    const int64_t *bucket_off;
};

// index of the row's 900-s bucket in P.bucket_id (binary search), -1 if absent
HM_HD int64_t position_bucket(const PosDocParams &P, int64_t ts_us) {
    const int64_t b = floordiv(floordiv(ts_us, 1000000), 900);
    int64_t lo = 0, hi = P.n_buckets;
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (P.bucket_id[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    return lo < P.n_buckets && P.bucket_id[lo] == b ? lo : -1;
}

// the row's codes and time bucket lie inside the caller's tables (else the host reports an error)
HM_HD bool position_ok(const PosDocParams &P, uint64_t vkey, int64_t ts_us) {
    if (P.n_vehicles <= 0 || vkey / (uint64_t)P.n_vehicles >= (uint64_t)P.n_providers) return false;
    return position_bucket(P, ts_us) >= 0;
}

HM_HD int64_t bson_date_ms(int64_t ts_us, int64_t off_s) {
    const int64_t s = floordiv(ts_us, 1000000);
    return (s + off_s) * 1000 + (ts_us - s * 1000000) / 1000;
}

HM_HD int position_statement(uint8_t *dst, const PosDocParams &P, uint64_t vkey, int64_t ts_us, double lat, double lon) {
    const int64_t pc = (int64_t)(vkey / (uint64_t)P.n_vehicles), vc = (int64_t)(vkey % (uint64_t)P.n_vehicles);
    const uint8_t *ps = P.p_bytes + P.p_off[pc], *vs = P.v_bytes + P.v_off[vc];
    const int pl = (int)(P.p_off[pc + 1] - P.p_off[pc]), vl = (int)(P.v_off[vc + 1] - P.v_off[vc]);
    const int64_t date = bson_date_ms(ts_us, P.bucket_off[position_bucket(P, ts_us)]);
    BsonW w{dst, 0};
    const int top = w.begin();
    w.key(0x03, "q");
    const int q = w.begin();
    w.key(0x02, "_id");
    w.i32(pl + 1 + vl + 1);
    for (int k = 0; k < pl; k++) w.u8(ps[k]);
    w.u8('|');
    for (int k = 0; k < vl; k++) w.u8(vs[k]);
    w.u8(0);
    w.key(0x04, "$or");
    const int arr = w.begin();
    w.key(0x03, "0");
    const int e0 = w.begin();
    w.key(0x03, "ts");
    const int e0t = w.begin();
    w.key(0x08, "$exists");
    w.u8(0);
    w.end(e0t);
    w.end(e0);
    w.key(0x03, "1");
    const int e1 = w.begin();
    w.key(0x03, "ts");
    const int e1t = w.begin();
    w.key(0x09, "$lt");
    w.i64(date);
    w.end(e1t);
    w.end(e1);
    w.end(arr);
    w.end(q);
    w.key(0x03, "u");
    const int u = w.begin();
    w.key(0x03, "$set");
    const int set = w.begin();
    str_field(w, "provider", ps, pl);
    str_field(w, "vehicleId", vs, vl);
    w.key(0x09, "ts");
    w.i64(date);
    w.key(0x03, "loc");
    const int c = w.begin();
    str_field(w, "type", (const uint8_t *)"Point", 5);
    w.key(0x04, "coordinates");
    const int a = w.begin();
    w.key(0x01, "0");
    w.f64(lon);
    w.key(0x01, "1");
    w.f64(lat);
    w.end(a);
    w.end(c);
    w.end(set);
    w.end(u);
    w.key(0x08, "multi");
    w.u8(0);
    w.key(0x08, "upsert");
    w.u8(1);
    w.end(top);
    return w.n;
}

// sizes (pass 1) and statements written straight to HBM (pass 2: one thread per statement; positions are at most
// one per vehicle, and their strings make the lengths vary, so there is no LDS staging)
__global__ __launch_bounds__(256) void k_pos_doc_sizes(PosDocParams P, const int64_t *__restrict__ rows, int64_t n,
                                                       const uint64_t *__restrict__ vk, const int64_t *__restrict__ ts,
                                                       unsigned *__restrict__ sizes, unsigned long long *bad) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t r = rows[i];
        const bool ok = position_ok(P, vk[r], ts[r]);
        if (!ok) atomicAdd(bad, 1ull);
        sizes[i] = ok ? (unsigned)position_statement(nullptr, P, vk[r], ts[r], 0.0, 0.0) : 0u;
    }
}
__global__ __launch_bounds__(256) void k_pos_docs(PosDocParams P, const int64_t *__restrict__ rows, int64_t n,
                                                  const uint64_t *__restrict__ vk, const int64_t *__restrict__ ts,
                                                  const double *__restrict__ lat, const double *__restrict__ lon,
                                                  const unsigned long long *__restrict__ off, uint8_t *__restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t r = rows[i];
        if (position_ok(P, vk[r], ts[r])) position_statement(out + off[i], P, vk[r], ts[r], lat[r], lon[r]);
    }
}

}  // namespace hm
