// Kafka values -> batch columns (from_json + to_timestamp, heatmap_stream.py:88-93) and the string dictionaries.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// =====================================================================================================
// K0: Kafka values -> batch columns (row f1: from_json + to_timestamp, heatmap_stream.py:88-93; json_decode.h),
// one thread per record; then the exact string dictionaries of provider and vehicleId (hash table keyed by a
// 64-bit string hash, every row verified byte for byte against its slot's representative; a hash collision
// reruns the dictionary with another seed) and vkey = provider_code * n_vehicles + vehicle_code.
// =====================================================================================================
constexpr int64_t SPAN_SCRATCH = INT64_C(1) << 62;   // span offset flag: the decoded bytes are in the scratch buffer
__global__ __launch_bounds__(256) void k_json_parse(const uint8_t *__restrict__ bytes, const int64_t *__restrict__ offs,
                                                    int64_t base, int64_t n, uint8_t *__restrict__ scratch,
                                                    double *__restrict__ lat, double *__restrict__ lon,
                                                    int64_t *__restrict__ ts, double *__restrict__ speed,
                                                    uint8_t *__restrict__ sv, uint8_t *__restrict__ rv,
                                                    int64_t *__restrict__ p_off, int32_t *__restrict__ p_len,
                                                    int64_t *__restrict__ v_off, int32_t *__restrict__ v_len,
                                                    uint8_t *__restrict__ unsup_row, unsigned long long *counts) {
    unsigned long long bad = 0, unsup = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        JsonRow r;
        parse_record(bytes, offs[i] - base, offs[i + 1] - base, scratch, r);
        const bool u = (r.flags & JF_UNSUPPORTED) != 0;
        const uint32_t f = u ? 0u : r.flags;   // an unsupported record stays an all-null row until the host splices it
        bad += (f & JF_MALFORMED) != 0;
        unsup += u;
        unsup_row[i] = u;
        lat[i] = (f & JF_LAT) ? r.lat : __builtin_nan("");
        lon[i] = (f & JF_LON) ? r.lon : __builtin_nan("");
        ts[i] = (f & JF_TS) ? r.ts_us : 0;
        speed[i] = (f & JF_SPEED) ? r.speed : 0.0;
        sv[i] = (f & JF_SPEED) ? 1 : 0;
        rv[i] = (f & JF_PROV) && (f & JF_VEH) && (f & JF_TS) ? 1 : 0;
        p_off[i] = r.p_off | ((f & JF_PROV_ESC) ? SPAN_SCRATCH : 0);
        p_len[i] = (f & JF_PROV) ? r.p_len : -1;
        v_off[i] = r.v_off | ((f & JF_VEH_ESC) ? SPAN_SCRATCH : 0);
        v_len[i] = (f & JF_VEH) ? r.v_len : -1;
    }
    bad = wave_sum(bad);
    unsup = wave_sum(unsup);
    if (lane_id() == 0) {
        if (bad) atomicAdd(&counts[0], bad);
        if (unsup) atomicAdd(&counts[1], unsup);
    }
}

__device__ __forceinline__ const uint8_t *span_ptr(const uint8_t *bytes, const uint8_t *scratch, int64_t off) {
    return (off & SPAN_SCRATCH) ? scratch + (off & ~SPAN_SCRATCH) : bytes + off;
}
__device__ __forceinline__ uint64_t str_hash(const uint8_t *s, int n, uint64_t seed) {
    uint64_t h = mix64(seed ^ ((uint64_t)n * UINT64_C(0x9e3779b97f4a7c15)));
    for (int k = 0; k < n; k += 8) {
        uint64_t x = 0;
        for (int q = 0; q < 8 && k + q < n; q++) x |= (uint64_t)s[k + q] << (8 * q);
        h = mix64(h ^ x) + UINT64_C(0x632be59bd9b4e019);
    }
    return h & ~(UINT64_C(1) << 63);   // (never DICT_EMPTY)
}
struct DictSlot {   // cleared to all-ones bytes
    unsigned long long key;   // str_hash, < 2^63; ~0 = empty
    unsigned rep;             // the smallest row holding the string
    unsigned pad;
};
constexpr unsigned long long DICT_EMPTY = ~0ull;
constexpr int DICT_PROBES = 64;
__global__ __launch_bounds__(256) void k_dict_insert(const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ scratch,
                                                     const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                                                     int64_t n, DictSlot *tab, unsigned long long mask, uint64_t seed,
                                                     unsigned *__restrict__ slot_of, unsigned long long *overflow) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // this lane's last string and its slot: a later row of the same string (a higher row index: its representative is
    // already at most the earlier one's) takes the slot without touching the table
    uint64_t last_h = DICT_EMPTY;
    unsigned last_s = ~0u;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        const int32_t L = i < n ? len[i] : -1;
        const bool live = L >= 0;
        const uint64_t h = live ? str_hash(span_ptr(bytes, scratch, off[i]), L, seed) : 0;
        // the lanes holding the same string as the wave's first live lane take the slot that lane finds: one probe and
        // one representative update per wave for a column of few distinct values (a batch's one provider string put
        // every lane's CAS on one address: 4.7 ms of hm_arrow_columns per 1e7 rows, profiles/r6/r6p)
        const unsigned long long m = __ballot(live);
        const int leader = m ? __ffsll((long long)m) - 1 : 0;
        const bool follower = live && lane_id() != leader && h == __shfl(h, leader, 64);
        unsigned got = ~0u;
        if (live && !follower && h == last_h) {
            got = last_s;
        } else if (live && !follower) {
            unsigned long long s = mix64(h ^ seed) & mask;
            for (int p = 0; p < DICT_PROBES; p++) {
                // (plain loads: a slot's key never changes once set, so a key read equal to h is final and a stale
                // EMPTY only costs the CAS that returns the real one; a stale representative only an atomicMin that
                // changes nothing)
                unsigned long long k = tab[s].key;
                // (an EMPTY from the CU's cache may be stale: read the L2's before the CAS -- a CAS from every wave
                // of the first grid pass on a single-valued column's one slot serialised there, 2.3 ms per 1e7 rows)
                if (k == DICT_EMPTY) k = __hip_atomic_load(&tab[s].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (k == DICT_EMPTY) k = atomicCAS(&tab[s].key, DICT_EMPTY, (unsigned long long)h);
                if (k == DICT_EMPTY || k == h) {
                    // (the representative only moves down: a row above it adds nothing -- the leader's row is the
                    // lowest of its followers')
                    // (the L2's value before the atomicMin: a stale cached one sent every first-pass wave's atomicMin
                    // to the one slot, 1.6-2.2 ms per 1e7 rows)
                    if ((unsigned)i < tab[s].rep &&
                        (unsigned)i < __hip_atomic_load(&tab[s].rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        atomicMin(&tab[s].rep, (unsigned)i);
                    got = (unsigned)s;
                    break;
                }
                s = (s + 1) & mask;
            }
            if (got != ~0u) { last_h = h; last_s = got; }
        }
        const unsigned lead_got = __shfl(got, leader, 64);
        if (follower) got = lead_got;
        if (i < n) slot_of[i] = got;
        if (live && got == ~0u) atomicAdd(overflow, 1ull);
    }
}
// every row's bytes against its slot's representative: a mismatch is a 64-bit hash collision
__global__ __launch_bounds__(256) void k_dict_verify(const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ scratch,
                                                     const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                                                     int64_t n, const DictSlot *__restrict__ tab,
                                                     const unsigned *__restrict__ slot_of, unsigned long long *collide) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned s = slot_of[i];
        if (s == ~0u) continue;
        const unsigned r = tab[s].rep;
        if (r == (unsigned)i) continue;
        bool eq = len[r] == len[i];
        if (eq) {
            const uint8_t *a = span_ptr(bytes, scratch, off[i]), *b = span_ptr(bytes, scratch, off[r]);
            for (int k = 0; k < len[i] && eq; k++) eq = a[k] == b[k];
        }
        if (!eq) atomicAdd(collide, 1ull);
    }
}
__global__ __launch_bounds__(256) void k_dict_occ(const DictSlot *__restrict__ tab, int64_t cap, uint8_t *__restrict__ occ) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += stride) occ[s] = tab[s].key != DICT_EMPTY;
}
// code c = the c-th occupied slot (ascending): code_of_slot, and the code's string length
__global__ __launch_bounds__(256) void k_dict_codes(const int64_t *__restrict__ slots, const unsigned long long *n_codes,
                                                    const DictSlot *__restrict__ tab, const int32_t *__restrict__ len,
                                                    unsigned *__restrict__ code_of_slot, unsigned *__restrict__ clen) {
    const int64_t m = (int64_t)*n_codes;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += stride) {
        const int64_t s = slots[c];
        code_of_slot[s] = (unsigned)c;
        clen[c] = (unsigned)len[tab[s].rep];
    }
}
__global__ __launch_bounds__(256) void k_dict_gather(const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ scratch,
                                                     const int64_t *__restrict__ off, const int32_t *__restrict__ len,
                                                     const int64_t *__restrict__ slots, const unsigned long long *n_codes,
                                                     const DictSlot *__restrict__ tab, const unsigned long long *__restrict__ coff,
                                                     uint8_t *__restrict__ out) {
    const int64_t m = (int64_t)*n_codes;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += stride) {
        const unsigned r = tab[slots[c]].rep;
        const uint8_t *a = span_ptr(bytes, scratch, off[r]);
        for (int k = 0; k < len[r]; k++) out[coff[c] + k] = a[k];
    }
}
__global__ __launch_bounds__(256) void k_json_vkey(const uint8_t *__restrict__ rv, const unsigned *__restrict__ pslot,
                                                   const unsigned *__restrict__ vslot, const unsigned *__restrict__ pcode,
                                                   const unsigned *__restrict__ vcode, int64_t n, uint64_t n_vehicles,
                                                   uint64_t *__restrict__ vkey) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        vkey[i] = rv[i] ? (uint64_t)pcode[pslot[i]] * n_vehicles + vcode[vslot[i]] : 0;
}
// hm_json_patch: every valid row's vkey re-encoded for the extended vehicle dictionary (nv_old -> nv_new), then the
// host-decoded rows written over the unsupported ones (P = m rows of JsonPatchRow)
struct JsonPatchRow {
    int64_t row, ts_us, pcode, vcode;
    double lat, lon, speed;
    uint8_t sv, rv, pad[6];
};
static_assert(sizeof(JsonPatchRow) == 64, "JsonPatchRow is 64 B");
__global__ __launch_bounds__(256) void k_json_rekey(const uint8_t *__restrict__ rv, int64_t n, uint64_t nv_old,
                                                    uint64_t nv_new, uint64_t *__restrict__ vkey) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (rv[i]) vkey[i] = vkey[i] / nv_old * nv_new + vkey[i] % nv_old;
}
__global__ __launch_bounds__(256) void k_json_patch(const JsonPatchRow *__restrict__ P, int64_t m, uint64_t nv,
                                                    double *__restrict__ lat, double *__restrict__ lon,
                                                    int64_t *__restrict__ ts, double *__restrict__ speed,
                                                    uint8_t *__restrict__ sv, uint8_t *__restrict__ rv,
                                                    uint64_t *__restrict__ vkey) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += stride) {
        const JsonPatchRow p = P[k];
        const int64_t i = p.row;
        lat[i] = p.lat;
        lon[i] = p.lon;
        ts[i] = p.ts_us;
        speed[i] = p.speed;
        sv[i] = p.sv;
        rv[i] = p.rv;
        vkey[i] = p.rv ? (uint64_t)p.pcode * nv + (uint64_t)p.vcode : 0;
    }
}
// the distinct 900-s buckets of the latest rows' eventTs (a set of int64, EMPTY = INT64_MIN), compacted into list
__global__ __launch_bounds__(256) void k_latest_buckets(const int64_t *__restrict__ rows, int64_t m,
                                                        const int64_t *__restrict__ ts, long long *set, unsigned long long mask,
                                                        long long *list, unsigned long long *n_list) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m; q += stride) {
        const long long b = (long long)floordiv(floordiv(ts[rows[q]], 1000000), 900);
        unsigned long long s = mix64((uint64_t)b) & mask;
        for (unsigned long long p = 0; p <= mask; p++) {
            long long k = __hip_atomic_load(&set[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == INT64_MIN) {
                k = atomicCAS((unsigned long long *)&set[s], (unsigned long long)INT64_MIN, (unsigned long long)b);
                if (k == INT64_MIN) { list[atomicAdd(n_list, 1ull)] = b; break; }
            }
            if (k == b) break;
            s = (s + 1) & mask;
        }
    }
}
__global__ __launch_bounds__(256) void k_fill_i64(long long *p, int64_t n, long long v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

// hm_arrow_columns: Arrow nulls -> the batch columns' conventions (lat / lon NaN, speed_valid, row_valid), in place on the
// values copied to the device; the string columns' spans (off into the column's bytes, len -1 = null) for dict_build
struct ArrowDevCol {
    const void *offs;         // string columns: n + 1 offsets (4 or 8 B), relative to data
    const uint8_t *valid;     // validity bitmap bytes from bit 0 = row 0 (shifted copy), nullptr = no nulls
    int64_t base;             // string columns: offs[0] (the bytes were copied from it)
    int32_t offset_bytes;
    int16_t present;          // 0: the column is absent (every row null)
    int16_t bit0;             // row 0's bit in valid[0]
    int32_t ns;               // eventTs in nanoseconds: truncated toward zero to microseconds here (hm_arrow_col.unit)
};
__device__ __forceinline__ bool arrow_valid(const ArrowDevCol &c, int64_t i) {
    const int64_t j = i + c.bit0;
    return c.present && (!c.valid || ((c.valid[j >> 3] >> (j & 7)) & 1));
}
__device__ __forceinline__ int64_t arrow_off(const ArrowDevCol &c, int64_t i) {
    return (c.offset_bytes == 4 ? (int64_t)((const int32_t *)c.offs)[i] : ((const int64_t *)c.offs)[i]) - c.base;
}
// a string column's offsets: non-decreasing, every string shorter than 2^31 bytes
__global__ __launch_bounds__(256) void k_arrow_check_offsets(ArrowDevCol c, int64_t n, unsigned long long *bad) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long b = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t d = arrow_off(c, i + 1) - arrow_off(c, i);
        b += d < 0 || d > INT32_MAX;
    }
    b = wave_sum(b);
    if (b && lane_id() == 0) atomicAdd(bad, b);
}
__global__ __launch_bounds__(256) void k_arrow_prep(int64_t n, ArrowDevCol lat_c, ArrowDevCol lon_c, ArrowDevCol sp_c,
                                                    ArrowDevCol ts_c, ArrowDevCol pv_c, ArrowDevCol vh_c,
                                                    double *__restrict__ lat, double *__restrict__ lon,
                                                    double *__restrict__ speed, uint8_t *__restrict__ sv,
                                                    int64_t *__restrict__ ts, uint8_t *__restrict__ rv,
                                                    int64_t *__restrict__ poff, int32_t *__restrict__ plen,
                                                    int64_t *__restrict__ voff, int32_t *__restrict__ vlen) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const double qnan = __builtin_nan("");
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (!arrow_valid(lat_c, i)) lat[i] = qnan;
        if (!arrow_valid(lon_c, i)) lon[i] = qnan;
        const bool s = arrow_valid(sp_c, i);
        sv[i] = s;
        if (!s) speed[i] = 0.0;
        const bool t = arrow_valid(ts_c, i);
        if (!t) ts[i] = 0;
        else if (ts_c.ns) ts[i] = ts[i] / 1000;   // (C division: toward zero, as Arrow's unsafe ns -> us cast)
        const bool p = arrow_valid(pv_c, i), v = arrow_valid(vh_c, i);
        if (p) {
            const int64_t a = arrow_off(pv_c, i), b = arrow_off(pv_c, i + 1);
            poff[i] = a;
            plen[i] = (int32_t)(b - a);
        } else {
            poff[i] = 0;
            plen[i] = -1;
        }
        if (v) {
            const int64_t a = arrow_off(vh_c, i), b = arrow_off(vh_c, i + 1);
            voff[i] = a;
            vlen[i] = (int32_t)(b - a);
        } else {
            voff[i] = 0;
            vlen[i] = -1;
        }
        rv[i] = p && v && t;
    }
}
