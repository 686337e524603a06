// Device kernels of the per-micro-batch hot path (reference heatmap_stream.py:96-133,198-207).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "h3_device.h"

namespace hm {

constexpr uint64_t EMPTY_CELL = 0;                        // H3 cells always have the mode bit set
constexpr int64_t EMPTY_WIN = INT64_MIN;                  // window starts are > INT64_MIN (rows near it are invalid)
constexpr uint64_t EMPTY_VKEY = ~UINT64_C(0);             // reserved by the ABI
constexpr int WAVE = 64;

enum : uint8_t { F_VALID = 1, F_AGG = 2, F_LATE = 4 };

// one persistent tile-state slot = one 64-B line. An all-zero slot is empty (tables are cleared with a
// memset): the window word holds wenc = windowStart ^ 2^63, and windowStart = INT64_MIN is never valid.
struct alignas(64) TileSlot {
    uint64_t cell;
    unsigned long long wenc;
    unsigned long long count;
    unsigned long long nspeed;
    double sspeed;
    double slat;
    double slon;
    unsigned long long touched;   // batch sequence number of the last update
};
static_assert(sizeof(TileSlot) == 64, "TileSlot must be one 64-B line");

// tile partial record exchanged between stages / ranks (HM_TILE_REC_BYTES = 56)
struct TilePartial {
    uint64_t cell;
    int64_t wstart;
    int64_t count;
    int64_t nspeed;
    double sspeed;
    double slat;
    double slon;
};
static_assert(sizeof(TilePartial) == 56, "TilePartial is 56 B");

// latest-position candidate (HM_CAND_REC_BYTES = 32)
struct Cand {
    uint64_t vkey;
    int64_t ts;
    int64_t row;
    int64_t origin;
};
static_assert(sizeof(Cand) == 32, "Cand is 32 B");

HM_HD unsigned long long wenc_of(int64_t w) { return (unsigned long long)w ^ (UINT64_C(1) << 63); }
HM_HD int64_t wdec(unsigned long long e) { return (int64_t)(e ^ (UINT64_C(1) << 63)); }

// live-key count per window (lazy eviction: dead keys stay in the table until the next compaction, so
// the number of live keys is the sum over windows whose end is after the watermark)
constexpr int WMAP_SLOTS = 4096;
struct WinCount {
    unsigned long long wenc;   // 0 = empty
    unsigned long long count;
};

struct alignas(16) DedupSlot {
    unsigned long long vkey;
    long long maxts;
};

// batch statistics written by the kernels (device), copied back once per batch
struct DevStats {
    unsigned long long n_valid;
    unsigned long long n_late;
    long long max_ts_ms;
    long long min_wstart;          // min window start inserted into the state since the last rebuild
    unsigned long long n_partials;
    unsigned long long n_touched;
    unsigned long long n_state_new; // keys created in the state table
    unsigned long long n_dedup_used;
    unsigned long long n_cands;
    unsigned long long overflow;    // nonzero: a hash table probe bound was exceeded
    unsigned long long bad_vkey;
    unsigned long long dedup_retry; // k_ingest: a vkey probe hit its bound; rerun k_dedup_max on a larger table
    unsigned long long pad[4];
};

HM_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= UINT64_C(0xff51afd7ed558ccd);
    x ^= x >> 33;
    x *= UINT64_C(0xc4ceb9fe1a85ec53);
    x ^= x >> 33;
    return x;
}
HM_HD uint64_t tile_hash(uint64_t cell, int64_t w) { return mix64(cell ^ mix64((uint64_t)w + UINT64_C(0x9e3779b97f4a7c15))); }
HM_HD uint64_t vkey_hash(uint64_t v) { return mix64(v ^ UINT64_C(0x2545f4914f6cdd1d)); }
// owner rank of a key: taken from high hash bits so it is independent of the table index bits
HM_HD int owner_of(uint64_t h, int nranks) { return (int)(((h >> 32) * (uint64_t)nranks) >> 32); }

}  // namespace hm
