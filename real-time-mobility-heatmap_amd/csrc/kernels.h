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

// F_CAND: the row's ts was >= its vkey's max when k_ingest's fused dedup saw it (every final winner is one)
enum : uint8_t { F_VALID = 1, F_AGG = 2, F_LATE = 4, F_CAND = 8 };

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

// tile partial record exchanged between stages / ranks (HM_TILE_REC_BYTES = 48): three 16-B parts, so that three
// lanes move one record with 16-B accesses.  count/nspeed are a batch's rows (< 2^32).  The key's
// hash is not carried: the consumers (partition, merge) recompute it -- they are memory-bound, and the bytes are
// read and written five times per batch and sent over xGMI on several GPUs.
struct alignas(16) TilePartial {
    uint64_t cell;
    int64_t wstart;
    uint32_t count;
    uint32_t nspeed;
    double sspeed;
    double slat;
    double slon;
};
static_assert(sizeof(TilePartial) == 48, "TilePartial is 48 B");
// a partial after the radix partition (k_rp_scatter): one 64-B line, so that the scatter's randomly placed records
// are whole-line writes (48-B records straddle 32-B sectors: partition 4.4 -> 7.3 ms), carrying the key's hash
// for the merge
struct alignas(64) SortedRec {
    uint64_t cell;
    int64_t wstart;
    uint64_t count;
    uint64_t nspeed;
    double sspeed;
    double slat;
    double slon;
    uint64_t hash;   // tile_hash(cell, wstart)
};
static_assert(sizeof(SortedRec) == 64, "SortedRec is 64 B");
// growth record: a live key of a window's old table moved into its new one (k_dump_gen -> rehash merge); keeps the
// slot's cumulative u64 counts and its touched word
struct alignas(64) GrowRec {
    uint64_t cell;
    int64_t wstart;
    uint64_t count;
    uint64_t nspeed;
    double sspeed;
    double slat;
    double slon;
    uint64_t touched;
};
static_assert(sizeof(GrowRec) == 64, "GrowRec is 64 B");

// ---- event keys (k_ingest's one output word per row) ----
// A cell of the context's resolution has constant bits 52-63 (mode 1, reserved 0, resolution), so a row's
// (cell, window) fits one word: the cell's low 52 bits and, in bits 52-63, 1 + the window's slot in the batch's
// window registry (WREG_SLOTS windows per batch).  0 = the row aggregates nothing (invalid, late, no window slot).
constexpr uint64_t CELL_LO = (UINT64_C(1) << 52) - 1;
constexpr int WREG_SLOTS = 4095;
HM_HD uint64_t ekey_make(uint64_t cell, unsigned widx) { return (cell & CELL_LO) | ((uint64_t)(widx + 1) << 52); }
HM_HD unsigned ekey_widx(uint64_t k) { return (unsigned)(k >> 52) - 1u; }
HM_HD uint64_t cell_hi_of(int res) { return (UINT64_C(1) << 59) | ((uint64_t)res << 52); }

// the direct path's partial record: one aggregated row (count 1), 32 B, so that the partition's randomly placed
// records are whole 32-B sectors.  speed = SPEED_NULL_BITS when speedKmh is null (a signalling-NaN payload: input
// NaNs are stored as the canonical quiet NaN, which Spark's double arithmetic yields too).
struct alignas(32) EventRec {
    uint64_t key;    // ekey
    double speed;
    double lat;
    double lon;
};
static_assert(sizeof(EventRec) == 32, "EventRec is 32 B");
constexpr uint64_t SPEED_NULL_BITS = UINT64_C(0x7ff0000000000001);
constexpr uint64_t CANON_NAN_BITS = UINT64_C(0x7ff8000000000000);

// per-window parameters of the batch, indexed by registry slot (the direct path's partition and merge)
struct alignas(32) WInfo {
    unsigned long long wenc;   // window start ^ 2^63
    uint64_t inner;            // mix64(windowStart + golden): tile_hash(cell, ws) = mix64(cell ^ inner)
    unsigned binp;             // radix bin parameters: (REGION_BITS - rbits) << 24 | (window salt & smask)
    unsigned gslot;            // multi-GPU sender: the window's slot in the batch's global registry
    unsigned pad[2];
};
static_assert(sizeof(WInfo) == 32, "WInfo is 32 B");
// A direct-mapped image of the batch's WInfo entries (slot & (WI_CACHE - 1)), built by the host next to the per-slot
// array; the partition and merge kernels copy it into LDS, so that a record's window parameters are an LDS read
// instead of a dependent global load (slots that collide in the image keep the global lookup).
constexpr int WI_CACHE = 64;
constexpr unsigned WI_NONE = 0xffffffffu, WI_CONFLICT = 0xfffffffeu;   // (never a registry slot)
struct WiCacheImg {
    unsigned tag[WI_CACHE];   // the registry slot held by the entry, or WI_NONE / WI_CONFLICT
    WInfo e[WI_CACHE];
};

// table mode (low cardinality): an aggregate evicted from k_agg's LDS table, bucketed by key hash for k_bin_reduce
struct alignas(16) AggRec {
    uint64_t key;              // ekey
    unsigned long long cnt;    // count | n_speed << 32
    double ssp;
    double slat;
    double slon;
    uint64_t pad;
};
static_assert(sizeof(AggRec) == 48, "AggRec is 48 B");

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

// Per-window state tables ("generations").  Every live window (windowStart) has its own open-addressing table
// of TileSlots; a window's keys never outlive it, so eviction releases the whole table (O(1), no compaction)
// and a released table is reused for a later window WITHOUT clearing: a slot belongs to window w iff its wenc
// is w's.  (Safe because a window never returns once evicted -- its rows are late from then on -- and a
// growing window only moves to larger tables, never back into one that still holds its stale keys.)
// A table of 2^L slots is split into 2^rbits regions of >= 256 slots; a key's region is taken from hash bits
// [32 - REGION_BITS, 32) and its slot from the low bits, linear probing wraps inside the region.  The radix partition
// sends all partials of (window, region) to ONE bin = (region << (REGION_BITS - rbits)) | (window salt), so the
// merge workgroup of a bin is the only writer of the regions it receives.
constexpr int GMAP_SLOTS = 4096;        // live windows per context (open addressing by wenc)
constexpr int REGION_MIN_BITS = 8;      // >= 256 slots per region (overflow-free at load <= 1/2)
// at most 2^REGION_BITS regions per table = radix bins of the partition (mobheat/distributed.py REGION_BITS: the
// multi-GPU owner ranges are ranges of this field)
constexpr int REGION_BITS = 13;
struct GenDesc {
    unsigned long long wenc;   // 0 = empty map slot
    TileSlot *tab;
    unsigned long long rmask;  // slots per region - 1
    unsigned short rshift;     // log2(slots per region)
    unsigned char rbits;       // log2(regions), <= REGION_BITS
    unsigned char sb;          // a key's table region is (region field >> sb) - rbase
    unsigned int rbase;        // (sb = REGION_BITS - rbits, rbase = 0: every region field has a region; sb = 0:
                               // the table holds the region fields [rbase, rbase + 2^rbits) -- a shard's owned range)
    unsigned long long count;  // keys of this window in its table (the merge adds created keys)
    unsigned long long batch_parts;   // partials of the current batch in this window (0: not merged into now)
};
static_assert(sizeof(GenDesc) == 48, "GenDesc is 48 B");
// Every table of 2^L slots is followed by 2^L one-byte slot tags (0 = empty, else tag8 of the key's hash), zeroed
// whenever the table is (re)acquired.  The owner merge keeps a region's tags in LDS, so finding a free slot for a
// new key reads nothing from HBM and an occupied slot is read only when its tag matches (1/255 of mismatches).
HM_HD uint8_t *gen_tags(const GenDesc &g) { return (uint8_t *)(g.tab + ((g.rmask + 1) << g.rbits)); }
HM_HD unsigned tag8(uint64_t h) { const unsigned t = (unsigned)(h >> 40) & 0xffu; return t ? t : 1u; }

// partial count per window of a batch (the census that sizes the tables)
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
    unsigned long long n_state_new; // keys created in the state tables
    unsigned long long n_dedup_used;
    unsigned long long n_cands;
    unsigned long long overflow;    // nonzero: a hash table probe bound was exceeded
    unsigned long long bad_vkey;
    unsigned long long dedup_retry; // k_ingest: a vkey probe hit its bound; rerun k_dedup_max on a larger table
    unsigned long long n_gaps;      // partial slots holding no record (gaps)
    unsigned long long win_overflow; // k_ingest: rows of windows beyond the batch's window registry (WREG_SLOTS)
    unsigned long long agg_spill;   // table mode: aggregates that did not fit a bucket (sent as partial records)
    unsigned long long n_evicted;   // table mode: aggregates k_agg evicted into the buckets
    unsigned long long sample_max_run;   // k_sample_heavy: occurrences of the most frequent key in a key sample
    unsigned long long bin_overflow;     // k_ingest<true>: rows whose bin slab was full (the batch re-partitions)
    unsigned long long vkey_max1;        // k_ingest: max vkey + 1 of its deduplicated rows (capped at 2^62; sizes the
                                         // next batch's dense dedup table)
};

// the dense dedup table's word: a max ts with its sign bit flipped (k_ingest.h: unsigned order = signed order, 0 = none)
constexpr unsigned long long DENSE_SIGN = 0x8000000000000000ull;

HM_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= UINT64_C(0xff51afd7ed558ccd);
    x ^= x >> 33;
    x *= UINT64_C(0xc4ceb9fe1a85ec53);
    x ^= x >> 33;
    return x;
}
HM_HD uint64_t window_inner(int64_t w) { return mix64((uint64_t)w + UINT64_C(0x9e3779b97f4a7c15)); }
HM_HD uint64_t tile_hash(uint64_t cell, int64_t w) { return mix64(cell ^ window_inner(w)); }
// floor(t / d) for d >= 1 by an invariant-divisor multiply (Granlund & Montgomery 1994, Fig. 4.1, N = 64):
// m = floor(2^64 (2^l - d) / d) + 1, l = ceil(log2 d); exact for every 64-bit dividend.  make_floor_div (host).
struct FloorDiv {
    uint64_t m;
    int s1, s2;
    int64_t d;
};
HM_HD uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
HM_HD uint64_t udiv_inv(uint64_t u, const FloorDiv &D) {
    const uint64_t hi = umulhi64(D.m, u);
    return (hi + ((u - hi) >> D.s1)) >> D.s2;
}
HM_HD int64_t floor_div(int64_t t, const FloorDiv &D) {
    if (t >= 0) return (int64_t)udiv_inv((uint64_t)t, D);
    return -(int64_t)udiv_inv((uint64_t)(-(t + 1)), D) - 1;   // floor((-1 - u) / d) = -(u / d) - 1
}
inline FloorDiv make_floor_div(int64_t d) {
    FloorDiv D;
    int l = 0;
    while ((UINT64_C(1) << l) < (uint64_t)d && l < 63) l++;
    if ((UINT64_C(1) << l) < (uint64_t)d) l = 64;
    const unsigned __int128 two_l = l == 64 ? ((unsigned __int128)1 << 64) : ((unsigned __int128)1 << l);
    D.m = (uint64_t)((((unsigned __int128)1 << 64) * (two_l - (uint64_t)d)) / (uint64_t)d + 1);
    D.s1 = l < 1 ? l : 1;
    D.s2 = l > 1 ? l - 1 : 0;
    D.d = d;
    return D;
}

HM_HD uint64_t vkey_hash(uint64_t v) { return mix64(v ^ UINT64_C(0x2545f4914f6cdd1d)); }
// owner rank of a vkey (latest-position candidates): high hash bits
HM_HD int owner_of(uint64_t h, int nranks) { return (int)(((h >> 32) * (uint64_t)nranks) >> 32); }
// a key's REGION_BITS-bit region field, hash bits [32 - REGION_BITS, 32) (independent of the table size)
HM_HD unsigned region_field(uint64_t h) { return (unsigned)(h >> (32 - REGION_BITS)) & ((1u << REGION_BITS) - 1); }
// A key's home slot inside its region (2^rshift slots, rshift >= 8): the hash's SUB_BITS bits below the region field
// pick one of 2^SUB_BITS sub-regions, its low bits the slot there -- so the records of one sub-bin (k_ingest's binning by
// region field and those bits, hm_process_batch) land in one eighth of every window's region, and the merge, taking a
// bin's sub-bins in order, writes its state lines inside a window of 1/8 of the region at a time (64-B lines written at
// random inside 64 KB instead of 512 KB: 1.55 vs 1.84 ms per 1e8, tools/microbench/line_scatter.hip)
constexpr int SUB_BITS = 3;
constexpr int SUB_SHIFT = 32 - REGION_BITS - SUB_BITS;   // bits [16, 19): below the region field, above every slot's low bits
HM_HD unsigned sub_field(uint64_t h) { return (unsigned)(h >> SUB_SHIFT) & ((1u << SUB_BITS) - 1); }
HM_HD unsigned long long inreg_slot(uint64_t h, unsigned long long rmask) {
    const unsigned long long low = rmask >> SUB_BITS;
    return ((unsigned long long)sub_field(h) * (low + 1)) | (h & low);
}
// owner rank of a tile key (hash h): contiguous ranges of region fields, so that a rank's (window, region) bins --
// k_ingest's fused binning -- are already grouped by owner, and an owner's tables hold only its range
HM_HD int tile_owner_of(uint64_t h, int nranks) { return (int)((region_field(h) * (unsigned)nranks) >> REGION_BITS); }
// the region fields rank r of nranks owns: [shard_lo(r), shard_lo(r + 1))
HM_HD unsigned shard_lo(int r, int nranks) { return (unsigned)(((r << REGION_BITS) + nranks - 1) / nranks); }
HM_HD unsigned window_salt(unsigned long long we) { return (unsigned)mix64(we ^ UINT64_C(0x51ed270b27e5b3c1)); }

}  // namespace hm
