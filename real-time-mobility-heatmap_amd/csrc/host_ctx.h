// Host side: the context (hm_ctx), allocation, per-window tables, partition / merge launchers.
// Part of the single translation unit mobheat.hip (included there in dependency order; not compiled alone).
#pragma once

// =====================================================================================================
// host side
// =====================================================================================================
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

struct Inputs {   // a batch's device columns
    const double *lat, *lon, *sp;
    const int64_t *ts;
    const uint8_t *sv, *rv;
    const uint64_t *vk;
    int64_t n;
};

struct hm_ctx {
    hm_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    hipEvent_t ev[11] = {};
    // host inputs: their copies run on copy_stream in row chunks, k_ingest on each chunk as soon as it has arrived
    // (stage_inputs records the sources, phase_local issues copies and launches)
    static constexpr int H2D_CHUNKS = 16;
    hipStream_t copy_stream = nullptr;
    // hm_process_batch's dedup (flag + compaction) runs on side_stream while the main stream partitions and merges:
    // the two bind on different units (the dedup streams flags and probes a cache-resident table; the partition is
    // write-pattern bound, the merge instruction-issue bound)
    hipStream_t side_stream = nullptr;
    hipEvent_t side_ev[4] = {};   // [3]: the pooled tables' tags cleared (table_release)
    bool dedup_side = false;
    bool dedup_main = false;   // MOBHEAT_DEDUP_STREAM=main: never the side stream
    bool dedup_early = false;  // this batch's side-stream dedup was launched behind k_ingest (phase_local)
    bool early_ok = true;      // MOBHEAT_DEDUP_EARLY=0: launched after the readback instead (A/B)
    bool offsets_early = true; // MOBHEAT_OFFSETS_EARLY=0: the bins' row offsets launched after the readback (A/B)
    hipEvent_t h2d_ev[H2D_CHUNKS] = {};
    struct H2D { const void *src; void *dst; size_t el; };
    H2D h2d[7] = {};
    int n_h2d = 0;
    double timings[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // host side of the last batch call (hm_last_timings [8, 14)): wall ms of the call, ms blocked in stream
    // synchronizations, ms in device/pinned allocations and frees, the longest single synchronization and its source
    // line, allocations + frees made
    double host_ms[6] = {0, 0, 0, 0, 0, 0};
    // per-event
    DevBuf in_lat, in_lon, in_ts, in_speed, in_sv, in_vkey, in_rv;
    DevBuf cell, wstart, flags, win, rows, block_counts, block_offs;
    DevBuf partials, cands, parts_sorted, rp_H, rp_O, rp_btot, rp_boff;
    DevBuf slow;   // k_ingest's fast-path exceptions (event indices) for k_ingest_exact
    // persistent tile state: one table per live window (kernels.h: GenDesc); released tables are pooled and
    // reused without clearing
    // a window's table: 2^log2cap slots in 2^rbits regions, a key's region (region field >> sb) - rbase (GenDesc)
    struct Gen { unsigned long long wenc; TileSlot *tab; int log2cap; unsigned rbits, sb, rbase; int64_t keys; int64_t batch_parts; };
    std::vector<Gen> gens;
    std::vector<std::pair<TileSlot *, int>> pool;   // (table, log2 slots)
    // state_arena_bytes: window tables carved from one zeroed reservation made at create (no driver allocation
    // inside a batch); carved tables are pooled like the others but never freed before the arena
    uint8_t *arena = nullptr;
    size_t arena_bytes = 0, arena_used = 0;
    GenDesc *d_gmap = nullptr, *h_gmap = nullptr;   // device map window -> table (host mirror)
    bool gmap_ready = false;                         // h_gmap holds the device map after this batch's merge
    GenDesc *d_glist = nullptr, *h_glist = nullptr; // the same descriptors as a dense list (kernels' LDS cache)
    int n_glist = 0;
    bool census_ready = false;                      // k_ingest filled d_cmap for this batch's partials
    WinCount *d_cmap = nullptr, *h_cmap = nullptr;  // census of the current batch's partials per window
    int64_t state_size = 0;           // live keys after the last batch
    DevBuf s_cell, s_ws, s_cnt, s_sp, s_spn, s_lon, s_lat;   // k_merge_owned's rows in per-bin segments (with gaps)
    DevBuf bin_cnt, bin_off;          // k_merge_owned: touched keys per bin, their output offsets
    DevBuf parts_regrow;              // growth: the old tables' keys as partial records
    int64_t touched_dump_seq = -1;    // parts_regrow holds hm_state_export_touched's dump of batch seq (-1: none)
    int64_t touched_dump_n = 0;
    int64_t export_dump_n = -1;       // hm_state_export_begin: records of the dump in parts_regrow (-1: none) ...
    unsigned long long export_dump_seq = 0;   // ... made after batch seq (hm_state_export_copy checks both)
    static constexpr int STM_PIECES = 64;
    hipEvent_t stm_ev[STM_PIECES] = {};   // HM_MEM_HOST_STREAM statements: piece k of the bytes landed
    int stm_pieces = 0;                   // pieces of the last streamed encode (0: none pending)
    int64_t stm_piece = 0, stm_total = 0;
    static constexpr int EXPORT_SLICES = 64;
    hipEvent_t export_ev[EXPORT_SLICES] = {};   // hm_state_export_copy_async: slice k landed
    DevBuf parts_regrow_sorted;       // growth: the same, partitioned (not parts_sorted: a binned batch's slabs are there)
    // multi-GPU exchange (api_stage.h): chunk starts and headers, the local -> global window slot map; the owner's
    // per-sender bin counts and their scan, its bins' segments, the received candidates and table-mode partials
    DevBuf stage_meta, stage_C, stage_P, stage_SO, stage_SP, stage_T, cands_recv, stage_tmp;
    DevBuf gapbuf;                    // k_gap_counts / k_fill_gaps: per-bin gap and donor counts + donor offsets
    unsigned long long seq = 0;
    // dedup table (persistent, cleared through its used list)
    // latest-position tables (16-B slots, cleared through their used lists): `fused` is k_ingest's, sized from the
    // last batch's distinct vkeys and kept small (cache residency is its speed); `full` serves the max pass when
    // the fused one gave up, and received candidates (multi-GPU): grow-only, so it is allocated once
    struct DedupTable {
        DedupSlot *tab = nullptr;
        unsigned long long cap = 0;
        DevBuf used;
        bool dirty = false;
        int used_word = 0;   // d_scratch word counting the used slots
    } dfused, dfull;
    DedupTable *dlast = nullptr;   // the table the last batch's flags were computed on
    int64_t dedup_seen = 0;
    int64_t n_partials_merged = 0;   // partial records of the last merge (hm_batch_out.n_partials)
    int ingest_grid = 0;             // k_ingest's persistent grid: resident workgroups per CU x CUs
    int ingest_grid_bin = 0;         // the same for k_ingest<true> (fused binning)
    int64_t last_binned = 0;         // hm_last_counts [8]: the last batch was binned in k_ingest
    int n_cus = 0;
    // aggregation path: direct (event records -> partition -> merge) or table (k_agg + k_bin_reduce, low
    // cardinality); MOBHEAT_INGEST_MODE pins one (0 adaptive, 1 direct, 2 table)
    int ingest_mode = 0;
    // k_merge_owned's grid: 0 = one workgroup per bin; else that many persistent workgroups looping over the bins
    // (MOBHEAT_MERGE_GRID, tuning)
    int merge_grid = 0;
    int64_t prev_agg_rows = 0, prev_keys = 0;   // aggregated rows and distinct keys of the last batch
    bool merge_coop = false;   // the last batch's keys were mostly existing ones: the merge's cooperative probe
    bool coop_predict = true;  // MOBHEAT_COOP_PREDICT=0: the merge variant from the last batch (merge_coop) alone
    bool last_table = false;
    int64_t last_counts[6] = {0, 0, 0, 0, 0, 0};   // hm_last_counts [0, 6) ([6], [7]: n_allocs, n_frees)
    int64_t n_allocs = 0, n_frees = 0;             // device + pinned-host allocations / frees since create
    int64_t table_evicted = 0;                   // table mode: aggregates k_agg evicted into its buckets (last batch)
    // hm_decode_json (row f1): the values on the device, the decoded columns, the string dictionaries
    struct Dict {
        DevBuf tab, slot_of, occ, slots, code_of_slot, clen, coff, cbytes, btot, boff;
        int64_t last_codes = 0;   // distinct strings of the last batch (sizes the next table: cache-resident)
        int64_t n_codes = 0;
        void *h_off = nullptr, *h_bytes = nullptr;   // pinned host copies of the dictionary
        size_t h_off_cap = 0, h_bytes_cap = 0;
    };
    DevBuf jd_bytes, jd_offs, jd_scratch, jd_lat, jd_lon, jd_ts, jd_speed, jd_sv, jd_rv, jd_vkey, jd_poff, jd_plen, jd_voff,
        jd_vlen, jd_un, jd_unrows, jd_patch;
    std::vector<int64_t> jd_unsup;      // the last hm_decode_json's unsupported rows (HM_JSON_SPLICE)
    int64_t jd_n = -1, jd_np = 0, jd_nv = 0;   // its row count (-1: none to patch) and dictionary sizes
    Dict jd_prov, jd_veh;
    DevBuf ar_bits[6], ar_offs[2], ar_data[2];   // hm_arrow_columns: validity bitmaps, the string columns' offsets / bytes
    DevBuf lb_set, lb_list;   // hm_last_latest_buckets
    DevBuf keys;                     // k_ingest's event key per row (kernels.h ekey)
    // k_ingest's fused binning (large direct-path batches): the bins' cursors (RP_BINS + 1 u32: the last stays 0, so
    // that their exclusive scan ends with the total) and the slab capacity; the slabs are parts_sorted
    DevBuf bin_cur;
    unsigned slab_cap = 0;           // records per bin slab of this batch (0: not binned in k_ingest)
    unsigned *h_bincur = nullptr;    // the cursors read back (pinned): the fullest bin sizes the next batch's slabs
    double bin_skew = 1.0;           // the last binned batch's fullest bin / mean bin
    bool binned = false;             // this batch's rows are in their bins (k_ingest<true>, no slab overflowed)
    bool keys_partial = false;       // k_ingest<true> wrote only the exception and sampled rows' keys (keys_complete)
    int64_t keys_late_us = 0;        // (the batch's late watermark, which keys_complete's pass needs again)
    bool bin_offsets_ready = false;  // the bins' row offsets (bin_offsets) already launched behind k_ingest
    // the bins split into sub-bins by sub-region (k_ingest sub_bits: SUB_BITS, or 0 = whole bins): on hm_process_batch's
    // binned batches when the last batch re-touched mostly existing keys (merge_coop) -- its merge then reads old state
    // lines inside 1/8 of each region at a time (state-read leg 6.6-6.75 -> 5.25-5.36 ms), while a batch of new keys
    // keeps whole bins (65536 cursors and slabs cost k_ingest +0.5-0.7 ms and gain its merge nothing: profiles/r5/r5sub/);
    // the stage API's senders keep whole bins.  MOBHEAT_SUBBINS=0 never, =1 always (tests, A/B)
    unsigned sub_bits = 0;
    int subbins_mode = 2;
    unsigned long long *d_wreg = nullptr, *h_wreg = nullptr;     // the batch's window registry (WREG_SLOTS wenc)
    unsigned long long *d_wcount = nullptr, *h_wcount = nullptr; // aggregated rows per registry slot (census)
    WInfo *d_winfo = nullptr, *h_winfo = nullptr;   // per registry slot: window parameters of the direct path
    hipEvent_t winfo_ev = nullptr;                    // recorded after the last upload from h_winfo
    hipEvent_t ext_ev = nullptr;                      // hm_stream_wait: recorded on the caller's stream
    DevBuf agg_bucket, agg_cursor;   // table mode: k_agg's buckets (AG_BINS x AG_SUB x cap AggRecs) + fill cursors
    unsigned agg_cap = 0;            // AggRecs per sub-bucket
    std::vector<unsigned long long> h_agg_cursor;
    // outputs (device + pinned host)
    DevBuf o_cell, o_ws, o_cnt, o_sp, o_spn, o_lon, o_lat;
    void *h_cell = nullptr, *h_ws = nullptr, *h_cnt = nullptr, *h_sp = nullptr, *h_spn = nullptr, *h_lon = nullptr,
         *h_lat = nullptr, *h_rows = nullptr;
    size_t h_tiles_cap = 0, h_rows_cap = 0;
    // stats
    DevStats *d_st = nullptr;
    DevStats *h_st = nullptr;
    unsigned long long *d_scratch = nullptr;   // 256 words: partition counts/cursors, totals
    unsigned long long *h_scratch = nullptr;
    // watermark (ms)
    int64_t wm_prev = 0, wm_cur = 0;
    int64_t epoch = -1;
    // tile update statements (hm_encode_tile_updates): the last batch's emitted tiles and their windows
    int64_t last_n_tiles = 0;
    int64_t last_n_latest = -1;   // the last batch's latest rows (ctx->rows) and its input columns (hm_process_batch,
                                  // or hm_stage_finish: the rank's own rows)
    const uint64_t *last_vk = nullptr;
    const int64_t *last_ts = nullptr;
    const double *last_lat = nullptr, *last_lon = nullptr;
    std::vector<int64_t> batch_windows;
    DevBuf td_sizes, td_off, td_btot, td_boff, td_bytes, td_params;
    void *h_td_bytes = nullptr, *h_td_off = nullptr;
    size_t h_td_bytes_cap = 0, h_td_off_cap = 0;
    // stage API state (hm_stage_ingest -> hm_stage_send -> hm_stage_merge -> hm_stage_finish)
    int stage = 0;
    bool staged = false;                               // the last batch ran through the stage API
    int nranks = 1, rank = 0;
    // the shard of a multi-GPU world this context's state is (hm_config.shard_count > 1, or adopted by the first
    // hm_stage_ingest): its tables hold only the region fields it owns (tile_owner_of), in range geometry
    int shard_rank = 0, shard_count = 0;
    int64_t stage_n_in = 0;
    int64_t stage_agg_rows = 0;
    hm_stage_sizes stage_sizes{};
    Inputs stage_I{};                                  // the batch's device columns (the caller's device buffers
                                                       // or the context's copies: valid until the next batch)
    DevStats stage_s1{};                               // this rank's ingest statistics
    bool stage_table = false;                          // the batch's aggregation path (the same on every rank)
    int64_t stage_gmax_ms = INT64_MIN;                 // the batch's max event time over all ranks
    int64_t stage_sent = 0;                            // tile records this rank sent
    // the direct path's records this rank owns itself, kept in its slabs instead of packed into the chunk it
    // addresses to itself (hm_stage_send: binned batch, local window slots = global ones); MOBHEAT_STAGE_SELF=copy
    // packs them like any other destination's (A/B)
    // k_ingest's dense dedup table (k_ingest.h): dense_cap words of this batch (0: none), sized from the last batch's
    // max vkey (vkey_bound; -1: no batch yet); MOBHEAT_DEDUP_DENSE=0 turns it off (the hash table for every vkey)
    DevBuf dense;
    unsigned long long dense_cap = 0;
    int64_t vkey_bound = -1;
    bool dense_ok = true;
    int64_t stage_self_recs = 0;
    bool stage_self_held = false;
    bool self_hold_ok = true;
    std::vector<unsigned> stage_cen;   // a world of one: the census of its self-held records (host -> its own chunk)
    std::vector<unsigned long long> stage_gwreg;       // the batch's global window registry (WREG_SLOTS wenc)
    std::vector<unsigned> stage_gslot;                 // this rank's registry slot -> global slot
    // a pipelined batch (host_pipe.h): its chunks' k_ingest<true> on the main stream, each chunk's merge on merge_stream
    // as soon as the chunk's records are binned; pipe_mode: MOBHEAT_PIPELINE (0 off -- the default: measured slower,
    // host_pipe.h --, K chunks, -1 "auto": PIPE_CHUNKS chunks from PIPE_MIN_ROWS rows)
    static constexpr int PIPE_MAX = 16;
    hipStream_t merge_stream = nullptr;
    hipEvent_t pipe_ev[PIPE_MAX] = {};   // chunk k's records binned (main stream)
    hipEvent_t pipe_rb = nullptr;        // the registry / census / statistics readback of the latest chunk
    hipEvent_t pipe_done = nullptr;      // the last merge (merge stream)
    int pipe_mode = 0;
    int last_pipe_chunks = 0;            // hm_last_counts [10]: chunks of the last batch (0: not pipelined)
    DevBuf pl_cur;                       // per chunk: the bin cursors after it (nbins + 1 words)
    DevBuf pl_slow;                      // per chunk: the exception count after it (K + 1 words, [0] = 0)
    DevBuf pl_O, pl_cnt;                 // the chunks' bins as row segments: offsets (K x RP_BINS + 1), touched keys
    DevBuf pl_T;                         // one chunk's records per bin (k_chunk_segments -> k_seg_scan)
    unsigned test_slab_cap = 0;          // MOBHEAT_TEST_SLAB_CAP: slabs of at most this many records (tests: overflow)
};

static std::string g_create_err;
// rows of one batch (and records of one stage merge): positions are 32-bit, and k_ev_scatter_rec's lanes past a tile
// store to the 64 slack records after the n-th (a bound of 2^32 - 2 let those slack positions wrap)
constexpr int64_t MAX_BATCH_ROWS = (int64_t)UINT32_MAX - 66;
// d_scratch word layout: [0,64) tile partition counts/cursors, [64,128) candidate counts/cursors,
// DUSED_WORD: used-slot count of the persistent dedup table (survives until the table is cleared),
// 255: result count of the last ordered compaction
constexpr int DUSED_WORD = 253;
constexpr int FULL_USED_WORD = 240;   // used-slot count of the full dedup table
constexpr int SLOW_WORD = 252;
constexpr size_t REG_BLOCK_BYTES = 2 * (WREG_SLOTS + 1) * 8 + sizeof(DevStats);   // d_wreg | d_wcount | d_st (hm_create)   // number of k_ingest fast-path exceptions of the current batch
constexpr int REGROW_WORD = 251; // records dumped by k_dump_gen
constexpr int GIVEUP_WORD = 232;
constexpr int GAPS_WORD = 242;   // 242-243: totals of the gap / donor scans
constexpr int POSBAD_WORD = 241; // position statements: rows outside the caller's dictionaries
constexpr int JSON_WORD = 244;   // 244-248: hm_decode_json's malformed / unsupported counts, dictionary overflow /
                                 // collisions; hm_last_latest_buckets' bucket count
// (GIVEUP_WORD: k_ingest's fused dedup gave up, a cache line of its own: words 232-239)

#define HIPCHK(ctx, expr)                                                                             \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) {                                                                       \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                           \
            return HM_E_HIP;                                                                          \
        }                                                                                             \
    } while (0)

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
// hipStreamSynchronize on the context's stream, timed into host_ms (site: the caller's source line)
static hipError_t ctx_sync(hm_ctx *ctx, int site) {
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = hipStreamSynchronize(ctx->stream);
    const double ms = ms_since(t0);
    ctx->host_ms[1] += ms;
    if (ms > ctx->host_ms[3]) { ctx->host_ms[3] = ms; ctx->host_ms[4] = site; }
    return e;
}
static void host_batch_begin(hm_ctx *ctx) { for (double &x : ctx->host_ms) x = 0; }
struct BatchClock {   // the call's wall time into host_ms[0] on every return path
    hm_ctx *ctx;
    std::chrono::steady_clock::time_point t0;
    explicit BatchClock(hm_ctx *c) : ctx(c), t0(std::chrono::steady_clock::now()) {}
    ~BatchClock() { ctx->host_ms[0] = ms_since(t0); }
};
struct AllocTimer {   // times a device/pinned allocation or free into host_ms[2]
    hm_ctx *ctx;
    std::chrono::steady_clock::time_point t0;
    explicit AllocTimer(hm_ctx *c) : ctx(c), t0(std::chrono::steady_clock::now()) {}
    ~AllocTimer() { ctx->host_ms[2] += ms_since(t0); ctx->host_ms[5] += 1; }
};
static int set_err(hm_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    ctx->err = buf;
    return code;
}

// MOBHEAT_TRACE=1: every device allocation of the library (size, host wall time) to stderr
static bool g_trace = getenv("MOBHEAT_TRACE") && getenv("MOBHEAT_TRACE")[0] == '1';
static double wall_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}
static hipError_t dev_malloc(hm_ctx *ctx, void **p, size_t bytes, const char *what) {
    const double t0 = g_trace ? wall_ms() : 0;
    AllocTimer at_(ctx);
    const hipError_t e = hipMalloc(p, bytes);
    ctx->n_allocs++;
    if (g_trace) fprintf(stderr, "[mobheat] hipMalloc %-12s %10.3f GB %8.1f ms\n", what, bytes / 1e9, wall_ms() - t0);
    return e;
}

static int ensure(hm_ctx *ctx, DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return HM_OK;
    size_t want = std::max<size_t>(bytes, 256);
    // a regrowth takes 1.5x headroom: a size that creeps up over a window's life (the census of a growing window,
    // its regrow records) then reallocates O(log) times instead of in every batch that grows it
    if (b.p) want = std::max(want, b.bytes + b.bytes / 2);
    if (b.p) {
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        { AllocTimer at_(ctx); HIPCHK(ctx, hipFree(b.p)); }
        ctx->n_frees++;
        b.p = nullptr;
        b.bytes = 0;
    }
    want = (want + 4095) & ~(size_t)4095;
    if (dev_malloc(ctx, &b.p, want, "buffer") != hipSuccess) {
        (void)hipGetLastError();
        want = (std::max<size_t>(bytes, 256) + 4095) & ~(size_t)4095;   // without the headroom
        if (dev_malloc(ctx, &b.p, want, "buffer") != hipSuccess) {
            (void)hipGetLastError();
            b.p = nullptr;
            return set_err(ctx, HM_E_NOMEM, "hipMalloc(%zu) failed", want);
        }
    }
    b.bytes = want;
    return HM_OK;
}

static int grid_for(int64_t n, int threads, int max_blocks = 256 * 16) {
    int64_t b = (n + threads - 1) / threads;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (int)b;
}

static uint64_t next_pow2(uint64_t v) {
    uint64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

// ---- per-window state tables (kernels.h: GenDesc) ----
static int ilog2(uint64_t v) { return 63 - __builtin_clzll(v); }

// Geometry of a window's table for `keys` keys receiving `parts` partials per batch: load <= 1/2, regions of
// >= 2^REGION_MIN_BITS slots, and enough regions that one merge workgroup gets <= ~16k of the window's partials
// (a hot window with few keys is still merged in parallel).
// H3 cells at a resolution (2 + 120 * 7^res): no window can hold more keys than that
static int64_t h3_cells_at(int res) {
    int64_t c = 120;
    for (int r = 0; r < res; r++) c *= 7;
    return c + 2;
}

// A window table's geometry.  Ordinary: 2^rbits regions of the region field's top rbits (sb = REGION_BITS - rbits),
// as many as keep a merge workgroup's share of the batch's partials <= ~16k.  Range (a shard's tables, and every table
// a batch binned in k_ingest merges into): one region per region field of the context's range [lo, hi) (sb = 0,
// rbase = lo), so that a bin -- a region field -- is one region of every window.
struct Geo { int log2cap; unsigned rbits, sb, rbase; bool range; };
// the region fields a range-mode table holds: the shard's owned range, else all of them
static void range_of(const hm_ctx *ctx, unsigned &lo, unsigned &hi) {
    if (ctx->shard_count > 1) {
        lo = shard_lo(ctx->shard_rank, ctx->shard_count);
        hi = shard_lo(ctx->shard_rank + 1, ctx->shard_count);
    } else {
        lo = 0;
        hi = 1u << REGION_BITS;
    }
}
static bool range_mode(const hm_ctx *ctx, bool binned) { return binned || ctx->shard_count > 1; }
// slots of a table that its keys can use (a range table's regions past the range stay empty)
static int64_t usable_slots(const hm_ctx *ctx, const hm_ctx::Gen &g) {
    if (g.sb != 0 || ctx->shard_count <= 1) return int64_t(1) << g.log2cap;
    unsigned lo, hi;
    range_of(ctx, lo, hi);
    return (int64_t)(hi - lo) << (g.log2cap - (int)g.rbits);
}
// the geometry for `keys` keys receiving `parts` partials, at least 2^min_log2 slots
static Geo gen_geometry(const hm_ctx *ctx, int64_t keys, int64_t parts, bool range, int min_log2 = 0) {
    keys = std::min(keys, h3_cells_at(ctx->cfg.h3_res));   // (the census bounds keys by rows; the grid bounds them too)
    Geo g{};
    g.range = range;
    if (range) {
        unsigned lo, hi;
        range_of(ctx, lo, hi);
        const int64_t nreg = hi - lo;
        g.rbits = (unsigned)ilog2(next_pow2((uint64_t)nreg));
        const int64_t per = (2 * std::max<int64_t>(keys, 1) + nreg - 1) / nreg;   // slots per region at load <= 1/2
        const int rs = std::max(REGION_MIN_BITS, ilog2(next_pow2((uint64_t)per)));
        g.log2cap = std::max((int)g.rbits + rs, min_log2);
        g.sb = 0;
        g.rbase = lo;
        return g;
    }
    int L = ilog2(next_pow2((uint64_t)std::max<int64_t>(2 * keys, 1024)));
    const int want_rb = std::min(RP_BITS, ilog2(next_pow2((uint64_t)std::max<int64_t>((parts + 16383) / 16384, 1))));
    L = std::max({L, want_rb + REGION_MIN_BITS, min_log2});
    g.rbits = (unsigned)std::min(RP_BITS, L - REGION_MIN_BITS);
    g.sb = REGION_BITS - g.rbits;
    g.rbase = 0;
    g.log2cap = L;
    return g;
}
// a table's descriptor (gens_upload, growth, the state dump)
static GenDesc gen_desc(const hm_ctx::Gen &g) {
    GenDesc d{};
    d.wenc = g.wenc;
    d.tab = g.tab;
    d.rbits = (unsigned char)g.rbits;
    d.sb = (unsigned char)g.sb;
    d.rbase = g.rbase;
    d.rshift = (unsigned short)(g.log2cap - (int)g.rbits);
    d.rmask = (UINT64_C(1) << d.rshift) - 1;
    d.count = (unsigned long long)g.keys;
    d.batch_parts = (unsigned long long)g.batch_parts;
    return d;
}
static hm_ctx::Gen gen_of(unsigned long long wenc, TileSlot *t, const Geo &g, int64_t keys, int64_t parts) {
    return hm_ctx::Gen{wenc, t, g.log2cap, g.rbits, g.sb, g.rbase, keys, parts};
}

static bool in_arena(const hm_ctx *ctx, const void *p) {
    return ctx->arena && (const uint8_t *)p >= ctx->arena && (const uint8_t *)p < ctx->arena + ctx->arena_bytes;
}

// A table of >= 2^log2cap slots: the smallest pooled table of 2^log2cap .. 2^(log2cap+2) slots (not cleared: see
// kernels.h; a window whose key count sits near a power of two must not miss the pool and pay a multi-GB hipMalloc
// every batch), else a new one zeroed once.  geo returns the table's actual geometry.
static int table_acquire(hm_ctx *ctx, Geo &geo, TileSlot **out) {
    int &log2cap = geo.log2cap;
    int best = -1;
    for (size_t i = 0; i < ctx->pool.size(); i++) {
        const int l = ctx->pool[i].second;
        if (l >= log2cap && l <= log2cap + 2 && (best < 0 || l < ctx->pool[best].second)) best = (int)i;
    }
    if (best >= 0) {
        *out = ctx->pool[best].first;
        log2cap = ctx->pool[best].second;
        if (!geo.range) {   // (a range table keeps its regions: larger ones)
            geo.rbits = (unsigned)std::min(RP_BITS, log2cap - REGION_MIN_BITS);
            geo.sb = REGION_BITS - geo.rbits;
        }
        ctx->pool.erase(ctx->pool.begin() + best);
        // the slots keep the previous window's keys (never matched: other wenc), the tags were cleared at release
        HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[3], 0));
        return HM_OK;
    }
    const size_t bytes = (size_t(1) << log2cap) * (sizeof(TileSlot) + 1);   // slots, then one tag byte per slot
    TileSlot *t = nullptr;
    if (ctx->arena && ctx->arena_used + bytes <= ctx->arena_bytes) {   // zeroed at create, never handed out before
        *out = (TileSlot *)(ctx->arena + ctx->arena_used);
        ctx->arena_used += (bytes + 255) & ~(size_t)255;
        return HM_OK;
    }
    if (dev_malloc(ctx, (void **)&t, bytes, "state table") != hipSuccess) {
        (void)hipGetLastError();
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        HIPCHK(ctx, hipStreamSynchronize(ctx->side_stream));   // (pooled tags being cleared: table_release)
        std::vector<std::pair<TileSlot *, int>> keep;
        for (auto &pt : ctx->pool)
            if (in_arena(ctx, pt.first)) keep.push_back(pt); else { AllocTimer at_(ctx); (void)hipFree(pt.first); ctx->n_frees++; }
        ctx->pool.swap(keep);
        ctx->n_allocs++;
        if (hipMalloc(&t, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return set_err(ctx, HM_E_NOMEM, "state table of 2^%d slots: out of device memory", log2cap);
        }
    }
    HIPCHK(ctx, hipMemsetAsync(t, 0, bytes, ctx->stream));
    *out = t;
    return HM_OK;
}
// (the stream must have drained every kernel that reads the table).  The table's tags are cleared at once on the
// side stream -- behind the main stream's work so far, concurrent with the next batch's first kernels (k_ingest does
// not use the HBM bandwidth) -- and table_acquire waits for that (side_ev[3]).
// Several tables at once (a batch's evicted windows): one event pair and one launch per ZR_MAX tables (one
// release at a time cost ~30 us of host API calls each between batches, profiles/r5/r5tl/).
static int table_release_all(hm_ctx *ctx, const std::vector<std::pair<TileSlot *, int>> &ts) {
    if (ts.empty()) return HM_OK;
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[0], ctx->stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->side_ev[0], 0));
    for (size_t a = 0; a < ts.size(); a += ZR_MAX) {
        ZeroRanges r = {};
        const int k = (int)std::min<size_t>(ZR_MAX, ts.size() - a);
        int64_t mx = 0;
        for (int j = 0; j < k; j++) {   // (2^log2cap >= 1024 tag bytes, 64-B aligned)
            r.p[j] = (uint4 *)(ts[a + j].first + (size_t(1) << ts[a + j].second));
            r.n16[j] = (int64_t(1) << ts[a + j].second) / 16;
            mx = std::max(mx, r.n16[j]);
        }
        hipLaunchKernelGGL(k_zero16_ranges, dim3(grid_for(mx, 256, 256 * 32), k), dim3(256), 0, ctx->side_stream, r);
        HIPCHK(ctx, hipGetLastError());
    }
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[3], ctx->side_stream));
    for (const auto &t : ts) ctx->pool.push_back(t);
    size_t own = 0;   // pooled tables of our own allocations (arena tables stay pooled)
    for (auto &pt : ctx->pool) own += !in_arena(ctx, pt.first);
    for (size_t i = 0; own > 8 && i < ctx->pool.size();) {
        if (in_arena(ctx, ctx->pool[i].first)) { i++; continue; }
        HIPCHK(ctx, hipStreamSynchronize(ctx->side_stream));   // (its tags may still be being cleared)
        { AllocTimer at_(ctx); (void)hipFree(ctx->pool[i].first); }
        ctx->n_frees++;
        ctx->pool.erase(ctx->pool.begin() + i);
        own--;
    }
    return HM_OK;
}
static int table_release(hm_ctx *ctx, TileSlot *t, int log2cap) { return table_release_all(ctx, {{t, log2cap}}); }

static int gens_upload(hm_ctx *ctx) {
    memset(ctx->h_gmap, 0, GMAP_SLOTS * sizeof(GenDesc));
    ctx->gmap_ready = false;   // (h_gmap is the upload's staging now)
    for (const auto &g : ctx->gens) {
        unsigned h = (unsigned)(mix64(g.wenc) & (GMAP_SLOTS - 1));
        while (ctx->h_gmap[h].wenc) h = (h + 1) & (GMAP_SLOTS - 1);
        ctx->h_gmap[h] = gen_desc(g);
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_gmap, ctx->h_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyHostToDevice, ctx->stream));
    ctx->n_glist = 0;
    for (int q = 0; q < GMAP_SLOTS; q++)
        if (ctx->h_gmap[q].wenc) ctx->h_glist[ctx->n_glist++] = ctx->h_gmap[q];
    if (ctx->n_glist)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_glist, ctx->h_glist, ctx->n_glist * sizeof(GenDesc), hipMemcpyHostToDevice, ctx->stream));
    return HM_OK;
}

// exclusive scan of the m = (nbins + 1) x ntiles tile histogram rp_H into rp_O (digit-major)
// exclusive scan of m u32 counts `in` into u64 offsets `out`
static int scan_counts(hm_ctx *ctx, const unsigned *in, int64_t m, unsigned long long *out) {
    const int64_t nb = (m + SC_PER - 1) / SC_PER;
    int rc;
    if ((rc = ensure(ctx, ctx->rp_btot, nb * 4)) || (rc = ensure(ctx, ctx->rp_boff, nb * 8))) return rc;
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, ctx->stream, in, m, out, (unsigned *)ctx->rp_btot.p);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, ctx->stream, (const unsigned *)ctx->rp_btot.p, nb,
                       (unsigned long long *)ctx->rp_boff.p, ctx->d_scratch + 254);
    hipLaunchKernelGGL(k_scan_add, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream, out, m,
                       (const unsigned long long *)ctx->rp_boff.p);
    return HM_OK;
}
static int rp_scan(hm_ctx *ctx, int64_t m) {
    return scan_counts(ctx, (const unsigned *)ctx->rp_H.p, m, (unsigned long long *)ctx->rp_O.p);
}

// radix partition of n partial records into RP_BINS bins (one per (window, region)); the sorted copy goes to
// ctx->parts_sorted, bin b starts at rp_O[b * ntiles]
// In -> Out: TilePartial -> SortedRec (table mode / stage merge, into parts_sorted), GrowRec -> GrowRec (growth, into
// parts_regrow_sorted), TilePartial -> TilePartial (the owner partition, into the caller's send buffer)
template <typename In, typename Out>
static int partition(hm_ctx *ctx, const In *parts, int64_t n, int64_t &ntiles, int nranks = 0, Out *dst = nullptr) {
    const int nbins = nranks > 0 ? nranks : RP_BINS;
    if (n >= (int64_t)UINT32_MAX) return set_err(ctx, HM_E_INVALID, "%lld partial records in one merge exceed 2^32-2", (long long)n);
    const int64_t tile = rp_tile_for(n);
    ntiles = std::max<int64_t>((n + tile - 1) / tile, 1);
    const int64_t m = (int64_t)(nbins + 1) * ntiles;   // digit nbins: gaps (cell 0), which the scatter drops
    int rc;
    if (!dst && (rc = ensure(ctx, ctx->parts_sorted, std::max<int64_t>(n, 1) * sizeof(Out)))) return rc;
    if ((rc = ensure(ctx, ctx->rp_H, m * 4)) || (rc = ensure(ctx, ctx->rp_O, m * 8))) return rc;
    hipLaunchKernelGGL(k_rp_hist<In>, dim3(ntiles), dim3(RP_THREADS), 0, ctx->stream, parts, n, tile, (const GenDesc *)ctx->d_gmap,
                       (const GenDesc *)ctx->d_glist, ctx->n_glist, nranks, nbins, (unsigned *)ctx->rp_H.p, ntiles, ctx->d_st);
    if ((rc = rp_scan(ctx, m))) return rc;
    hipLaunchKernelGGL((k_rp_scatter<In, Out>), dim3(ntiles), dim3(RP_THREADS), 0, ctx->stream, parts, n, tile,
                       (const GenDesc *)ctx->d_gmap, (const GenDesc *)ctx->d_glist, ctx->n_glist, nranks, nbins,
                       (const unsigned long long *)ctx->rp_O.p, ntiles, dst ? dst : (Out *)ctx->parts_sorted.p);
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

static int phase_dedup(hm_ctx *ctx, const Inputs *I, const Cand *cands, int64_t n, bool rerun_max, hipStream_t st);
// the batch's dedup on the side stream (hm_process_batch): side_ev[1] / [2] bracket it
static int launch_side_dedup(hm_ctx *ctx, const Inputs *I) {
    int rc;
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[1], ctx->side_stream));
    if ((rc = phase_dedup(ctx, I, nullptr, I->n, false, ctx->side_stream))) return rc;
    HIPCHK(ctx, hipEventRecord(ctx->side_ev[2], ctx->side_stream));
    return HM_OK;
}

// the direct path's partition: n event keys with the batch's columns (I) -> EventRecs in (window, region) bins
// (parts_sorted; the bins from the windows' WInfo.binp: with binp 0, one bin per region field -- the multi-GPU
// sender's grouping); rows without a key fall into digit RP_BINS (dropped)
static int ev_partition(hm_ctx *ctx, const uint64_t *keys, int64_t n, const Inputs *I, int64_t &ntiles) {
    const int nbins = RP_BINS;
    const int64_t tile = rp_tile_for(n);
    ntiles = std::max<int64_t>((n + tile - 1) / tile, 1);
    const int64_t m = (int64_t)(nbins + 1) * ntiles;
    int rc;
    // (+ 64 slack records: k_ev_scatter_rec's lanes past a tile store there)
    if ((rc = ensure(ctx, ctx->parts_sorted, (std::max<int64_t>(n, 1) + 64) * sizeof(EventRec)))) return rc;
    if ((rc = ensure(ctx, ctx->rp_H, m * 4)) || (rc = ensure(ctx, ctx->rp_O, m * 8))) return rc;
    const uint64_t ch = cell_hi_of(ctx->cfg.h3_res);
    hipLaunchKernelGGL(k_ev_hist, dim3(ntiles), dim3(EV_THREADS), 0, ctx->stream, keys, n, tile, (const WInfo *)ctx->d_winfo, ch,
                       0, nbins, (unsigned *)ctx->rp_H.p, ntiles);
    if ((rc = rp_scan(ctx, m))) return rc;
    hipLaunchKernelGGL(k_ev_scatter_rec, dim3(ntiles), dim3(SR_THREADS), 0, ctx->stream, keys, n, tile, I->sp, I->sv, I->lat, I->lon,
                       (const WInfo *)ctx->d_winfo, ch, nbins, (const unsigned long long *)ctx->rp_O.p, ntiles,
                       (EventRec *)ctx->parts_sorted.p);
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

static RowsOut rows_of(DevBuf &cell, DevBuf &ws, DevBuf &cnt, DevBuf &sp, DevBuf &spn, DevBuf &lon, DevBuf &lat) {
    return RowsOut{(uint64_t *)cell.p, (int64_t *)ws.p, (int64_t *)cnt.p, (double *)sp.p, (uint8_t *)spn.p,
                   (double *)lon.p, (double *)lat.p};
}
static RowsOut staged_rows(hm_ctx *ctx) {
    return rows_of(ctx->s_cell, ctx->s_ws, ctx->s_cnt, ctx->s_sp, ctx->s_spn, ctx->s_lon, ctx->s_lat);
}

// the batch sequence number kept in the slots' touched words (32 bits, never 0: fresh slots hold 0)
static unsigned seq32(const hm_ctx *ctx) { return (unsigned)(ctx->seq % 0xffffffffull) + 1u; }

// the segments of a multi-GPU owner's bins (k_stage_segments; merge_sorted's kSeg variant)
struct Segs {
    const unsigned long long *SO = nullptr;
    const unsigned *SP = nullptr;
    int nseg = 0;
    SegBounds bounds{};   // where the segments may lie (checked by the MOBHEAT_BOUNDS_CHECK build only)
};
// merge the partitioned records (ctx->parts_sorted, or src) of n_rows staging rows
// (O / cnt: the bins' row offsets and their touched-key counts; default rp_O and bin_cnt -- a pipelined batch's chunk k
// passes its own slices of pl_O / pl_cnt)
template <typename Rec>
static int merge_sorted(hm_ctx *ctx, int64_t n_rows, int64_t ntiles, int64_t slab = 0, const Rec *src = nullptr,
                        const Segs &seg = Segs(), const unsigned long long *O = nullptr, unsigned *cnt = nullptr) {
    constexpr bool rehash = std::is_same<Rec, GrowRec>::value;
    int rc;
    if ((rc = ensure(ctx, ctx->bin_cnt, RP_BINS * 4)) || (rc = ensure(ctx, ctx->bin_off, RP_BINS * 8)))
        return rc;
    if (!rehash) {
        const int64_t m = std::max<int64_t>(n_rows, 1);
        if ((rc = ensure(ctx, ctx->s_cell, m * 8)) || (rc = ensure(ctx, ctx->s_ws, m * 8)) || (rc = ensure(ctx, ctx->s_cnt, m * 8)) ||
            (rc = ensure(ctx, ctx->s_sp, m * 8)) || (rc = ensure(ctx, ctx->s_spn, m)) || (rc = ensure(ctx, ctx->s_lon, m * 8)) ||
            (rc = ensure(ctx, ctx->s_lat, m * 8)))
            return rc;
    }
    // resident tags: every window merged into this batch may have a region in a bin
    unsigned tag_bytes = 0;
    if (!rehash) {
        size_t need = 0;
        for (const auto &g : ctx->gens)
            if (g.batch_parts) need += size_t(1) << (g.log2cap - (int)g.rbits);
        tag_bytes = (unsigned)std::min<size_t>((need + 4095) & ~size_t(4095), MO_TAG_MAX);   // (attribute: hm_create)
    }
    const int grid = ctx->merge_grid > 0 ? std::min(ctx->merge_grid, RP_BINS) : RP_BINS;
    // every window of the batch resident in every bin (their regions' tags fit together): the variant without the
    // HBM-probing fallback
    bool resident = false;
    if (!rehash) {
        size_t need = 0;
        int nwin = 0;
        for (const auto &g : ctx->gens)
            if (g.batch_parts) { need += size_t(1) << (g.log2cap - (int)g.rbits); nwin++; }
        resident = need <= tag_bytes && nwin <= MO_RES_MAX && ctx->n_glist <= GC_MAX;
    }
    if (seg.nseg > MO_SEG_MAX) return set_err(ctx, HM_E_INVALID, "%d senders exceed %d", seg.nseg, MO_SEG_MAX);
#if MOBHEAT_BOUNDS_CHECK
    if (seg.nseg > 0) HIPCHK(ctx, hipMemcpyToSymbolAsync(HIP_SYMBOL(g_seg_bounds), &seg.bounds, sizeof(SegBounds), 0,
                                                         hipMemcpyHostToDevice, ctx->stream));
#endif
    // the cooperative probe (re-touched keys: old lines read) when this batch's windows already hold keys for most of
    // its records -- known here from the census and the tables, where the last batch's ratio (merge_coop) mispredicts
    // the batch after a window opened (all new keys, then all re-touched: 6.8-ms merges, profiles/r5/r5headprof)
    bool coop = ctx->merge_coop;
    if (!rehash && ctx->coop_predict) {
        int64_t old = 0, parts = 0;
        for (const auto &g : ctx->gens)
            if (g.batch_parts) { parts += g.batch_parts; old += std::min(g.keys, g.batch_parts); }
        coop = parts > 0 && 2 * old > parts;
    }
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(MO_THREADS), tag_bytes, ctx->stream, src ? src : (const Rec *)ctx->parts_sorted.p, slab,
                           seg.SO, seg.SP, seg.nseg,
                           O ? O : (const unsigned long long *)ctx->rp_O.p, ntiles, RP_BINS, ctx->d_gmap, (const GenDesc *)ctx->d_glist,
                           ctx->n_glist, (const WInfo *)ctx->d_winfo, cell_hi_of(ctx->cfg.h3_res), seq32(ctx), staged_rows(ctx),
                           cnt ? cnt : (unsigned *)ctx->bin_cnt.p, ctx->d_st, tag_bytes);
    };
    if constexpr (std::is_same<Rec, EventRec>::value) {
        if (seg.nseg > 0) {   // (the multi-GPU owner)
            if (resident && coop) launch(k_merge_owned<Rec, true, true, true>);
            else if (resident) launch(k_merge_owned<Rec, true, false, true>);
            else launch(k_merge_owned<Rec, false, false, true>);
            HIPCHK(ctx, hipGetLastError());
            return HM_OK;
        }
    }
    if constexpr (!rehash) {
        if (resident && coop) launch(k_merge_owned<Rec, true, true>);
        else if (resident) launch(k_merge_owned<Rec, true>);
        else launch(k_merge_owned<Rec, false>);
    } else {
        launch(k_merge_owned<Rec, false>);
    }
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

// census of partial records per window (the stage merge's received partials; table mode counts its own)
static int census_of_partials(hm_ctx *ctx, const TilePartial *parts, int64_t n, std::vector<WinCount> &census) {
    if (!ctx->census_ready) {
        HIPCHK(ctx, hipMemsetAsync(ctx->d_cmap, 0, GMAP_SLOTS * sizeof(WinCount), ctx->stream));
        hipLaunchKernelGGL(k_census, dim3(grid_for(n, 256, 256 * 8)), dim3(256), 0, ctx->stream, parts, n, ctx->d_cmap, ctx->d_st);
        HIPCHK(ctx, hipGetLastError());
    }
    ctx->census_ready = false;
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_cmap, ctx->d_cmap, GMAP_SLOTS * sizeof(WinCount), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_st, ctx->d_st, sizeof(DevStats), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    if (ctx->h_st->overflow) return set_err(ctx, HM_E_OVERFLOW, "more than %d windows in one batch", GMAP_SLOTS);
    census.clear();
    for (int q = 0; q < GMAP_SLOTS; q++)
        if (ctx->h_cmap[q].wenc) census.push_back(ctx->h_cmap[q]);
    return HM_OK;
}
// census of the direct path: the registry's windows and their aggregated rows (h_wreg / h_wcount, read back after
// k_ingest)
static void census_of_registry(const hm_ctx *ctx, std::vector<WinCount> &census) {
    census.clear();
    for (int w = 0; w < WREG_SLOTS; w++)
        if (ctx->h_wreg[w] && ctx->h_wcount[w]) census.push_back(WinCount{ctx->h_wreg[w], ctx->h_wcount[w]});
}

// WInfo of every registry slot in use (after gens_prepare when with_bins: the radix bin parameters need the
// window's table geometry)
static int winfo_upload(hm_ctx *ctx, bool with_bins) {
    HIPCHK(ctx, hipEventSynchronize(ctx->winfo_ev));   // (h_winfo is reused: the previous upload must be done)
    WInfo *h = ctx->h_winfo;
    int lo = WREG_SLOTS, hi = -1;
    for (int w = 0; w < WREG_SLOTS; w++) {
        const unsigned long long we = ctx->h_wreg[w];
        if (!we) continue;
        WInfo &x = h[w];
        memset(&x, 0, sizeof x);
        x.wenc = we;
        x.inner = window_inner(wdec(we));
        x.gslot = ctx->stage_gslot.empty() ? (unsigned)w : ctx->stage_gslot[w];
        if (with_bins) {
            unsigned sb = 0;
            bool found = false;
            for (const auto &g : ctx->gens)
                if (g.wenc == we) { sb = g.sb; found = true; break; }
            if (!found) return set_err(ctx, HM_E_STATE, "window without a state table");
            x.binp = (sb << 24) | (window_salt(we) & ((1u << sb) - 1));
        }
        lo = std::min(lo, w);
        hi = std::max(hi, w);
    }
    if (hi >= lo)
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_winfo + lo, h + lo, (size_t)(hi - lo + 1) * sizeof(WInfo), hipMemcpyHostToDevice,
                                   ctx->stream));
    // the direct-mapped image the kernels keep in LDS (kernels.h WiCacheImg)
    WiCacheImg *img = (WiCacheImg *)(h + WREG_SLOTS + 1);
    for (int e = 0; e < WI_CACHE; e++) img->tag[e] = WI_NONE;
    for (int w = lo; w <= hi; w++) {
        if (!ctx->h_wreg[w]) continue;
        const int e = w & (WI_CACHE - 1);
        if (img->tag[e] == WI_NONE) {
            img->tag[e] = (unsigned)w;
            img->e[e] = h[w];
        } else {
            img->tag[e] = WI_CONFLICT;   // (both slots keep the global lookup)
        }
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_winfo + WREG_SLOTS + 1, img, sizeof(WiCacheImg), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipEventRecord(ctx->winfo_ev, ctx->stream));
    return HM_OK;
}

// Give every window of the census a table large enough for its keys after this batch (new windows: a new table;
// windows that would pass load 1/2: a larger table, filled by dumping the old one and merging the dump in rehash
// mode); upload the window map.
// range: every window's table in range geometry (a shard's context, or a batch binned in k_ingest: a row's bin, chosen
// before the census, is then its region in every window)
static int gens_prepare(hm_ctx *ctx, const std::vector<WinCount> &census, bool range = false) {
    std::vector<hm_ctx::Gen> old;   // tables being replaced by larger ones
    int rc;
    range = range_mode(ctx, range);
    unsigned lo = 0, hi = 0;
    range_of(ctx, lo, hi);
    for (auto &g : ctx->gens) g.batch_parts = 0;
    for (const WinCount &w : census) {
        ctx->batch_windows.push_back(wdec(w.wenc));
        const int64_t c = (int64_t)w.count;
        auto it = std::find_if(ctx->gens.begin(), ctx->gens.end(), [&](const hm_ctx::Gen &g) { return g.wenc == w.wenc; });
        if (it == ctx->gens.end()) {
            Geo geo = gen_geometry(ctx, c, c, range);
            TileSlot *t = nullptr;
            if ((rc = table_acquire(ctx, geo, &t))) return rc;
            ctx->gens.push_back(gen_of(w.wenc, t, geo, 0, c));   // (keys: the merge counts the ones it creates)
            continue;
        }
        const bool full = std::min(it->keys + c, h3_cells_at(ctx->cfg.h3_res)) * 2 > usable_slots(ctx, *it);
        const bool misfit = range && (it->sb != 0 || it->rbase != lo || (int64_t(1) << it->rbits) < (int64_t)(hi - lo));
        if (full || misfit) {
            Geo geo = gen_geometry(ctx, it->keys + c, c, range, full ? it->log2cap + 1 : 0);
            TileSlot *t = nullptr;
            if ((rc = table_acquire(ctx, geo, &t))) return rc;
            old.push_back(*it);
            // keys unchanged: the rehash merge moves them without counting
            *it = gen_of(it->wenc, t, geo, it->keys, 0);
        }
        it->batch_parts = c;
    }
    if ((int)ctx->gens.size() > GMAP_SLOTS / 2)
        return set_err(ctx, HM_E_OVERFLOW, "%zu live windows exceed the window map (%d)", ctx->gens.size(), GMAP_SLOTS / 2);
    if ((rc = gens_upload(ctx))) return rc;
    if (!old.empty()) {
        int64_t moved = 0;
        for (const auto &g : old) moved += g.keys;
        ctx->touched_dump_seq = -1;
        ctx->bin_offsets_ready = false;   // (the regrow's partition below writes rp_O)
        if ((rc = ensure(ctx, ctx->parts_regrow, std::max<int64_t>(moved, 1) * sizeof(GrowRec)))) return rc;
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + REGROW_WORD, 0, 8, ctx->stream));
        ctx->touched_dump_seq = ctx->export_dump_n = -1;   // (parts_regrow is overwritten)
        for (const auto &g : old) {
            const GenDesc d = gen_desc(g);
            hipLaunchKernelGGL(k_dump_gen, dim3(grid_for(int64_t(1) << g.log2cap, 256 * DUMP_PER)), dim3(256), 0, ctx->stream, d,
                               (GrowRec *)ctx->parts_regrow.p, ctx->d_scratch + REGROW_WORD);
        }
        HIPCHK(ctx, hipGetLastError());
        int64_t ntiles;
        if ((rc = ensure(ctx, ctx->parts_regrow_sorted, std::max<int64_t>(moved, 1) * sizeof(GrowRec))) ||
            (rc = partition<GrowRec, GrowRec>(ctx, (const GrowRec *)ctx->parts_regrow.p, moved, ntiles, 0,
                                              (GrowRec *)ctx->parts_regrow_sorted.p)) ||
            (rc = merge_sorted<GrowRec>(ctx, moved, ntiles, 0, (const GrowRec *)ctx->parts_regrow_sorted.p)))
            return rc;
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        std::vector<std::pair<TileSlot *, int>> rel;
        for (const auto &g : old) rel.emplace_back(g.tab, g.log2cap);
        if ((rc = table_release_all(ctx, rel))) return rc;
    }
    return HM_OK;
}

// After a batch: every window's key count from the device; windows whose end <= the eviction watermark are
// released whole (their rows are late from now on); n_state = keys of the live windows.
static int state_account(hm_ctx *ctx, int64_t evict_wm_ms) {
    if (!ctx->gmap_ready) {
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_gmap, ctx->d_gmap, GMAP_SLOTS * sizeof(GenDesc), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
    }
    ctx->gmap_ready = false;
    const int64_t dead_end_us = evict_wm_ms * 1000;
    int64_t live = 0;
    std::vector<hm_ctx::Gen> keep;
    std::vector<std::pair<TileSlot *, int>> dead;
    for (auto &g : ctx->gens) {
        unsigned h = (unsigned)(mix64(g.wenc) & (GMAP_SLOTS - 1));
        for (int p = 0; p < GMAP_SLOTS && ctx->h_gmap[h].wenc; p++, h = (h + 1) & (GMAP_SLOTS - 1))
            if (ctx->h_gmap[h].wenc == g.wenc) { g.keys = (int64_t)ctx->h_gmap[h].count; break; }
        if (wdec(g.wenc) + ctx->cfg.tile_us <= dead_end_us) {
            dead.emplace_back(g.tab, g.log2cap);
        } else {
            live += g.keys;
            keep.push_back(g);
        }
    }
    if (int rc = table_release_all(ctx, dead)) return rc;
    ctx->gens.swap(keep);
    ctx->state_size = live;
    return HM_OK;
}

// Clear a dedup table through its used list and make sure it holds `n_keys` keys at <= 1/2 load; shrink: the
// table is also reallocated when it is more than twice the size needed (the fused table: cache residency).
static int dedup_prepare(hm_ctx *ctx, hm_ctx::DedupTable &d, int64_t n_keys, bool shrink) {
    if (d.dirty) {
        hipLaunchKernelGGL(k_clear_dedup, dim3(grid_for(d.cap, 256)), dim3(256), 0, ctx->stream, d.tab,
                           (const unsigned int *)d.used.p, ctx->d_scratch + d.used_word);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemsetAsync(ctx->d_scratch + d.used_word, 0, 8, ctx->stream));
        d.dirty = false;
    }
    unsigned long long want = next_pow2((unsigned long long)std::max<int64_t>(2 * n_keys, 1024));
    // (a 2 MB fused table stays in every XCD's L2, an 8 MB one does not: k_ingest 6.9 -> 28 ms on the bench)
    if (d.tab && d.cap >= want && (!shrink || d.cap <= 2 * want)) return HM_OK;
    if (d.tab) {
        HIPCHK(ctx, ctx_sync(ctx, __LINE__));
        { AllocTimer at_(ctx); HIPCHK(ctx, hipFree(d.tab)); }
        ctx->n_frees++;
        d.tab = nullptr;
    }
    if (dev_malloc(ctx, (void **)&d.tab, want * sizeof(DedupSlot), "dedup table") != hipSuccess) {
        (void)hipGetLastError();
        return set_err(ctx, HM_E_NOMEM, "dedup table alloc failed");
    }
    d.cap = want;
    hipLaunchKernelGGL(k_init_dedup, dim3(grid_for(want, 256)), dim3(256), 0, ctx->stream, d.tab, want);
    HIPCHK(ctx, hipGetLastError());
    return ensure(ctx, d.used, want * sizeof(unsigned int));
}
// k_ingest's table: sized from the last batch's distinct vkeys (small and cache-resident), not from n; a batch
// with many more keys makes the fused probes give up and phase_dedup reruns the max pass on a full-size table.
static int64_t dedup_fused_keys(const hm_ctx *ctx, int64_t n) {
    const int64_t guess = ctx->dedup_seen > 0 ? ctx->dedup_seen + ctx->dedup_seen / 4 : int64_t(1) << 18;   // first batch
    return std::min<int64_t>(n, std::max<int64_t>(int64_t(1) << 15, guess));
}

// ordered compaction of byte flags -> int64 indices into ctx->rows; count into d_scratch[255]
static int compact_flags(hm_ctx *ctx, const uint8_t *f, int64_t n, int64_t *out, hipStream_t st) {
    int64_t nb = (n + CP_TILE - 1) / CP_TILE;
    if (nb < 1) nb = 1;
    int rc;
    if ((rc = ensure(ctx, ctx->block_counts, nb * sizeof(unsigned)))) return rc;
    if ((rc = ensure(ctx, ctx->block_offs, nb * sizeof(unsigned long long)))) return rc;
    hipLaunchKernelGGL(k_cp_count, dim3(nb), dim3(CP_THREADS), 0, st, f, n, (unsigned *)ctx->block_counts.p);
    hipLaunchKernelGGL(k_cp_scan, dim3(1), dim3(1024), 0, st, (const unsigned *)ctx->block_counts.p, nb,
                       (unsigned long long *)ctx->block_offs.p, ctx->d_scratch + 255);
    hipLaunchKernelGGL(k_cp_write, dim3(nb), dim3(CP_THREADS), 0, st, f, n,
                       (const unsigned long long *)ctx->block_offs.p, out);
    HIPCHK(ctx, hipGetLastError());
    return HM_OK;
}

static int stage_inputs(hm_ctx *ctx, const hm_batch_in *in, const double **lat, const double **lon, const int64_t **ts,
                        const double **sp, const uint8_t **sv, const uint64_t **vk, const uint8_t **rv) {
    int64_t n = in->n;
    if (in->memory == HM_MEM_DEVICE || n == 0) {
        *lat = in->lat; *lon = in->lon; *ts = in->ts_us; *sp = in->speed; *sv = in->speed_valid; *vk = in->vkey;
        *rv = in->row_valid;
        return HM_OK;
    }
    struct { DevBuf *b; const void *src; size_t el; const void **dst; } items[] = {
        {&ctx->in_lat, in->lat, 8, (const void **)lat},     {&ctx->in_lon, in->lon, 8, (const void **)lon},
        {&ctx->in_ts, in->ts_us, 8, (const void **)ts},     {&ctx->in_speed, in->speed, 8, (const void **)sp},
        {&ctx->in_sv, in->speed_valid, 1, (const void **)sv}, {&ctx->in_vkey, in->vkey, 8, (const void **)vk},
        {&ctx->in_rv, in->row_valid, 1, (const void **)rv},
    };
    ctx->n_h2d = 0;
    for (auto &it : items) {
        if (!it.src) { *it.dst = nullptr; continue; }
        int rc = ensure(ctx, *it.b, n * it.el);
        if (rc) return rc;
        ctx->h2d[ctx->n_h2d++] = hm_ctx::H2D{it.src, it.b->p, it.el};   // copied by phase_local, chunk by chunk
        *it.dst = it.b->p;
    }
    return HM_OK;
}

// pinned host capacity for `need` elements, grown with 1.5x headroom (output row counts creep up as windows fill)
static size_t host_cap_for(size_t cap, size_t need) { return std::max<size_t>({need, cap + cap / 2, 1024}); }

static int ensure_host(hm_ctx *ctx, void **p, size_t &cap_el, size_t want_el, size_t el) {
    (void)cap_el;
    AllocTimer at_(ctx);
    if (*p) { HIPCHK(ctx, hipHostFree(*p)); ctx->n_frees++; }
    *p = nullptr;
    ctx->n_allocs++;
    HIPCHK(ctx, hipHostMalloc(p, std::max<size_t>(want_el, 1) * el, hipHostMallocDefault));
    return HM_OK;
}
