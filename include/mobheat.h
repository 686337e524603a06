/*
 * mobheat -- MI355X-native drop-in for the per-micro-batch hot path of
 * panosporf99/real-time-mobility-heatmap (reference heatmap_stream.py).
 *
 * C ABI only: plain pointers and sizes, no C++ or torch types. Every function returns 0 on success or a
 * negative HM_E_* code; hm_last_error() returns the message. The ctypes host binding raises RuntimeError
 * on a negative code, which keeps the reference's "exception fails the micro-batch" behaviour
 * (reference heatmap_stream.py:192,196,231,235 have no try/except; the query dies in awaitTermination, :249).
 *
 * What each entry point replaces (reference file:line):
 *   hm_create / hm_destroy       -- the Spark session + stateful query plan (heatmap_stream.py:41-47,241-249):
 *                                   config H3_RES (:26), TILE_MINUTES (:29), withWatermark 10 min (:107).
 *   hm_process_batch             -- everything between from_json (:88-93) and the Mongo writes for one
 *                                   micro-batch: the sanity filter (:96-104), the to_h3 UDF (:65-75,105-106),
 *                                   the watermark (:107), window(eventTs, TILE) x cellId count/avg aggregation
 *                                   in update mode (:111-133,243), and the in-batch latest-position dedup
 *                                   groupBy(provider,vehicleId).max(eventTs) + join back (:198-207).
 *   hm_latlng_to_cell            -- the per-row UDF alone: h3.latlng_to_cell(lat, lon, H3_RES) (:73).
 *   hm_stage_* (multi-GPU)       -- the same batch split into local pre-aggregation, an owner-partitioned
 *                                   exchange (the caller moves the records with RCCL all-to-all), and the
 *                                   owner-side merge; replaces Spark's shuffle (spark.sql.shuffle.partitions, :44).
 *   hm_state_export / _import    -- the state store behind .option("checkpointLocation", CHECKPOINT_DIR)
 *                                   (:37,244): the tile state + watermark after a committed epoch, and its
 *                                   restore into a fresh context after a restart (the epoch is then replayed).
 *   hm_encode_tile_updates       -- the tiles half of the batch writer (:164-196): one MongoDB `update`
 *                                   statement {q, u: {$set: doc}, multi, upsert} per emitted tile, BSON-encoded
 *                                   on the GPU exactly as pymongo encodes the reference's UpdateOne.
 *   hm_encode_position_updates   -- the positions half (:198-235): one positions_latest statement per latest row.
 */
#ifndef MOBHEAT_H
#define MOBHEAT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HM_ABI_VERSION 11

/* error codes */
#define HM_OK 0
#define HM_E_INVALID (-1)   /* bad argument */
#define HM_E_HIP (-2)       /* HIP runtime error */
#define HM_E_NOMEM (-3)     /* device or host allocation failed */
#define HM_E_OVERFLOW (-4)  /* a device hash table overflowed its probe bound */
#define HM_E_STATE (-5)     /* call out of order (stage API) */
#define HM_E_UNSUPPORTED (-6) /* input outside what the device decoder handles (hm_decode_json) */

/* memory kinds for batch pointers */
#define HM_MEM_HOST 0
#define HM_MEM_DEVICE 1
#define HM_MEM_HOST_STREAM 2   /* hm_encode_* outputs only: pinned host memory; the offsets have landed when the call
                                  returns, the bytes land in pieces after it (hm_statements_wait) */

typedef struct hm_config {
    int32_t abi_version;            /* must be HM_ABI_VERSION */
    int32_t h3_res;                 /* H3_RES, 0..15 (reference default 8, heatmap_stream.py:26) */
    int32_t device;                 /* HIP device ordinal */
    int32_t late_uses_prev_watermark; /* 1 = Spark 3.5 default: late rows filtered by the previous batch's
                                         watermark, state evicted by the current one; 0 = both current */
    int64_t tile_us;                /* window length in microseconds: TILE_MINUTES*60e6 (default 5 min) */
    int64_t watermark_delay_ms;     /* withWatermark delay (reference: 10 minutes = 600000) */
    int64_t state_capacity_hint;    /* expected keys of the largest window: its table is reserved at create
                                       (0 = allocate on demand) */
    int64_t batch_capacity_hint;    /* expected max events per batch (0 = grow on demand) */
    int64_t state_arena_bytes;      /* device memory reserved (and zeroed) at create for the window tables; tables
                                       are carved from it before any allocation in a batch (0 = none) */
    int32_t shard_rank;             /* multi-GPU: this context is rank shard_rank of shard_count (the stage API); its
                                       state holds only the keys that rank owns.  shard_count 0 = not fixed at create
                                       (the first hm_stage_ingest fixes it), 1 = a single GPU */
    int32_t shard_count;
} hm_config;

/* One micro-batch of raw events, structure of arrays. All arrays have n entries.
 * row_valid: 1 iff provider, vehicleId and eventTs are all non-null (NULL pointer = all 1).
 * lat/lon: degrees; a null lat/lon is passed as NaN (it then fails the range filter, like Spark's between).
 * ts_us: eventTs as Spark TimestampType, microseconds since the epoch, UTC.
 * speed/speed_valid: speedKmh and its non-null flag (speed_valid NULL = all non-null; speed NULL = all null).
 * vkey: identity of (provider, vehicleId); equal pairs must give equal keys, distinct pairs distinct keys.
 *       UINT64_MAX is reserved. */
typedef struct hm_batch_in {
    int64_t n;
    int32_t memory;        /* HM_MEM_HOST or HM_MEM_DEVICE */
    int32_t reserved;
    const double *lat;
    const double *lon;
    const int64_t *ts_us;
    const double *speed;
    const uint8_t *speed_valid;
    const uint64_t *vkey;
    const uint8_t *row_valid;
} hm_batch_in;

/* Per-batch results. Arrays are library-owned and stay valid until the next call on this context
 * (or hm_destroy). With out_memory == HM_MEM_DEVICE they are device pointers.
 * Tiles (update mode: every (cell, window) changed by this batch, with cumulative aggregates):
 *   cell, window_start_us, count, avg_speed (0.0 when speed_null), speed_null, avg_lon, avg_lat.
 *   window end = window_start_us + tile_us.
 * Latest positions: row indices (into this batch's input) of every row whose eventTs equals the max
 *   eventTs of its (provider, vehicleId) among this batch's valid rows; ties give several rows. Sorted. */
typedef struct hm_batch_out {
    int64_t n_tiles;
    const uint64_t *cell;
    const int64_t *window_start_us;
    const int64_t *count;
    const double *avg_speed;
    const uint8_t *speed_null;
    const double *avg_lon;
    const double *avg_lat;
    int64_t n_latest;
    const int64_t *latest_row;
    /* batch statistics */
    int64_t n_in;                 /* input rows */
    int64_t n_valid;              /* rows passing the filter (heatmap_stream.py:98-106) */
    int64_t n_late;               /* valid rows dropped by the watermark */
    int64_t n_state;              /* live keys in the persistent tile state after the batch */
    int64_t batch_max_event_ms;   /* max(eventTs/1000) over valid rows, INT64_MIN if none */
    int64_t watermark_ms;         /* watermark used for eviction in this batch */
    int64_t late_watermark_ms;    /* watermark used to drop late rows in this batch */
    int64_t n_partials;           /* partial records merged (after the in-batch LDS pre-aggregation) */
} hm_batch_out;

typedef struct hm_ctx hm_ctx;

int hm_create(const hm_config *cfg, hm_ctx **out);
void hm_destroy(hm_ctx *ctx);
const char *hm_last_error(const hm_ctx *ctx);   /* ctx may be NULL: last error of hm_create */

/* Single-GPU hot path for one micro-batch. epoch_id is recorded (Spark's batch id); batches must be
 * passed in order, including empty (no-data) batches. out_memory selects host or device result arrays. */
int hm_process_batch(hm_ctx *ctx, int64_t epoch_id, const hm_batch_in *in, int32_t out_memory,
                     hm_batch_out *out);

/* Per-row UDF: cells for n points (degrees) at resolution res; 0 for rows the UDF maps to None.
 * Pointers are in `memory` space (host pointers are copied). Runs on device `device`. */
int hm_latlng_to_cell(const double *lat, const double *lon, int64_t n, int32_t res, int32_t memory,
                      int32_t device, uint64_t *out);
/* Inputs of the last hm_latlng_to_cell call on `device` that the fast path handed to the exact path (its near-tie
 * exceptions; tests check that constructed near-ties exercise it). */
int64_t hm_latlng_to_cell_last_exact(int32_t device);

/* ---- multi-GPU stage API (one context per GPU/rank; the caller performs the exchanges) ----
 * Replaces Spark's shuffle of the groupBy and of the latest-position join (heatmap_stream.py:44,112-133,198-207).
 * Per micro-batch:
 * 1. hm_stage_ingest: snap + filter + window + late test + this rank's latest-position max; writes this rank's
 *    summary (HM_STAGE_SUMMARY_WORDS int64 words, host memory) for the caller to all-gather.
 * 2. hm_stage_send(all ranks' summaries, [nranks][HM_STAGE_SUMMARY_WORDS], rank-major): every rank derives the
 *    same batch-wide decisions from them -- the global max event time (the watermark's input, :107), the
 *    aggregation path and the batch's global window registry -- and writes ONE chunk per destination rank into the
 *    caller's device send buffer (send_cap bytes; hm_stage_send_capacity(n, nranks) bytes are always enough), its
 *    size in bytes into send_bytes[r].  A tile key's destination owns a contiguous range of the key hash's 13-bit
 *    region field (rank r: [ceil(r 8192 / nranks), ceil((r + 1) 8192 / nranks))); a candidate's is a hash of its
 *    vkey.  Chunk (little-endian, every part 32-B aligned):
 *      header, 8 int64: magic 0x314b4e5548434d48, records, candidates, record bytes, bins, records offset,
 *        candidates offset, chunk bytes
 *      direct path (sizes.table_mode == 0): u32 counts[bins] (the records of each region field the destination
 *        owns, in order), u32 census[4096] (records per global window slot), then one 32-B record per aggregated
 *        row, grouped by region field: u64 cell's low 52 bits | (1 + the window's global registry slot) << 52,
 *        speed bits (null = 0x7ff0000000000001, NaN canonical), f64 lat, f64 lon;
 *      table mode (sizes.table_mode == 1, low-cardinality batches): bins = 0, one 48-B tile partial per key of the
 *        rank's shard: u64 cell, i64 window_start_us, u32 count, u32 n_speed, f64 sum_speed, f64 sum_lat, f64 sum_lon;
 *      then the latest candidates, 32 B: u64 vkey, i64 ts_us, i64 row, i64 origin_rank.
 * 3. caller: one all_to_all of the chunks (sizes first); recv_buf holds the chunks of ranks 0..nranks-1 in order.
 * 4. hm_stage_merge: the owner merges the received tile records into the persistent state it owns (each of its
 *    (window, region) bins from its senders' segments: no second partition), emits the tiles it owns, reduces the
 *    received candidates to winners, and writes the winners' row indices grouped by origin rank into
 *    winner_send_buf (capacity >= the candidates received) with per-origin counts.
 * 5. caller: exchange winners back; hm_stage_finish takes the received winners (rows of this rank).
 * After hm_stage_merge the owner's tiles can be encoded (hm_last_windows, hm_encode_tile_updates); after hm_stage_finish
 * the rank's latest rows can (hm_last_latest_buckets, hm_encode_position_updates, with the batch's dictionaries): every
 * rank writes the statements of what it owns, so no statement crosses the exchange.  A device caller keeps its input
 * buffers until then.  A context serves one rank of one world size (hm_config.shard_rank / shard_count, or fixed by
 * its first hm_stage_ingest): its tables hold that rank's keys only. */
#define HM_STAGE_SUMMARY_WORDS 8200
#define HM_TILE_REC_BYTES 48
#define HM_EVENT_REC_BYTES 32
#define HM_CAND_REC_BYTES 32
typedef struct hm_stage_sizes {
    int64_t table_mode;                  /* the batch's aggregation path (the same on every rank) */
    int64_t n_tile_records;              /* tile records this rank sent */
    int64_t n_cands;                     /* latest candidates this rank sent */
    int64_t global_batch_max_event_ms;   /* max over all ranks */
    int64_t n_valid, n_late;             /* this rank's rows */
    int64_t n_self_records;              /* of n_tile_records: the ones of bins this rank owns, kept in its own slabs
                                            (the chunk it addresses to itself carries their counts and census, and
                                            records = 0 in its header; hm_stage_merge merges them from the slabs) */
} hm_stage_sizes;

int hm_stage_ingest(hm_ctx *ctx, int64_t epoch_id, const hm_batch_in *in, int32_t nranks, int32_t rank,
                    int64_t *summary);
int64_t hm_stage_send_capacity(int64_t n_rows, int32_t nranks);
int hm_stage_send(hm_ctx *ctx, const int64_t *summaries, void *send_buf, int64_t send_cap, int64_t *send_bytes,
                  hm_stage_sizes *sizes);
int hm_stage_merge(hm_ctx *ctx, const void *recv_buf, const int64_t *recv_bytes, int32_t out_memory, hm_batch_out *out,
                   void *winner_send_buf, int64_t winner_send_cap, int64_t *winner_send_counts);
int hm_stage_finish(hm_ctx *ctx, const void *winner_recv_dev, int64_t n_winner_recv, int32_t out_memory,
                    hm_batch_out *out);
/* Orders the context's stream after the work queued so far on `stream` (a hipStream_t of the caller: the stream its
 * collective ran on, e.g. torch's current stream after RCCL's all_to_all): an event recorded there and waited for on
 * the library's stream, so that the next stage reads the received buffer without a host synchronization.  NULL = the
 * legacy default stream. */
int hm_stream_wait(hm_ctx *ctx, void *stream);

/* device helpers for the caller's exchange buffers */
int hm_device_memory(int32_t device, int64_t *free_bytes, int64_t *total_bytes);   /* (sizes a state arena) */
int hm_device_alloc(int32_t device, int64_t bytes, void **ptr);
int hm_device_free(int32_t device, void *ptr);
int hm_memcpy(void *dst, const void *src, int64_t bytes, int32_t kind); /* 0 H2D 1 D2H 2 D2D */
/* page-locked host memory (the checkpoint's export buffer: a device-to-host copy into it runs at the link's rate) */
int hm_host_alloc(int64_t bytes, void **ptr);
int hm_host_free(void *ptr);

/* Self-test entry (host-side execution of the device numerics; no GPU needed): evaluates the
 * extended-precision emulation used by the kernels, op codes as oracle_ld_ops(). */
int hm_selftest_ld_ops(const double *a, int64_t n, int32_t op, double *out);
/* floor(t[i] / d) by k_ingest's invariant-divisor multiply (kernels.h FloorDiv), executed on the host */
int hm_selftest_floor_div(const int64_t *t, int64_t n, int64_t d, int64_t *out);
/* Host-side execution of the device latLngToCell exact path (upstream's sequence with glibc's transcendentals as
 * restated in csrc/glibc_libm.h: the same numerics as k_ingest_exact / k_cells_exact). */
int hm_selftest_latlng_to_cell_host(const double *lat, const double *lon, int64_t n, int32_t res,
                                    uint64_t *out);
/* Host-side execution of the kernels' fast path (latLngToCellFast: direct gnomonic projection with a margin
 * test) with the exact path as fallback, as k_ingest + k_ingest_exact run it; fell_back[i] = 1 where the
 * exact path was taken (may be NULL). */
int hm_selftest_latlng_to_cell_fast_host(const double *lat, const double *lon, int64_t n, int32_t res,
                                         uint64_t *out, uint8_t *fell_back);
/* glibc 2.35's sincos / acos / atan2 / tan as the exact path restates them (csrc/glibc_libm.h; what the
 * reference's h3 calls through the host libm, heatmap_stream.py:65-75): fn 0 sincos(a) -> out = sin, out2 = cos;
 * 1 acos(a); 2 atan2(a, b); 3 tan(a).  _host runs the code on the CPU, _device on GPU `device` (host arrays). */
int hm_selftest_glibc_libm_host(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2);
int hm_selftest_glibc_libm_device(int32_t fn, const double *a, const double *b, int64_t n, double *out, double *out2,
                                  int32_t device);

/* Tile-state checkpoint (Spark's state store version after an epoch, heatmap_stream.py:37,244).
 * One record per live (cellId, windowStart) key: the cumulative aggregates the next batches build on.
 * reserved must be 0 on import. Records are in no particular order. */
typedef struct hm_state_rec {
    uint64_t cell;
    int64_t window_start_us;
    int64_t count;        /* count(1) so far */
    int64_t n_speed;      /* non-null speedKmh rows so far */
    double sum_speed;
    double sum_lat;
    double sum_lon;
    int64_t reserved;
} hm_state_rec;   /* 64 B */

typedef struct hm_state_info {
    int64_t epoch_id;            /* last epoch processed by the context (-1: none) */
    int64_t n_keys;              /* records */
    int64_t watermark_ms;        /* the watermark the next batch evicts with */
    int64_t prev_watermark_ms;   /* the one it drops late rows with (late_uses_prev_watermark) */
    int64_t tile_us;             /* must match the importing context's config */
    int64_t watermark_delay_ms;  /* idem */
    int32_t h3_res;              /* idem */
    int32_t reserved;
} hm_state_info;

/* Fills *info; with recs != NULL also writes info->n_keys records to recs (host memory, cap records:
 * HM_E_INVALID if cap < n_keys). Call once with recs = NULL for the size. Not between stage calls. */
int hm_state_export(hm_ctx *ctx, hm_state_info *info, hm_state_rec *recs, int64_t cap);
/* Incremental checkpoint (Spark's state store delta files): the records of the keys the last batch touched (their
 * cumulative values), *n_out of them (recs = NULL: count only); info as hm_state_export (n_keys = all live keys).  The
 * state after that batch = the last-written record of every key of an older full export followed by the deltas of the
 * batches since, keeping keys whose window end > info->prev_watermark_ms * 1000. */
int hm_state_export_touched(hm_ctx *ctx, hm_state_info *info, hm_state_rec *recs, int64_t cap, int64_t *n_out);
/* The same exports in two halves, for a checkpoint file writer that overlaps the device-to-host copy with the
 * statements' encode and the file write (the reference's state store write, heatmap_stream.py:37,244): _begin dumps the
 * state -- every live key, or (touched_only) the last batch's touched keys -- into device memory and returns
 * *n_out; _copy writes records [first, first + count) of that dump to host memory `recs` (page-locked memory: the
 * copy runs at the link's rate).  _copy may run on another thread while hm_encode_tile_updates /
 * hm_encode_position_updates run on this context (it uses a stream of its own), never beside hm_process_batch, a
 * stage call or another export; a batch or another export in between makes it fail (HM_E_STATE). */
int hm_state_export_begin(hm_ctx *ctx, hm_state_info *info, int32_t touched_only, int64_t *n_out);
int hm_state_export_copy(hm_ctx *ctx, hm_state_rec *recs, int64_t first, int64_t count);
/* _copy split in two: _async enqueues the copy and marks its completion in slot (0..63) -- call it on the engine's
 * thread BEFORE the statements' encode, so that the encode's copies queue behind it, not the other way round -- and
 * _wait (any thread) blocks until the copy marked in slot has landed. */
int hm_state_export_copy_async(hm_ctx *ctx, hm_state_rec *recs, int64_t first, int64_t count, int32_t slot);
int hm_state_export_copy_wait(hm_ctx *ctx, int32_t slot);
/* Restores an exported state into a context that has processed no batch (HM_E_STATE otherwise); the
 * config fields of info must equal the context's (HM_E_INVALID). recs: info->n_keys distinct keys, host memory. */
int hm_state_import(hm_ctx *ctx, const hm_state_info *info, const hm_state_rec *recs);

/* Tiles of the last batch as MongoDB update statements (reference heatmap_stream.py:164-196): statement i is
 * bytes[offsets[i], offsets[i+1]), the BSON document {q: {_id}, u: {$set: doc}, multi: false, upsert: true}
 * that pymongo sends for the reference's UpdateOne({"_id": _id}, {"$set": doc}, upsert=True), doc as :164-188.
 * Datetimes are pyspark's naive local wall times: the caller gives, for each window of hm_last_windows (same
 * order), the local UTC offset in seconds at the window's start and at its end. Outputs are library-owned
 * until the next call (device or pinned host memory per out_memory). */
typedef struct hm_tile_doc_cfg {
    const char *city;               /* CITY, UTF-8, at most 64 bytes */
    int32_t city_len;
    int32_t reserved;
    int64_t ttl_ms;                 /* TTL_MINUTES * 60000 (staleAt = windowEnd + TTL) */
    int64_t n_windows;
    const int64_t *window_start_us; /* = hm_last_windows */
    const int64_t *start_offset_s;
    const int64_t *end_offset_s;
} hm_tile_doc_cfg;

/* The distinct window starts of the last batch's emitted tiles, ascending (*n = count; up to cap written). */
int hm_last_windows(hm_ctx *ctx, int64_t *window_start_us, int64_t cap, int64_t *n);
int hm_encode_tile_updates(hm_ctx *ctx, const hm_tile_doc_cfg *cfg, int32_t out_memory, const uint8_t **bytes,
                           const int64_t **offsets, int64_t *n_docs);

/* Latest positions of the last hm_process_batch as positions_latest update statements (reference
 * heatmap_stream.py:211-235): {q: {_id: "provider|vehicleId", $or: [{ts: {$exists: false}}, {ts: {$lt: ts}}]},
 * u: {$set: {provider, vehicleId, ts, loc}}, multi: false, upsert: true}, in latest_row order. The strings come
 * from the batch's dictionaries (the vkey the caller passed = provider_code * n_vehicles + vehicle_code; string k
 * of a dictionary = bytes[offsets[k], offsets[k+1]), UTF-8); ts is the naive local datetime of eventTs, with the
 * local UTC offset of the row's 900-s bucket floor(ts_s / 900): bucket_offset_s[k] for bucket_ids[k] (the distinct
 * buckets of the latest rows, strictly ascending; a row whose bucket is absent fails the call). After the stage API:
 * this rank's latest rows (hm_stage_finish). Outputs as hm_encode_tile_updates. */
typedef struct hm_position_doc_cfg {
    int64_t n_providers;
    const int64_t *provider_offsets;   /* n_providers + 1 */
    const char *provider_bytes;
    int64_t n_vehicles;
    const int64_t *vehicle_offsets;    /* n_vehicles + 1 */
    const char *vehicle_bytes;
    int64_t n_buckets;
    const int64_t *bucket_ids;         /* n_buckets, strictly ascending */
    const int64_t *bucket_offset_s;    /* n_buckets */
} hm_position_doc_cfg;
int hm_encode_position_updates(hm_ctx *ctx, const hm_position_doc_cfg *cfg, int32_t out_memory, const uint8_t **bytes,
                               const int64_t **offsets, int64_t *n_docs);
/* After an hm_encode_* call with HM_MEM_HOST_STREAM: blocks until bytes [0, upto) of its statements have landed in
 * the host buffer (any thread), so that a sink sends each command as soon as its statements are there -- the
 * statements' device-to-host copy overlaps the sink's writes instead of preceding them (reference :191-196,230-235). */
int hm_statements_wait(hm_ctx *ctx, int64_t upto);

/* Host execution of hm_encode_tile_updates' statement encoder on caller arrays (no GPU needed): statement i
 * is bytes[offsets[i], offsets[i+1]) (offsets: n+1 entries; HM_E_INVALID if cap bytes do not suffice). */
int hm_selftest_tile_statements(const hm_tile_doc_cfg *cfg, int32_t h3_res, int64_t tile_us, const uint64_t *cell,
                                const int64_t *ws, const int64_t *cnt, const double *sp, const uint8_t *spn,
                                const double *lon, const double *lat, int64_t n, uint8_t *bytes, int64_t cap,
                                int64_t *offsets);

/* Host execution of hm_encode_position_updates' encoder on caller rows (row i: vkey[i], ts[i], lat[i], lon[i]). */
int hm_selftest_position_statements(const hm_position_doc_cfg *cfg, const uint64_t *vkey, const int64_t *ts,
                                    const double *lat, const double *lon, int64_t n, uint8_t *bytes, int64_t cap,
                                    int64_t *offsets);

/* Timing of the last hm_process_batch / stage batch on the library's stream (HIP events), milliseconds
 * per phase: index 0 ingest (k_ingest: filter + cells + windows + event keys + latest max), 1 table-mode
 * aggregation (k_agg + k_bin_reduce), 2 merge, 3 emit, 4 dedup (flag + compaction), 5 total, 6 (window, region)
 * partition, 7 stage API: the sender's partition by owner rank.  Host side of the last hm_process_batch (wall
 * clock): 8 the call, 9 blocked in stream synchronizations, 10 in device/pinned allocations and frees, 11 the
 * longest single synchronization, 12 its source line in the library, 13 allocations + frees made. */
int hm_last_timings(const hm_ctx *ctx, double *ms, int32_t n);

/* ---- Kafka message values -> batch columns (reference heatmap_stream.py:51-61, 88-93) ----
 * The micro-batch's Kafka values (the producer's JSON records, mbta_to_kafka.py:66-74), back to back with
 * n + 1 offsets (Arrow binary/string layout; offsets[0] may be > 0), parsed on the device like
 * from_json(value, schema) in PERMISSIVE mode + to_timestamp(ts) (rules: csrc/json_decode.h): the columns of
 * hm_batch_in (device memory, valid until the next hm_decode_json on this context) with row_valid = provider,
 * vehicleId and eventTs non-null, and vkey = provider_code * n_vehicles + vehicle_code from the batch's exact
 * string dictionaries (code order unspecified; strings as Arrow offsets + UTF-8 bytes in pinned host memory, the
 * layout hm_encode_position_updates takes).  Records the device decoder does not handle (see json_decode.h) fail
 * the call with HM_E_UNSUPPORTED, unless flags holds HM_JSON_SPLICE: then they decode to all-null rows listed in
 * unsupported_rows, the dictionaries hold the other rows' strings only, and the caller decodes those records on the
 * host and writes them in with hm_json_patch before hm_process_batch (mobheat/engine.py decode_json).  Malformed
 * records decode to all-null rows (counted). */
#define HM_JSON_SPLICE 1
typedef struct hm_json_in {
    int64_t n;
    int32_t memory;            /* HM_MEM_HOST or HM_MEM_DEVICE: where bytes and offsets live */
    int32_t flags;             /* HM_JSON_SPLICE or 0 */
    const uint8_t *bytes;
    const int64_t *offsets;    /* n + 1 */
} hm_json_in;
typedef struct hm_json_out {
    hm_batch_in batch;         /* device columns, ready for hm_process_batch */
    int64_t n_providers;
    const int64_t *provider_offsets;   /* n_providers + 1 */
    const uint8_t *provider_bytes;
    int64_t n_vehicles;
    const int64_t *vehicle_offsets;    /* n_vehicles + 1 */
    const uint8_t *vehicle_bytes;
    int64_t n_malformed;       /* records that decoded to all-null rows (from_json's malformed records) */
    int64_t n_unsupported;     /* records outside the device decoder (HM_E_UNSUPPORTED, or spliced) */
    const int64_t *unsupported_rows;   /* HM_JSON_SPLICE: their row indices, ascending (host memory, valid until the
                                          next hm_decode_json) */
} hm_json_out;
int hm_decode_json(hm_ctx *ctx, const hm_json_in *in, hm_json_out *out);
/* The splice step: rows[k] (from unsupported_rows) of the last hm_decode_json get lat / lon / ts_us / speed /
 * speed_valid / row_valid and the dictionary codes pcode[k] / vcode[k] (host arrays, m entries; codes index the
 * extended dictionaries of n_providers / n_vehicles strings: the decoder's strings with the caller's appended);
 * every other valid row's vkey is re-encoded for the new n_vehicles.  The batch from hm_decode_json then holds the
 * whole micro-batch. */
int hm_json_patch(hm_ctx *ctx, int64_t m, const int64_t *rows, const double *lat, const double *lon,
                  const int64_t *ts_us, const double *speed, const uint8_t *speed_valid, const uint8_t *row_valid,
                  const int64_t *pcode, const int64_t *vcode, int64_t n_providers, int64_t n_vehicles);

/* ---- Arrow columns -> batch columns on the device (the boundary's Spark / Arrow / pandas frames; reference
 * heatmap_stream.py:51-61,150) ----
 * The micro-batch's columns in Arrow's memory layout, in host memory (zero-copy views of a pyarrow Table, of pyspark's
 * collected Arrow batches or of a pandas frame converted to Arrow): the library copies them to the device and builds
 * hm_batch_in there -- lat / lon null -> NaN (fails between(), :101-102), speedKmh null -> speed_valid 0, row_valid =
 * provider, vehicleId and eventTs non-null (:99-103) -- and factorises provider and vehicleId with the exact device
 * string dictionaries of hm_decode_json (vkey = provider_code * n_vehicles + vehicle_code; the dictionaries come back
 * as Arrow offsets + UTF-8 bytes for hm_encode_position_updates).  Outputs as hm_decode_json (n_malformed and
 * n_unsupported 0), valid until the next hm_decode_json / hm_arrow_columns on this context. */
typedef struct hm_arrow_col {
    const void *values;        /* float64 (lat, lon, speed) / int64 (ts_us, microseconds UTC) values, or a string column's
                                  n + 1 offsets into data; NULL = the column is absent (every row null) */
    const uint8_t *data;       /* string columns: the UTF-8 bytes the offsets point into */
    const uint8_t *validity;   /* Arrow validity bitmap (bit validity_offset + i, least significant bit first); NULL =
                                  no nulls */
    int64_t validity_offset;
    int32_t offset_bytes;      /* string columns: 4 (Arrow string) or 8 (large_string) */
    int32_t unit;              /* ts_us only: 0 = microseconds, 1 = nanoseconds (pandas' datetime64[ns], handed over as it
                                  is: the device truncates toward zero to microseconds, as Arrow's unsafe cast does);
                                  0 for every other column */
} hm_arrow_col;
typedef struct hm_arrow_in {
    int64_t n;
    hm_arrow_col lat, lon, speed, ts_us, provider, vehicle;
} hm_arrow_in;
int hm_arrow_columns(hm_ctx *ctx, const hm_arrow_in *in, hm_json_out *out);

/* The distinct 900-s buckets floor(ts_s / 900) of the last hm_process_batch's latest rows, ascending (computed on
 * the device; *n = count, up to cap written): the buckets whose local offsets hm_encode_position_updates needs. */
int hm_last_latest_buckets(hm_ctx *ctx, int64_t *bucket_ids, int64_t cap, int64_t *n);

/* Host execution of the record decoder (json_decode.h) on n records (bytes readable up to 16 bytes past the last
 * record: the decoder reads 16-B windows); scratch (same size as bytes) receives escaped strings' decoded bytes.
 * Per record: lat, lon, speed (NaN when null), ts_us, bearing, accuracy, the provider / vehicleId spans (absolute
 * offsets into bytes, or into scratch when the JF_*_ESC flag is set) and the field flags. */
int hm_selftest_json_records(const uint8_t *bytes, const int64_t *offsets, int64_t n, uint8_t *scratch, double *lat,
                             double *lon, double *speed, int64_t *ts_us, int32_t *bearing, int32_t *accuracy,
                             int64_t *p_off, int32_t *p_len, int64_t *v_off, int32_t *v_len, uint32_t *flags);
/* Host execution of the decoder's decimal -> binary64 conversion: bits[i] = w[i] * 10^q[i] correctly rounded. */
int hm_selftest_decimal_to_double(const uint64_t *w, const int64_t *q, int64_t n, uint64_t *bits);

/* ---- read side (reference app.py:19-41 h3_boundary_geojson -> h3.cell_to_boundary) ----
 * cellToBoundary of n cells: vertex k of cell i at lat[10 i + k], lng[10 i + k] (degrees, upstream's vertex order;
 * unused slots NaN), nverts[i] vertices (5-10; 0 for an invalid index).  memory as hm_latlng_to_cell. */
int hm_cells_to_boundary(const uint64_t *cells, int64_t n, int32_t memory, int32_t device, double *lat, double *lng,
                         int32_t *nverts);
/* Host execution of the same device code (no GPU; the CPU tests compare it with the oracle). */
int hm_selftest_cells_to_boundary_host(const uint64_t *cells, int64_t n, double *lat, double *lng, int32_t *nverts);

/* Counts of the last hm_process_batch / stage batch (up to n of them): [0] keys created in the tile state, [1] partial
 * records merged (direct path: aggregated rows; table mode: ~ distinct keys; stage API: the records this rank
 * received as owner), [2] tiles emitted, [3] 1 if table mode ran, [4] table mode: aggregates evicted from k_agg's
 * LDS tables into its buckets, [5] stage API: tile records this rank sent, [6] device + pinned-host allocations and
 * [7] frees the context made since hm_create (steady-state batches make none: tests/test_gpu_parity.py), [8] 1 if the
 * direct path's rows were binned by the ingest itself (no separate partition pass), [9] stage API: of [5], the records
 * of bins this rank owns, kept in its slabs (hm_stage_sizes.n_self_records), [10] hm_process_batch: the chunks the
 * batch was pipelined in (each chunk's ingest overlapping the previous chunk's merge; 0: not pipelined). */
int hm_last_counts(const hm_ctx *ctx, int64_t *c, int32_t n);
/* Version of the persistent tile state: incremented when a batch starts merging into it (hm_process_batch,
 * hm_stage_merge, growth).  A call that failed without changing it left the state as it was (-1: ctx NULL). */
int64_t hm_state_version(const hm_ctx *ctx);

/* HM_ABI_VERSION the library was built with (callers check it before hm_create). */
int32_t hm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
