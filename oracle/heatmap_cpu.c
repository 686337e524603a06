/* ORACLE -- test infrastructure only (the bench's cpu_baseline leg and tests/; never linked by the product).
 *
 * The reference's per-micro-batch work (heatmap_stream.py) restated as multi-threaded C with OpenMP, so that the
 * bench's CPU baseline is an honest compiled implementation of the whole batch rather than numpy glue:
 *   filter (:96-104, UDF guard :66-69) -> latLngToCell (:65-75, this directory's h3_oracle.c) -> tumbling window
 *   (:115, Spark TimeWindowing floor-mod) -> late rows against the previous batch's watermark (:107, Spark 3.5
 *   allowMultiple) -> groupBy(window, cellId) count / avg(speedKmh) / avg(lon) / avg(lat) in update mode (:112-133,
 *   :243; cumulative state, only touched keys emitted) -> eviction with the current watermark -> watermark for the
 *   next batch -> latest rows per vehicle, ties kept (:200-207).
 * Semantics are those of oracle/spark_oracle.py (tests/test_cpu_restatement.py checks the two agree batch by
 * batch); the structure is the usual shared-nothing CPU plan: rows hashed into P key partitions (each thread's rows
 * keep their order), one open-addressing state table per partition, partitions aggregated in parallel, the same for
 * the per-vehicle maxima.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

uint64_t oracle_latlng_to_cell(double lat_deg, double lng_deg, int res);

#define NPART 256
#define MAXT 256

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

typedef struct {
    uint64_t cell;     /* 0 = empty */
    int64_t ws;
    int64_t cnt, nsp;
    double ssp, sla, slo;
    uint64_t seq;      /* batch that last touched the key */
} Slot;

typedef struct {
    Slot *s;
    int64_t cap, n;
    int64_t min_ws;
    int64_t *touched;  /* slot indices touched by this batch, first-touch order */
    int64_t n_touched, touched_cap;
} Table;

typedef struct {
    uint64_t vkey;
    int64_t maxts;
    int used;
} VSlot;

typedef struct hmcpu {
    int res;
    int64_t tile, delay;
    int64_t wm_prev, wm_cur;
    uint64_t seq;
    Table part[NPART];
    /* per-row scratch */
    int64_t cap_rows;
    uint64_t *cell;
    int16_t *pid, *vpid;
    int64_t *idx, *vidx;
    /* outputs of the last batch */
    int64_t n_tiles, o_cap;
    uint64_t *o_cell;
    int64_t *o_ws, *o_cnt;
    double *o_sp, *o_lat, *o_lon;
    uint8_t *o_spn;
    int64_t n_latest;
    int64_t *latest;
    int64_t n_valid, n_late, batch_max_ms, watermark_ms, late_watermark_ms, n_state;
    /* per-vehicle max tables, one per partition */
    VSlot *vt[NPART];
    int64_t vcap[NPART];
} hmcpu;

static uint64_t key_hash(uint64_t cell, int64_t ws) { return mix64(cell ^ mix64((uint64_t)ws + 0x9e3779b97f4a7c15ULL)); }

static int table_reserve(Table *t, int64_t keys) {
    if (2 * keys <= t->cap) return 0;
    int64_t cap = t->cap ? t->cap : 1024;
    while (2 * keys > cap) cap *= 2;
    Slot *s = calloc((size_t)cap, sizeof(Slot));
    if (!s) return -1;
    for (int64_t i = 0; i < t->cap; i++) {
        if (!t->s[i].cell) continue;
        uint64_t h = key_hash(t->s[i].cell, t->s[i].ws) & (uint64_t)(cap - 1);
        while (s[h].cell) h = (h + 1) & (uint64_t)(cap - 1);
        s[h] = t->s[i];
    }
    free(t->s);
    t->s = s;
    t->cap = cap;
    return 0;
}

static int grow(void **p, int64_t *cap, int64_t need, size_t el) {
    if (need <= *cap) return 0;
    int64_t c = need + need / 4 + 1024;
    void *q = realloc(*p, (size_t)c * el);
    if (!q) return -1;
    *p = q;
    *cap = c;
    return 0;
}

hmcpu *hmcpu_create(int res, int64_t tile_us, int64_t delay_ms) {
    hmcpu *c = calloc(1, sizeof(hmcpu));
    if (!c) return 0;
    c->res = res;
    c->tile = tile_us;
    c->delay = delay_ms;
    for (int p = 0; p < NPART; p++) c->part[p].min_ws = INT64_MAX;
    return c;
}

void hmcpu_destroy(hmcpu *c) {
    if (!c) return;
    for (int p = 0; p < NPART; p++) {
        free(c->part[p].s);
        free(c->part[p].touched);
        free(c->vt[p]);
    }
    free(c->cell); free(c->pid); free(c->vpid); free(c->idx); free(c->vidx);
    free(c->o_cell); free(c->o_ws); free(c->o_cnt); free(c->o_sp); free(c->o_lat); free(c->o_lon); free(c->o_spn);
    free(c->latest);
    free(c);
}

static int ensure_rows(hmcpu *c, int64_t n) {
    if (n <= c->cap_rows) return 0;
    int64_t m = n + n / 4;
    free(c->cell); free(c->pid); free(c->vpid); free(c->idx); free(c->vidx); free(c->latest);
    c->cell = malloc((size_t)m * 8);
    c->pid = malloc((size_t)m * 2);
    c->vpid = malloc((size_t)m * 2);
    c->idx = malloc((size_t)m * 8);
    c->vidx = malloc((size_t)m * 8);
    c->latest = malloc((size_t)m * 8);
    if (!c->cell || !c->pid || !c->vpid || !c->idx || !c->vidx || !c->latest) return -1;
    c->cap_rows = m;
    return 0;
}

/* counting scatter of row indices by partition id (-1: none), each thread's rows in order, partitions contiguous:
 * rows of partition p are out[off[p] .. off[p + 1]) in ascending row order */
static void scatter_rows(const int16_t *pid, int64_t n, int T, int64_t *out, int64_t off[NPART + 1]) {
    static int64_t cnt[MAXT][NPART];
    int64_t chunk = (n + T - 1) / T;
#pragma omp parallel num_threads(T)
    {
        int t = omp_get_thread_num();
        int64_t a = t * chunk, b = a + chunk < n ? a + chunk : n;
        int64_t *ct = cnt[t];
        memset(ct, 0, sizeof(cnt[0]));
        for (int64_t i = a; i < b; i++)
            if (pid[i] >= 0) ct[pid[i]]++;
#pragma omp barrier
#pragma omp single
        {
            int64_t s = 0;
            for (int p = 0; p < NPART; p++) {
                off[p] = s;
                for (int u = 0; u < T; u++) {
                    int64_t v = cnt[u][p];
                    cnt[u][p] = s;
                    s += v;
                }
            }
            off[NPART] = s;
        }
        for (int64_t i = a; i < b; i++)
            if (pid[i] >= 0) out[ct[pid[i]]++] = i;
    }
}

/* One micro-batch.  speed/speed_valid/vkey/row_valid may be NULL (no speed column: every speed null; vkey 0;
 * every row valid).  Returns 0, or -1 when out of memory. */
int hmcpu_process(hmcpu *c, int64_t n, const double *lat, const double *lon, const int64_t *ts, const double *speed,
                  const uint8_t *speed_valid, const uint64_t *vkey, const uint8_t *row_valid, int nthreads) {
    int T = nthreads > 0 ? nthreads : omp_get_max_threads();
    if (T > MAXT) T = MAXT;
    if (ensure_rows(c, n)) return -1;
    const int64_t tile = c->tile, late_wm = c->wm_prev, lo_ts = INT64_MIN + 2 * tile, hi_ts = INT64_MAX - 2 * tile;
    int64_t n_valid = 0, n_late = 0, bmax = INT64_MIN;
    c->seq++;

    /* filter, window, late test, cell, key partition; vehicle partition of the valid rows */
#pragma omp parallel for num_threads(T) schedule(static) reduction(+ : n_valid, n_late) reduction(max : bmax)
    for (int64_t i = 0; i < n; i++) {
        const double la = lat[i], lo = lon[i];
        const int64_t t = ts[i];
        int valid = la >= -90.0 && la <= 90.0 && lo >= -180.0 && lo <= 180.0 && t > lo_ts && t < hi_ts &&
                    (!row_valid || row_valid[i]);
        c->pid[i] = -1;
        c->vpid[i] = -1;
        if (!valid) continue;
        n_valid++;
        const int64_t ms = t >= 0 ? t / 1000 : -((-t) / 1000);
        if (ms > bmax) bmax = ms;
        const uint64_t vk = vkey ? vkey[i] : 0;
        c->vpid[i] = (int16_t)(mix64(vk ^ 0x2545f4914f6cdd1dULL) >> 56);
        int64_t m = t % tile;
        if (m < 0) m += tile;
        const int64_t ws = t - m;
        if (ws + tile <= late_wm * 1000) {
            n_late++;
            continue;
        }
        const uint64_t cell = oracle_latlng_to_cell(la, lo, c->res);
        c->cell[i] = cell;
        c->pid[i] = (int16_t)(key_hash(cell, ws) >> 56);
    }

    /* aggregation into the partitions' state tables, touched keys in first-touch order */
    int64_t off[NPART + 1], voff[NPART + 1];
    scatter_rows(c->pid, n, T, c->idx, off);
    int oom = 0;
#pragma omp parallel for num_threads(T) schedule(dynamic, 1) reduction(| : oom)
    for (int p = 0; p < NPART; p++) {
        Table *tb = &c->part[p];
        const int64_t a = off[p], b = off[p + 1];
        tb->n_touched = 0;
        if (table_reserve(tb, tb->n + (b - a)) || grow((void **)&tb->touched, &tb->touched_cap, b - a, 8)) {
            oom = 1;
            continue;
        }
        const uint64_t mask = (uint64_t)tb->cap - 1;
        for (int64_t r = a; r < b; r++) {
            const int64_t i = c->idx[r];
            const int64_t t = ts[i];
            int64_t m = t % tile;
            if (m < 0) m += tile;
            const int64_t ws = t - m;
            const uint64_t cell = c->cell[i];
            uint64_t h = key_hash(cell, ws) & mask;
            while (tb->s[h].cell && !(tb->s[h].cell == cell && tb->s[h].ws == ws)) h = (h + 1) & mask;
            Slot *s = &tb->s[h];
            if (!s->cell) {
                s->cell = cell;
                s->ws = ws;
                tb->n++;
                if (ws < tb->min_ws) tb->min_ws = ws;
            }
            if (s->seq != c->seq) {
                s->seq = c->seq;
                tb->touched[tb->n_touched++] = (int64_t)h;
            }
            s->cnt++;
            if (speed && (!speed_valid || speed_valid[i])) {
                s->nsp++;
                s->ssp += speed[i];
            }
            s->sla += lat[i];
            s->slo += lon[i];
        }
    }
    if (oom) return -1;

    /* emission: the touched keys' cumulative aggregates */
    int64_t toff[NPART + 1];
    toff[0] = 0;
    for (int p = 0; p < NPART; p++) toff[p + 1] = toff[p] + c->part[p].n_touched;
    c->n_tiles = toff[NPART];
    if (c->n_tiles > c->o_cap) {
        int64_t cap = c->n_tiles + c->n_tiles / 4 + 1024;
        free(c->o_cell); free(c->o_ws); free(c->o_cnt); free(c->o_sp); free(c->o_lat); free(c->o_lon); free(c->o_spn);
        c->o_cell = malloc((size_t)cap * 8); c->o_ws = malloc((size_t)cap * 8); c->o_cnt = malloc((size_t)cap * 8);
        c->o_sp = malloc((size_t)cap * 8); c->o_lat = malloc((size_t)cap * 8); c->o_lon = malloc((size_t)cap * 8);
        c->o_spn = malloc((size_t)cap);
        if (!c->o_cell || !c->o_ws || !c->o_cnt || !c->o_sp || !c->o_lat || !c->o_lon || !c->o_spn) return -1;
        c->o_cap = cap;
    }
    const int64_t evict_end = c->wm_cur * 1000;
    int64_t n_state = 0;
#pragma omp parallel for num_threads(T) schedule(dynamic, 1) reduction(+ : n_state) reduction(| : oom)
    for (int p = 0; p < NPART; p++) {
        Table *tb = &c->part[p];
        for (int64_t k = 0; k < tb->n_touched; k++) {
            const Slot *s = &tb->s[tb->touched[k]];
            const int64_t o = toff[p] + k;
            c->o_cell[o] = s->cell;
            c->o_ws[o] = s->ws;
            c->o_cnt[o] = s->cnt;
            c->o_spn[o] = s->nsp == 0;
            c->o_sp[o] = s->nsp ? s->ssp / (double)s->nsp : 0.0;
            c->o_lon[o] = s->slo / (double)s->cnt;
            c->o_lat[o] = s->sla / (double)s->cnt;
        }
        /* eviction after emission (current batch's watermark): rebuild the partition without the closed windows */
        if (tb->n && tb->min_ws + tile <= evict_end) {
            Slot *old = tb->s;
            const int64_t cap = tb->cap;
            Slot *s = calloc((size_t)cap, sizeof(Slot));
            if (!s) {
                oom = 1;
                continue;
            }
            int64_t keep = 0, mn = INT64_MAX;
            for (int64_t i = 0; i < cap; i++) {
                if (!old[i].cell || old[i].ws + tile <= evict_end) continue;
                uint64_t h = key_hash(old[i].cell, old[i].ws) & (uint64_t)(cap - 1);
                while (s[h].cell) h = (h + 1) & (uint64_t)(cap - 1);
                s[h] = old[i];
                keep++;
                if (old[i].ws < mn) mn = old[i].ws;
            }
            free(old);
            tb->s = s;
            tb->n = keep;
            tb->min_ws = mn;
        }
        n_state += tb->n;
    }
    if (oom) return -1;

    /* watermark for the next batch */
    c->n_valid = n_valid;
    c->n_late = n_late;
    c->batch_max_ms = n_valid ? bmax : INT64_MIN;
    c->watermark_ms = c->wm_cur;
    c->late_watermark_ms = late_wm;
    c->n_state = n_state;
    int64_t nxt = c->wm_cur;
    if (n_valid && bmax - c->delay > nxt) nxt = bmax - c->delay;
    c->wm_prev = c->wm_cur;
    c->wm_cur = nxt;

    /* latest rows per vehicle (ties kept): per-partition max ts, then the rows at their vehicle's max */
    scatter_rows(c->vpid, n, T, c->vidx, voff);
    VSlot **vt = c->vt;
    int64_t *vcap = c->vcap;
#pragma omp parallel for num_threads(T) schedule(dynamic, 1) reduction(| : oom)
    for (int p = 0; p < NPART; p++) {
        const int64_t a = voff[p], b = voff[p + 1];
        int64_t cap = 1024;
        while (cap < 2 * (b - a)) cap *= 2;
        if (cap > vcap[p]) {
            free(vt[p]);
            vt[p] = malloc((size_t)cap * sizeof(VSlot));
            if (!vt[p]) {
                vcap[p] = 0;
                oom = 1;
                continue;
            }
            vcap[p] = cap;
        }
        cap = vcap[p];
        memset(vt[p], 0, (size_t)cap * sizeof(VSlot));
        const uint64_t mask = (uint64_t)cap - 1;
        for (int64_t r = a; r < b; r++) {
            const int64_t i = c->vidx[r];
            const uint64_t vk = vkey ? vkey[i] : 0;
            uint64_t h = mix64(vk) & mask;
            while (vt[p][h].used && vt[p][h].vkey != vk) h = (h + 1) & mask;
            VSlot *s = &vt[p][h];
            if (!s->used || ts[i] > s->maxts) {
                s->used = 1;
                s->vkey = vk;
                s->maxts = ts[i];
            }
        }
    }
    if (oom) return -1;
    /* winners in ascending row order: per-thread counts, then positions */
    static int64_t wcnt[MAXT + 1];
    const int64_t chunk = (n + T - 1) / T;
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        const int64_t a = t * chunk, b = a + chunk < n ? a + chunk : n;
        int64_t k = 0;
        for (int pass = 0; pass < 2; pass++) {
            if (pass == 1) {
#pragma omp barrier
#pragma omp single
                {
                    int64_t s = 0;
                    for (int u = 0; u < T; u++) {
                        const int64_t v = wcnt[u];
                        wcnt[u] = s;
                        s += v;
                    }
                    wcnt[T] = s;
                }
                k = wcnt[t];
            }
            int64_t m = 0;
            for (int64_t i = a; i < b; i++) {
                const int p = c->vpid[i];
                if (p < 0) continue;
                const uint64_t vk = vkey ? vkey[i] : 0;
                const uint64_t mask = (uint64_t)vcap[p] - 1;
                uint64_t h = mix64(vk) & mask;
                while (vt[p][h].vkey != vk) h = (h + 1) & mask;
                if (ts[i] != vt[p][h].maxts) continue;
                if (pass == 0) m++;
                else c->latest[k++] = i;
            }
            if (pass == 0) wcnt[t] = m;
        }
    }
    c->n_latest = wcnt[T];
    return 0;
}

/* the last batch's results */
int64_t hmcpu_n_tiles(const hmcpu *c) { return c->n_tiles; }
void hmcpu_tiles(const hmcpu *c, uint64_t *cell, int64_t *ws, int64_t *cnt, double *sp, uint8_t *spn, double *lat,
                 double *lon) {
    const size_t n = (size_t)c->n_tiles;
    memcpy(cell, c->o_cell, n * 8); memcpy(ws, c->o_ws, n * 8); memcpy(cnt, c->o_cnt, n * 8);
    memcpy(sp, c->o_sp, n * 8); memcpy(spn, c->o_spn, n); memcpy(lat, c->o_lat, n * 8); memcpy(lon, c->o_lon, n * 8);
}
int64_t hmcpu_n_latest(const hmcpu *c) { return c->n_latest; }
void hmcpu_latest(const hmcpu *c, int64_t *rows) { memcpy(rows, c->latest, (size_t)c->n_latest * 8); }
/* n_valid, n_late, batch_max_ms, watermark_ms, late_watermark_ms, n_state */
void hmcpu_stats(const hmcpu *c, int64_t *out) {
    out[0] = c->n_valid; out[1] = c->n_late; out[2] = c->batch_max_ms;
    out[3] = c->watermark_ms; out[4] = c->late_watermark_ms; out[5] = c->n_state;
}
