"""ORACLE -- test infrastructure only (never imported by the product path).

CPU restatement of what the reference's Spark plan computes per micro-batch (reference heatmap_stream.py),
with Spark 3.5.1 semantics:

* filter (:96-104): provider, vehicleId, eventTs non-null; lat between -90 and 90, lon between -180 and 180
  (inclusive; NaN fails).  The UDF (:65-75) repeats the range test; the cellId-not-null filter (:106) never
  fires for in-range input.
* to_h3 (:65-75): h3.latlng_to_cell(lat, lon, H3_RES) -> oracle/h3_oracle.c.
* window(eventTs, TILE) (:115): start = ts - floormod(ts, tile), end = start + tile  (Spark TimeWindowing).
* withWatermark(eventTs, 10 min) (:107) + update output mode (:243), Spark 3.5 defaults
  (spark.sql.streaming.statefulOperator.allowMultiple = true): late rows are dropped with the PREVIOUS batch's
  watermark (window.end <= wm_prev ms * 1000), state is evicted after emission with the CURRENT batch's
  watermark (window.end <= wm_cur * 1000); wm_next = max(wm_cur, max over this batch's valid rows of
  (eventTs_us / 1000, truncated like Java long division) - delay), starting at 0.
* groupBy(window, cellId).agg(count(1), avg(speedKmh), avg(lon), avg(lat)) (:112-123): avg = sum over
  non-null / count of non-null (null when none; NaN propagates); cumulative over batches for live keys; only
  keys updated by the batch are emitted.
* latest per (provider, vehicleId) (:200-207): groupBy max(eventTs) then equi-join back -> every row whose
  eventTs equals its group's max (ties give several rows); batch-local, over valid rows (late rows included).

Rows whose eventTs lies within 2 tiles of the int64 limits are treated as invalid (outside Spark's timestamp
range; the device does the same).
"""
import numpy as np

from . import h3_oracle

INT64_MIN = np.iinfo(np.int64).min
INT64_MAX = np.iinfo(np.int64).max


class SparkHeatmapOracle:
    def __init__(self, h3_res=8, tile_minutes=5, watermark_delay_ms=600_000, late_uses_prev_watermark=True,
                 tile_us=None):
        self.res = int(h3_res)
        self.tile = int(tile_us) if tile_us is not None else int(tile_minutes) * 60_000_000
        self.delay = int(watermark_delay_ms)
        self.late_prev = bool(late_uses_prev_watermark)
        self.state = {}      # (cell, wstart) -> [count, nspeed, sum_speed, sum_lat, sum_lon]
        self.wm_prev = 0
        self.wm_cur = 0

    def valid_mask(self, lat, lon, ts, row_valid):
        lat = np.asarray(lat, np.float64)
        lon = np.asarray(lon, np.float64)
        ts = np.asarray(ts, np.int64)
        with np.errstate(invalid="ignore"):
            v = (lat >= -90.0) & (lat <= 90.0) & (lon >= -180.0) & (lon <= 180.0)
        v &= (ts > INT64_MIN + 2 * self.tile) & (ts < INT64_MAX - 2 * self.tile)
        if row_valid is not None:
            v &= np.asarray(row_valid).astype(bool)
        return v

    def process_batch(self, lat, lon, ts_us, speed=None, speed_valid=None, vkey=None, row_valid=None):
        lat = np.asarray(lat, np.float64)
        lon = np.asarray(lon, np.float64)
        ts = np.asarray(ts_us, np.int64)
        n = lat.size
        if speed is None:
            speed = np.zeros(n)
            speed_valid = np.zeros(n, bool)
        speed = np.asarray(speed, np.float64)
        sv = np.ones(n, bool) if speed_valid is None else np.asarray(speed_valid).astype(bool)
        vkey = np.zeros(n, np.uint64) if vkey is None else np.asarray(vkey, np.uint64)
        valid = self.valid_mask(lat, lon, ts, row_valid)

        late_wm = self.wm_prev if self.late_prev else self.wm_cur
        ws = ts - np.mod(ts, self.tile)
        late = valid & (ws + self.tile <= late_wm * 1000)
        agg = valid & ~late

        # ---- tiles ----
        idx = np.nonzero(agg)[0]
        cells = h3_oracle.latlng_to_cell(lat[idx], lon[idx], self.res)
        touched = []
        if idx.size:
            keys = np.rec.fromarrays([cells, ws[idx]], names="c,w")
            uniq, inv = np.unique(keys, return_inverse=True)
            inv = inv.ravel()
            cnt = np.bincount(inv, minlength=uniq.size)
            s_sv = sv[idx]
            nsp = np.bincount(inv, weights=s_sv.astype(np.float64), minlength=uniq.size).astype(np.int64)
            ssp = np.bincount(inv[s_sv], weights=speed[idx][s_sv], minlength=uniq.size)
            sla = np.bincount(inv, weights=lat[idx], minlength=uniq.size)
            slo = np.bincount(inv, weights=lon[idx], minlength=uniq.size)
            for u in range(uniq.size):
                k = (int(uniq["c"][u]), int(uniq["w"][u]))
                st = self.state.get(k)
                if st is None:
                    st = self.state[k] = [0, 0, 0.0, 0.0, 0.0]
                st[0] += int(cnt[u])
                st[1] += int(nsp[u])
                st[2] += float(ssp[u])
                st[3] += float(sla[u])
                st[4] += float(slo[u])
                touched.append(k)
        tiles = []
        for k in touched:
            c, n_sp, s_sp, s_la, s_lo = self.state[k]
            tiles.append(dict(cell=k[0], window_start_us=k[1], window_end_us=k[1] + self.tile, count=c,
                              avg_speed=(None if n_sp == 0 else s_sp / n_sp), avg_lon=s_lo / c, avg_lat=s_la / c))

        # ---- eviction after emission (current batch's watermark) ----
        evict_end = self.wm_cur * 1000
        for k in [k for k in self.state if k[1] + self.tile <= evict_end]:
            del self.state[k]

        # ---- watermark for the next batch ----
        batch_max = None
        if valid.any():
            t = ts[valid]
            ms = np.where(t >= 0, t // 1000, -((-t) // 1000))
            batch_max = int(ms.max())
        nxt = self.wm_cur
        if batch_max is not None:
            nxt = max(nxt, batch_max - self.delay)
        used_wm = self.wm_cur
        self.wm_prev, self.wm_cur = self.wm_cur, nxt

        # ---- latest per vehicle ----
        vidx = np.nonzero(valid)[0]
        latest = np.zeros(0, np.int64)
        if vidx.size:
            vk = vkey[vidx]
            tv = ts[vidx]
            order = np.lexsort((tv, vk))
            vk_s, tv_s = vk[order], tv[order]
            last = np.r_[vk_s[1:] != vk_s[:-1], True]
            grp = np.cumsum(np.r_[True, vk_s[1:] != vk_s[:-1]]) - 1
            gmax = tv_s[last]
            win = tv_s == gmax[grp]
            latest = np.sort(vidx[order[win]])

        return dict(tiles=tiles, latest_rows=latest, n_valid=int(valid.sum()), n_late=int(late.sum()),
                    n_state=len(self.state), batch_max_event_ms=(INT64_MIN if batch_max is None else batch_max),
                    watermark_ms=used_wm, late_watermark_ms=late_wm)
