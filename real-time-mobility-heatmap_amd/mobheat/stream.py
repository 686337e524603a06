"""Host-side mirror of the reference job's batch writer (reference heatmap_stream.py).

Keeps the reference's interface for this path:
  * module-level configuration from the same environment variables (heatmap_stream.py:21-37):
    MONGO_URI, MONGO_DB, CITY, H3_RES, TILE_MINUTES, TTL_MINUTES
  * ``foreach_batch_func(df, epoch_id)`` with the same signature (:150), called once per micro-batch, in order;
  * the MongoDB ``tiles`` and ``positions_latest`` documents built exactly as :164-188 and :211-228, written
    with ``UpdateOne(..., upsert=True)`` in unordered bulks of 1000 (:191-196, :230-235), tiles first;
  * a MongoClient opened and closed per batch (:156, :237); any exception propagates and fails the batch.

What changes underneath: ``df`` carries the raw events of the micro-batch (columns provider,
vehicleId, lat, lon, speedKmh and eventTs -- or the raw ISO ``ts`` string, parsed like to_timestamp, :92) instead
of the union of Spark's pre-aggregated tiles and the latest_raw projection (:136-146).  The sanity filter,
the to_h3 UDF, the watermark, the window aggregation with its persistent state and the in-batch dedup all run
on the GPU inside ``HeatmapEngine.process_batch`` (libmobheat.so).  There is no CPU fallback.
"""
import datetime
import os
from datetime import timedelta

import numpy as np

from .engine import HeatmapEngine

# ------------------ Configuration via environment (reference heatmap_stream.py:21-37) ------------------
MONGO_URI = os.getenv("MONGO_URI", "mongodb://127.0.0.1:27017")
MONGO_DB = os.getenv("MONGO_DB", "mobility")
CITY = os.getenv("CITY", "ath")
H3_RES = int(os.getenv("H3_RES", "8"))
TILE_MIN = int(os.getenv("TILE_MINUTES", "5"))
TTL_MIN = int(os.getenv("TTL_MINUTES", "45"))
WATERMARK_DELAY_MS = 10 * 60 * 1000          # withWatermark("eventTs", "10 minutes"), :107
BULK_CHUNK = 1000                              # :191, :230
DEVICE = int(os.getenv("MOBHEAT_DEVICE", os.getenv("LOCAL_RANK", "0")))
# Spark keeps the aggregation state under checkpointLocation, default /tmp/heatmap-checkpoint (:37, :244), and always
# restores it from there; the GPU state is checkpointed beside it (CHECKPOINT_DIR/mobheat-state) after each committed
# batch, like Spark's HDFS state store: a delta file per batch (the keys the batch touched) and a full snapshot every
# STATE_FULL_EVERY batches (spark.sql.streaming.stateStore.minDeltasForSnapshot = 10).  MOBHEAT_STATE_CHECKPOINT=0
# turns it off.
CHECKPOINT_DIR = os.getenv("CHECKPOINT", "/tmp/heatmap-checkpoint")
# MOBHEAT_GPUS=N > 1: the batch is sharded over N GPUs of this node (mobheat.sharded: this process runs rank 0, N-1
# spawned workers the others; torch.distributed over RCCL, or MOBHEAT_DIST_BACKEND=gloo to rehearse on one GPU)
N_GPUS = int(os.getenv("MOBHEAT_GPUS", "1"))
DIST_BACKEND = os.getenv("MOBHEAT_DIST_BACKEND", "nccl")
# MOBHEAT_SHARDED=1: the sharded writer even at one GPU (a process group of one rank over RCCL: the N>1 code path on a
# one-GPU machine)
FORCE_SHARDED = os.getenv("MOBHEAT_SHARDED", "0") == "1"
STATE_CHECKPOINT = os.getenv("MOBHEAT_STATE_CHECKPOINT", "1") == "1"
STATE_FULL_EVERY = int(os.getenv("MOBHEAT_STATE_FULL_EVERY", "10"))
# The engine's window tables are carved from a zeroed reservation made at its creation (hm_config.state_arena_bytes)
# before any allocation inside a batch: "auto" sizes it from the first batch the process sees (ARENA_BYTES_PER_ROW per
# row, at most a quarter of the device), a number of bytes pins it, 0 turns it off.  (A window table's first
# hipMalloc inside a batch took seconds on some boxes)
STATE_ARENA = os.getenv("MOBHEAT_STATE_ARENA_BYTES", "auto")
ARENA_BYTES_PER_ROW = 16 * 65   # ~8 live or pooled window tables of 2 x rows 65-B slots

LAST_TIMINGS = {}   # host-side phases (ms) of the last foreach_batch_func call: columns, process, checkpoint, sink ...

_ENGINE = None
_LAST_EPOCH = None   # the last epoch committed (merged and written) from _ENGINE's state
_PENDING = None      # (epoch, result, dictionaries): a batch merged into _ENGINE's state whose writes did not complete
_LINEAGE = None      # the checkpoint chain _ENGINE's state continues (mobheat.checkpoint)


def _state_dir():
    return os.path.join(CHECKPOINT_DIR, "mobheat-state")


def _store(rank=0, world=1):
    from .checkpoint import StateCheckpoints
    return StateCheckpoints(_state_dir(), rank, world)


def _checkpoints():
    """[(epoch, kind, path)] of this stream's (rank 0 of 1) saved states, oldest first; kind "full" or "delta"."""
    return [(e.epoch, e.kind, e.path) for e in _store().scan() if e.rank == 0 and e.world == 1]


def restore_state(eng, epoch_id):
    """Load the state after the newest checkpointed epoch older than `epoch_id` into a fresh engine: the newest epoch
    at which an unbroken chain (snapshot + deltas, one lineage) ends for every rank of the world that wrote it
    (mobheat.checkpoint; a multi-GPU stream's chains are merged: one GPU owns every key).  Returns that epoch or None
    (a fresh lineage then starts)."""
    global _LINEAGE
    from .checkpoint import new_lineage
    st = _store()
    pt = st.restore_point(int(epoch_id))
    if pt is None:
        _LINEAGE = new_lineage()
        return None
    info, recs = st.load(pt)
    eng.import_state(info, recs)
    _LINEAGE = pt.lineage
    return pt.epoch


def _arena_bytes(n_rows):
    if STATE_ARENA != "auto":
        return int(STATE_ARENA)
    if not n_rows or n_rows < 100_000:
        return 0
    from . import _lib
    import ctypes
    free, total = ctypes.c_int64(), ctypes.c_int64()
    if _lib.load().hm_device_memory(DEVICE, ctypes.byref(free), ctypes.byref(total)) != 0:
        return 0
    return int(min(ARENA_BYTES_PER_ROW * int(n_rows), total.value // 4, free.value // 2))


def get_engine(epoch_id=None, n_rows=None):
    """The process's engine; a new one resumes from the newest state checkpoint older than `epoch_id` (Spark
    re-runs the first uncommitted epoch on the state of the one before it) and, created for a batch of `n_rows`
    rows, reserves its state arena and per-batch buffers for batches of that size."""
    global _ENGINE, _LAST_EPOCH, _LINEAGE
    if _ENGINE is not None and epoch_id is not None and _LAST_EPOCH is not None and int(epoch_id) <= _LAST_EPOCH:
        # Spark re-runs an epoch this engine already merged (the query restarted in this process): rebuild the state
        # of the epoch before it instead of merging the batch a second time
        reset_engine()
    if _ENGINE is None:
        from .checkpoint import new_lineage
        eng = HeatmapEngine(h3_res=H3_RES, tile_minutes=TILE_MIN, watermark_delay_ms=WATERMARK_DELAY_MS,
                            device=DEVICE, state_arena_bytes=_arena_bytes(n_rows),
                            batch_capacity_hint=int(n_rows) if n_rows and n_rows >= 100_000 else 0)
        if STATE_CHECKPOINT and epoch_id is not None:
            restore_state(eng, epoch_id)
        else:
            _LINEAGE = new_lineage()
        _ENGINE = eng
    return _ENGINE


def save_state_checkpoint(epoch_id):
    """Checkpoint the engine's state after epoch `epoch_id` into its chain (mobheat.checkpoint): a full snapshot when
    the chain has none or STATE_FULL_EVERY deltas followed the newest one, else the batch's delta; files of epochs >=
    epoch_id (an abandoned lineage) are deleted first, and the chain keeps its newest two snapshots."""
    return checkpoint_begin(epoch_id).result()


_IO = None


def checkpoint_begin(epoch_id):
    """save_state_checkpoint in two halves: the export from the GPU now (before the next batch changes the state), the
    file write on a background thread -- foreach_batch_func overlaps it with the sink's writes and waits for it before
    returning.  (Written before the writes succeed is safe: a restart re-runs an uncommitted epoch E on the newest
    chain ending BEFORE E, and a replay of E in this process rewrites E's file.)  Returns a Future of the kind."""
    global _IO
    if _IO is None:
        from concurrent.futures import ThreadPoolExecutor
        _IO = ThreadPoolExecutor(1, thread_name_prefix="mobheat-checkpoint")
    st, lineage = _store(), _LINEAGE
    job = st.prepare(epoch_id, get_engine(), lineage, STATE_FULL_EVERY)

    def write():
        kind = st.write(job)
        st.prune_other_worlds(lineage)
        return kind
    fut = _IO.submit(write)
    fut.job = job
    return fut


def reset_engine():
    """Drop the persistent state (a new streaming query, or a batch that failed after its merge began)."""
    global _ENGINE, _LAST_EPOCH, _PENDING
    if _ENGINE is not None:
        _ENGINE.close()
    _ENGINE = None
    _LAST_EPOCH = None
    _PENDING = None
    if _SHARDED is not None:
        _SHARDED.reset()


_SHARDED = None   # mobheat.sharded.ShardedStream when N_GPUS > 1 (or FORCE_SHARDED)
SHARDED_EXTRA = {}   # more ShardedStream config (the CPU tests: {"cpu": True, "runner": "module:Class"})


def get_sharded():
    """The process's sharded writer (N_GPUS ranks; started at the first batch)."""
    global _SHARDED
    if _SHARDED is None:
        from .sharded import ShardedStream
        _SHARDED = ShardedStream(N_GPUS, dict(h3_res=H3_RES, tile_minutes=TILE_MIN, delay_ms=WATERMARK_DELAY_MS,
                                              city=CITY, ttl_min=TTL_MIN, checkpoint_dir=CHECKPOINT_DIR,
                                              checkpoint=STATE_CHECKPOINT, full_every=STATE_FULL_EVERY,
                                              backend=DIST_BACKEND, **SHARDED_EXTRA))
    return _SHARDED


def close_sharded():
    """Stop the sharded writer's workers and its process group (a new query, or the end of the process)."""
    global _SHARDED, _LAST_EPOCH, _PENDING
    if _SHARDED is not None:
        _SHARDED.close()
    _SHARDED = None
    _LAST_EPOCH = None
    _PENDING = None


# ------------------ sinks ------------------
class MongoSink:
    """Per-batch connection, like the reference's MongoClient (:156-157, :237).  A plain ``mongodb://host:port`` URI
    (the reference's default) is written through ``wire.WireMongoSink``: each command's statements leave as one slice
    of the GPU-encoded buffer.  Any other URI (credentials, TLS, replica sets, options) goes through pymongo."""

    def __init__(self, uri=None, db=None):
        from . import wire
        uri = uri or MONGO_URI
        self._dbname = db or MONGO_DB
        self._wire = None
        self._client = None
        plain = wire.plain_uri(uri) if wire.wire_enabled() else None
        if plain is not None:
            self._wire = wire.WireMongoSink(plain[0], plain[1], self._dbname)
        else:
            from pymongo import MongoClient
            self._client = MongoClient(uri)
            self._db = self._client[self._dbname]

    def _pymongo_db(self):
        if getattr(self, "_db", None) is None:   # (the wire path writes the encoded statements; pymongo the rest)
            from pymongo import MongoClient
            self._client = MongoClient(f"mongodb://{self._wire.host}:{self._wire.port}")
            self._db = self._client[self._dbname]
        return self._db

    def bulk_write(self, collection, ops):
        self._pymongo_db()[collection].bulk_write(ops, ordered=False)

    def update_statements(self, collection, buf, offs, landed=None):
        """Pre-encoded update statements (bytes buf, offsets[n+1]) in unordered commands of <= BULK_CHUNK; landed as
        wire.WireSink.update_statements (the wire path sends each command as its bytes land)."""
        if self._wire is not None:
            self._wire.update_statements(collection, buf, offs, landed)
            return
        if landed is not None:
            landed(int(offs[-1]) if len(offs) else 0)
        from bson.raw_bson import RawBSONDocument
        from . import wire
        o = np.asarray(offs, dtype=np.int64)
        # pymongo checks a command against maxBsonObjectSize + 16 KiB: split by bytes as well as by count
        for i, j in wire.chunks(o, 16 * 1024 * 1024 - 64 * 1024, BULK_CHUNK):
            self.update_raw(collection, [RawBSONDocument(buf[o[k]:o[k + 1]].tobytes()) for k in range(i, j)])

    def update_raw(self, collection, statements):
        """One unordered `update` command of pre-encoded statements (RawBSONDocument): the command pymongo's
        bulk_write(ordered=False) sends for the same UpdateOne ops, with the collection's write concern; write
        errors raise BulkWriteError like it."""
        from bson.son import SON
        from . import wire
        cmd = SON([("update", collection), ("updates", statements), ("ordered", False)])
        db = self._pymongo_db()
        try:
            wc = db[collection].write_concern.document
        except (TypeError, AttributeError, KeyError):
            wc = None
        if wc:
            cmd["writeConcern"] = wc
        wire.raise_write_errors(db.command(cmd))

    def close(self):
        if self._wire is not None:
            self._wire.close()
        if self._client is not None:
            self._client.close()


SINK_FACTORY = MongoSink   # tests replace this with an in-memory capture sink


# ------------------ batch columns ------------------
def _pandas_to_arrow(pdf, pre=None):
    import pandas as pd
    """A pandas frame as Arrow WITHOUT pandas' NaN -> null mapping on float columns: a NaN speedKmh (Spark's JSON reader
    accepts NaN tokens, SURVEY App. A.2) must stay NaN so that avg(speedKmh) is NaN (App. A.4), while a missing value
    (None in an object column, pd.NA in a nullable column) is null.  pre: columns already converted (device_columns'
    _strcols arrays), taken as they are, in the frame's column order -- no copy of the frame without them."""
    import pyarrow as pa
    cols = {}
    for name in pdf.columns:
        if pre and name in pre:
            cols[str(name)] = pre[name]
            continue
        c = pdf[name]
        if isinstance(c.dtype, pd.api.extensions.ExtensionDtype) and hasattr(c.array, "__arrow_array__"):
            # nullable extension arrays (Float64, Int64, string, ...): their mask is the null set -- pd.NA -> null, a
            # NaN in a Float64 column stays NaN (pyarrow's __arrow_array__ protocol keeps the two apart)
            cols[str(name)] = pa.array(c.array)
        elif c.dtype.kind == "f":          # numpy float: NaN is a value, there is no null
            cols[str(name)] = pa.array(c.to_numpy(), from_pandas=False)
        elif c.dtype == np.dtype("datetime64[ns]"):   # the values buffer as it is (no copy), NaT -> null
            v = np.ascontiguousarray(c.to_numpy())
            nat = v.view(np.int64) == np.iinfo(np.int64).min
            k = int(np.count_nonzero(nat))
            bits = pa.py_buffer(np.packbits(~nat, bitorder="little")) if k else None
            cols[str(name)] = pa.Array.from_buffers(pa.timestamp("ns"), v.size, [bits, pa.py_buffer(v)], null_count=k)
        elif c.dtype == object:            # None -> null, float('nan') -> NaN
            try:
                cols[str(name)] = pa.array(c.to_numpy(), from_pandas=False)
            except (pa.ArrowInvalid, pa.ArrowTypeError):
                cols[str(name)] = pa.array(c, from_pandas=True)
        else:                              # nullable extension dtypes, datetimes (NaT -> null), ints, strings
            cols[str(name)] = pa.array(c, from_pandas=True)
    return pa.table(cols) if cols else pa.table({})


def _is_pandas(df):
    try:
        import pandas as pd
    except ImportError:
        return False
    return isinstance(df, pd.DataFrame)


def _to_arrow(df):
    import pyarrow as pa
    if isinstance(df, pa.Table):
        return df
    if isinstance(df, pa.RecordBatch):
        return pa.Table.from_batches([df])
    try:
        import pandas as pd
        if isinstance(df, pd.DataFrame):
            return _pandas_to_arrow(df)
    except ImportError:
        pass
    if hasattr(df, "toArrow"):           # pyspark >= 4: Arrow batches with Spark's nulls
        return df.toArrow()
    if hasattr(df, "_collect_as_arrow"):  # pyspark 3.x: the same batches (toPandas would turn null doubles into NaN)
        batches = df._collect_as_arrow()
        if batches:
            return pa.Table.from_batches(batches)
        return _pandas_to_arrow(df.limit(0).toPandas())
    if hasattr(df, "toPandas"):
        return _pandas_to_arrow(df.toPandas())
    raise TypeError(f"unsupported batch type {type(df)!r}")


def _event_ts_us(t):
    """eventTs as int64 microseconds (Spark TimestampType) + validity mask."""
    import pyarrow as pa
    import pyarrow.compute as pc
    if "eventTs" in t.column_names:
        col = t.column("eventTs")
        if pa.types.is_timestamp(col.type):
            us = pc.cast(col, pa.timestamp("us", tz=col.type.tz), safe=False)
            arr = us.combine_chunks() if isinstance(us, pa.ChunkedArray) else us
            valid = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False), dtype=bool)
            vals = np.asarray(pc.fill_null(arr.cast(pa.int64()), 0).to_numpy(zero_copy_only=False), dtype=np.int64)
            return vals, valid
        col = col.combine_chunks() if isinstance(col, pa.ChunkedArray) else col
        valid = ~np.asarray(col.is_null().to_numpy(zero_copy_only=False), dtype=bool)
        vals = np.asarray(pc.fill_null(col.cast(pa.int64()), 0).to_numpy(zero_copy_only=False), dtype=np.int64)
        return vals, valid
    # raw ISO-8601 strings: to_timestamp(col("ts")) (reference :92); malformed -> null.  Strings with and without a
    # zone are parsed apart: in one mixed Series pandas applies an offset it saw to the naive strings, where
    # to_timestamp reads them in the session time zone (UTC, :45)
    import pandas as pd
    raw = t.column("ts").to_pandas()
    # (a zone only after a time component: the day of a date-only '2024-01-15' is no offset)
    zoned = raw.astype("string").str.strip().str.contains(r"[T ]\d{2}:\d{2}.*(?:Z|[+-]\d{2}(?::?\d{2})?)$",
                                                          regex=True).fillna(False).to_numpy(bool)
    vals = np.zeros(len(raw), np.int64)
    valid = np.zeros(len(raw), bool)
    for sel in (zoned, ~zoned):
        if sel.any():
            s = pd.to_datetime(raw[sel], utc=True, errors="coerce", format="ISO8601")
            ok = ~s.isna().to_numpy()
            valid[sel] = ok
            vals[sel] = np.where(ok, s.astype("int64", copy=False).to_numpy() // 1000, 0)
    return vals, valid


def kafka_values(t):
    """The Kafka `value` column of an Arrow table as (bytes uint8, offsets int64[n+1]); a null value (tombstone)
    is an empty value, which from_json makes an all-null row (heatmap_stream.py:88-91)."""
    import pyarrow as pa
    import pyarrow.compute as pc
    col = t.column("value")
    col = col.combine_chunks() if isinstance(col, pa.ChunkedArray) else col
    if pa.types.is_string(col.type) or pa.types.is_large_string(col.type):
        col = col.cast(pa.large_binary())
    elif not pa.types.is_large_binary(col.type):
        col = col.cast(pa.large_binary())
    if col.null_count:
        col = pc.fill_null(col, b"")
    n = len(col)
    offs = np.frombuffer(col.buffers()[1], dtype=np.int64, count=n + 1, offset=col.offset * 8)
    data = col.buffers()[2]
    raw = np.frombuffer(data, dtype=np.uint8) if data is not None else np.zeros(0, np.uint8)
    return raw, offs


def batch_columns(df):
    """Extract the SoA buffers the C ABI takes (hm_batch_in) from a micro-batch frame.  A frame that carries the
    raw Kafka `value` column (binary or string: the producer's JSON, mbta_to_kafka.py:66-74) is decoded on the GPU
    instead (hm_decode_json): then the result is {"kafka": (bytes, offsets), "n": n}."""
    import pandas as pd
    import pyarrow as pa
    import pyarrow.compute as pc
    # a pandas frame's string columns are factorised where they are (pandas' hash table over the Python strings), not
    # turned into Arrow strings first (1.6 of a 1e7-row batch's 3.1 s of columns)
    pstr = {}
    if _is_pandas(df) and "value" not in df.columns:
        pstr = {c: df[c] for c in ("provider", "vehicleId") if c in df.columns}
        df = df.drop(columns=list(pstr))
    t = _to_arrow(df)
    n = t.num_rows if t.num_columns or not pstr else len(next(iter(pstr.values())))
    if "value" in t.column_names:
        return {"kafka": kafka_values(t), "n": n}

    def f64(name):
        if name not in t.column_names:
            return np.full(n, np.nan), np.zeros(n, bool)
        c = t.column(name).combine_chunks() if t.num_rows else t.column(name)
        nulls = np.asarray(c.is_null().to_numpy(zero_copy_only=False), dtype=bool) if n else np.zeros(0, bool)
        vals = np.asarray(pc.fill_null(c.cast("double"), float("nan")).to_numpy(zero_copy_only=False),
                          dtype=np.float64) if n else np.zeros(0)
        return vals, ~nulls

    lat, _ = f64("lat")           # null lat/lon -> NaN: fails between(), like Spark (:101-102)
    lon, _ = f64("lon")
    speed, speed_valid = f64("speedKmh")
    ts_us, ts_valid = _event_ts_us(t)
    def codes(name):
        """(the column, int64 codes -- -1 for null --, the dictionary as an Arrow string array in first-appearance
        order): pandas' factorize for a pandas frame's column, Arrow's dictionary encoding otherwise (before: the
        strings went to Arrow, back to pandas and were factorised, 2.4 of a 1e7-row batch's 3.6 s of columns)"""
        if name in pstr:
            c, u = pd.factorize(pstr[name])
            return pstr[name], np.asarray(c, np.int64), pa.array(np.asarray(u, dtype=object), type=pa.string())
        col = t.column(name) if name in t.column_names else pa.nulls(n, pa.string())
        col = col.combine_chunks() if isinstance(col, pa.ChunkedArray) else col
        if pa.types.is_dictionary(col.type):
            col = col.dictionary_decode()
        if not (pa.types.is_string(col.type) or pa.types.is_large_string(col.type)):
            col = pc.cast(col, pa.string())
        enc = pc.dictionary_encode(col)
        return col, np.asarray(pc.fill_null(enc.indices, -1).to_numpy(zero_copy_only=False), np.int64), enc.dictionary

    prov, pc_codes, p_uni = codes("provider")
    vid, vc_codes, v_uni = codes("vehicleId")
    row_valid = (pc_codes >= 0) & (vc_codes >= 0) & ts_valid        # provider/vehicleId/eventTs non-null (:99-103)
    vkey = np.where(row_valid, pc_codes.astype(np.int64) * max(len(v_uni), 1) + vc_codes, 0).astype(np.uint64)
    return dict(n=n, lat=lat, lon=lon, ts_us=ts_us, speed=speed, speed_valid=speed_valid, vkey=vkey,
                row_valid=row_valid, provider=prov, vehicleId=vid, provider_uniques=p_uni, vehicle_uniques=v_uni)


class ArrowColumns:
    """The micro-batch's columns as Arrow arrays (one chunk each) and the hm_arrow_in over their buffers (zero-copy):
    hm_arrow_columns copies them to the device, turns Arrow's nulls into the batch columns' conventions and factorises
    the provider / vehicleId strings there (engine.process_arrow).  The arrays are kept here: the struct points into
    them."""

    def __init__(self, t, n):
        import pyarrow as pa
        from ._lib import HmArrowIn
        self.n = n
        self.keep = []
        a = HmArrowIn(n=n)
        for field, name in (("lat", "lat"), ("lon", "lon"), ("speed", "speedKmh")):
            self._numeric(getattr(a, field), t, name, pa.float64())
        self._ts(a.ts_us, t)
        self._string(a.provider, t, "provider")
        self._string(a.vehicle, t, "vehicleId")
        self.struct = a

    @staticmethod
    def _chunk(t, name):
        import pyarrow as pa
        if name not in t.column_names:
            return None
        c = t.column(name)
        if isinstance(c, pa.ChunkedArray):   # (one chunk -- a converted pandas frame's: taken as it is, no copy)
            c = c.chunk(0) if c.num_chunks == 1 else c.combine_chunks()
        if pa.types.is_dictionary(c.type):
            c = c.dictionary_decode()
        return None if pa.types.is_null(c.type) or c.null_count == len(c) else c

    def _validity(self, col, arr):
        b = arr.buffers()[0]
        if b is not None and arr.null_count:
            col.validity, col.validity_offset = b.address, arr.offset
        self.keep.append(arr)

    def _numeric(self, col, t, name, typ):
        import pyarrow.compute as pc
        arr = self._chunk(t, name)
        if arr is None:
            return
        if arr.type != typ:
            arr = pc.cast(arr, typ)
        col.values = arr.buffers()[1].address + arr.offset * 8
        self._validity(col, arr)

    def _ts(self, col, t):
        import pyarrow as pa
        import pyarrow.compute as pc
        arr = self._chunk(t, "eventTs") if "eventTs" in t.column_names else None
        if arr is not None and pa.types.is_timestamp(arr.type):
            if arr.type.unit == "ns":   # (pandas' datetime64[ns]: the device truncates to microseconds, no host cast)
                col.unit = 1
            elif arr.type.unit != "us":
                arr = pc.cast(arr, pa.timestamp("us", tz=arr.type.tz), safe=False)
        elif arr is not None or "eventTs" not in t.column_names:
            # raw ISO strings (to_timestamp, :92), or eventTs of another type: parsed / cast on the host
            vals, valid = _event_ts_us(t)
            arr = pa.array(vals, mask=~valid) if not valid.all() else pa.array(vals)
        else:
            return
        col.values = arr.buffers()[1].address + arr.offset * 8
        self._validity(col, arr)

    def _string(self, col, t, name):
        import pyarrow as pa
        import pyarrow.compute as pc
        arr = self._chunk(t, name)
        if arr is None:
            return
        if not (pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type)):
            arr = pc.cast(arr, pa.string())
        w = 8 if pa.types.is_large_string(arr.type) else 4
        bufs = arr.buffers()
        col.values = bufs[1].address + arr.offset * w
        col.data = bufs[2].address if bufs[2] is not None else None
        col.offset_bytes = w
        self._validity(col, arr)


def _object_strings(values):
    """A pandas object column of Python str -> pa.large_string array (None / NaN / pd.NA -> null): the compact-ASCII
    strings measured and copied by _strcols' threads without the GIL, any other str encoded here.  None when the column
    holds a non-string value (the caller converts it another way)."""
    import pyarrow as pa
    from . import _strcols
    a = np.ascontiguousarray(values, dtype=object)
    n = a.size
    threads = min(16, os.cpu_count() or 1)
    if n and hasattr(_strcols, "measure"):
        # the fused form: lengths + per-block totals, then offsets, bytes and validity bitmap in one threaded pass
        offs = np.empty(n + 1, np.int64)
        total, nulls, others, per = _strcols.measure(a.ctypes.data, n, offs.ctypes.data, threads)
        if not others:
            data = np.empty(max(total, 1), np.uint8)
            bitmap = np.empty((n + 7) // 8, np.uint8) if nulls else None
            _strcols.fill(a.ctypes.data, n, offs.ctypes.data, data.ctypes.data,
                          0 if bitmap is None else bitmap.ctypes.data, per, threads)
            return pa.Array.from_buffers(pa.large_string(), n, [None if bitmap is None else pa.py_buffer(bitmap),
                                         pa.py_buffer(offs), pa.py_buffer(data)], null_count=nulls)
        lens = offs[1:].copy()
    else:
        lens = np.empty(n, np.int64)
        if n:
            _strcols.lengths(a.ctypes.data, n, lens.ctypes.data, threads)
    enc = {}
    for i in np.nonzero(lens == -2)[0].tolist():
        v = a[i]
        if isinstance(v, str):
            enc[i] = v.encode("utf-8", "surrogatepass")
            lens[i] = len(enc[i])
        elif isinstance(v, float) and v != v or v is getattr(__import__("pandas"), "NA", None):
            lens[i] = -1
        else:
            return None
    valid = lens >= 0
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(np.maximum(lens, 0), out=offs[1:])
    data = np.empty(max(int(offs[-1]), 1), np.uint8)
    if n:
        _strcols.copy(a.ctypes.data, n, offs.ctypes.data, data.ctypes.data, threads)
    for i, b in enc.items():
        data[offs[i]:offs[i + 1]] = np.frombuffer(b, np.uint8)
    nulls = int(n - valid.sum())
    bitmap = pa.py_buffer(np.packbits(valid, bitorder="little")) if nulls else None
    return pa.Array.from_buffers(pa.large_string(), n, [bitmap, pa.py_buffer(offs), pa.py_buffer(data)], null_count=nulls)


def _object_floats(values):
    """A pandas object column of Python float / None (how a nullable double column often arrives) -> pa.float64 array
    (None / pd.NA -> null, NaN stays a value): _strcols' threads read the float objects without the GIL; ints and other
    numbers are converted here.  None when a value is not a number."""
    import pyarrow as pa
    from . import _strcols
    a = np.ascontiguousarray(values, dtype=object)
    n = a.size
    vals = np.empty(n, np.float64)
    kinds = np.empty(n, np.uint8)
    if n:
        _strcols.floats(a.ctypes.data, n, vals.ctypes.data, kinds.ctypes.data, min(16, os.cpu_count() or 1))
    na = getattr(__import__("pandas"), "NA", None)
    for i in np.nonzero(kinds == 2)[0].tolist():
        v = a[i]
        if v is na:
            kinds[i] = 0
        elif isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
            vals[i], kinds[i] = float(v), 1
        else:
            return None
    # kinds is 0 / 1 now: packed straight into Arrow's validity bitmap, the values buffer taken as it is
    nulls = n - int(np.count_nonzero(kinds))
    bitmap = pa.py_buffer(np.packbits(kinds, bitorder="little")) if nulls else None
    return pa.Array.from_buffers(pa.float64(), n, [bitmap, pa.py_buffer(vals)], null_count=nulls)


def device_columns(df):
    """The frame's columns for the device path (hm_arrow_columns): {"arrow": ArrowColumns, "n": n}, or batch_columns'
    host columns when the frame is not columnar Arrow-convertible (MOBHEAT_COLUMNS=host pins the host path), or the raw
    Kafka values ({"kafka": ...})."""
    if os.getenv("MOBHEAT_COLUMNS", "device") == "host":
        return batch_columns(df)
    strs = {}
    if _is_pandas(df) and "value" not in df.columns:
        # the pandas frame's string columns straight to Arrow's layout (_strcols: threads, no GIL), the rest by pyarrow
        for c, conv in (("provider", _object_strings), ("vehicleId", _object_strings), ("lat", _object_floats),
                        ("lon", _object_floats), ("speedKmh", _object_floats)):
            if c in df.columns and df[c].dtype == object:
                try:
                    arr = conv(df[c].to_numpy())
                except ImportError:   # (the helper is not built: pyarrow converts the column)
                    arr = None
                if arr is not None:
                    strs[c] = arr
    try:
        t = _pandas_to_arrow(df, strs) if strs else _to_arrow(df)
    except Exception:
        return batch_columns(df)
    if "value" in t.column_names:
        return {"kafka": kafka_values(t), "n": t.num_rows}
    import pyarrow as pa
    try:
        return {"arrow": ArrowColumns(t, t.num_rows), "n": t.num_rows}
    except (pa.ArrowException, TypeError, ValueError):   # (a column Arrow cannot cast: the host path decides)
        return batch_columns(t)


# ------------------ document builders (reference :164-188 and :211-228) ------------------
def _spark_datetime(us):
    # pyspark TimestampType.fromInternal: naive local time; the reference's '...Z' ids assume a UTC driver
    us = int(us)
    return datetime.datetime.fromtimestamp(us // 1000000).replace(microsecond=us % 1000000)


def tile_ops(tiles, city=None, h3_res=None, ttl_min=None):
    from pymongo import UpdateOne
    city = CITY if city is None else city
    h3_res = H3_RES if h3_res is None else h3_res
    ttl_min = TTL_MIN if ttl_min is None else ttl_min
    ops = []
    for k in range(len(tiles)):
        windowStart = _spark_datetime(tiles.window_start_us[k])
        windowEnd = _spark_datetime(tiles.window_end_us[k])
        cellId = format(int(tiles.cell[k]), "x")                       # h3-py's str form of the UDF output
        count_val = int(int(tiles.count[k]) or 0)
        avg_speed = float((None if tiles.speed_null[k] else float(tiles.avg_speed[k])) or 0.0)
        avg_lat = float(float(tiles.avg_lat[k]) or 0.0)
        avg_lon = float(float(tiles.avg_lon[k]) or 0.0)
        _id = f"{city}|h3r{h3_res}|{cellId}|{windowStart.strftime('%Y-%m-%dT%H:%M:%SZ')}"
        staleAt = windowEnd + timedelta(minutes=ttl_min)
        doc = {
            "_id": _id,
            "city": city,
            "grid": f"h3r{h3_res}",
            "cellId": cellId,
            "windowStart": windowStart,
            "windowEnd": windowEnd,
            "count": count_val,
            "avgSpeedKmh": avg_speed,
            "centroid": {"type": "Point", "coordinates": [avg_lon, avg_lat]},
            "staleAt": staleAt,
        }
        ops.append(UpdateOne({"_id": _id}, {"$set": doc}, upsert=True))
    return ops


def position_ops(cols, rows):
    from pymongo import UpdateOne
    ops = []
    prov, vid = cols["provider"], cols["vehicleId"]
    for r in rows:
        r = int(r)
        provider = prov[r].as_py() if hasattr(prov, "to_pylist") else prov.iloc[r]   # (Arrow array or pandas Series)
        vehicleId = vid[r].as_py() if hasattr(vid, "to_pylist") else vid.iloc[r]
        ts = _spark_datetime(cols["ts_us"][r])
        lat = float(cols["lat"][r])
        lon = float(cols["lon"][r])
        filt = {"_id": f"{provider}|{vehicleId}"}
        ops.append(UpdateOne(
            {**filt, "$or": [{"ts": {"$exists": False}}, {"ts": {"$lt": ts}}]},
            {"$set": {
                "provider": provider,
                "vehicleId": vehicleId,
                "ts": ts,
                "loc": {"type": "Point", "coordinates": [lon, lat]},
            }},
            upsert=True,
        ))
    return ops


def _flush(sink, collection, ops):
    for i in range(0, len(ops), BULK_CHUNK):
        sink.bulk_write(collection, ops[i:i + BULK_CHUNK])


def _flush_statements(sink, collection, buf, offs, landed=None):
    """Pre-encoded update statements (hm_encode_tile_updates / hm_encode_position_updates) in unordered batches of
    BULK_CHUNK (:191-196, :230-235): the sink's update_statements when it has one (MongoSink), else one update_raw
    per chunk (capture sinks in the tests).  landed (a streamed encode's hm_statements_wait): handed to a sink whose
    update_statements takes it (it sends each command as its statements land), else waited for in full first."""
    if landed is not None and not _takes_landed(sink):
        landed(int(offs[-1]) if len(offs) else 0)
        landed = None
    if hasattr(sink, "update_statements"):
        if landed is not None:
            sink.update_statements(collection, buf, offs, landed=landed)
        else:
            sink.update_statements(collection, buf, offs)
        return
    from bson.raw_bson import RawBSONDocument
    o = offs.tolist()
    for i in range(0, len(o) - 1, BULK_CHUNK):
        j = min(i + BULK_CHUNK, len(o) - 1)
        sink.update_raw(collection, [RawBSONDocument(buf[o[k]:o[k + 1]].tobytes()) for k in range(i, j)])


def _encode(eng, name, *args):
    """eng.<name>_streamed(*args) -> (bytes, offsets, landed); an engine without the streamed form (the tests' stand-ins):
    eng.<name>(*args) with landed None."""
    f = getattr(eng, name + "_streamed", None)
    return f(*args) if f is not None else getattr(eng, name)(*args) + (None,)


def _takes_landed(sink):
    import inspect
    f = getattr(sink, "update_statements", None)
    try:
        return f is not None and "landed" in inspect.signature(f).parameters
    except (TypeError, ValueError):
        return False


# ------------------ the drop-in boundary ------------------
def _process(eng, epoch_id, cols):
    """Merge the batch into the engine's state; (result, the string dictionaries of its vkeys)."""
    # (the tile and latest rows stay on the device: the statements are encoded there from them)
    if "arrow" in cols:   # the frame's Arrow columns: nulls and the string dictionaries resolved on the GPU
        res, kb = eng.process_arrow(epoch_id, cols["arrow"].struct, rows_on_device=True)
        return res, (kb.providers, kb.vehicles)
    if "kafka" in cols:   # raw Kafka values: from_json + to_timestamp on the GPU (row f1; the records outside the
        # device decoder are decoded on the host and spliced in, engine.decode_json: one such record cannot stop the
        # stream, where Spark would replay the same offsets into the same failure)
        res, kb = eng.process_kafka(epoch_id, *cols["kafka"], rows_on_device=True)
        return res, (kb.providers, kb.vehicles)
    res = eng.process_batch(epoch_id, cols["lat"], cols["lon"], cols["ts_us"], cols["speed"], cols["speed_valid"],
                            cols["vkey"], cols["row_valid"], rows_on_device=True)
    return res, (cols["provider_uniques"], cols["vehicle_uniques"])


def _kafka_host_columns(eng, values, offsets):
    """Raw Kafka values decoded on `eng`'s GPU (hm_decode_json) and copied to host columns: the sharded writer hands
    every rank its share from host memory (the batch-wide string dictionaries keep the vkeys consistent across ranks)."""
    from . import _lib
    kb = eng.decode_json(values, offsets)
    b = kb.batch
    n = int(b.n)
    lib = _lib.load()

    def d2h(p, dt):
        a = np.empty(n, dt)
        if n:
            _lib.check(lib.hm_memcpy(a.ctypes.data, p, a.nbytes, 1), None, "hm_memcpy")
        return a
    cols = dict(n=n, lat=d2h(b.lat, np.float64), lon=d2h(b.lon, np.float64), ts_us=d2h(b.ts_us, np.int64),
                speed=d2h(b.speed, np.float64), speed_valid=d2h(b.speed_valid, np.uint8), vkey=d2h(b.vkey, np.uint64),
                row_valid=d2h(b.row_valid, np.uint8))
    return cols, (kb.providers, kb.vehicles)


def _foreach_sharded(df, epoch):
    """foreach_batch_func over N_GPUS ranks (mobheat.sharded): every rank merges the keys it owns and encodes the
    statements of its tiles and of its latest rows; they are written here, tiles first (:159-235), while every rank
    writes its checkpoint (a chain ending at an epoch whose writes failed is never restored from: the replay re-runs
    that epoch on the state before it).  Replay and failure semantics as the single-GPU path."""
    global _LAST_EPOCH, _PENDING
    from .engine import BatchResult
    sh = get_sharded()
    if _PENDING is not None and _PENDING[0] == epoch and sh.last is not None:
        per_rank = sh.last   # the replay of the epoch whose writes failed: every rank's state is in place
    else:
        if _PENDING is not None or (_LAST_EPOCH is not None and epoch <= _LAST_EPOCH):
            # another epoch while one is uncommitted, or a committed epoch re-run: every rank restores the state of
            # the epoch before it from the checkpoints
            sh.reset()
            _LAST_EPOCH = None
        _PENDING = None
        if sh.cfg.get("cpu"):   # (ranks without a GPU: the host columns)
            cols = batch_columns(df)
            if "kafka" in cols:
                cols, dicts = _kafka_host_columns(sh.rank0_engine(epoch), *cols["kafka"])
            else:
                dicts = (cols["provider_uniques"], cols["vehicle_uniques"])
            per_rank = sh.process(epoch, cols, dicts)
        else:
            # the columns built on rank 0's GPU -- the frame's Arrow buffers (hm_arrow_columns) or the raw Kafka values
            # (hm_decode_json) -- and every rank's slice moved device to device (ShardedStream.process_device)
            cols = device_columns(df)
            if "arrow" in cols:
                kb = sh.rank0_engine(epoch).arrow_columns(cols["arrow"].struct)
            elif "kafka" in cols:
                kb = sh.rank0_engine(epoch).decode_json(*cols["kafka"])
            else:
                kb = None
            if kb is not None:
                per_rank = sh.process_device(epoch, kb.batch, (kb.providers, kb.vehicles))
            else:
                per_rank = sh.process(epoch, cols, (cols["provider_uniques"], cols["vehicle_uniques"]))
        _PENDING = (epoch, per_rank, None)
    # every rank's state checkpoint, written while the statements go out (see checkpoint_begin)
    if STATE_CHECKPOINT:
        sh.commit_begin(epoch)
    sink = SINK_FACTORY()
    try:
        for _, tiles, _ in per_rank:
            _flush_statements(sink, "tiles", *tiles)
        for _, _, pos in per_rank:
            if pos is not None:
                _flush_statements(sink, "positions_latest", *pos)
    except BaseException as write_err:
        sink.close()
        if STATE_CHECKPOINT:
            try:   # (the checkpoints must be finished before a replay; their own failure must not hide the sink's)
                sh.commit_end()
            except Exception as ck_err:
                import warnings
                warnings.warn(f"mobheat: checkpoint of epoch {epoch} failed after its writes failed: {ck_err!r}")
        raise write_err
    sink.close()
    if STATE_CHECKPOINT:
        sh.commit_end()
    _PENDING = None
    _LAST_EPOCH = epoch
    st = [x[0] for x in per_rank]
    tot = lambda k: sum(int(x[k]) for x in st)   # noqa: E731
    return BatchResult(tiles=None, latest_rows=None, n_in=tot("n_in"), n_valid=tot("n_valid"), n_late=tot("n_late"),
                       n_state=tot("n_state"), batch_max_event_ms=int(st[0]["batch_max_event_ms"]),
                       watermark_ms=int(st[0]["watermark_ms"]), late_watermark_ms=int(st[0]["late_watermark_ms"]),
                       n_partials=tot("n_partials"), n_tiles=tot("n_tiles"), n_latest=tot("n_latest"))


def foreach_batch_func(df, epoch_id: int):
    """Runs on each micro-batch (reference heatmap_stream.py:150): tiles + latest positions -> MongoDB.

    Failures keep the reference's semantics (the exception fails the batch and Spark re-runs the epoch) without
    losing state: a batch that fails before its merge leaves the state untouched (hm_state_version); one that fails
    during the merge drops the state, which the retry rebuilds from the checkpoints; one whose writes fail keeps the
    merged state and, when Spark re-runs that epoch, writes the same documents again without merging twice."""
    global _LAST_EPOCH, _PENDING, LAST_TIMINGS
    import time
    epoch = int(epoch_id)
    if N_GPUS > 1 or FORCE_SHARDED:
        return _foreach_sharded(df, epoch)
    tm = {}
    clock = [time.perf_counter()]

    def lap(name):
        t = time.perf_counter()
        tm[name] = tm.get(name, 0.0) + 1e3 * (t - clock[0])
        clock[0] = t
    if _PENDING is not None and _PENDING[0] == epoch and _ENGINE is not None:
        res, dicts = _PENDING[1], _PENDING[2]   # the replay of the epoch whose writes failed: its state is in place
    else:
        if _PENDING is not None:   # another epoch while one is uncommitted: that merge never committed
            reset_engine()
        cols = device_columns(df)
        lap("columns")
        eng = get_engine(epoch, cols.get("n"))
        lap("engine")
        v0 = eng.state_version()
        try:
            res, dicts = _process(eng, epoch, cols)
        except BaseException:
            if _ENGINE is not None and _ENGINE.state_version() != v0:
                reset_engine()   # the merge began: the state may hold part of the batch
            raise
        lap("process")
        _PENDING = (epoch, res, dicts)
    eng = get_engine()
    # the batch's state checkpoint: exported now, its file written while the statements go out
    ckpt = checkpoint_begin(epoch) if STATE_CHECKPOINT else None
    lap("checkpoint_export")
    sink = SINK_FACTORY()
    try:
        # ---- 1) Upsert tiles (TTL via staleAt): the UpdateOne statements, BSON-encoded on the GPU ----
        # (streamed: the statements' bytes land in pieces while the sink sends the commands that have landed)
        buf, offs, landed = _encode(eng, "encode_tile_updates", CITY, TTL_MIN)
        lap("encode")
        _flush_statements(sink, "tiles", buf, offs, landed)
        lap("sink")
        # ---- 2) latest per (provider, vehicleId) within this micro-batch: statements encoded on the GPU ----
        if res.n_latest:
            # (local offsets of the rows' 900-s buckets)
            buf, offs, landed = _encode(eng, "encode_position_updates", *dicts)
            lap("encode")
            _flush_statements(sink, "positions_latest", buf, offs, landed)
            lap("sink")
    finally:
        sink.close()
        if ckpt is not None:   # (also when a write failed: a replay must not race the file)
            exc = ckpt.exception()
            lap("checkpoint_wait")
            tm.update(getattr(ckpt, "job", {}).get("timings", {}))
    if ckpt is not None and exc is not None:
        raise exc
    LAST_TIMINGS = tm
    _PENDING = None
    _LAST_EPOCH = epoch
    return res
