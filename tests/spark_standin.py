"""Test helper (not a test module): stand-ins for the pyspark DataFrame that Spark hands foreach_batch_func
(reference heatmap_stream.py:150,245), exposing exactly the Arrow surface mobheat.stream reads -- pyspark 3.5's
``_collect_as_arrow()`` (one Arrow RecordBatch per result partition; ``limit(0).toPandas()`` for the schema of an empty
result) or pyspark 4's ``toArrow()`` -- over the types Spark gives the job's columns (heatmap_stream.py:51-61,88-93):
StringType -> ``string`` with nulls, DoubleType -> nullable ``double`` (NaN is a value, null is null), IntegerType ->
``int32``, TimestampType -> ``timestamp[us, tz=<session time zone>]`` ("UTC", :45).  pyspark is not installed here, so
the stand-in is built from the micro-batch's pandas twin.
"""
import numpy as np
import pandas as pd
import pyarrow as pa

SPARK_SCHEMA = pa.schema([("provider", pa.string()), ("vehicleId", pa.string()), ("lat", pa.float64()),
                          ("lon", pa.float64()), ("speedKmh", pa.float64()), ("bearing", pa.int32()),
                          ("accuracyM", pa.int32()), ("eventTs", pa.timestamp("us", tz="UTC"))])


def spark_table(pdf):
    """The Arrow table Spark would collect for the events of pandas frame `pdf` (its pd.NA / None are Spark nulls, its
    NaN speeds NaN values)."""
    n = len(pdf)

    def col(name, typ):
        if name not in pdf.columns:
            return pa.nulls(n, typ)
        c = pdf[name]
        if typ == pa.float64():
            if isinstance(c.dtype, pd.api.extensions.ExtensionDtype):
                return pa.array(c.array, type=typ)
            return pa.array(c.to_numpy(dtype=np.float64), type=typ, from_pandas=False)
        if typ == pa.string():
            return pa.array(c.astype(object).where(c.notna(), None).tolist(), type=typ)
        if pa.types.is_timestamp(typ):
            return pa.array(pd.to_datetime(c, utc=True), type=typ)
        return pa.array(c, type=typ)
    return pa.table({f.name: col(f.name, f.type) for f in SPARK_SCHEMA}, schema=SPARK_SCHEMA)


class Spark35Frame:
    """pyspark 3.5's DataFrame as foreach_batch_func sees it: _collect_as_arrow() -> [RecordBatch] (one per result
    partition, `parts` of them; an empty result gives none), limit(0).toPandas() for the schema."""

    def __init__(self, pdf, parts=3):
        self._t = spark_table(pdf)
        self._parts = parts

    def _collect_as_arrow(self):
        n = self._t.num_rows
        if n == 0:
            return []
        cuts = [n * k // self._parts for k in range(self._parts + 1)]
        return [b for lo, hi in zip(cuts, cuts[1:]) if hi > lo for b in self._t.slice(lo, hi - lo).to_batches()]

    def limit(self, k):
        other = Spark35Frame.__new__(Spark35Frame)
        other._t, other._parts = self._t.slice(0, k), self._parts
        return other

    def toPandas(self):   # (Spark's conversion: nulls of double columns become NaN -- why stream.py avoids it)
        return self._t.to_pandas()


class Spark4Frame:
    """pyspark 4's DataFrame: toArrow() -> pyarrow.Table (chunked by partition)."""

    def __init__(self, pdf, parts=3):
        self._f = Spark35Frame(pdf, parts)

    def toArrow(self):
        b = self._f._collect_as_arrow()
        return pa.Table.from_batches(b, schema=SPARK_SCHEMA) if b else SPARK_SCHEMA.empty_table()
