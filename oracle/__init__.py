"""ORACLE -- CPU restatement of the reference's hot path, used ONLY as the checker by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing under real-time-mobility-heatmap_amd/ imports it.

h3_oracle.c / h3_oracle.py : H3 v4 latLngToCell (+ cellToLatLng for table validation), x87 long double semantics
spark_oracle.py            : Spark 3.5.1 filter / window / watermark / update-mode aggregation / latest dedup
Parity status vs the real reference: UNPINNED (h3-py and pyspark are absent; the reference ships no fixtures).
Anchors: public H3 known-answer vectors, table self-consistency, exact round trips.
"""
