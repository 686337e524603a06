// mobheat: MI355X-native per-micro-batch hot path of the reference's streaming job (heatmap_stream.py).
//
// One translation unit (the device code shares __constant__ tables and inlines across stages); its parts, in
// dependency order:
//   dev_common.h    wave primitives, per-window state-table lookups, census sinks, the batch's window registry
//   k_partition.h   radix partition into (window, region) bins / owner ranks (k_ev_hist, k_ev_scatter_rec, k_rp_*)
//   k_table.h       table mode for low-cardinality batches (k_agg, k_bin_reduce)
//   k_merge.h       census, growth dump, the region-owned merge into the update-mode state (k_merge_owned), rows
//   k_dedup.h       latest position per (provider, vehicleId) (k_dedup_*), ordered compaction
//   k_ingest.h      the per-event pass (k_ingest: filter + latLngToCell + window + late test + dedup max + event key)
//   k_json.h        Kafka values -> columns, string dictionaries
//   k_stage.h       multi-GPU exchange helpers
//   host_ctx.h      the context, allocation, per-window tables, launchers;  host_batch.h: the batch phases
//   api_*.h         the C ABI of include/mobheat.h (batch, UDF/read side, stage API, checkpoint, sink, JSON, self-tests)
//
// Pipeline per batch (one HIP stream per context; every arithmetic step runs on the GPU):
//   k_ingest      filter (heatmap_stream.py:96-104) + H3 latLngToCell UDF (:65-75,105) + tumbling window (:115) +
//                 late-row test against the watermark (:107) + batch max event time + per-vkey max ts for the dedup
//                 (:200-203) + one 8-B event key per row (cell, window slot) + the census of rows per window
//   direct path   k_ev_hist / k_ev_scatter_rec: 32-B event records into (window, region) bins; k_merge_owned: one
//                 workgroup per bin merges them into the persistent per-window state tables (update mode, :243;
//                 Spark's StateStoreRestore/Save) and writes each touched key's cumulative row (:124-132)
//   table mode    k_agg + k_bin_reduce aggregate in LDS first (one partial per key), then partition + merge
//   k_fill_gaps   the per-bin row segments -> dense update-mode rows (in place)
//   eviction      (watermark, :107) releases a window's whole table; k_dump_gen + a rehash merge grow one
//   k_dedup_flag  latest position per (provider, vehicleId): rows whose ts equals the max (:204-207)
//   [multi-GPU: records grouped by owner rank, exchanged by the caller with RCCL all-to-all (api_stage.h)]
//
// Semantics follow SURVEY.md App. A (Spark 3.5.1): see DESIGN.md for the rules and their provenance.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <ctime>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/mobheat.h"
#include "kernels.h"
#include "bson_docs.h"
#include "json_decode.h"
#include "h3_boundary.h"
#include <chrono>
#include <mutex>

#define H3T_CONST static const
#include "h3_tables.inc"

using namespace hm;

__constant__ H3Tables c_tab;
// glibc's sincos/acos/atan2/tan tables for the exact path (glibc_libm.h); c_tab.glm points here
__device__ glm::Tables g_glm = {GLM_TABLE_INIT};   // (not const: a const namespace-scope symbol has internal linkage, which hipGetSymbolAddress cannot resolve)

#include "h3_tables_host.h"
static H3Tables make_tables() { return hm_make_tables(); }
// c_tab of the current device, its glibc table pointer aimed at the device copy
static hipError_t upload_tables() {
    H3Tables T = make_tables();
    void *g = nullptr;
    hipError_t e = hipGetSymbolAddress(&g, HIP_SYMBOL(g_glm));
    if (e != hipSuccess) return e;
    T.glm = (const glm::Tables *)g;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &T, sizeof(T));
}

#include "dev_common.h"
#include "k_partition.h"
#include "k_table.h"
#include "k_merge.h"
#include "k_dedup.h"
#include "k_ingest.h"
#include "k_json.h"
#include "k_stage.h"
#include "host_ctx.h"
#include "host_batch.h"
#include "host_pipe.h"

extern "C" {

#include "api_batch.h"
#include "api_udf.h"
#include "api_stage.h"
#include "api_state.h"
#include "api_sink.h"
#include "api_json.h"
#include "api_selftest.h"

}  // extern "C"
