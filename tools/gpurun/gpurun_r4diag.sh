# Round 4 diagnostics: the binning write patterns (tools/microbench/bin_scatter) and k_ingest's VALU instructions by
# phase (tools/diag/ingest_phases under one PMC pass).  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4diag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/bin_scatter > $O/bin_scatter.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/phases -o run --output-format csv -- ./tools/diag/ingest_phases > $O/phases.log 2>&1 && \
python3 tools/diag/ingest_phases.py $O/phases > $O/phases.txt 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
