# SQ counters of the direct path's partition and merge kernels on the bench workload (one bench run per pass)
set -o pipefail
O=gpurun_out/${TAG:-msq}
mkdir -p $O
export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-state-leg"
R='k_merge_owned|k_ev_scatter|k_ev_hist|k_ingest'
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1 -o run --output-format csv -- $P > $O/sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM -d $O/sq2 -o run --output-format csv -- $P > $O/sq2.log 2>&1 && \
python3 tools/pmc_summary.py $O/sq1 $O/sq2 > $O/summary.txt 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
