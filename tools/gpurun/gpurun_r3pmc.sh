# Round 3: PMC passes (one rocprofv3 run per counter group) over the bench's partition and merge kernels, plus the
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE) of every kernel of the step.
set -o pipefail
O=gpurun_out/${TAG:-r3pmc}
mkdir -p $O
export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-state-leg"
R='k_merge_owned|k_ev_scatter_rec|k_ev_hist|k_ingest'
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/sq1 -o run --output-format csv -- $P > $O/sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM -d $O/sq2 -o run --output-format csv -- $P > $O/sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $P > $O/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $P > $O/write.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
