# Round 4: where the merge's and the ingest's wave cycles go (SQ quad-cycle counters: parked in s_waitcnt / barriers,
# issue stalls, active) and their LDS traffic, one PMC pass over both bench legs.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4pmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -d $O/pmc_wait -o run --output-format csv -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/pmc_wait.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
