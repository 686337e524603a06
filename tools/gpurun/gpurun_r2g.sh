# merge grid A/B (MOBHEAT_MERGE_GRID) + SQ wait/LDS counters of the bench's kernels and of the C3 shard's kernels
set -o pipefail
O=gpurun_out/${TAG:-r2g}
mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS"
CASES="${CASES:-g0:MOBHEAT_MERGE_GRID=0 g512:MOBHEAT_MERGE_GRID=512 g1024:MOBHEAT_MERGE_GRID=1024}" bash tools/gpurun/gpurun_abenv.sh || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_bench -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-state-leg > $O/pmc_bench.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_c3 -o run --output-format csv -- python3 tools/scale_check.py --config c3 > $O/pmc_c3.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
