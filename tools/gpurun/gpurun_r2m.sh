# Merge ablation (bench per-stage times, builds under abl/) + LDS/SQ counters of the C3 shard's kernels
set -o pipefail
O=gpurun_out/${TAG:-r2m}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in ${VARIANTS:-head noslot norows noboth}; do
    MOBHEAT_LIB=abl/libmobheat_$v.so timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-state-leg > $O/bench_${v}_$r.log 2>&1 || exit $?
  done
done
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES -d $O/pmc_c3 -o run --output-format csv -- python3 tools/scale_check.py --config c3 > $O/pmc_c3.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
