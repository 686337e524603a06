set -o pipefail
O=gpurun_out/h3bench
mkdir -p $O
export TMPDIR=/tmp
for v in base x87_plain trig_cheap face1 no_rot no_digits x87_plain_trig_cheap; do
  timeout -k 10 120 tools/h3bench/build/h3bench_$v 100000000 8 5 >> $O/times.jsonl || exit 1
done
timeout -k 10 120 tools/h3bench/build/h3bench_base 100000000 7 5 >> $O/times.jsonl && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES -d $O/pmc_base -o run --output-format csv -- tools/h3bench/build/h3bench_base 100000000 8 2 > $O/pmc.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
