# Round 6: k_ingest with ap7Quad read from global memory (tools/variants/ingest_quad_l1.patch):
# cells at every resolution against the oracle with the variant, SQ LDS counters of both builds, bench A/B
set -o pipefail
O=gpurun_out/${TAG:-r6q}
mkdir -p $O
export TMPDIR=/tmp
V=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_ingest_quad_l1.so
MOBHEAT_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "cell or res or modes" > $O/gpu_tests.log 2>&1 || exit 1
P="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-state-leg"
R='k_ingest'
for b in V0 Q; do
  if [ $b = Q ]; then export MOBHEAT_LIB=$V; else unset MOBHEAT_LIB; fi
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq_$b -o run --output-format csv -- $P > $O/sq_$b.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/sq_$b > $O/summary_$b.txt 2>&1 || exit 1
done
unset MOBHEAT_LIB
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_V0_$r.log 2>&1 || exit 1
  MOBHEAT_LIB=$V timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_Q_$r.log 2>&1 || exit 1
done
echo done
