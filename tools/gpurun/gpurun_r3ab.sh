# A/B of library variants (real-time-mobility-heatmap_amd/csrc/variants/libmobheat_<v>.so, "default" = the in-tree
# build) on one box: $ROUNDS rounds of the bench per variant, interleaved; then optional GPU tests ($TESTS) on the
# in-tree build and an optional SQ pass over k_ingest for each variant ($PMC=1).
set -o pipefail
O=gpurun_out/${TAG:-r3ab}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then L=; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
    MOBHEAT_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:---no-state-leg} > $O/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_${v}_$r.log; exit 1; }
    python3 -c "
import json,sys
for l in open('$O/bench_${v}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); k=d['roofline']['kernel_ms']; print('$v r$r', round(d['value']/1e9,3), 'e9/s', round(d['ms_per_step'],2), 'ms', k)
"
  done
done
if [ "${PMC:-0}" = 1 ]; then
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then L=; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
    MOBHEAT_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "${PMC_RE:-k_ingest}" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/pmc_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-state-leg > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  done
fi
echo "done"
