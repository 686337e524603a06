# A/B of library builds under abl/ (VARIANTS, interleaved ROUNDS times) on both aggregation paths: bench.py's
# per-stage times (direct path) and the C3 shard (table mode); optional TESTS with the default build first.
set -o pipefail
O=gpurun_out/${TAG:-abboth}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf ${KEXPR:+-k "$KEXPR"} > $O/gpu_tests.log 2>&1 || exit $?
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    MOBHEAT_LIB=abl/libmobheat_$v.so timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:---no-state-leg} > $O/bench_${v}_$r.log 2>&1 || exit $?
    MOBHEAT_LIB=abl/libmobheat_$v.so timeout -k 10 300 python3 tools/scale_check.py --config c3 > $O/c3_${v}_$r.log 2>&1 || exit $?
  done
done
echo "done rc=0"
