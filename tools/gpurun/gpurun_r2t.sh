# Full GPU test suite on the default build, then bench A/B of abl/ builds (VARIANTS, ROUNDS)
set -o pipefail
O=gpurun_out/${TAG:-r2t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit $?
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-head}; do
    MOBHEAT_LIB=abl/libmobheat_$v.so timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_${v}_$r.log 2>&1 || exit $?
  done
done
echo "done rc=0"
