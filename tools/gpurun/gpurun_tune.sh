# GPU parity tests on the default build, then bench.py on each tuning variant of libmobheat (csrc/variants/).
set -o pipefail
O=gpurun_out/${TAG:-tune}
mkdir -p $O
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
for v in ${VARIANTS:-}; do
  if [ "$v" = default ]; then L=; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
  MOBHEAT_LIB=$L timeout -k 10 240 python3 bench.py --steps ${STEPS:-4} --warmup ${WARMUP:-3} --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; exit 1; }
done
[ -n "$SKIP_PROF" ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
