# GPU tests (TESTS, default build), then bench.py (with its state-read leg) for the default build and each variant
# in $VARIANTS (real-time-mobility-heatmap_amd/csrc/variants/libmobheat_<v>.so)
set -o pipefail
O=gpurun_out/${TAG:-var}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { echo "tests failed"; exit 1; }
fi
for v in base $VARIANTS; do
  if [ $v = base ]; then L=""; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_$v.log 2>&1 || exit $?
done
echo "done rc=0"
