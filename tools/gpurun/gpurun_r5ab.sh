# Round 5: bench A/B of library variants interleaved on one box (V0 = the product library; others
# csrc/variants/libmobheat_$v.so built by tools/variants/build.sh from tools/variants/$v.patch), $ROUNDS rounds; then
# optionally GPU tests ($TESTS) with the library $TESTLIB.  $TAG names the output directory; $BENCHARGS extra bench flags.
set -o pipefail
O=gpurun_out/${TAG:-r5ab}
mkdir -p $O
export TMPDIR=/tmp
# (a throwaway warm-up run: the first bench process on a fresh box runs up to ~20% slow)
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
for v in ${MVARIANTS:-V0}; do
  L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so
  [ "$v" = V0 ] && L=real-time-mobility-heatmap_amd/csrc/libmobheat.so
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps ${STEPS:-8} --warmup 3 --no-cpu-baseline ${BENCHARGS:---no-state-leg} > $O/bench_${v}_$r.log 2>&1 || exit 1
done
done
if [ -n "$TESTS" ]; then
  L=${TESTLIB:-real-time-mobility-heatmap_amd/csrc/libmobheat.so}
  MOBHEAT_LIB=$L timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
fi
echo "done"; exit 0
