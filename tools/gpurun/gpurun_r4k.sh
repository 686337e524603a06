# Round 4: bench A/B of library variants interleaved (V0 = the product library; $MVARIANTS, two rounds), then GPU
# tests ($TESTS).  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4k}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for v in ${MVARIANTS:-V0 V4 V5}; do
  L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so
  [ "$v" = V0 ] && L=real-time-mobility-heatmap_amd/csrc/libmobheat.so
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_${v}_$r.log 2>&1 || exit 1
done
done
if [ -n "$TESTS" ]; then timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
