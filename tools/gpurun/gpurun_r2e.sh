# Full GPU test suite + smoke on the default build, the PCIe-inclusive and foreach_batch_func end-to-end rates,
# then a bench A/B of abl/ builds (VARIANTS)
set -o pipefail
O=gpurun_out/${TAG:-r2e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python3 tools/e2e_bench.py --steps 3 > $O/e2e.log 2>&1 && \
timeout -k 10 300 python3 tools/e2e_bench.py --foreach --events ${FOREACH_EVENTS:-5000000} --steps 2 > $O/e2e_foreach.log 2>&1 || exit $?
for v in $VARIANTS; do
  MOBHEAT_LIB=abl/libmobheat_$v.so timeout -k 10 200 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit $?
done
echo "done rc=0"
