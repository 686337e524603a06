# Round 5: an environment-switch A/B of the product library: the bench with $ENVA (default) and with $ENVB, interleaved,
# $ROUNDS rounds, then optional GPU tests ($TESTS).  $TAG names the output directory; $BENCHARGS extra bench flags.
set -o pipefail
O=gpurun_out/${TAG:-r5env}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  env $ENVA timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline $BENCHARGS > $O/bench_A_$r.log 2>&1 || exit 1
  env $ENVB timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline $BENCHARGS > $O/bench_B_$r.log 2>&1 || exit 1
done
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
fi
echo done
