# Round 6: the pipelined batch -- its GPU parity tests, then a bench A/B of MOBHEAT_PIPELINE settings interleaved on one
# box ($PIPES, default "0 4 2 8"; 0 = unpipelined), $ROUNDS rounds
set -o pipefail
O=gpurun_out/${TAG:-r6b}
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_pipeline.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
for p in ${PIPES:-0 4 2 8}; do
  MOBHEAT_PIPELINE=$p timeout -k 10 300 python3 bench.py --steps ${STEPS:-8} --warmup 3 --no-cpu-baseline ${BENCHARGS:---no-state-leg} > $O/bench_p${p}_$r.log 2>&1 || exit 1
done
done
echo done
