# Round 6: the wave-owned merge (k_merge_waves, MOBHEAT_MERGE_WAVES=1) -- parity tests with sub-bins forced, then a bench
# A/B on one box: V0 product defaults, S sub-bins forced (k_merge_owned), W sub-bins + k_merge_waves; both legs
set -o pipefail
O=gpurun_out/${TAG:-r6w}
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
MOBHEAT_MERGE_WAVES=1 MOBHEAT_SUBBINS=1 timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_pipeline.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V0_$r.log 2>&1 || exit 1
  MOBHEAT_SUBBINS=1 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_S_$r.log 2>&1 || exit 1
  MOBHEAT_SUBBINS=1 MOBHEAT_MERGE_WAVES=1 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_W_$r.log 2>&1 || exit 1
done
echo done
