# Round 6: sub-bins predicted from the stream's event-time advance (retouch_next) + the merge variant predicted from
# the census, both under MOBHEAT_COOP_PREDICT (=0: the last batch's ratio alone): parity tests, then a bench A/B
set -o pipefail
O=gpurun_out/${TAG:-r6l}
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_V0_$r.log 2>&1 || exit 1
  MOBHEAT_COOP_PREDICT=0 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_P0_$r.log 2>&1 || exit 1
done
echo done
