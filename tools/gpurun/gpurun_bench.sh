# bench (state-read leg included) + C3 shard check
set -o pipefail
O=gpurun_out/${TAG:-bench}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1 && \
timeout -k 10 300 python3 tools/scale_check.py --config c3 > $O/c3.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
