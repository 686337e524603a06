# Quick GPU pass (round 4): parity tests (TESTS), smoke, the bench without its CPU baseline (skipped with NOBENCH=1).
set -o pipefail
O=gpurun_out/${TAG:-r4c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
if [ -z "$NOBENCH" ]; then timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
