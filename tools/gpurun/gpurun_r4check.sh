# Quick GPU pass (round 4): parity tests, smoke, the bench without its CPU baseline.
set -o pipefail
O=gpurun_out/${TAG:-r4c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
