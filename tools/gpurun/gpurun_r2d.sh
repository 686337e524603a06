# GPU tests from a given file on (FROM), then bench with the state-read leg and the C3 shard check
set -o pipefail
O=gpurun_out/${TAG:-r2d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf ${PYARGS} > $O/gpu_tests.log 2>&1 && \
timeout -k 10 400 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 && \
timeout -k 10 300 python3 tools/scale_check.py --config c3 > $O/c3.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
