# Round 3 baseline on a fresh box: GPU tests, then the default bench (with CPU baseline and state leg).
set -o pipefail
O=gpurun_out/${TAG:-r3base}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
