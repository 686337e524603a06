# Round 3: the whole -m gpu suite alone (bench in gpurun_r3d.sh).
set -o pipefail
O=gpurun_out/${TAG:-r3t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf --durations=25 > $O/gpu_tests.log 2>&1
rc=$?; echo "done rc=$rc"; tail -40 $O/gpu_tests.log; exit $rc
