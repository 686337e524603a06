# Focused debug run: one test file (TESTS) with HIP error logging.
set -o pipefail
O=gpurun_out/${TAG:-dbg}
mkdir -p $O
export TMPDIR=/tmp
AMD_LOG_LEVEL=${LOGLVL:-1} timeout -k 10 300 python -u -m pytest ${TESTS} -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf -s > $O/dbg.log 2>&1
rc=$?; echo "done rc=$rc"; tail -50 $O/dbg.log; exit $rc
