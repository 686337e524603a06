# Round 4: ingest variants (PMC), merge/library variants (bench), then GPU tests.  $TAG names the output directory.
set -o pipefail
export TAG=${TAG:-r4combo}
VARIANTS="${IVARIANTS:-B C}" TESTS="" bash tools/gpurun/gpurun_r4var.sh && \
VARIANTS="${MVARIANTS:-V0 V1 V3}" bash tools/gpurun/gpurun_r4mv.sh && \
if [ -n "$TESTS" ]; then timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/$TAG/gpu_tests.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
