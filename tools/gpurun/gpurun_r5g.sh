# Round 5: the sharded writer on device columns (gloo on one GPU, RCCL at world 1) and the Arrow/Spark column tests.
set -o pipefail
O=gpurun_out/${TAG:-r5g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests/test_gpu_sharded_stream.py tests/test_gpu_rccl.py tests/test_gpu_arrow_columns.py tests/test_gpu_kafka.py -m gpu -x -v -p no:cacheprovider --timeout 170 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
