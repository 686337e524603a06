# Checkpoint tests + traced C5 (allocation timeline of the first 5e8-event batch)
set -o pipefail
O=gpurun_out/${TAG:-ckpt}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_checkpoint.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/gpu_ckpt_tests.log 2>&1 && \
MOBHEAT_TRACE=1 timeout -k 10 300 python3 tools/scale_check.py --config c5 > $O/c5_trace.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
