# Round 6: the concurrency probe (tools/diag/overlap_probe.py) and the GPU tests touched by this round's first commit
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag/overlap_probe.py > $O/probe.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
echo done
