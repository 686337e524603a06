set -o pipefail
mkdir -p gpurun_out/tune
export TMPDIR=/tmp
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -rf > gpurun_out/tune/gpu_tests.log 2>&1 && \
timeout -k 10 300 python $B > gpurun_out/tune/base.json 2>gpurun_out/tune/base.err && \
MOBHEAT_MERGE=atomic timeout -k 10 300 python $B > gpurun_out/tune/atomic.json 2>gpurun_out/tune/atomic.err
rc=$?; echo "done rc=$rc"; exit $rc
