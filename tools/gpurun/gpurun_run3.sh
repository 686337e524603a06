set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1f}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -rf > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
