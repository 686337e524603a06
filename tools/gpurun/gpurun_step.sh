# GPU parity (all GPU tests) + a bench run (no CPU baseline) + kernel-trace stats of a short bench
set -o pipefail
O=gpurun_out/${TAG:-step}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
