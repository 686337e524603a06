# Round 2 first pass: GPU parity tests, a short bench, the C3 shard check.
set -o pipefail
O=gpurun_out/${TAG:-r2a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 && \
timeout -k 10 300 python3 tools/scale_check.py --config c3 > $O/c3.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
