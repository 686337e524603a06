# Round 3: the whole -m gpu suite at the current build, then the default bench twice (state leg with the slowest
# step's host-side breakdown), and a rocprofv3 kernel-stats pass of the bench.
set -o pipefail
O=gpurun_out/${TAG:-r3e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_1.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-state-leg > $O/prof.log 2>&1
rc=$?; echo "done rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -1; tail -2 $O/bench_1.log | cut -c1-300; exit $rc
