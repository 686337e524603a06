# Round 5: this round's new GPU tests, then the default bench and the sharded N=1 line over RCCL.  $TAG names the
# output directory.
set -o pipefail
O=gpurun_out/${TAG:-r5b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_spark_frame.py tests/test_gpu_checkpoint.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --sharded > $O/bench_sharded.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --c1-baseline > $O/c1.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
