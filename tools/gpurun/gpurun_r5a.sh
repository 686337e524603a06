# Round 5: the RCCL world-1 tests, then the default bench (this round's baseline on this box) and the sharded N=1 line
# over RCCL.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r5a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_rccl.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --sharded > $O/bench_sharded.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench2.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
