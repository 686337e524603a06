# Round 5: the RCCL world-1 tests (one record exchange in rounds), then the sharded N=1 bench at 1e8 events (its first
# run faulted with one 3.2-GB all_to_all), then the default bench.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r5e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 5 60 ./tools/microbench/bin_chunk 100000000 coop > $O/bin_coop.txt 2>&1 && timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_rccl.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --sharded > $O/bench_sharded.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --sharded > $O/bench_sharded10.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
