# Round 5: the stage API's self-held records (the rank's own bins merged from its slabs) -- GPU tests of the stage
# path, then the sharded N=1 bench (RCCL world 1) with self-held records and with them packed (MOBHEAT_STAGE_SELF=copy),
# interleaved, and the direct bench once.
set -o pipefail
O=gpurun_out/${TAG:-r5self}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_rccl.py tests/test_gpu_sharded_stream.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --sharded --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_sharded_held_$r.log 2>&1 || exit 1
  MOBHEAT_STAGE_SELF=copy timeout -k 10 300 python3 bench.py --sharded --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_sharded_copy_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_direct.log 2>&1 || exit 1
echo done
