# Round 5: the binning microbenchmark (one process per pattern), this round's new GPU tests, the end-to-end boundary
# (foreach_batch_func: pandas / Arrow frames, device / host columns, wire / null sinks, 1e7 events), and the sharded N=1
# bench line over RCCL.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r5c}
mkdir -p $O
export TMPDIR=/tmp
for m in ${MB_MODES:-seq direct atomics pre xcdpre chunkx chunk}; do
  timeout -k 5 40 ./tools/microbench/bin_chunk 100000000 $m >> $O/bin_chunk.txt 2>&1 || { echo "$m failed rc=$?" >> $O/bin_chunk.txt; break; }
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_arrow_columns.py tests/test_gpu_spark_frame.py tests/test_gpu_rccl.py tests/test_gpu_checkpoint.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/e2e_bench.py --foreach --events 10000000 --steps 4 > $O/e2e_foreach.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --sharded > $O/bench_sharded.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
