# Round 4: the GPU tests the host-side changes touch (state files, batch columns, sinks, sharded stream), then the
# end-to-end foreach_batch_func run.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_checkpoint.py tests/test_gpu_sharded_stream.py tests/test_gpu_sink.py tests/test_gpu_kafka.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 tools/e2e_bench.py --foreach --events 10000000 > $O/e2e_foreach.log 2>&1
rc2=$?; echo "e2e rc=$rc2"; exit $(( rc > rc2 ? rc : rc2 ))
