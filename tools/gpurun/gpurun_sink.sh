# Sink encoder: GPU tests (sink + checkpoint + boundary), the throughput tool, and its kernel-trace profile
set -o pipefail
O=gpurun_out/${TAG:-sink}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sink.py tests/test_gpu_checkpoint.py tests/test_gpu_parity.py::test_foreach_batch_func_capture_sink -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/gpu_sink_tests.log 2>&1 && \
timeout -k 10 300 python3 tools/sink_bench.py > $O/sink_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/sink_bench.py --reps 3 --sample 1000 > $O/sink_prof.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
