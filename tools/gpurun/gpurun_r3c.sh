# Allocation-free steady-state test + host->device bandwidth microbenchmark.
set -o pipefail
O=gpurun_out/${TAG:-r3c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py::test_steady_state_batches_allocate_nothing -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf -s > $O/alloc.log 2>&1 &&
timeout -k 10 120 ./tools/microbench/h2d_bw $((1<<30)) > $O/h2d.log 2>&1
rc=$?; echo "done rc=$rc"; grep -a "passed\|failed\|Assert\|allocations" $O/alloc.log; cat $O/h2d.log; exit $rc
