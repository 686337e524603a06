# Round 4: parity tests (TESTS), smoke, the bench, its kernel-trace stats, and the VALU-rate microbenchmark under the
# SQ counters k_ingest's issue fraction is read with.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4p}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/prof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAVES -d $O/valu -o run --output-format csv -- ./tools/microbench/valu_rate > $O/valu.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
