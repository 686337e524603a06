# Round 4: the binned-write microbenchmark (tools/microbench/bin_scatter) timed, then its HBM traffic per kernel
# (FETCH_SIZE and WRITE_SIZE in separate PMC passes).  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4bs}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/bin_scatter > $O/bin_scatter.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- ./tools/microbench/bin_scatter > $O/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- ./tools/microbench/bin_scatter > $O/pmc_write.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
