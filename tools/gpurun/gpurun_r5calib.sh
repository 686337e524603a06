# Round 5: FETCH_SIZE / WRITE_SIZE calibration on k_ingest<true>'s access patterns (tools/microbench/pmc_calib), one
# counter pass each.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r5calib}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/microbench/pmc_calib > $O/calib_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/microbench/pmc_calib > $O/calib_write.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
