# Round 5: the end-to-end boundary after the device-column fixes (dictionary insert, pinned checkpoint export, pandas
# strings by _strcols).  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r5f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/e2e_bench.py --foreach --events 10000000 --steps 4 ${E2E_CASES:+--cases $E2E_CASES} > $O/e2e_foreach.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
