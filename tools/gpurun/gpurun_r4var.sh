# Round 4: k_ingest variants (tools/diag/ingest_phases_{A,B,C}: resolution specialised with the digit loop unrolled /
# rolled, and the generic kernel) under one PMC pass each, then GPU tests ($TESTS).  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4var}
mkdir -p $O
export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-A B C}; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $P -d $O/phases_$v -o run --output-format csv -- ./tools/diag/ingest_phases_$v > $O/phases_$v.log 2>&1 || exit 1
  python3 tools/diag/ingest_phases.py $O/phases_$v > $O/phases_$v.txt 2>&1 || exit 1
done
if [ -n "$TESTS" ]; then timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
