# Round 4: the product k_ingest's VALU phases (tools/diag/ingest_phases, one PMC pass), the bench with the product
# library and the merge variants (csrc/variants/), then GPU tests ($TESTS).  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4j}
mkdir -p $O
export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $P -d $O/phases -o run --output-format csv -- ./tools/diag/ingest_phases > $O/phases.log 2>&1 || exit 1
python3 tools/diag/ingest_phases.py $O/phases > $O/phases.txt 2>&1 || exit 1
for v in ${MVARIANTS:-V0 V1 V3}; do
  L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so
  [ "$v" = V0 ] && L=real-time-mobility-heatmap_amd/csrc/libmobheat.so
  MOBHEAT_LIB=$L timeout -k 10 400 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
done
if [ -n "$TESTS" ]; then timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
