# Round 4: packed base-cell tables in k_ingest's LDS (the product library) against the build before (variant P):
# ingest cell and parity tests of the product, its VALU phases, then the bench interleaved.
set -o pipefail
O=gpurun_out/${TAG:-r4pk}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/test.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
P="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $P -d $O/phases -o run --output-format csv -- ./tools/diag/ingest_phases > $O/phases.log 2>&1 || exit 1
python3 tools/diag/ingest_phases.py $O/phases > $O/phases.txt 2>&1 || exit 1
L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_P.so
for r in 1 2; do
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_P_$r.log 2>&1 || exit 1
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_new_$r.log 2>&1 || exit 1
done
echo done
