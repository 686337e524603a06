# PMC passes over the merge-side kernels (one bench run per pass) for each library variant in $VARIANTS.
set -o pipefail
O=gpurun_out/${TAG:-pmc}
mkdir -p $O
export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 3 --no-cpu-baseline"
R='k_merge_owned|k_rows_compact|k_rp_scatter|k_rp_hist|k_ingest|k_dedup_flag'
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
  export MOBHEAT_LIB=$L
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $O/$v/sq -o run --output-format csv -- $P > $O/${v}_sq.log 2>&1 || { echo "sq pass $v failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc FETCH_SIZE -d $O/$v/fetch -o run --output-format csv -- $P > $O/${v}_fetch.log 2>&1 || { echo "fetch pass $v failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$R" --pmc WRITE_SIZE -d $O/$v/write -o run --output-format csv -- $P > $O/${v}_write.log 2>&1 || { echo "write pass $v failed"; exit 1; }
  python3 tools/pmc_summary.py $O/$v/sq $O/$v/fetch $O/$v/write > $O/${v}_summary.txt 2>&1
done
echo "done"
