# k_ingest instruction counts (one SQ PMC pass per library variant in $VARIANTS; ablation builds: tools/ablate_ingest.sh)
set -o pipefail
O=gpurun_out/${TAG:-pmcabl}
mkdir -p $O
export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 3 --no-cpu-baseline"
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
  export MOBHEAT_LIB=$L
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "k_ingest" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d $O/$v/sq -o run --output-format csv -- $P > $O/${v}_sq.log 2>&1 || { echo "sq pass $v failed"; exit 1; }
  python3 tools/pmc_summary.py $O/$v/sq > $O/${v}_summary.txt 2>&1
done
echo "done"
