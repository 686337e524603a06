# k_ingest ablation: bench's per-stage times with variant builds (tools/ablate_ingest.sh)
set -o pipefail
O=gpurun_out/${TAG:-abl}
mkdir -p $O
export TMPDIR=/tmp
for v in base ${VARIANTS:-nodedup nocell bare}; do
  if [ $v = base ]; then L=""; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_abl_$v.so; fi
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-state-leg > $O/bench_$v.log 2>&1 || exit $?
done
echo "done rc=0"
