# near-tie diagnostic, then k_merge_owned ablation: bench's per-stage times with variant builds (tools/ablate_merge.sh)
set -o pipefail
O=gpurun_out/${TAG:-mabl}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/diag/neartie_gpu.py > $O/neartie.log 2>&1 || exit $?
for v in base ${VARIANTS:-nofence norows noslot noslotrows}; do
  if [ $v = base ]; then L=""; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_abl_$v.so; fi
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:---no-state-leg} > $O/bench_$v.log 2>&1 || exit $?
done
echo "done rc=0"
