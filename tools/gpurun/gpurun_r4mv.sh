# Round 4: library variants (real-time-mobility-heatmap_amd/csrc/variants/libmobheat_<V>.so, built from patched copies
# of the sources; V0 = the product library) timed by the bench, both legs.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4mv}
mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-V0 V1 V3}; do
  L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so
  [ "$v" = V0 ] && L=real-time-mobility-heatmap_amd/csrc/libmobheat.so
  MOBHEAT_LIB=$L timeout -k 10 400 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
done
rc=$?; echo "done rc=$rc"; exit $rc
