# A/B of the k_ingest LDS table size (HM_LA_SLOTS) on C3 (LDS mode) and the bench (direct mode), one box
set -o pipefail
O=gpurun_out/${TAG:-las}
mkdir -p $O
export TMPDIR=/tmp
for v in default s1024_w4 s2048_w4 s2048_w2; do
  if [ $v = default ]; then L=; else L=$PWD/real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
  MOBHEAT_LIB=$L timeout -k 10 200 python3 tools/scale_check.py --config c3 > $O/c3_$v.log 2>&1 || exit 1
  MOBHEAT_LIB=$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
done
echo "done"
