set -o pipefail
O=gpurun_out/r5pad; mkdir -p $O; export TMPDIR=/tmp
L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_merge_ldspad.so
MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in 1 2; do
  for pad in 0 24576; do
    MOBHEAT_LIB=$L MOBHEAT_MERGE_LDS_PAD=$pad timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_pad${pad}_$r.log 2>&1 || exit 1
  done
done
echo done
