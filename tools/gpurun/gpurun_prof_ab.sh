set -o pipefail
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
for v in default prev; do
  if [ "$v" = default ]; then L=; else L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so; fi
  MOBHEAT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline > $O/$v.log 2>&1 || exit 1
done
echo done
