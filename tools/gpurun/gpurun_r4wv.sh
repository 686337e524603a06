# Round 4: k_ingest at 7 and 8 waves per SIMD (variants W7 / W8: 72 / 64 VGPRs, with spills) against the product's 6,
# bench interleaved twice (the bench leg only).
set -o pipefail
O=gpurun_out/${TAG:-r4wv}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in V0 W7 W8; do
    L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so
    [ "$v" = V0 ] && L=real-time-mobility-heatmap_amd/csrc/libmobheat.so
    MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_${v}_$r.log 2>&1 || exit 1
  done
done
echo done
