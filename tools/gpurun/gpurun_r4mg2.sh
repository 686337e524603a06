# Round 4: the merge's grid -- one workgroup per bin (default) vs 512 / 1024 persistent workgroups looping over the bins
# (MOBHEAT_MERGE_GRID), bench interleaved twice.
set -o pipefail
O=gpurun_out/${TAG:-r4mg2}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for g in 0 512 1024; do
    MOBHEAT_MERGE_GRID=$g timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_g${g}_$r.log 2>&1 || exit 1
  done
done
echo done
