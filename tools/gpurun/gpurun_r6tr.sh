# Round 6: kernel-trace timelines of one bench step, unpipelined vs pipelined ($PIPES)
set -o pipefail
O=gpurun_out/${TAG:-r6tr}
mkdir -p $O
export TMPDIR=/tmp
for p in ${PIPES:-0 2}; do
  MOBHEAT_PIPELINE=$p timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p$p -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-state-leg > $O/tr_p$p.log 2>&1 || exit 1
  DB=$(find $O/tr_p$p -name "*.db" | head -1)
  python3 tools/trace_timeline.py "$DB" --anchor k_batch_reset --step -2 --min-gap-us 5 > $O/timeline_p$p.txt 2>&1 || exit 1
  rm -f "$DB"
done
echo done
