# Round 5: an environment-switch A/B with a throwaway warm-up run first (the first bench process on a fresh box runs
# up to ~20% slow) and the order alternating per round (A B, B A, ...): $ENVA vs $ENVB, $ROUNDS rounds.
set -o pipefail
O=gpurun_out/${TAG:-r5env2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-3}); do
  if [ $((r % 2)) -eq 1 ]; then first=A; second=B; else first=B; second=A; fi
  for v in $first $second; do
    if [ $v = A ]; then E="$ENVA"; else E="$ENVB"; fi
    env $E timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline $BENCHARGS > $O/bench_${v}_$r.log 2>&1 || exit 1
  done
done
echo done
