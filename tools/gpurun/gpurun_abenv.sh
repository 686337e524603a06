# A/B of environment settings on the default build: CASES="name:VAR=val,VAR2=val name2:..." (interleaved ROUNDS times)
# -> bench.py per-stage times per case; optional PMC pass (PMC="counters") on the first case's bench command.
set -o pipefail
O=gpurun_out/${TAG:-abenv}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CASES:-base:}; do
    name=${c%%:*}; envs=${c#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:---no-state-leg} > $O/bench_${name}_$r.log 2>&1 || exit $?
  done
done
if [ -n "$PMC" ]; then
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PMC -d $O/pmc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-state-leg > $O/pmc.log 2>&1 || exit $?
fi
echo "done rc=0"
