# Round 6: the sharded N=1 path over RCCL against the direct path on the same box, interleaved (VERDICT r5 item 6:
# sharded <= 1.05x direct), with the sharded step's kernel times
set -o pipefail
O=gpurun_out/${TAG:-r6s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-state-leg > $O/warmup.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_direct_$r.log 2>&1 || exit 1
  timeout -k 10 300 python3 bench.py --sharded --steps 10 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_sharded_$r.log 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --sharded --steps 6 --warmup 3 --no-cpu-baseline --no-state-leg > $O/prof.log 2>&1 || exit 1
echo done
