# Round 3: default bench, bench.py's N=2 path rehearsed on one GPU (two gloo ranks; RCCL refuses two ranks on one
# device) with its N=1 twin at the same per-rank size, and the host->device bandwidth microbenchmark.
set -o pipefail
O=gpurun_out/${TAG:-r3d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 && \
MOBHEAT_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 2 --events ${EVENTS:-20000000} > $O/bench_n2.log 2>&1 && \
timeout -k 10 120 python3 bench.py --gpus 1 --steps 4 --warmup 2 --events ${EVENTS:-20000000} --no-cpu-baseline --no-state-leg > $O/bench_n1_small.log 2>&1 && \
timeout -k 10 120 ./tools/microbench/h2d_bw $((1<<30)) > $O/h2d.log 2>&1
rc=$?; echo "done rc=$rc"; tail -3 $O/bench.log; cat $O/h2d.log | tail -20; exit $rc
