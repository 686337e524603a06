# Rehearsal of bench.py's N>1 path on a 1-GPU box: 2 ranks sharing cuda:0 (gloo: RCCL refuses two ranks on one device), small batches.
set -o pipefail
O=gpurun_out/${TAG:-dist}
mkdir -p $O
export TMPDIR=/tmp
MOBHEAT_DIST_BACKEND=${BACKEND:-gloo} timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 1 --events ${EVENTS:-10000000} > $O/bench_n2.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
