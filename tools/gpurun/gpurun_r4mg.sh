# Round 4: the multi-GPU path on one GPU -- the stage API tests, the sharded writer, the gloo N=2 bench rehearsal beside
# its N=1 twin -- then the single-GPU parity tests.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4mg}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_stages.py tests/test_gpu_sharded_stream.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 && \
MOBHEAT_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 2 --events 20000000 --no-state-leg > $O/bench_n2.log 2>&1 && \
timeout -k 10 120 python3 bench.py --gpus 1 --steps 4 --warmup 2 --events 20000000 --no-cpu-baseline --no-state-leg > $O/bench_n1_small.log 2>&1 && \
if [ -n "$MORE" ]; then timeout -k 10 900 python -u -m pytest $MORE -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests2.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
