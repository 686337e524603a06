# Round 4: foreach_batch_func end to end (default configuration: checkpoints on; wire and null sinks), the raw Kafka
# value path, then the bench in its default configuration.  $TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-r4e2e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/e2e_bench.py --foreach --events 10000000 > $O/e2e_foreach.log 2>&1 && \
timeout -k 10 300 python3 tools/e2e_bench.py --kafka --events 10000000 > $O/e2e_kafka.log 2>&1 && \
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
