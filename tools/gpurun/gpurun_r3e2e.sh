# Round 3: PCIe-inclusive boundary rates (tools/e2e_bench.py): host-input hm_process_batch with the chunked H2D on a
# copy stream, foreach_batch_func on the raw Kafka values (device JSON decode) and on pandas frames, both through
# the loopback wire sink.
set -o pipefail
O=gpurun_out/${TAG:-r3e2e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/e2e_bench.py --events 100000000 --steps 4 > $O/e2e_host.log 2>&1 && \
timeout -k 10 300 python3 tools/e2e_bench.py --kafka --events 10000000 > $O/e2e_kafka.log 2>&1 && \
timeout -k 10 300 python3 tools/e2e_bench.py --foreach --events 10000000 > $O/e2e_foreach.log 2>&1
rc=$?; echo "done rc=$rc"; tail -3 $O/e2e_host.log | cut -c1-400; tail -3 $O/e2e_kafka.log | cut -c1-400; tail -3 $O/e2e_foreach.log | cut -c1-400; exit $rc
