# Round 5: the dense dedup table -- GPU parity / stage tests, then the bench with it and without it
# (MOBHEAT_DEDUP_DENSE=0: the hash table for every vkey), interleaved.
set -o pipefail
O=gpurun_out/${TAG:-r5dense}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_stages.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_dense_$r.log 2>&1 || exit 1
  MOBHEAT_DEDUP_DENSE=0 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_hash_$r.log 2>&1 || exit 1
done
echo done
