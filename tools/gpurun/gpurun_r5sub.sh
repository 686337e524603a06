# Round 5: sub-bins (k_ingest bins by region field and sub-region; the merge takes a bin's sub-slabs in order) --
# GPU tests, then the bench with sub-bins ($SUBMODE: MOBHEAT_SUBBINS, default adaptive) and without (=0), interleaved.
set -o pipefail
O=gpurun_out/${TAG:-r5sub}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_checkpoint.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  MOBHEAT_SUBBINS=${SUBMODE:-2} timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_sub_$r.log 2>&1 || exit 1
  MOBHEAT_SUBBINS=0 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_whole_$r.log 2>&1 || exit 1
done
echo done
