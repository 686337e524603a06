set -o pipefail
O=gpurun_out/${TAG:-step}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -rf > $O/gpu_tests.log 2>&1 && \
for v in base x87_plain trig_cheap face1 no_rot no_digits x87_plain_trig_cheap; do
  timeout -k 10 120 tools/h3bench/build/h3bench_$v 100000000 8 5 >> $O/h3bench.jsonl || exit 1
done && \
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
