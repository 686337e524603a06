# Round 4: merge variant V7 (csrc/variants/libmobheat_V7.so: the next chunk's window parameters loaded with the store
# drain): its parity tests, then the bench interleaved with the product library.
set -o pipefail
O=gpurun_out/${TAG:-r4v7}
mkdir -p $O
export TMPDIR=/tmp
L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_V7.so
MOBHEAT_LIB=$L timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/test_V7.log 2>&1
rc=$?; echo "V7 tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V0_$r.log 2>&1 || exit 1
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V7_$r.log 2>&1 || exit 1
done
echo done
