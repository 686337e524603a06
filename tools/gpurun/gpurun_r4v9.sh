# Round 4: binning variant V9 (csrc/variants/libmobheat_V9.so: k_bin_rows on a second stream behind each ingest chunk)
# : its parity tests, then the bench interleaved with the product library.
set -o pipefail
O=gpurun_out/${TAG:-r4v7}
mkdir -p $O
export TMPDIR=/tmp
L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_V9.so
MOBHEAT_LIB=$L timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_full_size.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/test_V9.log 2>&1
rc=$?; echo "V9 tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V0_$r.log 2>&1 || exit 1
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V9_$r.log 2>&1 || exit 1
done
echo done
