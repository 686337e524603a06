# Round 4: two-pass binning variant (csrc/variants/libmobheat_V6.so: coarse bins in k_ingest, k_bin_split): its binned
# parity tests, then the bench interleaved with the product library.  A test failure (rc 1) skips the bench of V6.
set -o pipefail
O=gpurun_out/${TAG:-r4v6}
mkdir -p $O
export TMPDIR=/tmp
L6=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_V6.so
MOBHEAT_LIB=$L6 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stages.py tests/test_gpu_full_size.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread -rf > $O/test_V6.log 2>&1
rc=$?; echo "V6 tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V0_$r.log 2>&1 || exit 1
  MOBHEAT_LIB=$L6 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_V6_$r.log 2>&1 || exit 1
done
echo done
