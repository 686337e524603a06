# Round 4: the per-resolution ingest cell test and the bench for the product library and variants ($VARIANTS:
# csrc/variants/libmobheat_<V>.so; V0 = the product).  A test failure (rc 1) goes on to the next library; any other
# non-zero status (time limit, abort, fault) ends the script.
set -o pipefail
O=gpurun_out/${TAG:-r4w}
mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-V0 G A}; do
  L=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_$v.so
  [ "$v" = V0 ] && L=real-time-mobility-heatmap_amd/csrc/libmobheat.so
  MOBHEAT_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ingest_cells_every_resolution or state_read_regime" -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/test_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  MOBHEAT_LIB=$L timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_$v.log 2>&1 || exit 1
done
echo done
