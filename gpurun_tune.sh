set -o pipefail
mkdir -p gpurun_out/tune
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/tune/counters.txt 2>&1 || true
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 python $B > gpurun_out/tune/base.json 2>gpurun_out/tune/base.err && \
for w in 3 4 5; do
  MOBHEAT_LIB=$PWD/real-time-mobility-heatmap_amd/csrc/variants/libmobheat_w$w.so timeout -k 10 300 python $B > gpurun_out/tune/w$w.json 2>gpurun_out/tune/w$w.err || exit 1
done && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/tune/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_sq.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/tune/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/tune/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tune/pmc_write.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
