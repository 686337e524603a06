# kernel-trace stats of the bench (and optionally of the C3 check): $TAG names the output directory
set -o pipefail
O=gpurun_out/${TAG:-prof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/prof.log 2>&1 && \
if [ -n "$C3" ]; then timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 tools/scale_check.py --config c3 > $O/prof_c3.log 2>&1; fi
rc=$?; echo "done rc=$rc"; exit $rc
