# Round 6 full pass: GPU tests, smoke, kernel-trace stats of the bench, PMC passes of its first leg + the counter
# calibration on k_ingest's patterns -> profiles/r5/kernel_pmc.json (bench.py's roofline traffic, calibrated), the
# default bench (CPU baselines with C1) with the PMC file in place, the sharded N=1 bench over RCCL, the gloo N=2
# rehearsal beside its N=1 twin, and foreach_batch_func end to end.  $TAG names the output directory; NOTESTS=1 skips
# the tests, ONLYTESTS=1 stops after the tests and smoke, PART=A after the profiles and the default bench, PART=B
# runs only what follows them (each part fits one gpurun call).
set -o pipefail
O=gpurun_out/${TAG:-r6full}
mkdir -p $O
export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 3 --no-cpu-baseline --no-state-leg"
if [ -z "$NOTESTS" ]; then timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || exit 1; fi
if [ "$PART" != "B" ]; then timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1; fi
if [ -n "$ONLYTESTS" ]; then echo "done tests"; exit 0; fi
if [ "$PART" != "B" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 -d $O/pmc_f64 -o run --output-format csv -- $P > $O/pmc_f64.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc_sq -o run --output-format csv -- $P > $O/pmc_sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $P > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $P > $O/pmc_write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/microbench/pmc_calib > $O/calib_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/microbench/pmc_calib > $O/calib_write.log 2>&1 && \
python3 tools/ingest_pmc.py --res 8 --events 100000000 --out $O/kernel_pmc.json $O/pmc_f64 $O/pmc_sq $O/pmc_fetch $O/pmc_write > $O/ingest_pmc.log 2>&1 && \
python3 tools/pmc_calib.py --calib $O/calib_fetch $O/calib_write --pmc $O/kernel_pmc.json --records 100000000 > $O/pmc_calib.log 2>&1 && \
mkdir -p profiles/r6 && cp $O/kernel_pmc.json profiles/r6/kernel_pmc.json && \
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 && timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 1
if [ "$PART" = "A" ]; then echo "done part A"; exit 0; fi
fi
timeout -k 10 300 python3 bench.py --sharded --steps 8 --warmup 3 --no-cpu-baseline --no-state-leg > $O/bench_sharded.log 2>&1 && \
MOBHEAT_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 2 --events 20000000 --no-state-leg > $O/bench_n2.log 2>&1 && \
timeout -k 10 120 python3 bench.py --gpus 1 --sharded --steps 4 --warmup 2 --events 20000000 --no-cpu-baseline --no-state-leg > $O/bench_n1_small.log 2>&1 && \
timeout -k 10 400 python3 tools/e2e_bench.py --foreach --events 10000000 > $O/e2e_foreach.log 2>&1
rc=$?; echo "done rc=$rc"; exit $rc
