# Overlap experiment: k_ingest and k_ev_scatter_rec alone and on two streams together (experiment build
# variants/libmobheat_exp.so, -DHM_EXP_OVERLAP), then the usual A/B (tools/gpurun/gpurun_r3ab.sh).
set -o pipefail
O=gpurun_out/${TAG:-r3ov}
mkdir -p $O
export TMPDIR=/tmp
MOBHEAT_EXP_OVERLAP=1 MOBHEAT_LIB=real-time-mobility-heatmap_amd/csrc/variants/libmobheat_exp.so timeout -k 10 200 \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-state-leg > $O/exp_overlap.log 2>&1 || { echo "exp failed"; tail -20 $O/exp_overlap.log; exit 1; }
grep exp_overlap $O/exp_overlap.log
bash tools/gpurun/gpurun_r3ab.sh
