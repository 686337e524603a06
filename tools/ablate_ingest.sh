#!/bin/bash
# Ablation builds of k_ingest (profiling only; never loaded by the product): each removes one component so
# that bench.py's ingest time difference prices it.  Output: real-time-mobility-heatmap_amd/csrc/variants/.
set -e
cd "$(dirname "$0")/../real-time-mobility-heatmap_amd/csrc"
mkdir -p variants
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics -fPIC -shared"
build() { /opt/rocm/bin/hipcc $F $2 -o variants/libmobheat_abl_$1.so mobheat.hip; }
build nodedup "-DHM_ABL_NODEDUP" &
build noagg "-DHM_ABL_NOAGG" &
build nocell "-DHM_ABL_NOCELL" &
build cellsonly "-DHM_ABL_NOAGG -DHM_ABL_NODEDUP" &
build aggonly "-DHM_ABL_NOCELL -DHM_ABL_NODEDUP" &
build norec "-DHM_ABL_NOREC" &
build recnocell "-DHM_ABL_NOREC -DHM_ABL_NOCELL" &
wait
