#!/bin/bash
# Ablation builds of k_merge_owned (profiling only; never loaded by the product): each removes one component so
# that bench.py's merge time difference prices it.  Output: real-time-mobility-heatmap_amd/csrc/variants/.
set -e
cd "$(dirname "$0")/../real-time-mobility-heatmap_amd/csrc"
mkdir -p variants
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics -fPIC -shared"
build() { /opt/rocm/bin/hipcc $F $2 -o variants/libmobheat_abl_$1.so mobheat.hip; }
build nofence "-DHM_ABL_NOFENCE" &
build norows "-DHM_ABL_NOROWS" &
build noslot "-DHM_ABL_NOSLOT" &
build noslotrows "-DHM_ABL_NOSLOT -DHM_ABL_NOROWS" &
wait
