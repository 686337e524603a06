#!/bin/bash
# Builds kernel variants of libmobheat.so from patch files, so that every A/B this repo reports can be rebuilt:
#   tools/variants/build.sh NAME...      -> real-time-mobility-heatmap_amd/csrc/variants/libmobheat_NAME.so
# NAME.patch (this directory) is a unified diff against the product sources at the commit named in its header line
# ("# base: <commit>"); it is applied with `patch -p1` to a copy of csrc/ and include/ (git apply --directory style
# paths: a/real-time-mobility-heatmap_amd/csrc/...).  Select a build at run time with MOBHEAT_LIB=<path>.
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/real-time-mobility-heatmap_amd/csrc/variants
mkdir -p "$OUT"
for v in "$@"; do
  P=$ROOT/tools/variants/$v.patch
  [ -f "$P" ] || { echo "no $P"; exit 1; }
  W=$(mktemp -d /tmp/mobheat_var_XXXX)
  mkdir -p "$W/real-time-mobility-heatmap_amd"
  cp -r "$ROOT/real-time-mobility-heatmap_amd/csrc" "$W/real-time-mobility-heatmap_amd/"
  cp -r "$ROOT/include" "$W/"
  rm -rf "$W/real-time-mobility-heatmap_amd/csrc/variants" "$W"/real-time-mobility-heatmap_amd/csrc/*.so
  (cd "$W" && patch -s -p1 < "$P")
  make -s -C "$W/real-time-mobility-heatmap_amd/csrc" libmobheat.so
  cp "$W/real-time-mobility-heatmap_amd/csrc/libmobheat.so" "$OUT/libmobheat_$v.so"
  rm -rf "$W"
  echo "built $OUT/libmobheat_$v.so"
done
