#!/bin/bash
# Headline bench (decode call time) of the in-tree library and each exp_libs/lib_*.so.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for l in base exp_libs/lib_*.so; do
  n=$(basename "$l" .so)
  if [ "$l" = base ]; then unset QKD_AMD_LIB; else export QKD_AMD_LIB=$PWD/$l; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --steps 10 > "$OUT/exp_$n.json" 2>&1 || exit $?
  echo "$n $(grep -o '"kernel_ms": [0-9.]*' $OUT/exp_$n.json) $(grep -o '"replayed_frames": [0-9]*' $OUT/exp_$n.json)"
done
