#!/bin/bash
# Diagnostic: headline bench (phase timing) of each exp_libs/lib_*.so build.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for l in exp_libs/lib_*.so; do
  n=$(basename "$l" .so)
  QKD_AMD_LIB=$PWD/$l QKD_PHASE_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --steps 10 > "$OUT/exp2_$n.json" 2> "$OUT/exp2_$n.err" || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/exp2_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['roofline']['kernel_ms'],3), {k: round(v,3) for k,v in d.get('phase_share',{}).items()})"
done
