#!/bin/bash
# Diagnostic: decode time vs resident workgroups (QKD_DECODE_GRID) for the
# split decoder, binary64 and binary32 rules, and vs the LDS budget.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for v in sp_f64 sp_f32; do
  for g in 256 224 192 160 128; do
    QKD_DECODE_GRID=$g timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --variant $v --steps 5 > "$OUT/grid_${v}_$g.json" 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$OUT/grid_${v}_$g.json').read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$v grid $g', round(k,3), 'per-CU-frame us', round(k*1e3*$g/4096,2))"
  done
done
