#!/bin/bash
# Diagnostic: decode-kernel time of experiment builds (exp_libs/lib_*.so, built with
# QKD_EXP_* macros) on config 2 with a fixed iteration count.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
IT=${IT:-3}
for l in exp_libs/lib_*.so; do
  n=$(basename "$l" .so)
  QKD_AMD_LIB=$PWD/$l QKD_PHASE_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --max-iters $IT --steps 5 > "$OUT/exp_$n.json" 2> "$OUT/exp_$n.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open('$OUT/exp_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['roofline']['kernel_ms'],3), {k: round(v,3) for k,v in d.get('phase_share',{}).items()})"
done
