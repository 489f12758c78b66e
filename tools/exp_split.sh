#!/bin/bash
# Diagnostic runs of tools/exp_build.sh libraries (fixed IT iterations) and of
# the split kernel's LDS budget (QKD_SPLIT_BUDGET: fewer LDS slots).
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
bash tools/exp_run.sh || exit $?
for b in 163840 120000 80000 40000 20000; do
  QKD_AMD_LIB=$PWD/exp_libs/lib_base.so QKD_SPLIT_BUDGET=$b timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --max-iters 3 --steps 5 > "$OUT/budget_$b.json" 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/budget_$b.json').read().strip().splitlines()[-1]); print('budget $b', round(d['roofline']['kernel_ms'],3))"
done
