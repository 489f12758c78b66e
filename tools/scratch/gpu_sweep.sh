#!/bin/bash
# Run bench.py once per value of an environment knob: VAR="1 2 3" tools/gpu_sweep.sh NAME
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
name=$1; shift
for v in ${VALS}; do
  echo "== $name=$v"
  env "$name=$v" timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 "$@" > "$OUT/sweep_${name}_$v.log" 2>&1
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('$OUT/sweep_${name}_$v.log').read().strip().splitlines()[-1]); print('value %.4g ms/step %.3f kernel_ms %.3f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))" || tail -5 "$OUT/sweep_${name}_$v.log"
  if [ $rc -ne 0 ]; then echo "rc=$rc stop"; exit $rc; fi
done
