#!/bin/bash
# Decode time per 4096-frame batch with and without the speculative interval
# iterations (QKD_SPEC_CAP=0), across QBER; the default policy decides between
# speculating from the first iteration and from a checkpoint (decode_keys).
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for q in ${QS:-0.02 0.03 0.04 0.05 0.06 0.07 0.08}; do
  for cap in 0 8; do
    QKD_SPEC_CAP=$cap timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --no-e2e --qber $q --steps 8 > "$OUT/spec_${q}_$cap.json" 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$OUT/spec_${q}_$cap.json').read().strip().splitlines()[-1]); print('q $q cap $cap', round(d['roofline']['kernel_ms'],3), 'ms, mean it', round(d['mean_iterations'],3), 'replays', d.get('speculation'))"
  done
done
