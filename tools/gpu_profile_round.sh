#!/bin/bash
# Round profile of the shipped decoder: rocprofv3 kernel stats of the bench,
# then the PMC passes of tools/gpu_pmc.sh and tools/gpu_pmc2.sh. Each step has
# its own time limit; a failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -n 20 "$OUT/prof.log"; exit 3; }
tail -n 1 "$OUT/prof.log"
bash tools/gpu_pmc.sh || exit $?
bash tools/gpu_pmc2.sh || exit $?
echo "== done"
