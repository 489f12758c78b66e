#!/bin/bash
# GPU-box round check: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/abort/timeout (rc >= 2 other than
# an ordinary pytest failure) ends the script before any further GPU step.
set -u
cd "$(dirname "$0")/../.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name, stopping"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-"tests smoke bench prof"}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
  esac
done
echo "== done"
