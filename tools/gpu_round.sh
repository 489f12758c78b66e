# One GPU call: the whole -m gpu suite, smoke, the default bench line (all
# measurements), and the VALU issue microbenchmark. Outputs under gpurun_out/$TAG.
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
# a heartbeat under gpurun_out/ while the steps run (each step has its own limit)
( for i in $(seq 80); do sleep 30; date >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -x tools/mb/issue_mb ]; then
  timeout -k 10 120 ./tools/mb/issue_mb > $O/issue_mb.txt 2>&1 || { cat $O/issue_mb.txt; exit 1; }
  head -40 $O/issue_mb.txt
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_brief.py $O/bench.json
