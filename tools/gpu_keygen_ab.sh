# GPU: the whole -m gpu suite, then end-to-end bench A/B of the key generators
# (default two-wave kernel vs QKD_KEYGEN=lanes, the one-wave kernel), alternating.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-kgab}
mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 60); do sleep 30; date >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
for r in 1 2; do
  for m in split lanes; do
    if [ $m = lanes ]; then export QKD_KEYGEN=lanes; else unset QKD_KEYGEN; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --no-sweeps --steps 20 > $O/bench_$m.json 2> $O/bench_$m.err || { tail $O/bench_$m.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/bench_$m.json').read().strip().splitlines()[-1])
print('$m', 'step', round(d['ms_per_step'],4), 'e2e', round(d['end_to_end']['ms_per_step'],4), round(d['end_to_end']['value']/1e9,2), 'Gbit/s')"
  done
done
unset QKD_KEYGEN
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-variants --no-sweeps --steps 10 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof $O/kernel_summary.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/kernel_summary.json'))
for k in d['kernels'][:6]: print(round(k['warm_avg_ms'],4), k['dispatches'], k['kernel'][:70])"
