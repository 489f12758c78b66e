# GPU-box check: the -m gpu suite, then the bench (no CPU baseline), then the
# bench with per-phase clocks. Each GPU step under its own time limit; a crash,
# abort or timeout ends the script.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAILED|form [45]|pass [01]:|headroom" gpurun_out/pytest_gpu.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])
print('headline ms', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'e2e', d.get('end_to_end',{}).get('ms_per_step'))
for k,v in d.get('variants',{}).items(): print(k, v['kernel_ms'], v['fer'], v['mean_iterations'])"
QKD_PHASE_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --no-e2e > gpurun_out/phase.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/phase.log').read().strip().splitlines()[-1]);print(d['phase_share'], d['ms_per_step'])"
exit $rc
