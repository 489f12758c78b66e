# One GPU call: the -m gpu suite, the per-phase clock shares of the headline
# decoder, and the sp_f64 profile (kernel trace + PMC passes). Outputs under
# gpurun_out/$1.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
QKD_PHASE_TIMING=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-sweeps --no-e2e > $O/phase.json 2>&1 || exit 1
python -c "import json;d=json.loads(open('$O/phase.json').read().strip().splitlines()[-1]);print({k: round(v,3) for k,v in d['phase_share'].items()})"
VARIANTS="${VARIANTS:-sp_f64}" OUT=$O/prof bash tools/gpu_profile.sh || exit $?
