set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r03d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_brief.py $O/bench.json
QKD_PHASE_TIMING=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-sweeps --no-e2e > $O/phase.json 2>&1 || exit 1
python -c "import json;d=json.loads(open('$O/phase.json').read().strip().splitlines()[-1]);print({k: round(v,3) for k,v in d['phase_share'].items()})"
VARIANTS="${VARIANTS:-sp_f64}" OUT=$O/prof bash tools/gpu_profile.sh || exit $?
