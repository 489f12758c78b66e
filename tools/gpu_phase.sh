# GPU: per-phase shader-clock shares of the headline decoder (QKD_PHASE_TIMING=1)
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-phase}
mkdir -p $O
QKD_PHASE_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --no-sweeps --no-e2e --steps 10 > $O/phase.json 2> $O/phase.err || { tail $O/phase.err; exit 1; }
python -c "
import json;d=json.loads(open('$O/phase.json').read().strip().splitlines()[-1])
print({k: round(v,4) for k,v in d['phase_share'].items()})"
