# Round-5 profile call: rocprofv3 kernel trace + PMC passes (tools/gpu_profile.sh,
# VARIANTS as given) and the per-phase shader-clock shares. Outputs under $OUT.
set -u
cd "$(dirname "$0")/.."
export OUT=${OUT:-gpurun_out/r05prof}
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 100); do sleep 30; date >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/gpu_profile.sh > $OUT/profile.log 2>&1 || { tail -30 $OUT/profile.log; exit 1; }
tail -5 $OUT/profile.log
QKD_PHASE_TIMING=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-sweeps --no-variants --no-e2e --steps 20 > $OUT/phase.json 2> $OUT/phase.err || { tail $OUT/phase.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/phase.json').read().strip().splitlines()[-1]);print('phase', {k: round(v,4) for k,v in d['phase_share'].items()})"
