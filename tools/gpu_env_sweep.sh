# Bench under environment settings (one per line of $SWEEP, "name VAR=value ...").
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "$SWEEP" | while read -r name rest; do
  [ -z "$name" ] && continue
  env $rest timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-e2e --steps 20 ${BENCH_EXTRA:-} \
    > gpurun_out/sweep_$name.log 2>&1 || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/sweep_$name.log').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['speculation']['replayed_frames'], d.get('phase_share',''))"
done
