# Bench under environment settings (one per line of $SWEEP, "name VAR=value ...",
# e.g. QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=exp_libs/head/libqkd_ldpc_amd.so for another build), the
# whole list REPS times. Optional parity subset first ($PARITY_K, a pytest -k
# expression run with the in-tree library). Each GPU step time-limited; a
# crash or timeout ends the script.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=${REPS:-1}
if [ -n "${PARITY_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${PARITY_FILES:-tests} -m gpu -q -x --timeout 120 --timeout-method thread \
    -k "$PARITY_K" > gpurun_out/sweep_parity.log 2>&1
  rc=$?; echo "parity rc=$rc $(tail -n 1 gpurun_out/sweep_parity.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for r in $(seq $REPS); do
echo "$SWEEP" | while read -r name rest; do
  [ -z "$name" ] && continue
  env $rest timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-e2e --steps 20 ${BENCH_EXTRA:-} \
    > gpurun_out/sweep_$name.log 2>&1 || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/sweep_$name.log').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['speculation']['replayed_frames'], d.get('phase_share',''))"
done || exit $?
done
