# A/B of experimental builds of the library (exp_libs/<name>/libqkd_ldpc_amd.so,
# scratch, git-ignored) against the in-tree one: a quick parity subset and the
# headline bench, alternating builds, REPS rounds. Each GPU step time-limited;
# a crash or timeout ends the script.
set -u
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=${REPS:-3}
LIBS="base ${LIBS:-$(ls exp_libs)}"
libpath() { [ "$1" = base ] && echo qkd_ldpc_amd/lib/libqkd_ldpc_amd.so || echo exp_libs/$1/libqkd_ldpc_amd.so; }
for l in $LIBS; do
  [ "$l" = base ] && continue
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 300 python -u -m pytest tests/test_spec.py -q -x --timeout 120 \
    -k "config2_every_cap or fresh_frames or bits_match_oracle" > gpurun_out/ab_parity_$l.log 2>&1
  rc=$?; echo "$l parity rc=$rc $(tail -n 1 gpurun_out/ab_parity_$l.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for r in $(seq $REPS); do
  for l in $LIBS; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-e2e --steps 20 \
      ${BENCH_EXTRA:-} > gpurun_out/ab_$l.log 2>&1 || exit $?
    python -c "
import json,sys;d=json.loads(open('gpurun_out/ab_$l.log').read().strip().splitlines()[-1])
print('$l', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['speculation']['replayed_frames'])"
  done
done
