# GPU: key-generator A/B over library builds (exp_libs/<name>/, tools/ab_build.sh):
# each build's keygen parity tests, then the end-to-end bench alternating builds.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/kglibs
mkdir -p $O
export TMPDIR=/tmp
LIBS="base ${LIBS:-$(ls exp_libs)}"
libpath() { [ "$1" = base ] && echo qkd_ldpc_amd/lib/libqkd_ldpc_amd.so || echo exp_libs/$1/libqkd_ldpc_amd.so; }
for l in $LIBS; do
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    --timeout 120 --timeout-method thread -k "keygen or trials or config2" > $O/parity_$l.log 2>&1
  rc=$?; echo "$l parity rc=$rc $(tail -n 1 $O/parity_$l.log)"
  [ $rc -eq 0 ] || { tail -30 $O/parity_$l.log; exit $rc; }
done
for r in $(seq ${REPS:-2}); do
  for l in $LIBS; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants \
      --no-sweeps --steps 20 > $O/bench_$l.json 2> $O/bench_$l.err || { tail $O/bench_$l.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/bench_$l.json').read().strip().splitlines()[-1])
print('$l', 'step', round(d['ms_per_step'],4), 'e2e', round(d['end_to_end']['ms_per_step'],4))"
  done
done
