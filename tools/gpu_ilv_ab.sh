# A/B of interleaved-decoder builds (exp_libs/<name>) on the long-code bench
# (N = 40000, QBER 0.02, 4096 frames), alternating, after a parity subset.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ilv_ab
mkdir -p $O
export TMPDIR=/tmp
LIBS="base ${LIBS:-$(ls exp_libs)}"
libpath() { [ "$1" = base ] && echo qkd_ldpc_amd/lib/libqkd_ldpc_amd.so || echo exp_libs/$1/libqkd_ldpc_amd.so; }
for l in $LIBS; do
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 300 python -u -m pytest tests/test_large_codes.py -q -x \
    -k "interleaved" --timeout 200 --timeout-method thread > $O/parity_$l.log 2>&1 || { echo "$l parity failed"; tail -20 $O/parity_$l.log; exit 1; }
  echo "$l parity $(tail -n 1 $O/parity_$l.log)"
done
for r in $(seq ${REPS:-2}); do
  for l in $LIBS; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 200 python tools/large_code_bench.py --qber 0.02 --debug-opt QKD_ILV=1 \
      > $O/lc_$l.json 2> $O/lc_$l.err || { tail $O/lc_$l.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/lc_$l.json').read().strip().splitlines()[-1]);print('$l', round(d['ms_per_batch'],3))"
  done
done
