# Round-5 call: the frame-interleaved decoder's parity tests, then the
# long-code bench with it on and off.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_large_codes.py -x -v -k "interleaved" \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in 1 0; do
  QKD_ILV=$m timeout -k 10 200 python tools/large_code_bench.py --qber 0.02 > $O/lc_ilv$m.json 2> $O/lc_ilv$m.err || { tail $O/lc_ilv$m.err; exit 1; }
  cat $O/lc_ilv$m.json
done
