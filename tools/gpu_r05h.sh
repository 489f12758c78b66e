# Round-5 call: parity of the prefetching prologue, A/B against HEAD and the
# no-prefetch build, the issue microbenchmark, long-code iteration histograms.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_spec.py tests/test_large_codes.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
LIBS="head nopf" REPS=3 bash tools/gpu_ab.sh || exit 1
timeout -k 10 120 tools/mb/issue_mb > $O/issue_mb.txt 2>&1 || exit 1
grep "waves/SIMD  4.0" $O/issue_mb.txt | grep -E "cndmask|v_add_f32|v_mov"
for q in 0.02 0.03; do
  timeout -k 10 200 python tools/large_code_bench.py --qber $q > $O/lc_$q.json 2> $O/lc_$q.err || { tail $O/lc_$q.err; exit 1; }
  cat $O/lc_$q.json
done
