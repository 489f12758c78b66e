# A/B of experimental library builds (exp_libs/<name>/, tools/ab_build.sh)
# against the in-tree one on one GPU: a parity subset per build, then the
# headline bench alternating builds for REPS rounds (decoder-kernel and step
# times). Every GPU step has its own time limit; a failure ends the script.
set -u
cd "$(dirname "$0")/.."
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
REPS=${REPS:-3}
LIBS="base ${LIBS:-$(ls exp_libs)}"
# a name "lib@NAME=value" runs build `lib` with that library debug option
# (qkd_debug_set_option, passed as bench.py --debug-opt; its parity subset
# runs without it)
libpath() { local b=${1%%@*}; [ "$b" = base ] && echo qkd_ldpc_amd/lib/libqkd_ldpc_amd.so || echo exp_libs/$b/libqkd_ldpc_amd.so; }
libopt() { case "$1" in *@*) echo "--debug-opt ${1#*@}";; *) echo "";; esac; }
for l in $LIBS; do
  QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 300 python -u -m pytest tests/test_spec.py -q -x \
    --timeout 120 --timeout-method thread -k "${PARITY_K:-config2_every_cap or bits_match_oracle}" > $O/parity_$l.log 2>&1
  rc=$?; echo "$l parity rc=$rc $(tail -n 1 $O/parity_$l.log)"
  [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
done
for r in $(seq $REPS); do
  for l in $LIBS; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants \
      --no-sweeps --steps 20 $(libopt $l) ${BENCH_EXTRA:-} > $O/bench_$l.json 2> $O/bench_$l.err || { tail $O/bench_$l.err; exit 1; }
    python -c "
import json;d=json.loads(open('$O/bench_$l.json').read().strip().splitlines()[-1])
print('$l', 'step', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'call', round(d['roofline']['call_ms'],4), 'e2e', round(d['end_to_end']['ms_per_step'],4) if 'end_to_end' in d else '', 'replays', d['speculation']['replayed_frames'])"
  done
done
# PMC="WRITE_SIZE" (one counter group): per build, one rocprofv3 --pmc pass over a
# short bench; the decode kernel's mean counter values per dispatch
if [ -n "${PMC:-}" ]; then
  for l in $LIBS; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv \
      -d $O/pmc_$l -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-e2e \
      --no-sweeps $(libopt $l) > $O/pmc_$l.log 2>&1 || { echo "pmc $l failed"; tail $O/pmc_$l.log; exit 1; }
    python3 - $O/pmc_$l $l ${PMC_KERNEL:-decode} <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[3] in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(x) / len(x)) for k, x in v.items()})
PY
  done
fi
# TRACE=1: per build, one rocprofv3 --kernel-trace pass over a short bench (with
# the end-to-end line); warm per-kernel averages (tools/prof_summary.py)
if [ -n "${TRACE:-}" ]; then
  for l in $LIBS; do
    QKD_AMD_DIAGNOSTIC=1 QKD_AMD_LIB=$(libpath $l) timeout -k 10 300 rocprofv3 --kernel-trace \
      --output-format csv -d $O/trace_$l -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      --no-variants --no-sweeps $(libopt $l) > $O/trace_$l.log 2>&1 || { echo "trace $l failed"; tail $O/trace_$l.log; exit 1; }
    f=$(find $O/trace_$l -name "run_kernel_trace.csv" | head -1)
    python3 tools/prof_summary.py "$(dirname $f)" $O/trace_$l.json && python3 - $O/trace_$l.json $l <<'PY'
import json, sys
for r in json.load(open(sys.argv[1]))["kernels"][:8]:
    print(sys.argv[2], f"{r['warm_avg_ms']*1e3:9.1f} us x{r['warm_dispatches']:4d}", r["kernel"][:90])
PY
  done
fi
